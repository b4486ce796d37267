// Receive-chain kernels next to the filter path:
//   * AutoCorrelator  src/filter/auto_correlator/mod.rs:26-214
//   * NCO mixing      src/nco/mod.rs:94-172
//
// AutoCorrelator.  After pushing x[n] the reference returns
//     execute() = sum_{j < W} window[j] * delayed[j]     (:156-163)
// with window[j] = x[n - j] and delayed[j] = conj(x[n - j - d]) for j + d < W and
// 0 otherwise: the delayed Window keeps W + d zeroed slots but shifts only the
// first W - 1 (src/window/mod.rs:63-71), so its tail slots [W, W + d) stay zero.
// With K = max(W - d, 0) the sum is
//     y[n] = (((0 + p[n]) + p[n-1]) + ...) + p[n-K+1],   p[m] = x[m] * conj(x[m-d]),
// the zero-product terms j >= K leave the sum unchanged (it starts at +0 and is
// never -0).  Each workgroup owns 256 consecutive outputs; p over the window the
// outputs need is built once in LDS (one num-complex product per input, the
// reference's rounding) and every lane adds its K terms newest first, in chunks
// of kChunk so W is unbounded.  Bit-identical to the restatement at the handle's
// precision; HBM traffic is one read of x and one write of y per sample.
//
// energy (:106-111, :212-214) is the sum of |x|^2 over the last W inputs; the
// reference keeps it as a running f64 sum (add the new e2, subtract the one
// leaving).  One workgroup per channel re-sums the last W e2 values in f64.
//
// NCO.  theta_i = theta_0 + i * dtheta (u32, wrapping, :94-96); the phasor is
// (table[(idx + 256) & 1023], table[idx]), idx = ((theta + 2^21) >> 22) & 1023
// (:99-121) from the handle's 1024-entry f64 sine table, staged in LDS;
// mix_up = phasor * x, mix_down = conj(phasor) * x (num-complex Mul).
#include "sdsp_device.hpp"
#include "sdsp_kernels.hpp"

namespace sdsp {

namespace {

constexpr int kTile = 256;    // outputs per workgroup
constexpr int kChunk = 1024;  // j-terms staged per pass

template <typename T> __device__ inline cpx<T> conj_(cpx<T> a) { return {a.re, -a.im}; }

template <typename T>
__device__ inline cpx<T> ext_at(const cpx<T>* __restrict__ x, const cpx<T>* __restrict__ hist, long long j, int H) {
    if (j >= 0) return x[j];
    if (j >= -(long long)H) return hist[H + j];
    return zero_v<cpx<T>>();
}

template <typename T>
__global__ void __launch_bounds__(kTile) acorr_kernel(const cpx<T>* __restrict__ x, const cpx<T>* __restrict__ hist,
                                                      cpx<T>* __restrict__ y, long long n, int H, int d, int K) {
    __shared__ cpx<T> p[kTile + kChunk - 1];
    const int ch = blockIdx.y;
    x += (long long)ch * n;
    y += (long long)ch * n;
    hist += (long long)ch * H;
    const int t = threadIdx.x;
    const long long n0 = (long long)blockIdx.x * kTile;
    const long long me = n0 + t;
    cpx<T> acc = zero_v<cpx<T>>();
    for (int j0 = 0; j0 < K; j0 += kChunk) {
        const int cj = K - j0 < kChunk ? K - j0 : kChunk;
        // p[m] for m in [n0 - j0 - cj + 1, n0 + kTile - 1 - j0]: slot s <-> m = base + s
        const long long base = n0 - j0 - cj + 1;
        const int cnt = kTile + cj - 1;
        __syncthreads();  // previous chunk's readers are done
        for (int s = t; s < cnt; s += kTile) {
            const long long m = base + s;
            p[s] = mul_(ext_at(x, hist, m, H), conj_(ext_at(x, hist, m - d, H)));
        }
        __syncthreads();
        // output me adds p[me - j] for j = j0 .. j0 + cj - 1, newest first (slot t + cj - 1 - j)
        const int s0 = t + cj - 1;
#pragma unroll 4
        for (int j = 0; j < cj; ++j) acc = add_(acc, p[s0 - j]);
    }
    if (me < n) y[me] = acc;
}

// execute() on the current window (no push): the output for the newest history sample
template <typename T>
__global__ void acorr_current_kernel(const cpx<T>* __restrict__ hist, cpx<T>* __restrict__ out, int H, int d, int K) {
    const int ch = blockIdx.x;
    hist += (long long)ch * H;
    if (threadIdx.x != 0) return;
    cpx<T> acc = zero_v<cpx<T>>();
    for (int j = 0; j < K; ++j) {
        const long long m = -1 - j;
        acc = add_(acc, mul_(ext_at<T>(nullptr, hist, m, H), conj_(ext_at<T>(nullptr, hist, m - d, H))));
    }
    out[ch] = acc;
}

// sum of e2 = (x * conj(x)).re over the W newest samples of (hist ++ x), in f64
template <typename T>
__global__ void __launch_bounds__(256) acorr_energy_kernel(const cpx<T>* __restrict__ x, const cpx<T>* __restrict__ hist,
                                                           long long n, int H, int W, double* __restrict__ energy) {
    __shared__ double part[256];
    const int ch = blockIdx.x;
    x += (long long)ch * n;
    hist += (long long)ch * H;
    double s = 0.0;
    for (int i = threadIdx.x; i < W; i += 256) {
        const cpx<T> v = ext_at(x, hist, n - W + i, H);
        s += (double)mul_(v, conj_(v)).re;
    }
    part[threadIdx.x] = s;
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
        if (threadIdx.x < w) part[threadIdx.x] += part[threadIdx.x + w];
        __syncthreads();
    }
    if (threadIdx.x == 0) energy[ch] = part[0];
}

template <typename T, bool DOWN>
__global__ void __launch_bounds__(256) nco_mix_kernel(const cpx<T>* __restrict__ x, cpx<T>* __restrict__ y, long long n,
                                                      const double* __restrict__ table, uint32_t theta0,
                                                      uint32_t dtheta) {
    __shared__ T lut[1024];
    for (int i = threadIdx.x; i < 1024; i += 256) lut[i] = (T)table[i];
    __syncthreads();
    for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
        const uint32_t th = theta0 + (uint32_t)i * dtheta;  // wrapping u32: theta_0 + i dtheta mod 2^32
        const uint32_t idx = ((th + (1u << 21)) >> 22) & 0x3ffu;
        cpx<T> ph = {lut[(idx + 256) & 0x3ffu], lut[idx]};
        if constexpr (DOWN) ph = conj_(ph);
        y[i] = mul_(ph, x[i]);
    }
}

}  // namespace

hipError_t launch_acorr(int prec, const void* x, const void* hist, void* y, size_t n, int H, int d, int K,
                        size_t channels, hipStream_t s) {
    if (n == 0) return hipSuccess;
    dim3 grid((unsigned)((n + kTile - 1) / kTile), (unsigned)channels);
    if (prec == 0)
        hipLaunchKernelGGL(acorr_kernel<float>, grid, dim3(kTile), 0, s, (const c32*)x, (const c32*)hist, (c32*)y,
                           (long long)n, H, d, K);
    else
        hipLaunchKernelGGL(acorr_kernel<double>, grid, dim3(kTile), 0, s, (const c64*)x, (const c64*)hist, (c64*)y,
                           (long long)n, H, d, K);
    return hipGetLastError();
}

hipError_t launch_acorr_current(int prec, const void* hist, void* out, int H, int d, int K, size_t channels,
                                hipStream_t s) {
    if (prec == 0)
        hipLaunchKernelGGL(acorr_current_kernel<float>, dim3((unsigned)channels), dim3(64), 0, s, (const c32*)hist,
                           (c32*)out, H, d, K);
    else
        hipLaunchKernelGGL(acorr_current_kernel<double>, dim3((unsigned)channels), dim3(64), 0, s, (const c64*)hist,
                           (c64*)out, H, d, K);
    return hipGetLastError();
}

hipError_t launch_acorr_energy(int prec, const void* x, const void* hist, size_t n, int H, int W, size_t channels,
                               double* energy, hipStream_t s) {
    if (prec == 0)
        hipLaunchKernelGGL(acorr_energy_kernel<float>, dim3((unsigned)channels), dim3(256), 0, s, (const c32*)x,
                           (const c32*)hist, (long long)n, H, W, energy);
    else
        hipLaunchKernelGGL(acorr_energy_kernel<double>, dim3((unsigned)channels), dim3(256), 0, s, (const c64*)x,
                           (const c64*)hist, (long long)n, H, W, energy);
    return hipGetLastError();
}

hipError_t launch_nco_mix(int prec, bool down, const void* x, void* y, size_t n, const double* table, uint32_t theta0,
                          uint32_t dtheta, int num_cus, hipStream_t s) {
    if (n == 0) return hipSuccess;
    long long blocks = ((long long)n + 255) / 256;
    const long long cap = (long long)num_cus * 16;
    if (blocks > cap) blocks = cap;
    dim3 grid((unsigned)blocks);
#define SDSP_NCO(T, D)                                                                                        \
    hipLaunchKernelGGL((nco_mix_kernel<T, D>), grid, dim3(256), 0, s, (const cpx<T>*)x, (cpx<T>*)y, (long long)n, \
                       table, theta0, dtheta)
    if (prec == 0) {
        if (down) SDSP_NCO(float, true); else SDSP_NCO(float, false);
    } else {
        if (down) SDSP_NCO(double, true); else SDSP_NCO(double, false);
    }
#undef SDSP_NCO
    return hipGetLastError();
}

}  // namespace sdsp
