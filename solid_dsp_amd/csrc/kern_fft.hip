// Batched FFT and the PFB + FFT channeliser (gfx950).
//
// FFT semantics (src/fft/mod.rs:175-215): FORWARD X[k] = sum_n x[n] e^{-j2pi nk/N},
// REVERSE with e^{+j...}, neither normalised.  The reference plans power-of-two
// sizes as recursive mixed radix over hard-coded DFT leaves; on the device a
// power-of-two transform is a radix-4 (+ one radix-2) Stockham autosort FFT in
// LDS with an exact f64-computed twiddle table, and any other size uses a
// direct DFT with the same table.  Results agree with the reference within
// its own accuracy (its DFT16 constants are truncated to ~1e-8).
//
// Channeliser (build-defined composition):
//   v_p[m] = sum_{i<K} cb[p][i] * x[(m-i)M + (M-1-p)],  cb[p][i] = h[p+(K-1-i)M]
//   X[m]   = FFT_M(v[m])
// one workgroup per (frame, stream); the branch dot products write v straight
// into the LDS buffer the FFT runs in.
#include <cstdlib>

#include "sdsp_device.hpp"
#include "sdsp_kernels.hpp"

namespace sdsp {

template <typename T> struct c2 { T re, im; };
template <typename T> __device__ __forceinline__ c2<T> ca(c2<T> a, c2<T> b) { return {a.re + b.re, a.im + b.im}; }
template <typename T> __device__ __forceinline__ c2<T> cs(c2<T> a, c2<T> b) { return {a.re - b.re, a.im - b.im}; }
template <typename T> __device__ __forceinline__ c2<T> cm(c2<T> a, c2<T> b) {
    return {a.re * b.re - a.im * b.im, a.re * b.im + a.im * b.re};
}
template <typename T, bool INV> __device__ __forceinline__ c2<T> twl(const c2<T>* __restrict__ tw, int m) {
    c2<T> w = tw[m];
    if constexpr (INV) w.im = -w.im;
    return w;
}
template <typename T, bool INV> __device__ __forceinline__ c2<T> rot(c2<T> a) {  // *(-j) fwd, *(+j) inv
    if constexpr (INV) return {-a.im, a.re};
    else return {a.im, -a.re};
}

// Stockham passes on an LDS transform `a` (natural order in), result in `a` or
// `b` (returned).  `lane` in [0, nthr), nthr threads cooperate on this transform.
template <typename T, bool INV>
__device__ c2<T>* stockham(c2<T>* a, c2<T>* b, int N, int logN, const c2<T>* __restrict__ tw, int lane, int nthr) {
    int Ns = 1;
    if (logN & 1) {  // one radix-2 pass
        for (int j = lane; j < N / 2; j += nthr) {
            const c2<T> v0 = a[j], v1 = a[j + N / 2];
            // Ns = 1: no twiddle
            b[2 * j] = ca(v0, v1);
            b[2 * j + 1] = cs(v0, v1);
        }
        __syncthreads();
        c2<T>* t = a; a = b; b = t;
        Ns = 2;
    }
    for (; Ns < N; Ns *= 4) {
        for (int j = lane; j < N / 4; j += nthr) {
            const int k = j % Ns;
            const int stride = N / (Ns * 4);  // twiddle index step
            c2<T> v0 = a[j], v1 = a[j + N / 4], v2 = a[j + N / 2], v3 = a[j + 3 * (N / 4)];
            if (Ns > 1) {
                v1 = cm(v1, twl<T, INV>(tw, (1 * k * stride) & (N - 1)));
                v2 = cm(v2, twl<T, INV>(tw, (2 * k * stride) & (N - 1)));
                v3 = cm(v3, twl<T, INV>(tw, (3 * k * stride) & (N - 1)));
            }
            const c2<T> s02 = ca(v0, v2), d02 = cs(v0, v2), s13 = ca(v1, v3), d13 = rot<T, INV>(cs(v1, v3));
            const int o = (j / Ns) * Ns * 4 + k;
            b[o] = ca(s02, s13);
            b[o + Ns] = ca(d02, d13);
            b[o + 2 * Ns] = cs(s02, s13);
            b[o + 3 * Ns] = cs(d02, d13);
        }
        __syncthreads();
        c2<T>* t = a; a = b; b = t;
    }
    return a;
}

// batched power-of-two FFT: block = `tpb` transforms of N points, nthr threads each
template <typename T, bool INV>
__global__ void __launch_bounds__(1024)
fft_pow2_kernel(const c2<T>* __restrict__ x, c2<T>* __restrict__ y, const c2<T>* __restrict__ tw, int N, int logN,
                long long batch, int nthr, int tpb) {
    extern __shared__ __attribute__((aligned(16))) char lds_raw[];
    c2<T>* buf = reinterpret_cast<c2<T>*>(lds_raw);
    const int sub = threadIdx.x / nthr, lane = threadIdx.x % nthr;
    const long long tr = (long long)blockIdx.x * tpb + sub;
    c2<T>* a = buf + (size_t)sub * 2 * N;
    c2<T>* b = a + N;
    if (tr < batch)
        for (int i = lane; i < N; i += nthr) a[i] = x[tr * N + i];
    __syncthreads();
    c2<T>* r = stockham<T, INV>(a, b, N, logN, tw, lane, nthr);
    if (tr < batch)
        for (int i = lane; i < N; i += nthr) y[tr * N + i] = r[i];
}

// direct DFT for sizes that are not powers of two: one thread per output bin
template <typename T, bool INV>
__global__ void __launch_bounds__(256)
dft_direct_kernel(const c2<T>* __restrict__ x, c2<T>* __restrict__ y, const c2<T>* __restrict__ tw, int N,
                  long long batch) {
    const long long tr = blockIdx.y;
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (tr >= batch || k >= N) return;
    const c2<T>* xi = x + tr * N;
    c2<T> acc = {T(0), T(0)};
    int m = 0;  // (n k) mod N, advanced incrementally
    for (int n = 0; n < N; ++n) {
        acc = ca(acc, cm(xi[n], twl<T, INV>(tw, m)));
        m += k;
        if (m >= N) m -= N;
    }
    y[tr * N + k] = acc;
}

// channeliser: block (frame m, stream s); M = N power of two
template <typename T>
__global__ void __launch_bounds__(256)
chan_kernel(const c2<T>* __restrict__ x, const c2<T>* __restrict__ hist, const T* __restrict__ cb,
            c2<T>* __restrict__ y, const c2<T>* __restrict__ tw, int M, int logM, int K, long long n) {
    extern __shared__ __attribute__((aligned(16))) char lds_raw[];
    c2<T>* a = reinterpret_cast<c2<T>*>(lds_raw);
    c2<T>* b = a + M;
    const long long m = blockIdx.x;
    const int s = blockIdx.y;
    x += (long long)s * n;
    const long long H = (long long)(K - 1) * M;
    hist += (long long)s * H;
    y += (long long)s * n + m * M;
    for (int p = threadIdx.x; p < M; p += blockDim.x) {
        const T* c = cb + (long long)p * K;
        c2<T> acc = {T(0), T(0)};
        for (int i = 0; i < K; ++i) {
            const long long j = (m - i) * M + (M - 1 - p);
            const c2<T> v = j >= 0 ? x[j] : hist[H + j];
            acc = ca(acc, c2<T>{c[i] * v.re, c[i] * v.im});
        }
        a[p] = acc;
    }
    __syncthreads();
    c2<T>* r = stockham<T, false>(a, b, M, logM, tw, threadIdx.x, blockDim.x);
    for (int c = threadIdx.x; c < M; c += blockDim.x) y[c] = r[c];
}

// Strided pass of the four-step FFT (power-of-two N = N1 N2 > 4096, both factors
// <= 4096): transform t of L points reads element i at
//   x[(t / G) S0 + (t % G) S1 + i Si]  and writes  y[(t / G) S0 + (t % G) T1 + i So],
// times W_Ntw^{(t % G) i} when TW (the inter-pass twiddle, from f64 sincospi of
// the exact phase (t % G) i mod Ntw).  A workgroup runs `tpb` consecutive
// transforms (tpb divides G): when their elements interleave with unit stride
// (S1 == 1 or T1 == 1) the group loads / stores them with consecutive lanes on
// consecutive transforms, so every wave touches 8 * tpb-byte runs instead of one
// 8-byte element per row.
template <typename T, bool INV, bool TW>
__global__ void __launch_bounds__(1024)
fft_pass_kernel(const c2<T>* __restrict__ x, c2<T>* __restrict__ y, const c2<T>* __restrict__ tw, int L, int logL,
                long long count, long long G, long long S0, long long S1, long long Si, long long T1, long long So,
                long long Ntw, int nthr, int tpb) {
    extern __shared__ __attribute__((aligned(16))) char lds_raw[];
    c2<T>* buf = reinterpret_cast<c2<T>*>(lds_raw);
    const int sub = threadIdx.x / nthr, lane = threadIdx.x % nthr;
    const int nth = blockDim.x, tot = tpb * L;
    const int ltpb = __builtin_ctz(tpb);  // tpb and L are powers of two
    const long long t0 = (long long)blockIdx.x * tpb;
    const long long g0 = t0 % G;
    const long long ib = (t0 / G) * S0 + g0 * S1, ob = (t0 / G) * S0 + g0 * T1;
    const int ntr = count - t0 < tpb ? (int)(count - t0) : tpb;
    if (S1 == 1) {
        for (int e = threadIdx.x; e < tot; e += nth) {
            const int c = e & (tpb - 1), i = e >> ltpb;
            if (c < ntr) buf[(size_t)c * 2 * L + i] = x[ib + c + i * Si];
        }
    } else {
        for (int e = threadIdx.x; e < tot; e += nth) {
            const int i = e & (L - 1), c = e >> logL;
            if (c < ntr) buf[(size_t)c * 2 * L + i] = x[ib + c * S1 + i * Si];
        }
    }
    __syncthreads();
    c2<T>* a = buf + (size_t)sub * 2 * L;
    c2<T>* r = stockham<T, INV>(a, a + L, L, logL, tw, lane, nthr);
    const int roff = (int)(r - a);  // 0 or L, the same for every transform of the group
    auto out = [&](int c, int i) {
        c2<T> v = buf[(size_t)c * 2 * L + roff + i];
        if constexpr (TW) {
            const long long m = ((g0 + c) * (long long)i) & (Ntw - 1);  // Ntw = N, a power of two
            double sn, cs;
            sincospi((INV ? 2.0 : -2.0) * (double)m / (double)Ntw, &sn, &cs);
            v = cm(v, c2<T>{(T)cs, (T)sn});
        }
        y[ob + c * T1 + i * So] = v;
    };
    if (T1 == 1) {
        for (int e = threadIdx.x; e < tot; e += nth) {
            const int c = e & (tpb - 1), i = e >> ltpb;
            if (c < ntr) out(c, i);
        }
    } else {
        for (int e = threadIdx.x; e < tot; e += nth) {
            const int i = e & (L - 1), c = e >> logL;
            if (c < ntr) out(c, i);
        }
    }
}

// Bluestein (chirp-z) steps for sizes that are not powers of two: w[n] = the
// chirp of the transform direction, B = FFT_M(conj chirp, wrapped) / M
template <typename T>
__global__ void bluestein_in_kernel(const c2<T>* __restrict__ x, c2<T>* __restrict__ a, const c2<T>* __restrict__ w,
                                    long long N, long long M, long long batch) {
    const long long total = batch * M;
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
         i += (long long)gridDim.x * blockDim.x) {
        const long long b = i / M, m = i % M;
        a[i] = m < N ? cm(x[b * N + m], w[m]) : c2<T>{T(0), T(0)};
    }
}
template <typename T>
__global__ void bluestein_mul_kernel(c2<T>* __restrict__ a, const c2<T>* __restrict__ B, long long M, long long batch) {
    const long long total = batch * M;
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
         i += (long long)gridDim.x * blockDim.x)
        a[i] = cm(a[i], B[i % M]);
}
template <typename T>
__global__ void bluestein_out_kernel(const c2<T>* __restrict__ a, c2<T>* __restrict__ y, const c2<T>* __restrict__ w,
                                     long long N, long long M, long long batch) {
    const long long total = batch * N;
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
         i += (long long)gridDim.x * blockDim.x) {
        const long long b = i / N, k = i % N;
        y[i] = cm(a[b * M + k], w[k]);
    }
}

// ---------------------------------------------------------------- launchers
template <typename T>
hipError_t launch_fft_pass_t(const FftPass& p, hipStream_t s) {
    const int L = p.L;
    // transforms per workgroup: up to kMaxGroup interleaved transforms in <= kLdsCap
    // bytes of LDS (two L-point buffers each), dividing G; <= 1024 threads
    const int kMaxGroup = p.group >= 1 && p.group <= 64 ? p.group : 4;
    constexpr size_t kLdsCap = 128 * 1024;
    const size_t per = 2 * (size_t)L * sizeof(c2<T>);
    int tpb = 1;
    while (tpb * 2 <= kMaxGroup && (size_t)tpb * 2 * per <= kLdsCap && p.G % (tpb * 2) == 0) tpb *= 2;
    int nthr = L >= 4 ? L / 4 : 1;
    while (nthr * tpb > 1024) nthr /= 2;
    const size_t lds = (size_t)tpb * per;
    dim3 grid((unsigned)((p.count + tpb - 1) / tpb));
#define SDSP_PASS(INV, TW)                                                                                       \
    hipLaunchKernelGGL((fft_pass_kernel<T, INV, TW>), grid, dim3(nthr * tpb), lds, s, (const c2<T>*)p.x,          \
                       (c2<T>*)p.y, (const c2<T>*)p.tw, L, p.logL, p.count, p.G, p.S0, p.S1, p.Si, p.T1, p.So, p.Ntw, \
                       nthr, tpb)
    if (p.inverse) {
        if (p.Ntw) SDSP_PASS(true, true); else SDSP_PASS(true, false);
    } else {
        if (p.Ntw) SDSP_PASS(false, true); else SDSP_PASS(false, false);
    }
#undef SDSP_PASS
    return hipGetLastError();
}

hipError_t launch_fft_pass(bool f64, const FftPass& p, hipStream_t s) {
    if (p.count == 0) return hipSuccess;
    hipError_t err;
    if (!f64 && try_launch_fft1024_pass(p, s, &err)) return err;  // L = 1024 on the wave FFT
    return f64 ? launch_fft_pass_t<double>(p, s) : launch_fft_pass_t<float>(p, s);
}

hipError_t launch_bluestein(bool f64, int step, const void* in, void* out, const void* w_or_B, long long N, long long M,
                            long long batch, hipStream_t s) {
    const long long total = batch * (step == 2 ? N : M);
    long long blocks = (total + 255) / 256;
    if (blocks > 65536) blocks = 65536;
    dim3 grid((unsigned)blocks);
#define SDSP_BLU(T)                                                                                               \
    do {                                                                                                          \
        if (step == 0)                                                                                            \
            hipLaunchKernelGGL(bluestein_in_kernel<T>, grid, dim3(256), 0, s, (const c2<T>*)in, (c2<T>*)out,      \
                               (const c2<T>*)w_or_B, N, M, batch);                                                \
        else if (step == 1)                                                                                       \
            hipLaunchKernelGGL(bluestein_mul_kernel<T>, grid, dim3(256), 0, s, (c2<T>*)out, (const c2<T>*)w_or_B, \
                               M, batch);                                                                         \
        else                                                                                                      \
            hipLaunchKernelGGL(bluestein_out_kernel<T>, grid, dim3(256), 0, s, (const c2<T>*)in, (c2<T>*)out,     \
                               (const c2<T>*)w_or_B, N, M, batch);                                                \
    } while (0)
    if (f64) SDSP_BLU(double);
    else SDSP_BLU(float);
#undef SDSP_BLU
    return hipGetLastError();
}

template <typename T>
hipError_t launch_fft_t(const FftArgs& a, hipStream_t s) {
    const int N = a.N;
    if (a.pow2) {
        const int nthr = N >= 4 ? N / 4 : 1;
        const int tpb = nthr >= 256 ? 1 : 256 / nthr;
        const size_t lds = (size_t)tpb * 2 * N * sizeof(c2<T>);
        dim3 grid((unsigned)((a.batch + tpb - 1) / tpb));
        if (a.inverse)
            hipLaunchKernelGGL((fft_pow2_kernel<T, true>), grid, dim3(nthr * tpb), lds, s, (const c2<T>*)a.x,
                               (c2<T>*)a.y, (const c2<T>*)a.tw, N, a.logN, (long long)a.batch, nthr, tpb);
        else
            hipLaunchKernelGGL((fft_pow2_kernel<T, false>), grid, dim3(nthr * tpb), lds, s, (const c2<T>*)a.x,
                               (c2<T>*)a.y, (const c2<T>*)a.tw, N, a.logN, (long long)a.batch, nthr, tpb);
    } else {
        dim3 grid((unsigned)((N + 255) / 256), (unsigned)a.batch);
        if (a.inverse)
            hipLaunchKernelGGL((dft_direct_kernel<T, true>), grid, dim3(256), 0, s, (const c2<T>*)a.x, (c2<T>*)a.y,
                               (const c2<T>*)a.tw, N, (long long)a.batch);
        else
            hipLaunchKernelGGL((dft_direct_kernel<T, false>), grid, dim3(256), 0, s, (const c2<T>*)a.x, (c2<T>*)a.y,
                               (const c2<T>*)a.tw, N, (long long)a.batch);
    }
    return hipGetLastError();
}

hipError_t launch_fft(bool f64, const FftArgs& a, hipStream_t s) {
    if (a.batch == 0) return hipSuccess;
    return f64 ? launch_fft_t<double>(a, s) : launch_fft_t<float>(a, s);
}

template <typename T>
hipError_t launch_chan_t(const ChanArgs& a, hipStream_t s) {
    const size_t lds = 2 * (size_t)a.M * sizeof(c2<T>);
    const int thr = a.M >= 1024 ? 256 : (a.M >= 256 ? a.M / 4 : 64);
    dim3 grid((unsigned)a.frames, (unsigned)a.streams);
    hipLaunchKernelGGL((chan_kernel<T>), grid, dim3(thr), lds, s, (const c2<T>*)a.x, (const c2<T>*)a.hist,
                       (const T*)a.cb, (c2<T>*)a.y, (const c2<T>*)a.tw, a.M, a.logM, a.K, (long long)a.n);
    return hipGetLastError();
}

hipError_t launch_chan(bool f64, const ChanArgs& a, hipStream_t s) {
    if (a.frames == 0) return hipSuccess;
    hipError_t err;
    if (!f64 && try_launch_chan1024(a, s, &err)) return err;
    return f64 ? launch_chan_t<double>(a, s) : launch_chan_t<float>(a, s);
}

}  // namespace sdsp
