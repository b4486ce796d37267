// Direct-form FIR and decimating FIR kernels (gfx950).
//
// Semantics (reference: FIRFilter::execute src/filter/fir/mod.rs:209-212 over
// Window::push/to_vec src/window/mod.rs:44-71 and DotProduct::execute
// src/dot_product/mod.rs:159-170):
//     y[n] = (sum_{i=0}^{L-1} cr[i] * x[n-i]) * scale,   cr[i] = h[L-1-i]
// accumulated from zero in increasing i.  With EXACT=true every output is the
// reference's own sequence of rounded multiplies and adds (this TU is built
// with -ffp-contract=off), so results are bit-identical to the reference
// algorithm at the handle's precision.  EXACT=false uses fused multiply-add.
//
// The reference's per-sample memmove delay line becomes an LDS tile: a block
// stages TILE + LC samples of the stream (coalesced), each lane owns R
// adjacent outputs and slides a 2R-sample register window down the tile, so
// one LDS row read feeds R*R multiply-adds.  Samples before the start of the
// block come from the handle's HBM-resident history (the last L-1 inputs of
// the previous call), which is what makes the delay line persist across
// execute_block calls exactly as the reference's Window does.
#include "sdsp_device.hpp"
#include "sdsp_kernels.hpp"

namespace sdsp {

constexpr int kThreads = 256;
constexpr int kLC = 256;  // taps per LDS chunk

template <typename I> struct rows_of { static constexpr int R = sizeof(I) >= 16 ? 4 : 8; };

// LDS image: rows of R samples, each row followed by 16 bytes of padding so
// that lanes reading rows R samples apart hit distinct 16-byte bank slots.
template <typename I> struct LdsImg {
    static constexpr int R = rows_of<I>::R;
    static constexpr int kRowBytes = R * (int)sizeof(I) + 16;
    __device__ static inline I* at(char* base, int s) {
        return reinterpret_cast<I*>(base + (s / R) * kRowBytes + (s % R) * (int)sizeof(I));
    }
    __device__ static inline const I* row(const char* base, int r) {
        return reinterpret_cast<const I*>(base + r * kRowBytes);
    }
};

// extended stream: history (last L-1 samples, oldest first) then x
template <typename I>
__device__ inline I ext_load(const I* __restrict__ x, const I* __restrict__ hist, long long j, long long n, int Lm1) {
    if (j >= 0) return j < n ? x[j] : zero_v<I>();
    long long h = (long long)Lm1 + j;
    return h >= 0 ? hist[h] : zero_v<I>();
}

template <typename C, typename I, bool EXACT>
__global__ void __launch_bounds__(kThreads)
fir_direct_kernel(const I* __restrict__ x, const I* __restrict__ hist, const C* __restrict__ cr,
                  C scale, I* __restrict__ y, long long n, int L) {
    using Img = LdsImg<I>;
    constexpr int R = Img::R;
    constexpr int TILE = kThreads * R;
    constexpr int NS = TILE + kLC;
    extern __shared__ __attribute__((aligned(16))) char lds[];

    const int ch = blockIdx.y;
    x += (long long)ch * n;
    y += (long long)ch * n;
    hist += (long long)ch * (L - 1);
    const long long t0 = (long long)blockIdx.x * TILE;
    const int tid = threadIdx.x;
    const int b = tid * R;

    I acc[R];
#pragma unroll
    for (int r = 0; r < R; ++r) acc[r] = zero_v<I>();

    for (int c0 = 0; c0 < L; c0 += kLC) {
        // stage samples j = t0 - c0 - LC + s, s in [0, NS)
        const long long jbase = t0 - c0 - kLC;
        if (c0) __syncthreads();
        for (int s = tid; s < NS; s += kThreads) *Img::at(lds, s) = ext_load(x, hist, jbase + s, n, L - 1);
        __syncthreads();

        const int taps = min(kLC, L - c0);
        const int full = taps / R;
        I hi[R], lo[R];
        {
            const I* p = Img::row(lds, (b + kLC) / R);
#pragma unroll
            for (int e = 0; e < R; ++e) hi[e] = p[e];
        }
        for (int g = 0; g < full; ++g) {
            const I* p = Img::row(lds, (b + kLC) / R - g - 1);
#pragma unroll
            for (int e = 0; e < R; ++e) lo[e] = p[e];
            const C* cg = cr + c0 + g * R;
#pragma unroll
            for (int q = 0; q < R; ++q) {
                const C tap = cg[q];
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    const int e = R + r - q;
                    acc[r] = mac<EXACT>(acc[r], tap, e < R ? lo[e] : hi[e - R]);
                }
            }
#pragma unroll
            for (int e = 0; e < R; ++e) hi[e] = lo[e];
        }
        const int rem = taps - full * R;
        if (rem) {  // last partial group: taps beyond L are skipped, never multiplied by zero
            const I* p = Img::row(lds, (b + kLC) / R - full - 1);
#pragma unroll
            for (int e = 0; e < R; ++e) lo[e] = p[e];
            const C* cg = cr + c0 + full * R;
#pragma unroll
            for (int q = 0; q < R; ++q) {
                if (q < rem) {
                    const C tap = cg[q];
#pragma unroll
                    for (int r = 0; r < R; ++r) {
                        const int e = R + r - q;
                        acc[r] = mac<EXACT>(acc[r], tap, e < R ? lo[e] : hi[e - R]);
                    }
                }
            }
        }
    }
    const long long o = t0 + b;
    if (o + R <= n) {
#pragma unroll
        for (int r = 0; r < R; ++r) y[o + r] = mul_(acc[r], scale);  // plain: nontemporal +5 %
    } else {
#pragma unroll
        for (int r = 0; r < R; ++r)
            if (o + r < n) y[o + r] = mul_(acc[r], scale);
    }
}

// Decimating FIR: output m sits at block-relative input index j_m = j0 + m*M
// (DecimatingFIRFilter::push advances the phase, emission when it wraps to 0,
// src/filter/fir/decim.rs:115-118,221-228).
//   y[m] = (sum_{i<L} cr[i] * ext(j_m - i)) * scale
// Tap i = k*M + p.  LDS row rho holds the M samples ext(j_{m0} + (rho-K+1)*M - p),
// p = 0..M-1, so lane u reads row u-k+K-1 left to right for tap group k — the
// reference order — and lanes hit rows 16 bytes apart in bank space.
constexpr int kStageU = 16;  // staging loads in flight per lane (32 or 40 measured slower)

template <typename C, typename I, bool EXACT>
__global__ void __launch_bounds__(kThreads)
decim_direct_kernel(const I* __restrict__ x, const I* __restrict__ hist, const C* __restrict__ cr,
                    C scale, I* __restrict__ y, long long n, long long nout, int L, int M, long long j0,
                    int T) {
    extern __shared__ __attribute__((aligned(16))) char lds[];
    const int ch = blockIdx.y;
    x += (long long)ch * n;
    y += (long long)ch * nout;
    hist += (long long)ch * (L - 1);
    const int K = (L + M - 1) / M;
    const int rowBytes = M * (int)sizeof(I) + 16;
    const int rows = T + K - 1;
    const long long m0 = (long long)blockIdx.x * T;
    const long long jm0 = j0 + m0 * M;
    const int tid = threadIdx.x;

    // stage: interior tiles read the contiguous inputs x[base + f] with kStageU loads in
    // flight per lane (f -> row f / M, slot M-1 - f % M); edge tiles go through ext_load
    const long long base = jm0 - (long long)(K - 1) * M - (M - 1);
    const int total = rows * M;
    if (base >= 0 && base + total <= n) {
        for (int f0 = 0; f0 < total; f0 += kStageU * (int)blockDim.x) {
            I v[kStageU];
#pragma unroll
            for (int u = 0; u < kStageU; ++u) {
                const int f = f0 + u * (int)blockDim.x + tid;
                if (f < total) v[u] = x[base + f];
            }
#pragma unroll
            for (int u = 0; u < kStageU; ++u) {
                const int f = f0 + u * (int)blockDim.x + tid;
                if (f < total) {
                    const int rho = f / M, q = f - rho * M;
                    *reinterpret_cast<I*>(lds + rho * rowBytes + (M - 1 - q) * (int)sizeof(I)) = v[u];
                }
            }
        }
    } else {
        for (int f = tid; f < total; f += blockDim.x) {
            const int rho = f / M, p = f - rho * M;
            const long long j = jm0 + (long long)(rho - K + 1) * M - p;
            *reinterpret_cast<I*>(lds + rho * rowBytes + p * (int)sizeof(I)) = ext_load(x, hist, j, n, L - 1);
        }
    }
    __syncthreads();
    const long long m = m0 + tid;
    if (tid >= T || m >= nout) return;
    I acc = zero_v<I>();
    for (int k = 0; k < K; ++k) {
        const I* row = reinterpret_cast<const I*>(lds + (tid - k + K - 1) * rowBytes);
        const C* ck = cr + k * M;
        const int pe = min(M, L - k * M);
        // unrolled so that a run of LDS reads is in flight before the (ordered) sums
        // consume it; the summation order is unchanged
        if (pe == M) {
#pragma unroll 16
            for (int p = 0; p < M; ++p) acc = mac<EXACT>(acc, ck[p], row[p]);
        } else {
#pragma unroll 16
            for (int p = 0; p < pe; ++p) acc = mac<EXACT>(acc, ck[p], row[p]);
        }
    }
    y[m] = mul_(acc, scale);
}

// Same arithmetic with no LDS (very large M*L tiles).
template <typename C, typename I, bool EXACT>
__global__ void __launch_bounds__(kThreads)
decim_global_kernel(const I* __restrict__ x, const I* __restrict__ hist, const C* __restrict__ cr,
                    C scale, I* __restrict__ y, long long n, long long nout, int L, int M, long long j0) {
    const int ch = blockIdx.y;
    x += (long long)ch * n;
    y += (long long)ch * nout;
    hist += (long long)ch * (L - 1);
    const long long m = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (m >= nout) return;
    const long long jm = j0 + m * M;
    I acc = zero_v<I>();
    for (int i = 0; i < L; ++i) acc = mac<EXACT>(acc, cr[i], ext_load(x, hist, jm - i, n, L - 1));
    y[m] = mul_(acc, scale);
}

// new_hist[k] = ext(n - (L-1) + k), k in [0, L-1)   (bit copies)
struct u128 { uint64_t a, b; };
template <typename I>
__global__ void hist_update_kernel(const I* __restrict__ x, const I* __restrict__ old_hist, I* __restrict__ new_hist,
                                   long long n, int Lm1) {
    const int ch = blockIdx.y;
    x += (long long)ch * n;
    old_hist += (long long)ch * Lm1;
    new_hist += (long long)ch * Lm1;
    for (int k = blockIdx.x * blockDim.x + threadIdx.x; k < Lm1; k += gridDim.x * blockDim.x) {
        const long long j = n - Lm1 + k;
        new_hist[k] = j >= 0 ? x[j] : old_hist[Lm1 + j];
    }
}

// --------------------------------------------------------------------------
// launchers
// --------------------------------------------------------------------------
template <typename C, typename I>
hipError_t launch_fir_direct_t(const FirArgs& a, hipStream_t s) {
    using Img = LdsImg<I>;
    constexpr int R = Img::R;
    constexpr int TILE = kThreads * R;
    const size_t lds = (size_t)((TILE + kLC) / R) * Img::kRowBytes;
    dim3 grid((unsigned)((a.n + TILE - 1) / TILE), (unsigned)a.channels);
    const C scale = *reinterpret_cast<const C*>(a.scale);
    if (a.exact)
        hipLaunchKernelGGL((fir_direct_kernel<C, I, true>), grid, dim3(kThreads), lds, s, (const I*)a.x,
                           (const I*)a.hist, (const C*)a.taps_rev, scale, (I*)a.y, (long long)a.n, a.L);
    else
        hipLaunchKernelGGL((fir_direct_kernel<C, I, false>), grid, dim3(kThreads), lds, s, (const I*)a.x,
                           (const I*)a.hist, (const C*)a.taps_rev, scale, (I*)a.y, (long long)a.n, a.L);
    return hipGetLastError();
}

template <typename C, typename I>
hipError_t launch_decim_direct_t(const FirArgs& a, hipStream_t s) {
    const C scale = *reinterpret_cast<const C*>(a.scale);
    const int M = a.M, L = a.L, K = (L + M - 1) / M;
    const size_t rowBytes = (size_t)M * sizeof(I) + 16;
    // outputs (= lanes) per workgroup: the largest multiple of 64 whose LDS rows fit
    // in 40 KB, so that several workgroups per CU overlap their staging and sums
    int T = kThreads;
    while (T > 64 && (size_t)(T + K - 1) * rowBytes > 40 * 1024) T -= 64;
    if ((size_t)(T + K - 1) * rowBytes > 64 * 1024) T = 64;
    const size_t lds = (size_t)(T + K - 1) * rowBytes;
    if (lds <= 64 * 1024) {
        dim3 grid((unsigned)((a.nout + T - 1) / T), (unsigned)a.channels);
        if (a.exact)
            hipLaunchKernelGGL((decim_direct_kernel<C, I, true>), grid, dim3(T), lds, s, (const I*)a.x,
                               (const I*)a.hist, (const C*)a.taps_rev, scale, (I*)a.y, (long long)a.n,
                               (long long)a.nout, L, M, (long long)a.j0, T);
        else
            hipLaunchKernelGGL((decim_direct_kernel<C, I, false>), grid, dim3(T), lds, s, (const I*)a.x,
                               (const I*)a.hist, (const C*)a.taps_rev, scale, (I*)a.y, (long long)a.n,
                               (long long)a.nout, L, M, (long long)a.j0, T);
    } else {
        dim3 grid((unsigned)((a.nout + kThreads - 1) / kThreads), (unsigned)a.channels);
        if (a.exact)
            hipLaunchKernelGGL((decim_global_kernel<C, I, true>), grid, dim3(kThreads), 0, s, (const I*)a.x,
                               (const I*)a.hist, (const C*)a.taps_rev, scale, (I*)a.y, (long long)a.n,
                               (long long)a.nout, L, M, (long long)a.j0);
        else
            hipLaunchKernelGGL((decim_global_kernel<C, I, false>), grid, dim3(kThreads), 0, s, (const I*)a.x,
                               (const I*)a.hist, (const C*)a.taps_rev, scale, (I*)a.y, (long long)a.n,
                               (long long)a.nout, L, M, (long long)a.j0);
    }
    return hipGetLastError();
}

template <typename I>
hipError_t launch_hist_update_t(const void* x, const void* old_hist, void* new_hist, size_t n, int Lm1,
                                size_t channels, hipStream_t s) {
    if (Lm1 <= 0) return hipSuccess;
    dim3 grid((unsigned)((Lm1 + 255) / 256), (unsigned)channels);
    hipLaunchKernelGGL((hist_update_kernel<I>), grid, dim3(256), 0, s, (const I*)x, (const I*)old_hist,
                       (I*)new_hist, (long long)n, Lm1);
    return hipGetLastError();
}

#define SDSP_DISPATCH_DTYPE(dtype, FN, ...)                          \
    switch (dtype) {                                                 \
        case 0: return FN<float, float>(__VA_ARGS__);                \
        case 1: return FN<float, c32>(__VA_ARGS__);                  \
        case 2: return FN<c32, c32>(__VA_ARGS__);                    \
        case 3: return FN<double, double>(__VA_ARGS__);              \
        case 4: return FN<double, c64>(__VA_ARGS__);                 \
        case 5: return FN<c64, c64>(__VA_ARGS__);                    \
    }                                                                \
    return hipErrorInvalidValue;

hipError_t launch_fir_direct(int dtype, const FirArgs& a, hipStream_t s) {
    if (a.n == 0) return hipSuccess;
    SDSP_DISPATCH_DTYPE(dtype, launch_fir_direct_t, a, s)
}
hipError_t launch_decim_direct(int dtype, const FirArgs& a, hipStream_t s) {
    if (a.nout == 0) return hipSuccess;
    hipError_t err;
    if (try_launch_decim_poly(dtype, a, s, &err)) return err;
    SDSP_DISPATCH_DTYPE(dtype, launch_decim_direct_t, a, s)
}
hipError_t launch_hist_update(int dtype, const void* x, const void* old_hist, void* new_hist, size_t n, int Lm1,
                              size_t channels, hipStream_t s) {
    switch (dtype) {
        case 0: return launch_hist_update_t<uint32_t>(x, old_hist, new_hist, n, Lm1, channels, s);
        case 1: case 2: case 3: return launch_hist_update_t<uint64_t>(x, old_hist, new_hist, n, Lm1, channels, s);
        case 4: case 5: return launch_hist_update_t<u128>(x, old_hist, new_hist, n, Lm1, channels, s);
    }
    return hipErrorInvalidValue;
}

}  // namespace sdsp
