// Polyphase filterbank / interpolating FIR kernel (gfx950).
//
// PolyPhaseFilterBank (src/filter/fir/pfb.rs:24-90): branch p holds
// cb[p][i] = h[p + (K-1-i) M] (stored FORWARD after the in-place reversal at
// pfb.rs:33-40) and execute(p) = sum_{i<K} cb[p][i] * w[i] over the shared
// newest-first Window(K) — no scale.  InterpolatingFIRFilter::execute_block
// (src/filter/fir/interp.rs:102-111) pushes each input and emits all M
// branches, so
//     out[j*M + p] = sum_{i<K} cb[p][i] * x[j-i]
// Three kernels, same sums: interp_tile_kernel (M = 2^m, K in {4, 8, 16}, the
// interpolator shape), pfb_stage_kernel (every other shape whose tile fits in
// LDS) and pfb_kernel (one lane per output, the fallback for very long
// branches).  Summation order is the reference's (EXACT) or fused.
#include "sdsp_device.hpp"
#include "sdsp_kernels.hpp"

namespace sdsp {

template <typename I>
__device__ inline I pfb_ext(const I* __restrict__ x, const I* __restrict__ hist, long long j, int H) {
    if (j >= 0) return x[j];
    const long long h = (long long)H + j;
    return h >= 0 ? hist[h] : zero_v<I>();
}

template <typename C, typename I, bool EXACT>
__global__ void __launch_bounds__(256)
pfb_kernel(const I* __restrict__ x, const I* __restrict__ hist, const C* __restrict__ cb, I* __restrict__ y,
           long long n, int K, int M, int H) {
    const int ch = blockIdx.y;
    x += (long long)ch * n;
    hist += (long long)ch * H;
    const long long total = n * M;
    y += (long long)ch * total;
    const long long stride = (long long)gridDim.x * blockDim.x;
    for (long long o = (long long)blockIdx.x * blockDim.x + threadIdx.x; o < total; o += stride) {
        const long long j = o / M;
        const int p = (int)(o - j * M);
        const C* c = cb + (long long)p * K;
        I acc = zero_v<I>();
        for (int i = 0; i < K; ++i) acc = mac<EXACT>(acc, c[i], pfb_ext(x, hist, j - i, H));
        y[o] = acc;
    }
}

// Staged form for every other shape: a 256-lane workgroup owns T consecutive
// inputs of one channel (T M ~ 4096 outputs); the T + K - 1 samples they need
// and (when they fit) the M K branch coefficients are staged once in LDS with
// coalesced loads, then the lanes walk the tile's outputs in order (stores
// contiguous across the workgroup), each the reference dot product
// sum_{i<K} cb[p][i] x[j-i] in the reference order -- where pfb_kernel above
// re-read K samples and K coefficients from global memory per output and
// divided 64-bit indices.
constexpr int kPfbStageBytes = 48 * 1024;

template <typename C, typename I, bool EXACT, bool CB_LDS>
__global__ void __launch_bounds__(256)
pfb_stage_kernel(const I* __restrict__ x, const I* __restrict__ hist, const C* __restrict__ cb, I* __restrict__ y,
                 long long n, int K, int M, int H, int T) {
    extern __shared__ __attribute__((aligned(16))) unsigned char pfb_lds[];
    I* xs = reinterpret_cast<I*>(pfb_lds);  // xs[s] = x[j0 - K + 1 + s]
    const int ch = blockIdx.y;
    x += (long long)ch * n;
    hist += (long long)ch * H;
    y += (long long)ch * n * M;
    const long long j0 = (long long)blockIdx.x * T;
    const int nt = n - j0 < T ? (int)(n - j0) : T;
    const int ns = nt + K - 1;
    const C* cbs = cb;
    if constexpr (CB_LDS) {
        C* c = reinterpret_cast<C*>(pfb_lds + ((size_t)(T + K - 1) * sizeof(I) + 15) / 16 * 16);
        for (int i = threadIdx.x; i < M * K; i += 256) c[i] = cb[i];
        cbs = c;
    }
    const long long base = j0 - K + 1;
    if (base >= 0) {
        for (int i = threadIdx.x; i < ns; i += 256) xs[i] = x[base + i];
    } else {
        for (int i = threadIdx.x; i < ns; i += 256) xs[i] = pfb_ext(x, hist, base + i, H);
    }
    __syncthreads();
    const unsigned um = (unsigned)M, total = (unsigned)nt * um;
    I* yt = y + j0 * M;
    for (unsigned o = threadIdx.x; o < total; o += 256) {
        const unsigned j = o / um, p = o - j * um;
        const C* c = cbs + (size_t)p * K;
        const I* w = xs + j + K - 1;  // w[-i] = x[j0 + j - i]
        I acc = zero_v<I>();
        for (int i = 0; i < K; ++i) acc = mac<EXACT>(acc, c[i], w[-i]);
        yt[o] = acc;
    }
}

// Tiled form for M = 2^m (8 <= M <= 512) and K in {4, 8, 16}: the interpolator
// shape (InterpolatingFIRFilter::execute_block, one input in, M outputs out).
// A 256-lane workgroup owns T = 16 * 512 / M consecutive inputs of one channel
// (XCD-ordered: each XCD streams one contiguous stretch of the output).  Lane
// (g, q) -- q = 0 .. M/2-1 a pair of branches (2q, 2q + 1), g = 0 .. 512/M - 1
// a run of R = 16 inputs -- keeps its 2K branch coefficients and the R + K - 1
// samples its run needs in registers (staged once through LDS, read as
// wave-broadcasts) and writes its 2R outputs as 16-byte stores: for one input
// the M/2 lanes of a run cover M contiguous outputs.  Every output is the
// reference dot product sum_{i<K} cb[p][i] x[j-i] in the reference order.
constexpr int kInterpR = 16;

template <typename I> struct alignas(2 * sizeof(I)) Pair {
    I a, b;
};

template <typename C, typename I, bool EXACT, int K>
__global__ void __launch_bounds__(256)
interp_tile_kernel(const I* __restrict__ x, const I* __restrict__ hist, const C* __restrict__ cb,
                   I* __restrict__ y, long long n, int M, int H, long long q8) {
    constexpr int R = kInterpR;
    __shared__ I xs[1024 + 16];  // T + K - 1 <= 16 * 64 + 15 samples (M >= 8)
    const int ch = blockIdx.y;
    const int xc = blockIdx.x & 7;
    const long long tile = (long long)xc * q8 + (blockIdx.x >> 3);
    const int P = M >> 1, G = 256 / P, T = G * R;
    const long long j0 = tile * T;
    if (j0 >= n) return;  // uniform
    x += (long long)ch * n;
    hist += (long long)ch * H;
    y += (long long)ch * n * M;
    const int t = threadIdx.x;
    // stage x[j0 - K + 1, j0 + T) (zero past n, history before 0)
    for (int i = t; i < T + K - 1; i += 256) {
        const long long j = j0 - (K - 1) + i;
        xs[i] = j < n ? pfb_ext(x, hist, j, H) : zero_v<I>();
    }
    const int g = t / P, q = t - g * P;
    C c0[K], c1[K];
#pragma unroll
    for (int i = 0; i < K; ++i) {
        c0[i] = cb[(long long)(2 * q) * K + i];
        c1[i] = cb[(long long)(2 * q + 1) * K + i];
    }
    __syncthreads();
    I w[R + K - 1];  // w[m] = x[jg - K + 1 + m], jg = j0 + g R
#pragma unroll
    for (int m = 0; m < R + K - 1; ++m) w[m] = xs[g * R + m];
    const long long jg = j0 + (long long)g * R;
    I* yo = y + jg * M + 2 * q;
#pragma unroll
    for (int r = 0; r < R; ++r) {
        I a0 = zero_v<I>(), a1 = zero_v<I>();
#pragma unroll
        for (int i = 0; i < K; ++i) {
            const I s = w[r + K - 1 - i];  // x[jg + r - i]
            a0 = mac<EXACT>(a0, c0[i], s);
            a1 = mac<EXACT>(a1, c1[i], s);
        }
        if (jg + r < n) store_nt(reinterpret_cast<Pair<I>*>(yo + (long long)r * M), Pair<I>{a0, a1});
    }
}

template <typename C, typename I, bool EXACT>
hipError_t launch_interp_tile(const PfbArgs& a, hipStream_t s) {
    const int P = a.M / 2, T = (256 / P) * kInterpR;
    const long long tiles = ((long long)a.n + T - 1) / T;
    const long long q8 = (tiles + 7) / 8;
    if (8 * q8 > 0x7fffffffLL) return hipErrorInvalidValue;
    const dim3 grid((unsigned)(8 * q8), (unsigned)a.channels);
#define SDSP_INTERP_K(KK)                                                                                        \
    if (a.K == KK) {                                                                                             \
        hipLaunchKernelGGL((interp_tile_kernel<C, I, EXACT, KK>), grid, dim3(256), 0, s, (const I*)a.x,          \
                           (const I*)a.hist, (const C*)a.cb, (I*)a.y, (long long)a.n, a.M, a.H, q8);             \
        return hipGetLastError();                                                                                \
    }
    SDSP_INTERP_K(4)
    SDSP_INTERP_K(8)
    SDSP_INTERP_K(16)
#undef SDSP_INTERP_K
    return hipErrorInvalidValue;
}

template <typename I>
bool interp_tile_applies(const PfbArgs& a) {
    return a.M >= 8 && a.M <= 512 && (a.M & (a.M - 1)) == 0 && (a.K == 4 || a.K == 8 || a.K == 16) &&
           a.H == a.K && ((uintptr_t)a.y % (2 * sizeof(I))) == 0;
}

template <typename C, typename I>
hipError_t launch_pfb_t(const PfbArgs& a, hipStream_t s) {
    if (interp_tile_applies<I>(a))
        return a.exact ? launch_interp_tile<C, I, true>(a, s) : launch_interp_tile<C, I, false>(a, s);
#ifndef SDSP_PFB_LAB  // lab builds keep the per-output kernel for A/B (tools/lab.mk)
    {
        const int T = a.M >= 4096 ? 1 : 4096 / a.M;
        const size_t xb = ((size_t)(T + a.K - 1) * sizeof(I) + 15) / 16 * 16, cbb = (size_t)a.M * a.K * sizeof(C);
        if (xb <= kPfbStageBytes && (unsigned long long)T * a.M < (1ULL << 31)) {
            const bool cb_lds = xb + cbb <= kPfbStageBytes;
            const size_t lds = xb + (cb_lds ? cbb : 0);
            dim3 g((unsigned)((a.n + T - 1) / T), (unsigned)a.channels);
#define SDSP_PFB_STAGE(EX, CBL)                                                                                  \
    hipLaunchKernelGGL((pfb_stage_kernel<C, I, EX, CBL>), g, dim3(256), lds, s, (const I*)a.x, (const I*)a.hist, \
                       (const C*)a.cb, (I*)a.y, (long long)a.n, a.K, a.M, a.H, T)
            if (a.exact) {
                if (cb_lds) SDSP_PFB_STAGE(true, true); else SDSP_PFB_STAGE(true, false);
            } else {
                if (cb_lds) SDSP_PFB_STAGE(false, true); else SDSP_PFB_STAGE(false, false);
            }
#undef SDSP_PFB_STAGE
            return hipGetLastError();
        }
    }
#endif
    const long long total = (long long)a.n * a.M;
    long long blocks = (total + 255) / 256;
    if (blocks > 65536) blocks = 65536;
    dim3 grid((unsigned)blocks, (unsigned)a.channels);
    if (a.exact)
        hipLaunchKernelGGL((pfb_kernel<C, I, true>), grid, dim3(256), 0, s, (const I*)a.x, (const I*)a.hist,
                           (const C*)a.cb, (I*)a.y, (long long)a.n, a.K, a.M, a.H);
    else
        hipLaunchKernelGGL((pfb_kernel<C, I, false>), grid, dim3(256), 0, s, (const I*)a.x, (const I*)a.hist,
                           (const C*)a.cb, (I*)a.y, (long long)a.n, a.K, a.M, a.H);
    return hipGetLastError();
}

hipError_t launch_pfb(int dtype, const PfbArgs& a, hipStream_t s) {
    if (a.n == 0) return hipSuccess;
    switch (dtype) {
        case 0: return launch_pfb_t<float, float>(a, s);
        case 1: return launch_pfb_t<float, c32>(a, s);
        case 2: return launch_pfb_t<c32, c32>(a, s);
        case 3: return launch_pfb_t<double, double>(a, s);
        case 4: return launch_pfb_t<double, c64>(a, s);
        case 5: return launch_pfb_t<c64, c64>(a, s);
    }
    return hipErrorInvalidValue;
}

// ---- synthetic stream (build-defined generator) ---------------
__device__ inline uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

__global__ void synth_kernel(float* __restrict__ out, uint64_t key, uint64_t start, long long count) {
    const uint64_t g = 0x9E3779B97F4A7C15ULL;
    const long long stride = (long long)gridDim.x * blockDim.x;
    for (long long j = (long long)blockIdx.x * blockDim.x + threadIdx.x; j < count; j += stride) {
        const uint64_t v = mix64(key + (start + (uint64_t)j + 1) * g);
        out[j] = (float)(v >> 40) * (1.0f / 16777216.0f) * 2.0f - 1.0f;
    }
}

hipError_t launch_synth_f32(float* out, uint64_t seed, uint64_t channel, uint64_t start, size_t count,
                            hipStream_t s) {
    if (count == 0) return hipSuccess;
    const uint64_t key = seed ^ (channel * 0x9E3779B97F4A7C15ULL);
    long long blocks = ((long long)count + 255) / 256;
    if (blocks > 16384) blocks = 16384;
    hipLaunchKernelGGL(synth_kernel, dim3((unsigned)blocks), dim3(256), 0, s, out, key, start, (long long)count);
    return hipGetLastError();
}

}  // namespace sdsp

namespace sdsp {
// ---- STREAM-style copy used to calibrate achievable HBM bandwidth ----------
// One-shot grid, one 16-byte vector per lane: the fastest copy shape measured
// on the box (tools/bw_probe.hip: 6.3 TB/s read + write vs 5.0-5.9 for
// persistent grid-stride copies).
__global__ void __launch_bounds__(256) bw_copy_kernel(const float4* __restrict__ a, float4* __restrict__ b,
                                                      long long n16) {
    const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
    if (i < n16) b[i] = a[i];
}
hipError_t launch_bw_copy(const void* a, void* b, size_t bytes, int num_cus, hipStream_t s) {
    (void)num_cus;
    const long long n16 = (long long)(bytes / 16);
    if (n16 == 0) return hipSuccess;
    const long long blocks = (n16 + 255) / 256;
    if (blocks > 0x7fffffffLL) return hipErrorInvalidValue;
    hipLaunchKernelGGL(bw_copy_kernel, dim3((unsigned)blocks), dim3(256), 0, s, (const float4*)a, (float4*)b, n16);
    return hipGetLastError();
}
}  // namespace sdsp
