// Overlap-save fast-convolution FIR for 32-bit complex streams (gfx950).
//
// Same filter as FIRFilter::execute (src/filter/fir/mod.rs:209-212):
//     y[n] = scale * sum_{i<L} h[L-1-i] x[n-i]
// computed per 4096-sample segment as a circular convolution with the
// zero-padded impulse response g[i] = scale*h[L-1-i] (spectrum precomputed in
// f64 on the host).  Segment s reads x[s*V - H, s*V - H + 4096) and writes the
// V = 4096 - H outputs that do not wrap (H = 256*h2 >= L-1).
//
// Data flow (one 256-thread workgroup per segment, 16 points per lane, all
// three radix-16 passes of the forward DIF FFT, the spectral multiply and
// the three passes of the inverse in registers; the segment visits LDS only
// for the four transposes between passes):
//     n = 256 n2 + 16 n1 + n0,  k = k0 + 16 k1 + 256 k2
//   load   lane t=(n1,n0)   holds x over n2     (coalesced: stride 256 samples)
//   P1     DFT16 n2->k0, * W4096^(t k0)        -> LDS A[k0][t]
//   P2     lane (k0,n0)     DFT16 n1->k1, * W256^(n0 k1) -> LDS B[k0,k1][n0]
//   P3     lane (k0,k1)     DFT16 n0->k2, * H[k0+16k1+256k2]/N,
//                           IDFT16 k2->n0, * W256^-(k1 n0) -> LDS B
//   P4     lane (k0,n0)     IDFT16 k1->n1                    -> LDS A
//   P5     lane t=(n1,n0)   * W4096^-(t k0), IDFT16 k0->n2, store n2 >= h2
// The DIF output order is exactly the order the inverse DIT consumes, so no
// bit-reversal pass exists.  Twiddle rows and the spectrum slice each lane
// needs are constant across segments and live in registers.
//
// This file holds the scalar form of the transform: the boundary-segment
// kernel (first / last segments of a call, whose windows reach into the
// history or past the end of the block), the scalar persistent kernel used when
// rows are not 16-byte aligned, and the dispatcher.  The interior segments of
// aligned streams run in kern_fir_ols_os.hip (default) or kern_fir_ols_pk.hip.
#include "sdsp_device.hpp"
#include "sdsp_kernels.hpp"

namespace sdsp {

namespace {

struct cf { float re, im; };

__device__ __forceinline__ cf cadd(cf a, cf b) { return {a.re + b.re, a.im + b.im}; }
__device__ __forceinline__ cf csub(cf a, cf b) { return {a.re - b.re, a.im - b.im}; }
__device__ __forceinline__ cf cmul(cf a, cf b) {
    return {__builtin_fmaf(a.re, b.re, -(a.im * b.im)), __builtin_fmaf(a.re, b.im, a.im * b.re)};
}
__device__ __forceinline__ cf cmulc(cf a, cf b) {  // a * conj(b)
    return {__builtin_fmaf(a.re, b.re, a.im * b.im), __builtin_fmaf(a.im, b.re, -(a.re * b.im))};
}
// multiply by -j (forward) / +j (inverse)
template <bool INV> __device__ __forceinline__ cf rotj(cf a) {
    if constexpr (INV) return {-a.im, a.re};
    else return {a.im, -a.re};
}

template <bool INV> __device__ __forceinline__ void dft4(cf& x0, cf& x1, cf& x2, cf& x3) {
    cf a = cadd(x0, x2), b = csub(x0, x2), c = cadd(x1, x3), d = rotj<INV>(csub(x1, x3));
    x0 = cadd(a, c);
    x2 = csub(a, c);
    x1 = cadd(b, d);
    x3 = csub(b, d);
}

constexpr float kC1 = 0.92387953251128674f;  // cos(pi/8)
constexpr float kS1 = 0.38268343236508978f;  // sin(pi/8)
constexpr float kR2 = 0.70710678118654752f;  // sqrt(1/2)

// v *= W16^m (forward: e^{-j 2 pi m/16}; inverse: conjugate)
template <bool INV, int m> __device__ __forceinline__ cf tw16(cf v) {
    constexpr float s = INV ? -1.0f : 1.0f;
    if constexpr (m == 0) return v;
    else if constexpr (m == 1) return cmul(v, cf{kC1, -s * kS1});
    else if constexpr (m == 2) return cf{kR2 * (v.re + s * v.im), kR2 * (v.im - s * v.re)};
    else if constexpr (m == 3) return cmul(v, cf{kS1, -s * kC1});
    else if constexpr (m == 4) return rotj<INV>(v);
    else if constexpr (m == 6) return cf{kR2 * (-v.re + s * v.im), kR2 * (-v.im - s * v.re)};
    else if constexpr (m == 9) return cmul(v, cf{-kC1, s * kS1});
    else return v;
}

// in-place 16-point DFT, natural order in and out
template <bool INV> __device__ __forceinline__ void dft16(cf (&v)[16]) {
    // n = 4 na + nb ; k = ka + 4 kb
#pragma unroll
    for (int nb = 0; nb < 4; ++nb) dft4<INV>(v[nb], v[4 + nb], v[8 + nb], v[12 + nb]);
    // v[4 ka + nb] now holds stage-1 output (nb, ka); twiddle W16^(nb ka)
    v[5] = tw16<INV, 1>(v[5]);
    v[6] = tw16<INV, 2>(v[6]);
    v[7] = tw16<INV, 3>(v[7]);
    v[9] = tw16<INV, 2>(v[9]);
    v[10] = tw16<INV, 4>(v[10]);
    v[11] = tw16<INV, 6>(v[11]);
    v[13] = tw16<INV, 3>(v[13]);
    v[14] = tw16<INV, 6>(v[14]);
    v[15] = tw16<INV, 9>(v[15]);
#pragma unroll
    for (int ka = 0; ka < 4; ++ka) dft4<INV>(v[4 * ka + 0], v[4 * ka + 1], v[4 * ka + 2], v[4 * ka + 3]);
    // v[4 ka + kb] = X[ka + 4 kb]  -> transpose to natural order
    cf t[16];
#pragma unroll
    for (int ka = 0; ka < 4; ++ka)
#pragma unroll
        for (int kb = 0; kb < 4; ++kb) t[ka + 4 * kb] = v[4 * ka + kb];
#pragma unroll
    for (int i = 0; i < 16; ++i) v[i] = t[i];
}

constexpr int kRowA = 272;  // A image: 16 rows of 256 (+16 pad) samples
constexpr int kRegion = 16 * kRowA;  // samples per LDS region

// B image: 256 rows x 16 samples, pairs XOR-swizzled by (row>>1)&7
__device__ __forceinline__ int bidx(int r, int c) { return r * 16 + ((((c >> 1) ^ (r >> 1)) & 7) << 1) + (c & 1); }

template <bool CHECK>
__device__ __forceinline__ cf ext_ld(const cf* __restrict__ x, const cf* __restrict__ hist, long long j, long long n,
                                     int Lm1) {
    if constexpr (!CHECK) {
        return x[j];
    } else {
        cf s = {0.0f, 0.0f};
        if (j >= 0) {
            if (j < n) s = x[j];
        } else if (Lm1 + j >= 0) {
            s = hist[Lm1 + j];
        }
        return s;
    }
}

// P1..P5 of one segment on v (loaded: lane t holds x over n2).  `after_p1` runs
// right after P1's LDS writes (the next segment's loads go out there).  On return
// v holds the segment's outputs over rows n2.
template <typename F>
__device__ __forceinline__ void ols_segment(cf (&v)[16], cf* __restrict__ rA, cf* __restrict__ rB,
                                            const cf (&w1)[16], const cf (&w2)[16], const cf (&Hr)[16], int t,
                                            F&& after_p1) {
    const int hi4 = t >> 4, lo4 = t & 15;
    auto bar = [] { __syncthreads(); };
    // P1: DFT over n2 -> k0, twiddle, A[k0][t]
    dft16<false>(v);
#pragma unroll
    for (int k = 0; k < 16; ++k) rA[k * kRowA + t] = cmul(v[k], w1[k]);
    after_p1();
    bar();
    // P2: lane (k0=hi4, n0=lo4) reads n1
#pragma unroll
    for (int k = 0; k < 16; ++k) v[k] = rA[hi4 * kRowA + 16 * k + lo4];
    dft16<false>(v);
#pragma unroll
    for (int k = 0; k < 16; ++k) rB[bidx(16 * hi4 + k, lo4)] = cmul(v[k], w2[k]);
    bar();
    // P3: lane (k0=hi4, k1=lo4) reads its row over n0
    {
        const float4* row = reinterpret_cast<const float4*>(rB + t * 16);
#pragma unroll
        for (int p = 0; p < 8; ++p) {
            const float4 q = row[(p ^ (t >> 1)) & 7];
            v[2 * p] = {q.x, q.y};
            v[2 * p + 1] = {q.z, q.w};
        }
    }
    dft16<false>(v);
#pragma unroll
    for (int k = 0; k < 16; ++k) v[k] = cmul(v[k], Hr[k]);
    dft16<true>(v);
    // back to A region (its readers all passed the barrier above)
    {
        float4* row = reinterpret_cast<float4*>(rA + t * 16);
#pragma unroll
        for (int p = 0; p < 8; ++p) {
            const cf a = cmulc(v[2 * p], w2[2 * p]);
            const cf b = cmulc(v[2 * p + 1], w2[2 * p + 1]);
            row[(p ^ (t >> 1)) & 7] = make_float4(a.re, a.im, b.re, b.im);
        }
    }
    bar();
    // P4: lane (k0=hi4, n0=lo4) reads k1
#pragma unroll
    for (int k = 0; k < 16; ++k) v[k] = rA[bidx(16 * hi4 + k, lo4)];
    dft16<true>(v);
#pragma unroll
    for (int k = 0; k < 16; ++k) rB[hi4 * kRowA + 16 * k + lo4] = v[k];
    bar();
    // P5: lane t=(n1,n0) reads k0
#pragma unroll
    for (int k = 0; k < 16; ++k) v[k] = cmulc(rB[k * kRowA + t], w1[k]);
    dft16<true>(v);
    // the next segment's P1 writes region A: every lane has finished reading
    // region A (P4) before the barrier that precedes P5.
}

}  // namespace

// Scalar persistent kernel: the fallback for streams whose rows are not 16-byte
// aligned (odd channel stride, unaligned device pointers).  Segments are split
// into interior ones (input window [base, base+4096) and all outputs inside the
// stream) and at most a first and a last boundary segment.  Block b takes
// segments b, b+G, b+2G, ... so the blocks resident at any moment stream one
// contiguous window of HBM.  The main loop runs interior segments only, with
// straight-line loads and stores and an unconditional one-segment-ahead
// prefetch; stores are deferred by one segment (they go out after P1 of the next
// segment, ahead of the loads for the one after), so the loop-head wait for the
// prefetched data never covers freshly issued stores.
// H2 > 0: halo rows known at compile time (the interior stores are then
// unconditional and the loop-head wait counts them exactly); H2 = 0: runtime h2.
template <int H2>
__global__ void __launch_bounds__(256, 2)
fir_ols4096_kernel(const cf* __restrict__ x, const cf* __restrict__ hist, const cf* __restrict__ Hs,
                   const cf* __restrict__ tw1, const cf* __restrict__ tw2, cf* __restrict__ y, long long n,
                   int Lm1, int h2_rt, long long nseg) {
    const int h2 = H2 > 0 ? H2 : h2_rt;
    __shared__ __attribute__((aligned(16))) cf lds[2 * kRegion];
    cf* const rA = lds;
    cf* const rB = lds + kRegion;
    const int ch = blockIdx.y;
    x += (long long)ch * n;
    y += (long long)ch * n;
    hist += (long long)ch * Lm1;

    const int t = threadIdx.x;
    const int lo4 = t & 15;
    cf w1[16], w2[16], Hr[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        w1[k] = tw1[t * 16 + k];
        w2[k] = tw2[lo4 * 16 + k];
        Hr[k] = Hs[t * 16 + k];
    }
    const int V = 4096 - 256 * h2;
    const long long s1 = nseg, sstep = gridDim.x;
    auto base_of = [&](long long sg) { return sg * V - 256 * h2; };
    auto interior = [&](long long sg) { return sg < s1 && base_of(sg) >= 0 && base_of(sg) + 4096 <= n; };

    // boundary segment: guarded element loads and stores, no prefetch
    auto boundary = [&](long long sg) {
        cf v[16];
        const long long base = base_of(sg);
#pragma unroll
        for (int r = 0; r < 16; ++r) v[r] = ext_ld<true>(x, hist, base + 256 * r + t, n, Lm1);
        ols_segment(v, rA, rB, w1, w2, Hr, t, [] {});
        const long long ob = base + t;
#pragma unroll
        for (int k = 0; k < 16; ++k)
            if (k >= h2 && ob + 256 * k < n) y[ob + 256 * k] = v[k];
        __syncthreads();  // region A/B reuse by the next segment
    };

    long long seg = blockIdx.x;
    if (seg < s1 && !interior(seg)) {
        boundary(seg);
        seg += sstep;
    }
    cf nv[16];
    auto load = [&](long long sg) {
        const cf* xb = x + base_of(sg);
#pragma unroll
        for (int r = 0; r < 16; ++r) nv[r] = xb[256 * r + t];
    };
    cf ov[16];
    long long oseg = -1;
    auto store_out = [&]() {
        cf* yb = y + base_of(oseg) + t;
#pragma unroll
        for (int k = 0; k < 16; ++k)
            if (k >= h2) yb[256 * k] = ov[k];
    };
    if (interior(seg)) load(seg);
    for (; interior(seg); seg += sstep) {
        cf v[16];
#pragma unroll
        for (int r = 0; r < 16; ++r) v[r] = nv[r];
        // next interior segment, or this one again (keeps the loop body uniform)
        const long long nxt = interior(seg + sstep) ? seg + sstep : seg;
        ols_segment(v, rA, rB, w1, w2, Hr, t, [&] {
            if (oseg >= 0) store_out();
            load(nxt);
        });
#pragma unroll
        for (int k = 0; k < 16; ++k) ov[k] = v[k];
        oseg = seg;
    }
    if (oseg >= 0) store_out();
    for (; seg < s1; seg += sstep) boundary(seg);
}

// Boundary segments only (first segments whose window starts before the stream,
// last ones whose window runs past its end), for calls whose interior segments
// run in the packed kernel (kern_fir_ols_pk.hip): block b takes segment b when
// b < lo, else segment hi + (b - lo).
__global__ void __launch_bounds__(256)
fir_ols4096_edge_kernel(const cf* __restrict__ x, const cf* __restrict__ hist, const cf* __restrict__ Hs,
                        const cf* __restrict__ tw1, const cf* __restrict__ tw2, cf* __restrict__ y, long long n,
                        int Lm1, int h2, long long lo, long long hi) {
    __shared__ __attribute__((aligned(16))) cf lds[2 * kRegion];
    const int ch = blockIdx.y;
    x += (long long)ch * n;
    y += (long long)ch * n;
    hist += (long long)ch * Lm1;
    const int t = threadIdx.x;
    const int lo4 = t & 15;
    cf w1[16], w2[16], Hr[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        w1[k] = tw1[t * 16 + k];
        w2[k] = tw2[lo4 * 16 + k];
        Hr[k] = Hs[t * 16 + k];
    }
    const long long b = blockIdx.x;
    const long long sg = b < lo ? b : hi + (b - lo);
    const long long base = sg * (4096 - 256 * h2) - 256 * h2;
    cf v[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) v[r] = ext_ld<true>(x, hist, base + 256 * r + t, n, Lm1);
    ols_segment(v, lds, lds + kRegion, w1, w2, Hr, t, [] {});
    const long long ob = base + t;
#pragma unroll
    for (int k = 0; k < 16; ++k)
        if (k >= h2 && ob + 256 * k < n) y[ob + 256 * k] = v[k];
}

// interior segment range of a call: [lo, hi) with input window and outputs in range
void ols_interior_range(long long n, int h2, long long* lo, long long* hi) {
    const long long V = 4096 - 256LL * h2, H = 256LL * h2;
    const long long nseg = (n + V - 1) / V;
    long long a = (H + V - 1) / V;  // first s with s V - H >= 0
    if (a > nseg) a = nseg;
    // last s with s V - H + 4096 <= n
    long long b = n - 4096 + H >= 0 ? (n - 4096 + H) / V + 1 : 0;
    if (b > nseg) b = nseg;
    if (b < a) b = a;
    *lo = a;
    *hi = b;
}

// Kernel choice (OlsPlan::kernel, SDSP_TUNE_OLS_KERNEL): with 16-byte rows every
// segment runs in the one-shot kernel (default; it also writes the next history), or
// the interior segments in the persistent packed kernel (h2 <= 4) and the boundary
// segments in fir_ols4096_edge_kernel; otherwise
// everything runs in the scalar persistent kernel.  All choices compute the same
// transform (rounding differs only in the one-shot kernel's twiddle products).
hipError_t launch_fir_ols(const OlsPlan& p, const void* x, const void* hist, void* new_hist, void* y, size_t n,
                          int L, size_t channels, int num_cus, hipStream_t s, bool* hist_done) {
    *hist_done = false;
    if (n == 0) return hipSuccess;
    const int h2 = p.halo_rows;
    const long long V = 4096 - 256 * h2;
    const long long nseg = ((long long)n + V - 1) / V;
    const bool rows16 = ((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(y)) & 15) == 0 &&
                        (channels == 1 || n % 2 == 0);
    const bool os = p.kernel == kOlsOneShot || p.kernel == kOlsOneShotWide;
    const bool pk = p.kernel == kOlsPersistent && h2 <= 4;
    if (rows16 && os) {
        // one grid: boundary segments, interior segments and (n >= L - 1) the history update
        const bool fused_hist = n >= (size_t)(L - 1);
        hipError_t e = launch_fir_ols_os(p, x, hist, fused_hist ? new_hist : nullptr, y, n, L - 1, channels, s,
                                         p.kernel == kOlsOneShotWide);
        if (e == hipSuccess) *hist_done = fused_hist;
        return e;
    }
    if (rows16 && pk) {
        long long lo, hi;
        ols_interior_range((long long)n, h2, &lo, &hi);
        const long long nedge = lo + (nseg - hi);
        if (nedge > 0) {
            hipLaunchKernelGGL(fir_ols4096_edge_kernel, dim3((unsigned)nedge, (unsigned)channels), dim3(256), 0, s,
                               (const cf*)x, (const cf*)hist, (const cf*)p.d_H, (const cf*)p.d_tw1,
                               (const cf*)p.d_tw2, (cf*)y, (long long)n, L - 1, h2, lo, hi);
            hipError_t e = hipGetLastError();
            if (e != hipSuccess) return e;
        }
        return launch_fir_ols_pk(p, x, y, n, channels, s, lo, hi);
    }
    long long blocks = (long long)num_cus * 2;
    if (blocks > nseg) blocks = nseg;
    const dim3 grid((unsigned)blocks, (unsigned)channels);
#define SDSP_OLS_LAUNCH(H)                                                                                         \
    hipLaunchKernelGGL((fir_ols4096_kernel<H>), grid, dim3(256), 0, s, (const cf*)x, (const cf*)hist,             \
                       (const cf*)p.d_H, (const cf*)p.d_tw1, (const cf*)p.d_tw2, (cf*)y, (long long)n, L - 1, h2, \
                       nseg)
    if (h2 == 1) SDSP_OLS_LAUNCH(1);
    else SDSP_OLS_LAUNCH(0);
#undef SDSP_OLS_LAUNCH
    return hipGetLastError();
}

}  // namespace sdsp
