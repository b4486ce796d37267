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
// needs are constant across segments and live in registers; the workgroup is
// persistent over a contiguous run of segments so each segment's halo is an
// L2 hit on the previous segment's tail.
#include "sdsp_device.hpp"
#include "sdsp_kernels.hpp"

namespace sdsp {

namespace {

struct cf { float re, im; };
typedef float f2v __attribute__((ext_vector_type(2)));

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

// LDS hand-off between the lanes of one wave (LDS counter only; global loads
// and stores stay in flight)
__device__ __forceinline__ void wave_sync_lds() {
    __builtin_amdgcn_s_waitcnt(0xC07F);
    __builtin_amdgcn_wave_barrier();
}

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
// NOBAR: profiling ablation only (wrong results): the four barriers become
// wave barriers, to price workgroup synchronisation
template <bool NOBAR = false, typename F>
__device__ __forceinline__ void ols_segment(cf (&v)[16], cf* __restrict__ rA, cf* __restrict__ rB,
                                            const cf (&w1)[16], const cf (&w2)[16], const cf (&Hr)[16], int t,
                                            F&& after_p1) {
    const int hi4 = t >> 4, lo4 = t & 15;
    auto bar = [] {
        if constexpr (NOBAR) __builtin_amdgcn_wave_barrier();
        else __syncthreads();
    };
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

// Segments are split into interior ones (input window [base, base+4096) and
// all outputs inside the stream) and at most a first and a last boundary
// segment.  The main loop runs interior segments only, with straight-line
// loads and stores and an unconditional one-segment-ahead prefetch, so the
// compiler's wait for the prefetched data at the loop head counts only the
// loads (vmcnt(16 stores)) instead of draining every store (vmcnt(0)).
// H2 > 0: halo rows known at compile time (the interior stores are then
// unconditional and the loop-head wait counts them exactly); H2 = 0: runtime h2.
template <bool INTERLEAVE, int ABL, int H2, int NT = 0>
__global__ void __launch_bounds__(256, 2)
fir_ols4096_kernel(const cf* __restrict__ x, const cf* __restrict__ hist, const cf* __restrict__ Hs,
                   const cf* __restrict__ tw1, const cf* __restrict__ tw2, cf* __restrict__ y, long long n,
                   int Lm1, int h2_rt, long long nseg, long long segs_per_block) {
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
    // Segment order.  INTERLEAVE: block b takes segments b, b+G, b+2G, ... so
    // the blocks resident at any moment stream one contiguous window of HBM
    // (DRAM-page friendly; the halo is the previous segment's tail, read at
    // about the same time by the neighbouring block).  Otherwise each block
    // walks a contiguous run of segments.
    long long s0, s1, sstep;
    if constexpr (INTERLEAVE) {
        s0 = blockIdx.x;
        s1 = nseg;
        sstep = gridDim.x;
    } else {
        s0 = (long long)blockIdx.x * segs_per_block;
        s1 = s0 + segs_per_block;
        if (s1 > nseg) s1 = nseg;
        sstep = 1;
    }
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

    long long seg = s0;
    if (seg < s1 && !interior(seg)) {
        boundary(seg);
        seg += sstep;
    }
    cf nv[16];
    auto load = [&](long long sg) {
        if constexpr (ABL == 1 || ABL == 2 || ABL == 4) {  // ablation builds: no input traffic, same arithmetic
#pragma unroll
            for (int r = 0; r < 16; ++r) nv[r] = cf{(float)(t + r), (float)(sg & 1023)};
        } else {
            const cf* xb = x + base_of(sg);
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                if constexpr (NT & 1) {  // streaming loads
                    const f2v q = __builtin_nontemporal_load(reinterpret_cast<const f2v*>(xb + 256 * r + t));
                    nv[r] = cf{q.x, q.y};
                } else {
                    nv[r] = xb[256 * r + t];
                }
            }
        }
    };
    // Interior segments.  Stores are deferred by one segment: segment s's outputs
    // go out after P1 of segment s+1, ahead of the loads for segment s+2, so the
    // loop-head wait for those loads never waits on freshly issued stores.
    cf ov[16];
    long long oseg = -1;
    auto store_out = [&]() {
        cf* yb = y + base_of(oseg) + t;
        if constexpr (ABL == 1 || ABL == 3 || ABL == 4) {  // ablation builds: no output traffic
#pragma unroll
            for (int k = 0; k < 16; ++k)
                if (ov[k].re == 1234.5678f && k >= h2) yb[256 * k] = ov[k];
        } else {
#pragma unroll
            for (int k = 0; k < 16; ++k) {
                if (k >= h2) {
                    if constexpr (NT & 2) __builtin_nontemporal_store(f2v{ov[k].re, ov[k].im}, reinterpret_cast<f2v*>(yb + 256 * k));
                    else yb[256 * k] = ov[k];
                }
            }
        }
    };
    if (interior(seg)) load(seg);
    for (; interior(seg); seg += sstep) {
        cf v[16];
#pragma unroll
        for (int r = 0; r < 16; ++r) v[r] = nv[r];
        // next interior segment, or this one again (keeps the loop body uniform)
        const long long nxt = interior(seg + sstep) ? seg + sstep : seg;
        if constexpr (NT & 4) {
            ols_segment(v, rA, rB, w1, w2, Hr, t, [&] { load(nxt); });
#pragma unroll
            for (int k = 0; k < 16; ++k) ov[k] = v[k];
            oseg = seg;
            store_out();
        } else {
            ols_segment<ABL == 4>(v, rA, rB, w1, w2, Hr, t, [&] {
                if (oseg >= 0) store_out();
                load(nxt);
            });
#pragma unroll
            for (int k = 0; k < 16; ++k) ov[k] = v[k];
            oseg = seg;
        }
    }
    if (!(NT & 4) && oseg >= 0) store_out();
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

// ---------------------------------------------------------------------------
// Wave-per-segment overlap-save, N = 1024 (`SDSP_TUNE_OLS_WAVE`).  Each wave
// owns whole segments, 16 points per lane, and transposes only through its
// own LDS buffer, so a segment needs no workgroup barrier:
//     n = n0 + 4 n1 + 64 n2,  k = k2 + 16 k1 + 256 k0
//   P1  lane L = n0 + 4 n1: DFT16 n2 -> k2, * W1024^(L k2)      -> LDS rows n0 + 4 k2
//   P2  lane (n0, k2):      DFT16 n1 -> k1, * W1024^(16 n0 k1)   -> LDS [k2 + 16 k1][n0]
//   P3  lane l, c = l + 64 j: DFT4 n0 -> k0, * H[c + 256 k0] (natural order, /N, scale),
//                           IDFT4 k0 -> n0                    -> LDS [c][n0]
//   P2' lane (n0, k2):      * W1024^-(16 n0 k1), IDFT16 k1 -> n1 -> LDS rows
//   P1' lane (n0, n1):      * W1024^-(L k2), IDFT16 k2 -> n2, store rows n2 >= HR
// The halo is HR rows of 64 samples (64 HR >= L - 1); a segment yields 1024 - 64 HR
// outputs.  A 1024-thread workgroup shares the twiddle and spectrum tables in
// LDS, one 8.7 KB transpose buffer per wave (rows of 17: 16 lanes reading the
// same slot of consecutive rows hit distinct banks).
constexpr int kWRow = 17;
constexpr int kWBuf = 64 * kWRow;

template <int HR, int NOMEM>
__global__ void __launch_bounds__(1024)
fir_ols1024_wave_kernel(const cf* __restrict__ x, const cf* __restrict__ hist, const cf* __restrict__ H1k,
                        const cf* __restrict__ tw1k, cf* __restrict__ y, long long n, int Lm1, long long nseg) {
    __shared__ cf sTw[1024];
    __shared__ cf sH[1024];
    __shared__ cf sBuf[16 * kWBuf];
    const int tid = threadIdx.x, L = tid & 63;
    const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    for (int i = tid; i < 1024; i += 1024) {
        sTw[i] = tw1k[i];
        sH[i] = H1k[i];
    }
    __syncthreads();
    const int ch = blockIdx.y;
    x += (long long)ch * n;
    y += (long long)ch * n;
    hist += (long long)ch * Lm1;
    cf* const buf = sBuf + wv * kWBuf;
    constexpr int V = 1024 - 64 * HR;
    const int n0 = L & 3, n1 = L >> 2;  // P1 / P1' view
    const int k2v = L >> 2;             // P2 / P2' view: lane = n0 + 4 k2

    const long long gw = (long long)blockIdx.x * 16 + wv;
    const long long GW = (long long)gridDim.x * 16;
    auto base_of = [&](long long sg) { return sg * V - 64 * HR; };
    auto interior = [&](long long sg) { return sg < nseg && base_of(sg) >= 0 && base_of(sg) + 1024 <= n; };

    auto segment = [&](cf (&v)[16], auto&& after_p1) {
        // P1
        dft16<false>(v);
#pragma unroll
        for (int k = 1; k < 16; ++k) v[k] = cmul(v[k], sTw[(L * k) & 1023]);
        after_p1();
#pragma unroll
        for (int k = 0; k < 16; ++k) buf[(n0 + 4 * k) * kWRow + n1] = v[k];
        wave_sync_lds();
        // P2
#pragma unroll
        for (int i = 0; i < 16; ++i) v[i] = buf[L * kWRow + i];
        dft16<false>(v);
#pragma unroll
        for (int k = 1; k < 16; ++k) v[k] = cmul(v[k], sTw[(16 * n0 * k) & 1023]);
        wave_sync_lds();
#pragma unroll
        for (int k = 0; k < 16; ++k) buf[(k2v + 16 * k) * 4 + n0] = v[k];
        wave_sync_lds();
        // P3: DFT4, spectrum, IDFT4 per column c
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int c = L + 64 * j;
            cf a0 = buf[c * 4 + 0], a1 = buf[c * 4 + 1], a2 = buf[c * 4 + 2], a3 = buf[c * 4 + 3];
            dft4<false>(a0, a1, a2, a3);
            a0 = cmul(a0, sH[c]);
            a1 = cmul(a1, sH[c + 256]);
            a2 = cmul(a2, sH[c + 512]);
            a3 = cmul(a3, sH[c + 768]);
            dft4<true>(a0, a1, a2, a3);
            buf[c * 4 + 0] = a0;
            buf[c * 4 + 1] = a1;
            buf[c * 4 + 2] = a2;
            buf[c * 4 + 3] = a3;
        }
        wave_sync_lds();
        // P2'
#pragma unroll
        for (int k = 0; k < 16; ++k) v[k] = buf[(k2v + 16 * k) * 4 + n0];
#pragma unroll
        for (int k = 1; k < 16; ++k) v[k] = cmulc(v[k], sTw[(16 * n0 * k) & 1023]);
        dft16<true>(v);
        wave_sync_lds();
#pragma unroll
        for (int i = 0; i < 16; ++i) buf[L * kWRow + i] = v[i];
        wave_sync_lds();
        // P1'
#pragma unroll
        for (int k = 0; k < 16; ++k) v[k] = buf[(n0 + 4 * k) * kWRow + n1];
#pragma unroll
        for (int k = 1; k < 16; ++k) v[k] = cmulc(v[k], sTw[(L * k) & 1023]);
        dft16<true>(v);
        wave_sync_lds();  // buffer free for the next segment
    };

    // boundary segments: guarded element loads and stores
    auto boundary = [&](long long sg) {
        cf v[16];
        const long long base = base_of(sg);
#pragma unroll
        for (int r = 0; r < 16; ++r) v[r] = ext_ld<true>(x, hist, base + L + 64 * r, n, Lm1);
        segment(v, [] {});
#pragma unroll
        for (int r = HR; r < 16; ++r)
            if (base + L + 64 * r < n) y[base + L + 64 * r] = v[r];
    };

    long long seg = gw;
    if (seg < nseg && !interior(seg)) {
        boundary(seg);
        seg += GW;
    }
    cf nv[16];
    auto load = [&](long long sg) {
        if constexpr (NOMEM) {
#pragma unroll
            for (int r = 0; r < 16; ++r) nv[r] = cf{(float)(L + r), (float)(sg & 1023)};
        } else {
            const cf* xb = x + base_of(sg) + L;
#pragma unroll
            for (int r = 0; r < 16; ++r) nv[r] = xb[64 * r];
        }
    };
    if (interior(seg)) load(seg);
    for (; interior(seg); seg += GW) {
        cf v[16];
#pragma unroll
        for (int r = 0; r < 16; ++r) v[r] = nv[r];
        const long long nxt = interior(seg + GW) ? seg + GW : seg;
        segment(v, [&] { load(nxt); });
        cf* yb = y + base_of(seg) + L;
        if constexpr (NOMEM) {
#pragma unroll
            for (int r = HR; r < 16; ++r)
                if (v[r].re == 1234.5678f) yb[64 * r] = v[r];
        } else {
#pragma unroll
            for (int r = HR; r < 16; ++r) yb[64 * r] = v[r];
        }
    }
    for (; seg < nseg; seg += GW) boundary(seg);
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

hipError_t launch_fir_ols(const OlsPlan& p, const void* x, const void* hist, void* y, size_t n, int L,
                          size_t channels, int num_cus, hipStream_t s) {
    if (n == 0) return hipSuccess;
    const int h2 = p.halo_rows;
    const long long V = 4096 - 256 * h2;
    const long long nseg = ((long long)n + V - 1) / V;
    long long blocks = (long long)num_cus * 2;
    long long per = (nseg + blocks - 1) / blocks;
    if (per < 1) per = 1;
    if (!p.interleave) blocks = (nseg + per - 1) / per;
    else if (blocks > nseg) blocks = nseg;
    dim3 grid((unsigned)blocks, (unsigned)channels);
#define SDSP_OLS_LAUNCH(I, NM, H)                                                                                \
    hipLaunchKernelGGL((fir_ols4096_kernel<I, NM, H, 0>), grid, dim3(256), 0, s, (const cf*)x, (const cf*)hist,      \
                       (const cf*)p.d_H, (const cf*)p.d_tw1, (const cf*)p.d_tw2, (cf*)y, (long long)n, L - 1, h2, \
                       nseg, per)
    if (p.wave && p.d_H1k) {
        const int hr = p.halo_rows_1k;
        const long long V1 = 1024 - 64 * hr;
        const long long nseg1 = ((long long)n + V1 - 1) / V1;
        long long wg = ((nseg1 + 15) / 16 + 3) / 4;  // about four segments per wave
        const long long cap = (long long)num_cus * 8;
        if (wg > cap) wg = cap;
        if (wg < 1) wg = 1;
        dim3 g1((unsigned)wg, (unsigned)channels);
#define SDSP_OLS_WAVE(HRV, NM)                                                                                   \
    hipLaunchKernelGGL((fir_ols1024_wave_kernel<HRV, NM>), g1, dim3(1024), 0, s, (const cf*)x, (const cf*)hist,   \
                       (const cf*)p.d_H1k, (const cf*)p.d_tw1k, (cf*)y, (long long)n, L - 1, nseg1)
        const int nm = p.nomem == 1 ? 1 : 0;
        switch (hr) {
            case 1: if (nm) SDSP_OLS_WAVE(1, 1); else SDSP_OLS_WAVE(1, 0); break;
            case 2: if (nm) SDSP_OLS_WAVE(2, 1); else SDSP_OLS_WAVE(2, 0); break;
            case 3: if (nm) SDSP_OLS_WAVE(3, 1); else SDSP_OLS_WAVE(3, 0); break;
            case 4: if (nm) SDSP_OLS_WAVE(4, 1); else SDSP_OLS_WAVE(4, 0); break;
            default: return hipErrorInvalidValue;
        }
#undef SDSP_OLS_WAVE
        return hipGetLastError();
    }
    // packed interior kernel: by default only with 16-byte rows (its 8-byte form is slower than this file's)
    const bool rows16 = ((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(y)) & 15) == 0 &&
                        (channels == 1 || n % 2 == 0);
    if (p.packed && (rows16 || !p.wide) && p.interleave && p.nomem != 2 && p.nomem != 3 && h2 >= 1 && h2 <= 4) {
        // interior segments in packed arithmetic, the boundary ones here
        long long lo, hi;
        ols_interior_range((long long)n, h2, &lo, &hi);
        const long long nedge = lo + (nseg - hi);
        if (nedge > 0 && !p.nomem) {
            hipLaunchKernelGGL(fir_ols4096_edge_kernel, dim3((unsigned)nedge, (unsigned)channels), dim3(256), 0, s,
                               (const cf*)x, (const cf*)hist, (const cf*)p.d_H, (const cf*)p.d_tw1,
                               (const cf*)p.d_tw2, (cf*)y, (long long)n, L - 1, h2, lo, hi);
            hipError_t e = hipGetLastError();
            if (e != hipSuccess) return e;
        }
        static const int kAbl[11] = {0, 1, 0, 0, 3, 3, 7, 8, 24, 40, 16};  // 40: HBM only + spectrum table
        const int abl = kAbl[p.nomem];
        if (p.packed <= 2) return pk_default::launch_fir_ols_pk(p, x, y, n, channels, num_cus, s, lo, hi, abl);
        if (p.packed <= 4) return pk_ilp::launch_fir_ols_pk(p, x, y, n, channels, num_cus, s, lo, hi, abl);
        return pk_iilp::launch_fir_ols_pk(p, x, y, n, channels, num_cus, s, lo, hi, abl);
    }
    if (p.nomem) {  // profiling ablations (h2 = 1 only): 1 no HBM traffic, 2 no loads, 3 no stores
        if (p.nomem == 2) SDSP_OLS_LAUNCH(true, 2, 1);
        else if (p.nomem == 4) SDSP_OLS_LAUNCH(true, 4, 1);
        else if (p.nomem == 3) SDSP_OLS_LAUNCH(true, 3, 1);
        else SDSP_OLS_LAUNCH(true, 1, 1);
    } else if (p.interleave && h2 == 1 && p.nt) {
#define SDSP_OLS_NT(NTV)                                                                                          \
    hipLaunchKernelGGL((fir_ols4096_kernel<true, 0, 1, NTV>), grid, dim3(256), 0, s, (const cf*)x, (const cf*)hist, \
                       (const cf*)p.d_H, (const cf*)p.d_tw1, (const cf*)p.d_tw2, (cf*)y, (long long)n, L - 1, h2,  \
                       nseg, per)
        if (p.nt == 1) SDSP_OLS_NT(1);
        else if (p.nt == 2) SDSP_OLS_NT(2);
        else if (p.nt == 3) SDSP_OLS_NT(3);
        else if (p.nt == 4) SDSP_OLS_NT(4);
        else SDSP_OLS_NT(7);
#undef SDSP_OLS_NT
    } else if (p.interleave) {
        if (h2 == 1) SDSP_OLS_LAUNCH(true, 0, 1);
        else if (h2 == 2) SDSP_OLS_LAUNCH(true, 0, 2);
        else SDSP_OLS_LAUNCH(true, 0, 0);
    } else {
        SDSP_OLS_LAUNCH(false, 0, 0);
    }
#undef SDSP_OLS_LAUNCH
    return hipGetLastError();
}

}  // namespace sdsp
