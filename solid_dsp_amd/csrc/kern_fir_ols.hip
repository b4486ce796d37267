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

// ---- 16-byte-per-lane global access --------------------------------------
// Lane t needs x[base + 256 r + t] for rows r = 0..15 (8 bytes, coalesced).
// For a row pair (a, b) = (2q, 2q+1) an even lane reads x[base+256a+t .. +1]
// and an odd lane x[base+256b+t-1 .. +1], each one 16-byte access; one DPP
// swap between lanes t and t^1 then gives every lane its own two values.
// Stores use the inverse.  base and V are even, so every 16-byte access is
// aligned.
__device__ __forceinline__ float swap_pair(float v) {  // value of lane t^1 (DPP quad_perm [1,0,3,2])
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0xB1, 0xF, 0xF, false));
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

// raw[q] = the 16 bytes this lane reads for row pair q
template <bool CHECK>
__device__ __forceinline__ void load_raw(float4 (&raw)[8], const cf* __restrict__ x, const cf* __restrict__ hist,
                                         long long base, int t, long long n, int Lm1) {
    const int odd = t & 1;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
        const long long j = base + 256 * (2 * q + odd) + t - odd;  // even index
        if constexpr (!CHECK) {
            raw[q] = *reinterpret_cast<const float4*>(x + j);
        } else {
            const cf a = ext_ld<true>(x, hist, j, n, Lm1), b = ext_ld<true>(x, hist, j + 1, n, Lm1);
            raw[q] = make_float4(a.re, a.im, b.re, b.im);
        }
    }
}

__device__ __forceinline__ void unpack_raw(cf (&v)[16], const float4 (&raw)[8], int t) {
    const bool odd = t & 1;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
        const float4 r = raw[q];
        // even lane sends its partner's row-a value (hi), odd lane its partner's row-b value (lo)
        const float sre = odd ? r.x : r.z, sim = odd ? r.y : r.w;
        const float gre = swap_pair(sre), gim = swap_pair(sim);
        v[2 * q] = odd ? cf{gre, gim} : cf{r.x, r.y};
        v[2 * q + 1] = odd ? cf{r.z, r.w} : cf{gre, gim};
    }
}

// store rows >= h2 of v (row r at y[ob + 256 r], ob = segment output base + t)
template <bool CHECK>
__device__ __forceinline__ void store_rows(cf* __restrict__ y, const cf (&v)[16], long long ob, int t, int h2,
                                           long long n) {
    const bool odd = t & 1;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
        const cf a = v[2 * q], b = v[2 * q + 1];
        // even lane needs the odd partner's row-a value, odd lane the even partner's row-b value
        const float sre = odd ? a.re : b.re, sim = odd ? a.im : b.im;
        const float gre = swap_pair(sre), gim = swap_pair(sim);
        const int row = 2 * q + (odd ? 1 : 0);
        const long long j = ob + 256 * row - (odd ? 1 : 0);  // even index
        const float4 w = odd ? make_float4(gre, gim, b.re, b.im) : make_float4(a.re, a.im, gre, gim);
        if (row >= h2) {
            if constexpr (!CHECK) {
                *reinterpret_cast<float4*>(y + j) = w;
            } else {
                if (j >= 0 && j < n) y[j] = cf{w.x, w.y};
                if (j + 1 >= 0 && j + 1 < n) y[j + 1] = cf{w.z, w.w};
            }
        }
    }
}

}  // namespace

template <bool WIDE, bool INTERLEAVE, bool DEPTH2, bool NOMEM = false>
__global__ void __launch_bounds__(256, 2)
fir_ols4096_kernel(const cf* __restrict__ x, const cf* __restrict__ hist, const cf* __restrict__ Hs,
                   const cf* __restrict__ tw1, const cf* __restrict__ tw2, cf* __restrict__ y, long long n,
                   int Lm1, int h2, long long nseg, long long segs_per_block) {
    __shared__ __attribute__((aligned(16))) cf lds[2 * kRegion];
    cf* const rA = lds;
    cf* const rB = lds + kRegion;
    const int ch = blockIdx.y;
    x += (long long)ch * n;
    y += (long long)ch * n;
    hist += (long long)ch * Lm1;

    const int t = threadIdx.x;
    const int hi4 = t >> 4, lo4 = t & 15;
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

    // software pipeline: the next segment's loads are issued right after this
    // segment's P1 and land while P2..P5 run (2 waves/SIMD cannot hide HBM
    // latency otherwise)
    float4 nx[8];
    cf nv[16], nv2[16];
    auto load_plain = [&](cf (&dst)[16], long long sg) {
        const long long base = sg * V - 256 * h2;
        if constexpr (NOMEM) {  // ablation build: no HBM traffic, same arithmetic
#pragma unroll
            for (int r = 0; r < 16; ++r) dst[r] = cf{(float)(t + r), (float)(sg & 1023)};
            return;
        }
        // branch once per segment: a per-element "load or select" makes hipcc
        // wait for every load separately
        if (base >= 0 && base + 4096 <= n) {
#pragma unroll
            for (int r = 0; r < 16; ++r) dst[r] = x[base + 256 * r + t];
        } else {
#pragma unroll
            for (int r = 0; r < 16; ++r) dst[r] = ext_ld<true>(x, hist, base + 256 * r + t, n, Lm1);
        }
    };
    auto prefetch = [&](long long sg) {
        if constexpr (WIDE) {
            const long long base = sg * V - 256 * h2;
            if (base >= 0 && base + 4096 <= n) load_raw<false>(nx, x, hist, base, t, n, Lm1);
            else load_raw<true>(nx, x, hist, base, t, n, Lm1);
        } else if constexpr (DEPTH2) {
#pragma unroll
            for (int r = 0; r < 16; ++r) nv[r] = nv2[r];
            if (sg + sstep < s1) load_plain(nv2, sg + sstep);
        } else {
            load_plain(nv, sg);
        }
    };
    if (s0 < s1) {
        if constexpr (!WIDE && DEPTH2) {
            load_plain(nv2, s0);
            prefetch(s0);
        } else {
            prefetch(s0);
        }
    }
    for (long long seg = s0; seg < s1; seg += sstep) {
        cf v[16];
        if constexpr (WIDE) {
            unpack_raw(v, nx, t);
        } else {
#pragma unroll
            for (int r = 0; r < 16; ++r) v[r] = nv[r];
        }

        // P1: DFT over n2 -> k0, twiddle, A[k0][t]
        dft16<false>(v);
#pragma unroll
        for (int k = 0; k < 16; ++k) rA[k * kRowA + t] = cmul(v[k], w1[k]);
        if (seg + sstep < s1) prefetch(seg + sstep);
        __syncthreads();
        // P2: lane (k0=hi4, n0=lo4) reads n1
#pragma unroll
        for (int k = 0; k < 16; ++k) v[k] = rA[hi4 * kRowA + 16 * k + lo4];
        dft16<false>(v);
#pragma unroll
        for (int k = 0; k < 16; ++k) rB[bidx(16 * hi4 + k, lo4)] = cmul(v[k], w2[k]);
        __syncthreads();
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
        __syncthreads();
        // P4: lane (k0=hi4, n0=lo4) reads k1
#pragma unroll
        for (int k = 0; k < 16; ++k) v[k] = rA[bidx(16 * hi4 + k, lo4)];
        dft16<true>(v);
#pragma unroll
        for (int k = 0; k < 16; ++k) rB[hi4 * kRowA + 16 * k + lo4] = v[k];
        __syncthreads();
        // P5: lane t=(n1,n0) reads k0
#pragma unroll
        for (int k = 0; k < 16; ++k) v[k] = cmulc(rB[k * kRowA + t], w1[k]);
        dft16<true>(v);
        const long long ob = seg * V - 256 * h2 + t;
        if constexpr (NOMEM) {
#pragma unroll
            for (int k = 0; k < 16; ++k)
                if (v[k].re == 1234.5678f && k >= h2) y[ob + 256 * k] = v[k];
        } else if constexpr (WIDE) {
            if (ob - 1 >= 0 && ob + 256 * 16 <= n) store_rows<false>(y, v, ob, t, h2, n);
            else store_rows<true>(y, v, ob, t, h2, n);
        } else {
            if (ob + 256 * 16 <= n) {
#pragma unroll
                for (int k = 0; k < 16; ++k)
                    if (k >= h2) y[ob + 256 * k] = v[k];
            } else {
#pragma unroll
                for (int k = 0; k < 16; ++k)
                    if (k >= h2 && ob + 256 * k < n) y[ob + 256 * k] = v[k];
            }
        }
        // next segment's P1 writes region A: every lane has finished reading
        // region A (P4) before the barrier that precedes P5.
    }
}

// ---------------------------------------------------------------------------
// Occupancy variant: one LDS region (8 barriers per segment), the spectrum
// slice read from L2 inside P3 instead of living in registers, no register
// prefetch (thread-level parallelism hides the loads instead).  Targets 3-4
// waves per SIMD: the 2-wave kernel above is VALU-issue bound (an ablation
// without HBM traffic runs at 80% of its time).
template <int WAVES_PER_SIMD, bool NOMEM>
__global__ void __launch_bounds__(256, WAVES_PER_SIMD)
fir_ols4096_occ_kernel(const cf* __restrict__ x, const cf* __restrict__ hist, const cf* __restrict__ Hs,
                       const cf* __restrict__ tw1, const cf* __restrict__ tw2, cf* __restrict__ y, long long n,
                       int Lm1, int h2, long long nseg) {
    __shared__ __attribute__((aligned(16))) cf lds[kRegion];
    const int ch = blockIdx.y;
    x += (long long)ch * n;
    y += (long long)ch * n;
    hist += (long long)ch * Lm1;
    const int t = threadIdx.x;
    const int hi4 = t >> 4, lo4 = t & 15;
    cf w1[16], w2[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        w1[k] = tw1[t * 16 + k];
        w2[k] = tw2[lo4 * 16 + k];
    }
    const int V = 4096 - 256 * h2;
    for (long long seg = blockIdx.x; seg < nseg; seg += gridDim.x) {
        cf v[16];
        const long long base = seg * V - 256 * h2;
        if constexpr (NOMEM) {
#pragma unroll
            for (int r = 0; r < 16; ++r) v[r] = cf{(float)(t + r), (float)(seg & 1023)};
        } else if (base >= 0 && base + 4096 <= n) {
#pragma unroll
            for (int r = 0; r < 16; ++r) v[r] = x[base + 256 * r + t];
        } else {
#pragma unroll
            for (int r = 0; r < 16; ++r) v[r] = ext_ld<true>(x, hist, base + 256 * r + t, n, Lm1);
        }
        // P1
        dft16<false>(v);
        __syncthreads();  // previous segment's P5 reads of the region are done
#pragma unroll
        for (int k = 0; k < 16; ++k) lds[k * kRowA + t] = cmul(v[k], w1[k]);
        __syncthreads();
        // P2
#pragma unroll
        for (int k = 0; k < 16; ++k) v[k] = lds[hi4 * kRowA + 16 * k + lo4];
        dft16<false>(v);
        __syncthreads();
#pragma unroll
        for (int k = 0; k < 16; ++k) lds[bidx(16 * hi4 + k, lo4)] = cmul(v[k], w2[k]);
        __syncthreads();
        // P3
        {
            const float4* row = reinterpret_cast<const float4*>(lds + t * 16);
#pragma unroll
            for (int p = 0; p < 8; ++p) {
                const float4 q = row[(p ^ (t >> 1)) & 7];
                v[2 * p] = {q.x, q.y};
                v[2 * p + 1] = {q.z, q.w};
            }
        }
        cf Hr[16];
#pragma unroll
        for (int k = 0; k < 16; ++k) Hr[k] = Hs[t * 16 + k];
        dft16<false>(v);
#pragma unroll
        for (int k = 0; k < 16; ++k) v[k] = cmul(v[k], Hr[k]);
        dft16<true>(v);
        __syncthreads();
        {
            float4* row = reinterpret_cast<float4*>(lds + t * 16);
#pragma unroll
            for (int p = 0; p < 8; ++p) {
                const cf a = cmulc(v[2 * p], w2[2 * p]);
                const cf b = cmulc(v[2 * p + 1], w2[2 * p + 1]);
                row[(p ^ (t >> 1)) & 7] = make_float4(a.re, a.im, b.re, b.im);
            }
        }
        __syncthreads();
        // P4
#pragma unroll
        for (int k = 0; k < 16; ++k) v[k] = lds[bidx(16 * hi4 + k, lo4)];
        dft16<true>(v);
        __syncthreads();
#pragma unroll
        for (int k = 0; k < 16; ++k) lds[hi4 * kRowA + 16 * k + lo4] = v[k];
        __syncthreads();
        // P5
#pragma unroll
        for (int k = 0; k < 16; ++k) v[k] = cmulc(lds[k * kRowA + t], w1[k]);
        dft16<true>(v);
        const long long ob = seg * V - 256 * h2 + t;
        if constexpr (NOMEM) {
#pragma unroll
            for (int k = 0; k < 16; ++k)
                if (v[k].re == 1234.5678f && k >= h2) y[ob + 256 * k] = v[k];
        } else if (ob + 256 * 16 <= n) {
#pragma unroll
            for (int k = 0; k < 16; ++k)
                if (k >= h2) y[ob + 256 * k] = v[k];
        } else {
#pragma unroll
            for (int k = 0; k < 16; ++k)
                if (k >= h2 && ob + 256 * k < n) y[ob + 256 * k] = v[k];
        }
    }
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
#define SDSP_OLS_LAUNCH(W, I)                                                                              \
    hipLaunchKernelGGL((fir_ols4096_kernel<W, I, false>), grid, dim3(256), 0, s, (const cf*)x, (const cf*)hist,      \
                       (const cf*)p.d_H, (const cf*)p.d_tw1, (const cf*)p.d_tw2, (cf*)y, (long long)n, L - 1, h2, \
                       nseg, per)
#define SDSP_OLS_LAUNCH_D2(I)                                                                              \
    hipLaunchKernelGGL((fir_ols4096_kernel<false, I, true>), grid, dim3(256), 0, s, (const cf*)x, (const cf*)hist, \
                       (const cf*)p.d_H, (const cf*)p.d_tw1, (const cf*)p.d_tw2, (cf*)y, (long long)n, L - 1, h2, \
                       nseg, per)
    if (p.occ) {
        long long ob = (long long)num_cus * p.occ;
        if (ob > nseg) ob = nseg;
        dim3 g2((unsigned)ob, (unsigned)channels);
#define SDSP_OLS_OCC(WV, NM)                                                                                   \
    hipLaunchKernelGGL((fir_ols4096_occ_kernel<WV, NM>), g2, dim3(256), 0, s, (const cf*)x, (const cf*)hist,      \
                       (const cf*)p.d_H, (const cf*)p.d_tw1, (const cf*)p.d_tw2, (cf*)y, (long long)n, L - 1, h2, nseg)
        if (p.occ >= 4) { if (p.nomem) SDSP_OLS_OCC(4, true); else SDSP_OLS_OCC(4, false); }
        else { if (p.nomem) SDSP_OLS_OCC(3, true); else SDSP_OLS_OCC(3, false); }
#undef SDSP_OLS_OCC
    } else if (p.nomem) {
        hipLaunchKernelGGL((fir_ols4096_kernel<false, true, false, true>), grid, dim3(256), 0, s, (const cf*)x,
                           (const cf*)hist, (const cf*)p.d_H, (const cf*)p.d_tw1, (const cf*)p.d_tw2, (cf*)y,
                           (long long)n, L - 1, h2, nseg, per);
    } else if (p.depth2 && !p.wide) {
        if (p.interleave) SDSP_OLS_LAUNCH_D2(true);
        else SDSP_OLS_LAUNCH_D2(false);
    } else if (p.wide) {
        if (p.interleave) SDSP_OLS_LAUNCH(true, true);
        else SDSP_OLS_LAUNCH(true, false);
    } else {
        if (p.interleave) SDSP_OLS_LAUNCH(false, true);
        else SDSP_OLS_LAUNCH(false, false);
    }
#undef SDSP_OLS_LAUNCH
#undef SDSP_OLS_LAUNCH_D2
    return hipGetLastError();
}

}  // namespace sdsp
