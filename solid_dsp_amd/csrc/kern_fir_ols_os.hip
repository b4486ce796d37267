// One-shot, XCD-ordered overlap-save FIR for 32-bit complex streams (gfx950):
// the default interior-segment kernel of FIRFilter::execute_block for c32.
//
// Same filter as FIRFilter::execute (src/filter/fir/mod.rs:209-212),
//     y[n] = scale * sum_{i<L} h[L-1-i] x[n-i],
// per 4096-sample segment as a circular convolution with the zero-padded
// g[i] = scale h[L-1-i] (spectrum H/N precomputed in f64 on the host).
// Segment s reads x[s V - H, s V - H + 4096) and writes the V = 4096 - H
// outputs that do not wrap (H = 256 h2 >= L - 1).  The transform is the one of
// kern_fir_ols.hip / kern_fir_ols_pk.hip (three radix-16 passes each way,
// n = 256 n2 + 16 n1 + n0, k = k0 + 16 k1 + 256 k2, no bit reversal), in packed
// FP32 with the fused DFT16 of sdsp_pk.hpp (72 packed instructions per DFT16).
// What differs is the shape, chosen for the HBM stream:
//
//  * one segment per 256-thread workgroup, one workgroup per segment (no
//    persistent loop): the dispatcher deals workgroup b to XCD b % 8, so
//    segment(b) = lo + (b % 8) q + b / 8 makes every XCD stream one contiguous
//    eighth of the call in order (the halo row of a segment is the tail its XCD
//    neighbour just read, an L2 hit);
//  * 4 workgroups per CU (16 waves): 116 VGPRs and one 34 KB LDS image.  The
//    image is ALIASED across phases: in P2/P4 lane (k0, n0) owns the 16
//    positions (k0, 16 j + n0), in P3 lane (k0, k1) owns (k0, 16 k1 + j), in
//    P1/P5 lane t owns column t -- each lane reads and rewrites only its own
//    positions inside a phase, so one region suffices.  P2, P3 and P4 of wave w
//    touch only rows k0 = 4w .. 4w + 3, so only P1 -> P2 and P4 -> P5 need a
//    workgroup barrier;
//  * lane t owns column t in P1 / P5: 8-byte buffer loads and stores per row
//    (row offsets in SGPRs, no address arithmetic in VGPRs);
//  * no twiddle tables in LDS or per-lane tables in registers: W4096^(t k) =
//    D_{k>>2} C_{k&3} and W256^(l k) = F_{k>>2} E_{k&3} from per-lane bases
//    (C1, D1, E1, F1: two float4 from L2; C2 = C1 C1, C3 = C2 C1, ...), the
//    spectrum slice of P3 loaded from L2 in P2;
//  * nontemporal input loads and stores (the stream is read and written once).
//
// LDS image: element (r, c) at r * 272 + c + (c >> 4) (one 8-byte pad per
// 16-column block; rows 544 dwords apart, i.e. opposite halves of the 64
// banks).  Every access is a per-lane base plus a compile-time offset and is
// conflict-free except P5's reads (lanes 0 and 31 of a 32-lane group share a
// bank pair: SQ_LDS_BANK_CONFLICT counts 2 extra cycles per ds_read_b64,
// tools/lds_probe.hip).
//
// Numerics: bit-identical across calls and launch shapes; against the f64
// restatement rel-RMS ~2.2e-7 on the cfg2 taps (§8d tolerance 1e-6).
//
// The variants measured against this kernel (ablations, load orders, table forms, segment
// pairs, half spectra, ...) live in the lab copy tools/lab/ols_os_lab_kernel.hip (tools only);
// the history is in profiles/LABLOG.md and profiles/r06/LAB.md.
#include "sdsp_device.hpp"
#include "sdsp_kernels.hpp"
#include "sdsp_pk.hpp"

namespace sdsp {

using namespace pk;

namespace {

constexpr int kRow = 272;

typedef unsigned int u2v __attribute__((ext_vector_type(2)));
typedef unsigned int u4v __attribute__((ext_vector_type(4)));
constexpr int kBufWord3 = 0x00020000;  // raw buffer descriptor word 3 (gfx9 family)
constexpr int kNT = 2;                 // nontemporal cache policy of a buffer access

// P2 -> P3 -> P4 hand-offs stay inside one wave: the next phase reads only what this wave wrote
// (the LDS operations of one wave complete in order), so a compiler-level fence replaces the
// block barrier
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// x = D_{k>>2} C_{k&3} for C_b = c[b-1], D_a = d[a-1] (k = 0 -> 1)
__device__ __forceinline__ f2 tw_pair(const f2 (&c)[3], const f2 (&d)[3], int k) {
    const int a = k >> 2, b = k & 3;
    if (a == 0) return b == 0 ? f2{1.0f, 0.0f} : c[b - 1];
    if (b == 0) return d[a - 1];
    return pmul(d[a - 1], c[b - 1]);
}

// lane pair (2c, 2c + 1) exchange: even lanes lo = a, odd lanes lo = the partner's b; odd lanes
// hi = b, even lanes hi = the partner's a.  Loads: (a, b) = columns (2c, 2c + 1) of row k + 8h ->
// (lo, hi) = rows (k, 8 + k) of column 2c + h.  Stores: (a, b) = rows (k, 8 + k) of column 2c + h
// -> (lo, hi) = columns (2c, 2c + 1) of row k + 8h.  One v_cndmask_b32 with a quad_perm DPP
// operand per dword (the partner's register read in the same instruction); the s_nop covers
// the DPP read-after-VALU-write hazard of an operand the compiler computed just before.
__device__ __forceinline__ void pair_exchange(f2 a, f2 b, f2& lo, f2& hi) {
    float l0, l1, h0, h1;
    asm("s_nop 1\n\t"
        "s_mov_b32 vcc_lo, 0x55555555\n\t"
        "s_mov_b32 vcc_hi, 0x55555555\n\t"
        "v_cndmask_b32_dpp %0, %6, %4, vcc quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
        "v_cndmask_b32_dpp %1, %7, %5, vcc quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
        "s_not_b64 vcc, vcc\n\t"
        "v_cndmask_b32_dpp %2, %4, %6, vcc quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
        "v_cndmask_b32_dpp %3, %5, %7, vcc quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf"
        : "=&v"(l0), "=&v"(l1), "=&v"(h0), "=&v"(h1)
        : "v"(a.x), "v"(a.y), "v"(b.x), "v"(b.y)
        : "vcc");
    lo = f2{l0, l1};
    hi = f2{h0, h1};
}

}  // namespace

// One segment of the transform.  Template parameters (the product's instances only):
//   HALO1  the halo is one row (L <= 257, every cfg2-like filter): rows 1..15 are stored without a
//          test per row, and the two rows a neighbouring segment also reads (row 0, the halo, and
//          row 15, the next segment's halo) load with the default cache policy, the others
//          nontemporal (traffic 1.00005x instead of 1.029x, profiles/r05);
//   WIDE   16-byte lanes (SDSP_TUNE_OLS_KERNEL = 3): lane pair (2c, 2c + 1) moves columns
//          (2c, 2c + 1) of rows k + 8h and swaps halves by DPP (1-2.5 % slower: the exchange costs
//          more than the wider accesses save);
//   EDGE   the boundary segments of a call (launched apart, so the interior kernel carries no
//          boundary code): past the end of the stream loads return 0 and stores are dropped, rows
//          before it come from the history, and the call's last segment writes the next history.
template <bool HALO1, bool WIDE, bool EDGE>
__device__ __forceinline__ void ols_os_segment(const f2* __restrict__ x, const f2* __restrict__ hist,
                                               f2* __restrict__ new_hist, const float4* __restrict__ Hs,
                                               const float4* __restrict__ tb, f2* __restrict__ y, long long base,
                                               long long n, int Lm1, int h2, f2* img, int t) {
    const int hi4 = t >> 4, lo4 = t & 15;
    if constexpr (HALO1) h2 = 1;  // compiled in (the launcher checks h2 == 1)
    // the segment's window x[base, base + 4096) as a raw buffer
    const long long rem = n - base;
    const int nrec = (!EDGE || rem >= 4096) ? 32768 : (int)(8 * rem);
    const auto rx = __builtin_amdgcn_make_buffer_rsrc((void*)(x + base), (short)0, nrec, kBufWord3);
    const auto ry = __builtin_amdgcn_make_buffer_rsrc((void*)(y + base), (short)0, nrec, kBufWord3);
    const auto rt = __builtin_amdgcn_make_buffer_rsrc((void*)tb, (short)0, kOlsOsTabF4 * 16, kBufWord3);
    const auto rh = __builtin_amdgcn_make_buffer_rsrc((void*)Hs, (short)0, 2048 * 16, kBufWord3);
    // twiddle bases: {C1, D1} of column t and {E1, F1} of row lo4 (runtime.cpp ols_build), requested
    // before the segment's rows (L2 hits that land while the rows stream in)
    const float4 cd = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rt, 16 * t, 16 * kOlsOsTabCD, 0));
    const float4 ef = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rt, 16 * lo4, 16 * kOlsOsTabEF, 0));
    f2 v[16];
    if constexpr (EDGE) {
        // rows inside the stream through rx, rows before it from the handle's history (the last
        // Lm1 inputs, oldest first; positions before the history read as 0 through an
        // out-of-range offset)
        const auto rp = __builtin_amdgcn_make_buffer_rsrc((void*)hist, (short)0, 8 * Lm1, kBufWord3);
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const long long pos = base + 256 * r;
            if (pos >= 0) {
                v[r] = __builtin_bit_cast(f2, __builtin_amdgcn_raw_buffer_load_b64(rx, 8 * t, 2048 * r, 0));
            } else {
                const long long e = Lm1 + pos + t;
                v[r] = __builtin_bit_cast(f2, __builtin_amdgcn_raw_buffer_load_b64(rp, e >= 0 ? (int)(8 * e) : 0x7ffffff0, 0, 0));
            }
        }
        if (new_hist != nullptr) {
            // the call's last segment: its window holds the last Lm1 inputs (halo >= Lm1), which
            // become the history of the next call (ping-pong buffer: never the one read above)
            const long long h0 = n - Lm1;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const long long i = base + 256 * r + t - h0;
                if (i >= 0 && i < Lm1) new_hist[i] = v[r];
            }
        }
    } else if constexpr (WIDE) {
        // 16-byte lanes: lane t = 2c + h loads columns (2c, 2c + 1) of rows k + 8h, then one DPP
        // exchange per dword with its partner lane t ^ 1 gives it column t over the rows
        f4v q[8];
#pragma unroll
        for (int k = 0; k < 8; ++k)
            q[k] = __builtin_bit_cast(f4v, __builtin_amdgcn_raw_buffer_load_b128(rx, 16 * (t >> 1) + 16384 * (t & 1),
                                                                                2048 * k, kNT));
#pragma unroll
        for (int k = 0; k < 8; ++k) pair_exchange(f2{q[k].x, q[k].y}, f2{q[k].z, q[k].w}, v[k], v[8 + k]);
    } else {
        // the rows in row order (the compiler interleaves them as 0, 4, 1, 5, 8, 12, 9, 13, ...):
        // 2 % faster than the first radix-4 stage's order and than either order enforced with
        // scheduling barriers (profiles/r05/lab/r05h_olsburst.log, r05i_olsburst.log)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            if (HALO1 && (r == 0 || r == 15))
                v[r] = __builtin_bit_cast(f2, __builtin_amdgcn_raw_buffer_load_b64(rx, 8 * t, 2048 * r, 0));
            else
                v[r] = __builtin_bit_cast(f2, __builtin_amdgcn_raw_buffer_load_b64(rx, 8 * t, 2048 * r, kNT));
        }
    }
    // the first power of each base from L2, the others as products (W^2 = W W, W^3 = W^2 W)
    f2 Cb[3], Da[3], Eb[3], Fa[3];
    {
        const f2 c1 = f2{cd.x, cd.y}, d1 = f2{cd.z, cd.w}, e1 = f2{ef.x, ef.y}, f1 = f2{ef.z, ef.w};
        const f2 c2 = pmul(c1, c1), d2 = pmul(d1, d1), e2 = pmul(e1, e1), f2_ = pmul(f1, f1);
        Cb[0] = c1, Cb[1] = c2, Cb[2] = pmul(c2, c1);
        Da[0] = d1, Da[1] = d2, Da[2] = pmul(d2, d1);
        Eb[0] = e1, Eb[1] = e2, Eb[2] = pmul(e2, e1);
        Fa[0] = f1, Fa[1] = f2_, Fa[2] = pmul(f2_, f1);
    }
    f2* col = img + t + (t >> 4);  // (r, t) at col[r * kRow]

    // P1: DFT16 n2 -> k0, * W4096^(t k0) -> (k0, t)
    pdft16f<false>(v);
#pragma unroll
    for (int k = 0; k < 16; ++k) col[k * kRow] = k == 0 ? v[0] : pmul(v[kout(k)], tw_pair(Cb, Da, k));
    __syncthreads();

    // P2: lane (k0 = hi4, n0 = lo4): DFT16 n1 -> k1, * W256^(n0 k1) -> (k0, 16 k1 + n0)
    f2* r2 = img + hi4 * kRow + lo4;  // (hi4, 16 j + lo4) at r2[17 j]
#pragma unroll
    for (int j = 0; j < 16; ++j) v[j] = r2[17 * j];
    float4 hq[8];  // the spectrum slice of lane (k0, k1) = t for P3, k-pair major
#pragma unroll
    for (int p = 0; p < 8; ++p) hq[p] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rh, 16 * t, 4096 * p, 0));
    f2 w2[16];  // W256^(lo4 k), used by P2 (n0 = lo4) and P3 (k1 = lo4)
#pragma unroll
    for (int k = 1; k < 16; ++k) w2[k] = tw_pair(Eb, Fa, k);
    pdft16f<false>(v);
#pragma unroll
    for (int k = 0; k < 16; ++k) r2[17 * k] = k == 0 ? v[0] : pmul(v[kout(k)], w2[k]);
    wave_sync();

    // P3: lane (k0 = hi4, k1 = lo4) over n0: DFT16 n0 -> k2, * H, IDFT16 k2 -> n0, * conj W256^(k1 n0)
    {
        f2* r3 = img + hi4 * kRow + 17 * lo4;  // (hi4, 16 lo4 + j) at r3[j]
#pragma unroll
        for (int j = 0; j < 16; ++j) v[j] = r3[j];
        pdft16f<false>(v);
        f2 u[16];
#pragma unroll
        for (int p = 0; p < 8; ++p) {
            u[2 * p] = pmul(v[kout(2 * p)], f2{hq[p].x, hq[p].y});
            u[2 * p + 1] = pmul(v[kout(2 * p + 1)], f2{hq[p].z, hq[p].w});
        }
        pdft16f<true>(u);
#pragma unroll
        for (int j = 0; j < 16; ++j) r3[j] = j == 0 ? u[kout(0)] : pmulc(u[kout(j)], w2[j]);
    }
    wave_sync();

    // P4: lane (k0 = hi4, n0 = lo4): IDFT16 k1 -> n1 -> (k0, 16 n1 + n0)
#pragma unroll
    for (int j = 0; j < 16; ++j) v[j] = r2[17 * j];
    pdft16f<true>(v);
#pragma unroll
    for (int k = 0; k < 16; ++k) r2[17 * k] = v[kout(k)];
    __syncthreads();

    // P5: lane t: * conj W4096^(t k0), IDFT16 k0 -> n2; row n2 at v[kout(n2)].  The bases are
    // made opaque first so the products are recomputed here rather than kept live from P1.
#pragma unroll
    for (int i = 0; i < 3; ++i) asm volatile("" : "+v"(Cb[i]), "+v"(Da[i]));
#pragma unroll
    for (int k = 0; k < 16; ++k) v[k] = k == 0 ? col[0] : pmulc(col[k * kRow], tw_pair(Cb, Da, k));
    pdft16f<true>(v);
    // nontemporal stores (3.14 -> 3.08 ms on cfg2); rows < h2 wrap and are dropped, positions past
    // the stream fall outside the descriptor (dropped)
    if constexpr (WIDE && !EDGE) {
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            f2 a, b;
            pair_exchange(v[kout(k)], v[kout(8 + k)], a, b);
            if (k + 8 * (t & 1) >= h2)
                __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4v, f4v{a.x, a.y, b.x, b.y}), ry,
                                                       16 * (t >> 1) + 16384 * (t & 1), 2048 * k, kNT);
        }
    } else {
#pragma unroll
        for (int r = 0; r < 16; ++r)
            if (r >= h2) __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u2v, v[kout(r)]), ry, 8 * t, 2048 * r, kNT);
    }
}

// Interior segments [lo, hi) of every channel (whole window inside the stream): workgroup b runs on
// XCD b % 8 and takes segment lo + (b % 8) q + b / 8, so each XCD streams one contiguous eighth of
// the call in order.  EDGE: the boundary segments [0, lo) and [hi, nseg) (block b takes segment
// b < lo ? b : hi + b - lo), the last one writing the next history (new_hist).
template <bool HALO1, bool WIDE, bool EDGE>
__global__ void __launch_bounds__(256, 4)
fir_ols_os_kernel(const f2* __restrict__ x, const f2* __restrict__ hist, f2* __restrict__ new_hist,
                  const float4* __restrict__ Hs, const float4* __restrict__ tb, f2* __restrict__ y, long long n,
                  long long lo, long long hi, long long q, long long nseg, int h2, int Lm1) {
    __shared__ __attribute__((aligned(16))) f2 img[16 * kRow];
    long long seg;
    if constexpr (EDGE) {
        seg = (long long)blockIdx.x < lo ? (long long)blockIdx.x : hi + ((long long)blockIdx.x - lo);
    } else {
        const int xc = blockIdx.x & 7;
        seg = lo + (long long)xc * q + (long long)(blockIdx.x >> 3);
        const long long xe = lo + (long long)(xc + 1) * q;
        if (seg >= (xe < hi ? xe : hi)) return;  // uniform over the workgroup
    }
    const int V = 4096 - 256 * h2;
    const long long ch = blockIdx.y;
    ols_os_segment<HALO1, WIDE, EDGE>(x + ch * n, hist + ch * Lm1,
                                      (EDGE && new_hist != nullptr && seg == nseg - 1) ? new_hist + ch * Lm1 : nullptr,
                                      Hs, tb, y + ch * n, seg * V - 256 * h2, n, Lm1, h2, img, threadIdx.x);
}

// every segment of every channel: the boundary segments (and the next history) in one small
// launch, the interior ones in the XCD-ordered grid
template <bool HALO1, bool WIDE>
hipError_t launch_fir_ols_os_t(const OlsPlan& p, const void* x, const void* hist, void* new_hist, void* y, size_t n,
                               int Lm1, size_t channels, hipStream_t s) {
    if (n == 0) return hipSuccess;
    const int h2 = p.halo_rows;
    if (h2 < 1 || h2 > 15 || Lm1 > 256 * h2 || (HALO1 && h2 != 1)) return hipErrorInvalidValue;
    const long long V = 4096 - 256 * h2;
    const long long nseg = ((long long)n + V - 1) / V;
    long long lo, hi;
    ols_interior_range((long long)n, h2, &lo, &hi);
    if (hi > nseg - 1) hi = nseg - 1;  // the last segment always runs in the boundary launch (history)
    if (hi < lo) hi = lo;
    const long long nedge = lo + (nseg - hi);
    const long long q = (hi - lo + 7) / 8;
    hipLaunchKernelGGL((fir_ols_os_kernel<false, false, true>), dim3((unsigned)nedge, (unsigned)channels), dim3(256),
                       0, s, (const f2*)x, (const f2*)hist, (f2*)new_hist, (const float4*)p.d_pkt,
                       (const float4*)p.d_ostab, (f2*)y, (long long)n, lo, hi, 0LL, nseg, h2, Lm1);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess || hi <= lo) return e;
    hipLaunchKernelGGL((fir_ols_os_kernel<HALO1, WIDE, false>), dim3((unsigned)(8 * q), (unsigned)channels), dim3(256),
                       0, s, (const f2*)x, (const f2*)hist, (f2*)nullptr, (const float4*)p.d_pkt,
                       (const float4*)p.d_ostab, (f2*)y, (long long)n, lo, hi, q, nseg, h2, Lm1);
    return hipGetLastError();
}

hipError_t launch_fir_ols_os(const OlsPlan& p, const void* x, const void* hist, void* new_hist, void* y, size_t n,
                             int Lm1, size_t channels, hipStream_t s, bool wide) {
    if (wide) return launch_fir_ols_os_t<false, true>(p, x, hist, new_hist, y, n, Lm1, channels, s);
    if (p.halo_rows == 1) return launch_fir_ols_os_t<true, false>(p, x, hist, new_hist, y, n, Lm1, channels, s);
    return launch_fir_ols_os_t<false, false>(p, x, hist, new_hist, y, n, Lm1, channels, s);
}

}  // namespace sdsp
