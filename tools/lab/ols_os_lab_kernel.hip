// LAB COPY (tools only, never part of libsdsp.so): the one-shot overlap-save kernel of
// solid_dsp_amd/csrc/kern_fir_ols_os.hip with every ablation / variant bit of rounds 2-6 (ABL,
// below), compiled by tools/lab/ols_lab.hip for in-process A/B runs.  ABL 24 is the product
// configuration; the product source carries none of the other bits.
//
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
// FP32 (sdsp_pk.hpp).  What differs is the shape, chosen for the HBM stream:
//
//  * one segment per 256-thread workgroup, one workgroup per segment (no
//    persistent loop): the dispatcher deals workgroup b to XCD b % 8, so
//    segment(b) = lo + (b % 8) q + b / 8 makes every XCD stream one contiguous
//    eighth of the call in order (the halo row of a segment is the tail its XCD
//    neighbour just read, an L2 hit).  Measured against the alternatives in
//    persistent grids (any order) and more or fewer workgroups per
//    CU are slower;
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
// restatement rel-RMS ~1.8e-7 on the cfg2 taps (§8d tolerance 1e-6).
#include "sdsp_device.hpp"
#include "sdsp_kernels.hpp"
#include "sdsp_pk.hpp"

namespace sdsp {

using namespace pk;

namespace {

constexpr int kRow = 272;

// WAVE: the next phase reads only what this wave wrote (the LDS operations of one
// wave complete in order), so a compiler-level fence replaces the block barrier
template <bool WAVE> __device__ __forceinline__ void phase_sync() {
    if constexpr (WAVE) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    } else {
        __syncthreads();
    }
}

typedef unsigned int u2v __attribute__((ext_vector_type(2)));
typedef unsigned int u4v __attribute__((ext_vector_type(4)));
constexpr int kBufWord3 = 0x00020000;  // raw buffer descriptor word 3 (gfx9 family)

// x = D_{k>>2} C_{k&3} for C_b = c[b-1], D_a = d[a-1] (k = 0 -> 1)
__device__ __forceinline__ f2 tw_pair(const f2 (&c)[3], const f2 (&d)[3], int k) {
    const int a = k >> 2, b = k & 3;
    if (a == 0) return b == 0 ? f2{1.0f, 0.0f} : c[b - 1];
    if (b == 0) return d[a - 1];
    return pmul(d[a - 1], c[b - 1]);
}

// e^{-j th} for 0 <= th <= pi/8 as packed Horner polynomials (degree 8 / 9; |error| < 5e-8, the
// size of a table entry's own rounding): {cos th, -sin th}
// lab phase markers (ABL 64): a recognisable s_nop triple in the disassembly
template <int ABL, int M> __device__ __forceinline__ void phase_mark() {
    if constexpr ((ABL & 64) != 0) asm volatile("s_nop 7\n\ts_nop 6\n\ts_nop %0" ::"n"(M));
}

[[maybe_unused]] __device__ __forceinline__ f2 wpoly(float th) {
    const float x2 = th * th;
    const f2 xx = {x2, x2};
    f2 q = {1.0f / 40320.0f, 1.0f / 362880.0f};
    q = __builtin_elementwise_fma(q, xx, f2{-1.0f / 720.0f, -1.0f / 5040.0f});
    q = __builtin_elementwise_fma(q, xx, f2{1.0f / 24.0f, 1.0f / 120.0f});
    q = __builtin_elementwise_fma(q, xx, f2{-0.5f, -1.0f / 6.0f});
    q = __builtin_elementwise_fma(q, xx, f2{1.0f, 1.0f});
    return q * f2{1.0f, -th};
}

// lane pair (2c, 2c + 1) exchange: even lanes lo = a, odd lanes lo = the partner's b; odd lanes
// hi = b, even lanes hi = the partner's a.  Loads: (a, b) = columns (2c, 2c + 1) of row k + 8h ->
// (lo, hi) = rows (k, 8 + k) of column 2c + h.  Stores: (a, b) = rows (k, 8 + k) of column 2c + h
// -> (lo, hi) = columns (2c, 2c + 1) of row k + 8h.  One v_cndmask_b32 with a quad_perm DPP
// operand per dword (the partner's register read in the same instruction); the s_nop covers
// the DPP read-after-VALU-write hazard of an operand the compiler computed just before.
[[maybe_unused]] __device__ __forceinline__ void pair_exchange(f2 a, f2 b, f2& lo, f2& hi) {
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

// ABL selects compile-time variants of the segment transform.  The product kernels
// are ABL = 24 (one halo row, L <= 257) and ABL = 0 (longer filters), see launch_fir_ols_os;
// tools/lab/ols_lab.hip instantiates the others for in-process A/B runs
// (never part of libsdsp.so).  Bits: 1 block barriers at the wave-local phase
// boundaries; 2 no HBM traffic (ablation: outputs dropped); 4 HBM traffic only
// (ablation: no transform); 128 plain (not nontemporal) stores; 256 input rows
// loaded last to first; 512 output rows stored last to first; 1024 each XCD walks the
// even segments of its eighth, then the odd ones (a segment's halo row is then read
// long after its neighbour's tail: from HBM, not as a hit on an in-flight L2 miss); 2097152 rows
// loaded in the first radix-4 stage's order (the product: row order); 4194304 the
// twiddle-base tables requested after the rows; 16777216 the rows issued exactly in the loop's
// order (a scheduling barrier after each load); 33554432 the boundary segments as extra
// workgroups of the interior launch (a branch at the kernel's entry);
// 16 one halo row compiled in (h2 = 1: rows 1..15 stored without a test per row);
// 8 the rows a neighbouring segment also reads when h2 = 1 (row 0, the halo, and row 15, the next
// segment's halo) with temporal loads, the others nontemporal;
// ablations of the per-segment table reads from L2: 2048 no spectrum loads, 4096 no
// twiddle-base loads (wrong results, timing only); 8192 write-through (sc1) stores; 16384
// plain (not nontemporal) input loads; 32768 all six twiddle bases loaded (the round-3 form;
// 49152 = the round-3 kernel); 131072 with 4: the HBM-only pattern in 16-byte lanes (the NCO
// kernel's shape); 262144 clock stamps (lab builds that define SDSP_OLS_STAMPS only: every 32nd
// workgroup records s_memtime / s_memrealtime at entry and exit into g_ols_stamps, a buffer no
// other code reads; the in-kernel clock of MI355X_MICROARCH.md "DVFS give-back" item 6).
template <int ABL, bool EDGE>
__device__ __forceinline__ void ols_os_segment(const f2* __restrict__ x, const f2* __restrict__ hist,
                                               f2* __restrict__ new_hist, const float4* __restrict__ Hs,
                                               const float4* __restrict__ tb, f2* __restrict__ y, long long base,
                                               long long n, int Lm1, int h2, f2* img, int t, float4 (&tq)[6],
                                               float4 (&hq)[8], bool first = true) {
    const int hi4 = t >> 4, lo4 = t & 15;
    if constexpr ((ABL & 16) != 0) h2 = 1;  // one halo row compiled in (the launcher checks h2 == 1)
    // the segment's window x[base, base + 4096) as a raw buffer.  EDGE (the boundary segments of a
    // call, launched apart so that the interior kernel carries no boundary code: its presence
    // alone cost the interior segments 1.9 %, profiles/r05/lab/r05e_olsburst.log): past the end of
    // the stream loads return 0 and stores are dropped, rows before it come from the history
    const long long rem = n - base;
    const int nrec = (!EDGE || rem >= 4096) ? 32768 : (int)(8 * rem);
    const auto rx = __builtin_amdgcn_make_buffer_rsrc((void*)(x + base), (short)0, nrec, kBufWord3);
    const auto ry = __builtin_amdgcn_make_buffer_rsrc((void*)(y + base), (short)0, nrec, kBufWord3);
    const auto rt = __builtin_amdgcn_make_buffer_rsrc((void*)tb, (short)0, kOlsOsTabF4 * 16, kBufWord3);
    const auto rh = __builtin_amdgcn_make_buffer_rsrc((void*)Hs, (short)0,
                                                      (ABL & 268435456) ? 4 * kOlsHalfRow * 16 : 2048 * 16, kBufWord3);
    constexpr int kLdAux = (ABL & 16384) ? 0 : 2;  // nontemporal (aux 2)
    // twiddle bases: column t of W4096, row lo4 of W256 (runtime.cpp ols_build), requested
    // before the segment's rows (L2 hits that land while the rows stream in)
    auto tab = [&](int lane, int off) {
        if constexpr ((ABL & 4096) != 0) {
            const float u = 1e-3f * (float)lane + 1e-6f * (float)off;
            return float4{u, 0.5f - u, 0.25f + u, 1.0f - u};
        } else {
            return __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rt, 16 * lane, off, 0));
        }
    };
    // tq: the raw table loads (products formed once the rows are requested); hq: the spectrum
    // slice.  With `first` false (a workgroup's second segment, ABL 134217728) both are reused.
    auto load_tables = [&] {
        if (!first || (ABL & 65536)) return;
        if constexpr ((ABL & (32768 | 4096)) == 0) {
            tq[0] = tab(t, 16 * kOlsOsTabCD), tq[1] = tab(lo4, 16 * kOlsOsTabEF);
        } else {
            tq[0] = tab(t, 0), tq[1] = tab(t, 4096), tq[2] = tab(t, 8192);
            tq[3] = tab(lo4, 12288), tq[4] = tab(lo4, 12544), tq[5] = tab(lo4, 12800);
        }
    };
    f2 v[16];
    if constexpr (EDGE) {
        // rows inside the stream through rx, rows before it from the handle's history (the last
        // Lm1 inputs, oldest first; positions before the history read as 0 through an
        // out-of-range offset)
        load_tables();
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
    } else {
        if constexpr ((ABL & 4194304) == 0) load_tables();
        // the rows in row order (the compiler interleaves them as 0, 4, 1, 5, 8, 12, 9, 13, ...):
        // 2 % faster than the first radix-4 stage's order (0, 4, 8, 12, 1, 5, ...) and than either
        // order enforced with scheduling barriers (profiles/r05/lab/r05h_olsburst.log,
        // r05i_olsburst.log)
        if constexpr ((ABL & 524288) != 0) {
            // 16-byte lanes: lane t = 2c + h loads columns (2c, 2c + 1) of rows k + 8h, then one
            // DPP exchange per dword with its partner lane t ^ 1 gives it column t over the rows
            f4v q[8];
#pragma unroll
            for (int k = 0; k < 8; ++k)
                q[k] = __builtin_bit_cast(f4v, __builtin_amdgcn_raw_buffer_load_b128(rx, 16 * (t >> 1) + 16384 * (t & 1),
                                                                                    2048 * k, kLdAux));
#pragma unroll
            for (int k = 0; k < 8; ++k) pair_exchange(f2{q[k].x, q[k].y}, f2{q[k].z, q[k].w}, v[k], v[8 + k]);
        } else {
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                const int r = (ABL & 256) ? 15 - i : (ABL & 2097152) ? 4 * (i & 3) + (i >> 2) : i;
                if constexpr ((ABL & 131072) != 0) v[r] = f2{0.0f, 0.0f};  // (the 16-byte-lane ablation loads its own)
                else if constexpr (ABL & 2) v[r] = f2{1e-3f * t + r, 1e-9f * (float)base};
                else if ((ABL & 8) && (r == 0 || r == 15))
                    v[r] = __builtin_bit_cast(f2, __builtin_amdgcn_raw_buffer_load_b64(rx, 8 * t, 2048 * r, 0));
                else v[r] = __builtin_bit_cast(f2, __builtin_amdgcn_raw_buffer_load_b64(rx, 8 * t, 2048 * r, kLdAux));
                if constexpr ((ABL & 16777216) != 0) __builtin_amdgcn_sched_barrier(0);  // lab: issue in this order
            }
        }
        if constexpr ((ABL & 4194304) != 0) load_tables();  // lab: the tables after the rows
    }
    if constexpr ((ABL & 4) && (ABL & 131072)) {
        // HBM-only with the NCO kernel's lane shape: the segment as eight 4 KB rows of 16-byte
        // lanes (lane t: bytes 16 t + 4096 k), the halo's bytes not stored
        u4v w[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) w[k] = __builtin_bit_cast(u4v, __builtin_amdgcn_raw_buffer_load_b128(rx, 16 * t, 4096 * k, 2));
#pragma unroll
        for (int k = 0; k < 8; ++k) asm volatile("" : "+v"(w[k]));
#pragma unroll
        for (int k = 0; k < 8; ++k)
            if (4096 * k + 16 * t >= 2048 * h2) __builtin_amdgcn_raw_buffer_store_b128(w[k], ry, 16 * t, 4096 * k, 2);
        return;
    } else if constexpr (ABL & 4) {
        // every row's load in flight before the first store, as in the transform (without this
        // the compiler sinks each load into its store's `r >= h2` branch: one round trip per row)
#pragma unroll
        for (int r = 0; r < 16; ++r) asm volatile("" : "+v"(v[r]));
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const int r = (ABL & 512) ? 15 - i : i;
            if (r >= h2)
                __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u2v, v[r]), ry, 8 * t, 2048 * r,
                                                      (ABL & 8192) ? 16 : (ABL & 128) ? 0 : 2);
        }
        return;
    }
    f2 Cb[3], Da[3], Eb[3], Fa[3];
    if constexpr ((ABL & 65536) != 0) {
        // lab: no table loads -- C1 = W4096^t and E1 = W256^lo4 by polynomial (angles < pi/8),
        // D1 = C2 C2 = W4096^(4t), F1 = E2 E2
        const f2 c1 = wpoly((float)t * (float)(6.283185307179586 / 4096.0));
        const f2 e1 = wpoly((float)lo4 * (float)(6.283185307179586 / 256.0));
        const f2 c2 = pmul(c1, c1), e2 = pmul(e1, e1);
        const f2 d1 = pmul(c2, c2), f1 = pmul(e2, e2);
        const f2 d2 = pmul(d1, d1), f2_ = pmul(f1, f1);
        Cb[0] = c1, Cb[1] = c2, Cb[2] = pmul(c2, c1);
        Da[0] = d1, Da[1] = d2, Da[2] = pmul(d2, d1);
        Eb[0] = e1, Eb[1] = e2, Eb[2] = pmul(e2, e1);
        Fa[0] = f1, Fa[1] = f2_, Fa[2] = pmul(f2_, f1);
    } else if constexpr ((ABL & (32768 | 4096)) == 0) {
        // the first power of each base from L2 ({C1, D1} per column, {E1, F1} per row: two
        // 16-byte loads where the six-base form takes six), the others as products (W^2 = W W,
        // W^3 = W^2 W): a third of the table traffic per segment, results within rounding of the
        // six-base form (rel-RMS 2.2e-7 between the two on cfg2)
        const float4 cd = tq[0], ef = tq[1];
        const f2 c1 = f2{cd.x, cd.y}, d1 = f2{cd.z, cd.w}, e1 = f2{ef.x, ef.y}, f1 = f2{ef.z, ef.w};
        const f2 c2 = pmul(c1, c1), d2 = pmul(d1, d1), e2 = pmul(e1, e1), f2_ = pmul(f1, f1);
        Cb[0] = c1, Cb[1] = c2, Cb[2] = pmul(c2, c1);
        Da[0] = d1, Da[1] = d2, Da[2] = pmul(d2, d1);
        Eb[0] = e1, Eb[1] = e2, Eb[2] = pmul(e2, e1);
        Fa[0] = f1, Fa[1] = f2_, Fa[2] = pmul(f2_, f1);
    } else {
        const float4 b0 = tq[0], b1 = tq[1], b2 = tq[2], e0 = tq[3], e1 = tq[4], e2 = tq[5];
        Cb[0] = f2{b0.x, b0.y}, Cb[1] = f2{b0.z, b0.w}, Cb[2] = f2{b1.x, b1.y};
        Da[0] = f2{b1.z, b1.w}, Da[1] = f2{b2.x, b2.y}, Da[2] = f2{b2.z, b2.w};
        Eb[0] = f2{e0.x, e0.y}, Eb[1] = f2{e0.z, e0.w}, Eb[2] = f2{e1.x, e1.y};
        Fa[0] = f2{e1.z, e1.w}, Fa[1] = f2{e2.x, e2.y}, Fa[2] = f2{e2.z, e2.w};
    }
    f2* col = img + t + (t >> 4);  // (r, t) at col[r * kRow]
    // the fused DFT16 (72 instead of 81 packed instructions, sdsp_pk.hpp: 3.112 -> 3.056 ms sustained,
    // profiles/r06/lab/r06b_olsab.log); 67108864 the round-5 DFT16 (lab)
    auto dft = [](f2(&w)[16]) {
        if constexpr ((ABL & 67108864) != 0) pdft16<false>(w);
        else pdft16f<false>(w);
    };
    auto idft = [](f2(&w)[16]) {
        if constexpr ((ABL & 67108864) != 0) pdft16<true>(w);
        else pdft16f<true>(w);
    };

    constexpr bool kReal = (ABL & 268435456) != 0;
    auto load_h = [&] {
        // hq: the spectrum slice of lane (k0, k1) = t for P3, k-pair major.  kOlsRealTaps (real taps,
        // H[N - k] = conj H[k]): pairs p < 4 from the half table at lane t, pairs p >= 4 as the
        // conjugates of pair 7 - p of the mirror lane (16 - k0, 15 - k1) (k0 = 0: (0, 16 - k1); lane
        // (0, 0): the table's tail entry), halves swapped -- a 16 KB table instead of 32 KB, read with
        // the same eight loads (runtime.cpp ols_build)
        if constexpr (kReal) {
            const int k0 = hi4, k1 = lo4;
            const int ml = k0 ? 16 * (16 - k0) + (15 - k1) : (k1 ? 16 - k1 : 256);
#pragma unroll
            for (int p = 0; p < 4 && first; ++p) {
                hq[p] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rh, 16 * t, 16 * kOlsHalfRow * p, 0));
                hq[7 - p] =
                    __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rh, 16 * ml, 16 * kOlsHalfRow * p, 0));
            }
        } else {
#pragma unroll
            for (int p = 0; p < 8 && first; ++p) {
                if constexpr ((ABL & 2048) != 0) hq[p] = float4{1e-3f * (float)t, (float)p, 0.5f, 1e-4f * (float)t};
                else hq[p] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rh, 16 * t, 4096 * p, 0));
            }
        }
    };
    // lab placements of the spectrum loads: 1073741824 with the rows (before P1), 536870912 after
    // P1's LDS stores, before the barrier; the product issues them in P2
    if constexpr ((ABL & 1073741824) != 0) load_h();

    phase_mark<ABL, 0>();
    // P1: DFT16 n2 -> k0, * W4096^(t k0) -> (k0, t)
    dft(v);
#pragma unroll
    for (int k = 0; k < 16; ++k) col[k * kRow] = k == 0 ? v[0] : pmul(v[kout(k)], tw_pair(Cb, Da, k));
    if constexpr ((ABL & 536870912) != 0) load_h();
    __syncthreads();

    phase_mark<ABL, 1>();
    // P2: lane (k0 = hi4, n0 = lo4): DFT16 n1 -> k1, * W256^(n0 k1) -> (k0, 16 k1 + n0)
    f2* r2 = img + hi4 * kRow + lo4;  // (hi4, 16 j + lo4) at r2[17 j]
#pragma unroll
    for (int j = 0; j < 16; ++j) v[j] = r2[17 * j];
    if constexpr ((ABL & (1073741824 | 536870912)) == 0) load_h();
    f2 w2[16];  // W256^(lo4 k), used by P2 (n0 = lo4) and P3 (k1 = lo4)
#pragma unroll
    for (int k = 1; k < 16; ++k) w2[k] = tw_pair(Eb, Fa, k);
    dft(v);
#pragma unroll
    for (int k = 0; k < 16; ++k) r2[17 * k] = k == 0 ? v[0] : pmul(v[kout(k)], w2[k]);
    phase_sync<!(ABL & 1)>();

    phase_mark<ABL, 2>();
    // P3: lane (k0 = hi4, k1 = lo4) over n0: DFT16 n0 -> k2, * H, IDFT16 k2 -> n0, * conj W256^(k1 n0)
    {
        f2* r3 = img + hi4 * kRow + 17 * lo4;  // (hi4, 16 lo4 + j) at r3[j]
#pragma unroll
        for (int j = 0; j < 16; ++j) v[j] = r3[j];
        dft(v);
        f2 u[16];
#pragma unroll
        for (int p = 0; p < 8; ++p) {
            if (kReal && p >= 4) {  // {conj m.zw, conj m.xy} of the mirror's pair
                u[2 * p] = pmulc(v[kout(2 * p)], f2{hq[p].z, hq[p].w});
                u[2 * p + 1] = pmulc(v[kout(2 * p + 1)], f2{hq[p].x, hq[p].y});
            } else {
                u[2 * p] = pmul(v[kout(2 * p)], f2{hq[p].x, hq[p].y});
                u[2 * p + 1] = pmul(v[kout(2 * p + 1)], f2{hq[p].z, hq[p].w});
            }
        }
        idft(u);
#pragma unroll
        for (int j = 0; j < 16; ++j) r3[j] = j == 0 ? u[kout(0)] : pmulc(u[kout(j)], w2[j]);
    }
    phase_sync<!(ABL & 1)>();

    phase_mark<ABL, 3>();
    // P4: lane (k0 = hi4, n0 = lo4): IDFT16 k1 -> n1 -> (k0, 16 n1 + n0)
#pragma unroll
    for (int j = 0; j < 16; ++j) v[j] = r2[17 * j];
    idft(v);
#pragma unroll
    for (int k = 0; k < 16; ++k) r2[17 * k] = v[kout(k)];
    __syncthreads();

    phase_mark<ABL, 4>();
    // P5: lane t: * conj W4096^(t k0), IDFT16 k0 -> n2; row n2 at v[kout(n2)].  The bases are
    // made opaque first so the products are recomputed here rather than kept live from P1.
#pragma unroll
    for (int i = 0; i < 3; ++i) asm volatile("" : "+v"(Cb[i]), "+v"(Da[i]));
#pragma unroll
    for (int k = 0; k < 16; ++k) v[k] = k == 0 ? col[0] : pmulc(col[k * kRow], tw_pair(Cb, Da, k));
    idft(v);
    if constexpr (ABL & 2) {  // outputs kept live, not stored
        f2 acc = v[0];
#pragma unroll
        for (int r = 1; r < 16; ++r) acc += v[r];
        if (acc.x == 1.2345e30f) __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u2v, acc), ry, 8 * t, 0, 0);
        return;
    }
    // nontemporal stores (3.14 -> 3.08 ms on cfg2, in-process A/B); rows < h2 wrap and are dropped,
    // positions past the stream fall outside the descriptor (dropped)
    constexpr int kStAux = (ABL & 8192) ? 16 : (ABL & 128) ? 0 : 2;  // 16: write-through (sc1), lab
    if constexpr ((ABL & 524288) != 0 && !EDGE) {
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            f2 a, b;
            pair_exchange(v[kout(k)], v[kout(8 + k)], a, b);
            if (k + 8 * (t & 1) >= h2)
                __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4v, f4v{a.x, a.y, b.x, b.y}), ry,
                                                       16 * (t >> 1) + 16384 * (t & 1), 2048 * k, kStAux);
        }
    } else {
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const int r = (ABL & 512) ? 15 - i : i;
            if (r >= h2)
                __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u2v, v[kout(r)]), ry, 8 * t, 2048 * r, kStAux);
        }
    }
}

#ifdef SDSP_OLS_STAMPS
__device__ unsigned long long g_ols_stamps[4 * 8192];
#endif

// Interior segments [lo, hi) of every channel (whole window inside the stream): workgroup b
// runs on XCD b % 8 and takes segment lo + (b % 8) q + b / 8, so each XCD streams one contiguous
// eighth of the call in order.  EDGE: the boundary segments [0, lo) and [hi, nseg) (block b takes
// segment b < lo ? b : hi + b - lo), the last one writing the next history (new_hist).
template <int ABL, bool EDGE>
__global__ void __launch_bounds__(256, 4)
fir_ols_os_kernel(const f2* __restrict__ x, const f2* __restrict__ hist, f2* __restrict__ new_hist,
                  const float4* __restrict__ Hs, const float4* __restrict__ tb, f2* __restrict__ y, long long n,
                  long long lo, long long hi, long long q, long long nseg, int h2, int Lm1) {
    __shared__ __attribute__((aligned(16))) f2 img[16 * kRow];
    long long seg;
    if constexpr (!EDGE && (ABL & 33554432) != 0) {
        // lab: the boundary segments as extra workgroups past the interior grid, on their own
        // code path (one launch instead of two)
        const long long nb = 8 * q;
        if ((long long)blockIdx.x >= nb) {
            const long long b = (long long)blockIdx.x - nb;
            const long long sg = b < lo ? b : hi + (b - lo);
            const long long c = blockIdx.y;
            float4 tq[6], hq[8];
            ols_os_segment<0, true>(x + c * n, hist + c * Lm1,
                                    (new_hist != nullptr && sg == nseg - 1) ? new_hist + c * Lm1 : nullptr, Hs, tb,
                                    y + c * n, sg * (4096 - 256 * h2) - 256 * h2, n, Lm1, h2, img, threadIdx.x, tq,
                                    hq);
            return;
        }
    }
    const int V = 4096 - 256 * h2;
    const long long ch = blockIdx.y;
    float4 tq[6], hq[8];
    if constexpr (!EDGE && (ABL & 134217728) != 0) {
        // lab: two segments per workgroup, the tables and the spectrum slice loaded once.  The XCD's
        // eighth is walked as two fronts (segments j and j + qh), so a segment's halo row is still the
        // tail its neighbouring workgroup just read (consecutive segments per workgroup broke that:
        // +8.7 %, profiles/r06/lab/r06d_olsab_variants.log)
        const int xc = blockIdx.x & 7;
        const long long qh = (q + 1) / 2;
        const long long s0 = lo + (long long)xc * q + (long long)(blockIdx.x >> 3);
        const long long xe0 = lo + (long long)(xc + 1) * q;
        const long long xe = xe0 < hi ? xe0 : hi;
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            const long long sg = s0 + k * qh;
            if (sg >= xe) return;    // uniform over the workgroup
            if (k) __syncthreads();  // the first segment's P5 reads are done before P1 rewrites the image
            ols_os_segment<ABL, false>(x + ch * n, hist + ch * Lm1, nullptr, Hs, tb, y + ch * n,
                                       sg * V - 256 * h2, n, Lm1, h2, img, threadIdx.x, tq, hq, k == 0);
        }
        return;
    }
    if constexpr (EDGE) {
        seg = (long long)blockIdx.x < lo ? (long long)blockIdx.x : hi + ((long long)blockIdx.x - lo);
    } else {
        const int xc = blockIdx.x & 7;
        long long j = blockIdx.x >> 3;
        if constexpr ((ABL & 1024) != 0) j = j < (q + 1) / 2 ? 2 * j : 2 * (j - (q + 1) / 2) + 1;
        seg = lo + (long long)xc * q + j;
        const long long xe = lo + (long long)(xc + 1) * q;
        if (seg >= (xe < hi ? xe : hi)) return;  // uniform over the workgroup
    }
#ifdef SDSP_OLS_STAMPS
    unsigned long long m0 = 0, r0 = 0;
    if constexpr ((ABL & 262144) != 0) m0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
#endif
    ols_os_segment<ABL, EDGE>(x + ch * n, hist + ch * Lm1,
                              (EDGE && new_hist != nullptr && seg == nseg - 1) ? new_hist + ch * Lm1 : nullptr, Hs,
                              tb, y + ch * n, seg * V - 256 * h2, n, Lm1, h2, img, threadIdx.x, tq, hq);
#ifdef SDSP_OLS_STAMPS
    if constexpr ((ABL & 262144) != 0) {
        const unsigned long long m1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
        if (threadIdx.x == 0 && (blockIdx.x & 31) == 0) {
            unsigned long long* o = g_ols_stamps + 4 * ((blockIdx.x >> 5) & 8191);
            o[0] = m0, o[1] = r0, o[2] = m1, o[3] = r1;
        }
    }
#endif
}

// every segment of every channel: the boundary segments (and the next history) in one small
// launch, the interior ones in the XCD-ordered grid; ABL as above for the interior kernel (0 = the
// product kernel)
template <int ABL>
hipError_t launch_fir_ols_os_t(const OlsPlan& p, const void* x, const void* hist, void* new_hist, void* y, size_t n,
                               int Lm1, size_t channels, hipStream_t s, size_t dyn_lds) {
    if (n == 0) return hipSuccess;
    const int h2 = p.halo_rows;
    if (h2 < 1 || h2 > 15 || Lm1 > 256 * h2) return hipErrorInvalidValue;
    const long long V = 4096 - 256 * h2;
    const long long nseg = ((long long)n + V - 1) / V;
    long long lo, hi;
    ols_interior_range((long long)n, h2, &lo, &hi);
    if (hi > nseg - 1) hi = nseg - 1;  // the last segment always runs in the boundary launch (history)
    if (hi < lo) hi = lo;
    const long long nedge = lo + (nseg - hi);
    const long long q = (hi - lo + 7) / 8;
    const long long qg = (ABL & 134217728) ? (q + 1) / 2 : q;  // workgroups per XCD
    if constexpr ((ABL & 33554432) != 0) {  // lab: one launch, the boundary segments past the grid
        hipLaunchKernelGGL((fir_ols_os_kernel<ABL, false>), dim3((unsigned)(8 * q + nedge), (unsigned)channels),
                           dim3(256), dyn_lds, s, (const f2*)x, (const f2*)hist, (f2*)new_hist, (const float4*)p.d_pkt,
                           (const float4*)p.d_ostab, (f2*)y, (long long)n, lo, hi, q, nseg, h2, Lm1);
        return hipGetLastError();
    }
    hipLaunchKernelGGL((fir_ols_os_kernel<0, true>), dim3((unsigned)nedge, (unsigned)channels), dim3(256), 0, s,
                       (const f2*)x, (const f2*)hist, (f2*)new_hist, (const float4*)p.d_pkt, (const float4*)p.d_ostab,
                       (f2*)y, (long long)n, lo, hi, 0LL, nseg, h2, Lm1);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess || hi <= lo) return e;
    // the interior kernel's spectrum table: the half table for real taps (ABL 268435456)
    const float4* hs = (const float4*)((ABL & 268435456) ? p.d_hhalf : p.d_pkt);
    hipLaunchKernelGGL((fir_ols_os_kernel<ABL, false>), dim3((unsigned)(8 * qg), (unsigned)channels), dim3(256), dyn_lds,
                       s, (const f2*)x, (const f2*)hist, (f2*)nullptr, hs, (const float4*)p.d_ostab,
                       (f2*)y, (long long)n, lo, hi, q, nseg, h2, Lm1);
    return hipGetLastError();
}

// the interior kernel's product variants: kOlsOneHalo | kOlsHaloTemporal when the halo is one
// row (L <= 257, every cfg2-like filter), ABL = 0 for longer filters, 524288 the 16-byte-lane form
// (SDSP_TUNE_OLS_KERNEL = 3)
constexpr int kOlsHaloTemporal = 8, kOlsOneHalo = 16;

hipError_t launch_fir_ols_os(const OlsPlan& p, const void* x, const void* hist, void* new_hist, void* y, size_t n,
                             int Lm1, size_t channels, hipStream_t s, bool wide) {
    if (wide) return launch_fir_ols_os_t<524288>(p, x, hist, new_hist, y, n, Lm1, channels, s, 0);
    if (p.halo_rows == 1)
        return launch_fir_ols_os_t<kOlsOneHalo | kOlsHaloTemporal>(p, x, hist, new_hist, y, n, Lm1, channels, s, 0);
    return launch_fir_ols_os_t<0>(p, x, hist, new_hist, y, n, Lm1, channels, s, 0);
}

}  // namespace sdsp
