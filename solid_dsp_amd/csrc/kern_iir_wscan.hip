// Wave-level block-parallel scan for SOS cascades (gfx950), SDSP_ALGO_FMA /
// AUTO path of IIRFilter SecondOrder (src/filter/iir/sos.rs:92-114,
// mod.rs:270-289) when the handle neither decimates nor interpolates.
//
// The cascade is linear in its D = 2S state:  S[n+1] = A S[n] + b x[n],
// y[n] = c S[n] + d x[n].  Each wave walks its own segment of the stream as a
// sequence of tiles of 64 chunks x B samples (one chunk per lane), with no
// block barriers:
//   1. the tile is staged in the wave's LDS slab with coalesced 16-byte
//      nontemporal loads, one padded row per chunk;
//   2. lane l runs its row from zero state, writing y0 back in place, and
//      keeps its local final state s_l;
//   3. the exact state entering the tile (`carry`, wave-uniform) is folded in
//      at lane 0: s_0 += A^B carry; a Hillis-Steele scan across the 64 lanes
//      with P_k = A^(B 2^k) gives every lane the true state at the end of its
//      chunk, G_l; the initial state of chunk l is I_l = G_{l-1} (I_0 = carry)
//      and the next tile's carry is G_63.  A and its powers are lower block
//      triangular (section q depends on sections <= q), so only those blocks
//      are multiplied;
//   4. outputs are corrected instead of rerun:  y[i] = y0[i] + Cr[i] . I_l,
//      Cr[i] = c A^i (the output response to the state, precomputed on the
//      host in f64, read as wave-uniform scalar loads), then leave with
//      coalesced write-through (sc1) 16-byte stores.
// A wave's first tile starts `wc` chunks before its segment: those lanes run
// the preceding input as warm-up (outputs dropped), which makes the carried-in
// state exact to ||A^(wc B)|| < 1e-9 (f32) / 1e-17 (f64), the criterion the
// host applies before it selects any scan.  Wave 0 instead injects the call's
// exact carried state at lane wc-1 of its first tile.  The lane holding the
// call's last sample reruns its chunk from I_l and writes the exact final
// state for the next call.
#include "sdsp_device.hpp"
#include "sdsp_kernels.hpp"

#include <type_traits>

namespace sdsp {

namespace {

constexpr int kWsThreads = 256;

constexpr int kWsWaves = kWsThreads / 64;

// chunk of CB bytes per lane (B = CB / sizeof(I) samples); LDS rows padded by
// 16 bytes so that 16 lanes reading the same slot of their rows are conflict-free
template <int CB> struct WsGeom {
    static constexpr int kRowBytes = CB + 16;
    static constexpr int kVecPerRow = CB / 16;
    static constexpr int kSlabBytes = 64 * kRowBytes;  // one tile per wave
};
template <typename I, int CB> struct ws_chunk { static constexpr int B = CB / (int)sizeof(I); };

template <typename T> __device__ __forceinline__ T shfl_up_v(T v, int d) { return __shfl_up(v, d); }
template <typename T> __device__ __forceinline__ cpx<T> shfl_up_v(cpx<T> v, int d) {
    return {__shfl_up(v.re, d), __shfl_up(v.im, d)};
}
template <typename T> __device__ __forceinline__ T readlane_v(T v, int l) { return __shfl(v, l); }

// the whole-wave shift by one lane (lane l gets lane l - 1's value; lane 0's result is not used)
// as DPP moves (wave_shr:1) instead of LDS-routed ds_bpermute shuffles: a few cycles of latency
// instead of an LDS round trip on the scan's dependent chain.  Eight dwords per statement, one
// s_nop 1 for the DPP read-after-VALU-write hazard of values computed just before.
[[maybe_unused]] __device__ __forceinline__ void shfl_up1_x8(const float (&a)[8], float (&r)[8]) {
    asm("s_nop 1\n\t"
        "v_mov_b32_dpp %0, %8 wave_shr:1 row_mask:0xf bank_mask:0xf\n\t"
        "v_mov_b32_dpp %1, %9 wave_shr:1 row_mask:0xf bank_mask:0xf\n\t"
        "v_mov_b32_dpp %2, %10 wave_shr:1 row_mask:0xf bank_mask:0xf\n\t"
        "v_mov_b32_dpp %3, %11 wave_shr:1 row_mask:0xf bank_mask:0xf\n\t"
        "v_mov_b32_dpp %4, %12 wave_shr:1 row_mask:0xf bank_mask:0xf\n\t"
        "v_mov_b32_dpp %5, %13 wave_shr:1 row_mask:0xf bank_mask:0xf\n\t"
        "v_mov_b32_dpp %6, %14 wave_shr:1 row_mask:0xf bank_mask:0xf\n\t"
        "v_mov_b32_dpp %7, %15 wave_shr:1 row_mask:0xf bank_mask:0xf"
        : "=&v"(r[0]), "=&v"(r[1]), "=&v"(r[2]), "=&v"(r[3]), "=&v"(r[4]), "=&v"(r[5]), "=&v"(r[6]), "=&v"(r[7])
        : "v"(a[0]), "v"(a[1]), "v"(a[2]), "v"(a[3]), "v"(a[4]), "v"(a[5]), "v"(a[6]), "v"(a[7]));
}
// lane l - 1's values of an I[D] state (the DPP form for real f32 with D = 8, else shuffles)
template <bool DPP, int D, typename I> __device__ __forceinline__ void shfl_up1_state(const I (&a)[D], I (&r)[D]) {
    if constexpr (DPP && D == 8 && std::is_same<I, float>::value) {
        shfl_up1_x8(a, r);
    } else {
#pragma unroll
        for (int d = 0; d < D; ++d) r[d] = shfl_up_v(a[d], 1);
    }
}
template <typename T> __device__ __forceinline__ cpx<T> readlane_v(cpx<T> v, int l) {
    return {__shfl(v.re, l), __shfl(v.im, l)};
}

// LDS hand-off between the lanes of one wave: wait for this wave's LDS
// operations only (lgkmcnt(0); vmcnt/expcnt left at their maxima so that
// in-flight global loads and stores keep running), and keep the compiler from
// moving memory operations across
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_s_waitcnt(0xC07F);
    __builtin_amdgcn_wave_barrier();
}

// one cascade step, fused form: w = x - a1 w1 - a2 w2;  y = b0 w + b1 w1 + b2 w2
template <int S, typename C, typename I>
__device__ __forceinline__ I sos_step_f(const C* __restrict__ c, I v, I (&w1)[S], I (&w2)[S]) {
#pragma unroll
    for (int s = 0; s < S; ++s) {
        const I w = fmac_(fmac_(v, -c[5 * s + 4], w2[s]), -c[5 * s + 3], w1[s]);
        v = fmac_(fmac_(mul_(c[5 * s + 2], w2[s]), c[5 * s + 1], w1[s]), c[5 * s + 0], w);
        w2[s] = w1[s];
        w1[s] = w;
    }
    return v;
}

// the state scales of an SOS group's wave-scan coefficient set (see sys_step): state d of the
// kernel = the reference's state d * wscan_inv(d); the reference's = the kernel's * wscan_scale(d)
template <int S, typename C> __device__ __forceinline__ C wscan_scale(const C* __restrict__ c, int d) {
    return c[5 * S + d];
}
template <int S, typename C> __device__ __forceinline__ C wscan_inv(const C* __restrict__ c, int d) {
    return c[5 * S + 2 * S + d];
}

// y = P x for a lower block-triangular P (2x2 blocks), wave-uniform
template <int D, typename C, typename I>
__device__ __forceinline__ void matvec_lt(const C* __restrict__ P, const I (&x)[D], I (&y)[D]) {
#pragma unroll
    for (int r = 0; r < D; ++r) {
        const int cmax = (r / 2) * 2 + 2;
        I acc = mul_(P[r * D], x[0]);
#pragma unroll
        for (int c = 1; c < cmax; ++c) acc = fmac_(acc, P[r * D + c], x[c]);
        y[r] = acc;
    }
}

template <int D, typename C, typename I>
__device__ __forceinline__ void matvec_full(const C* __restrict__ P, const I (&x)[D], I (&y)[D]) {
#pragma unroll
    for (int r = 0; r < D; ++r) {
        I acc = mul_(P[r * D], x[0]);
#pragma unroll
        for (int c = 1; c < D; ++c) acc = fmac_(acc, P[r * D + c], x[c]);
        y[r] = acc;
    }
}

// one step of the scanned system.  ND == 0: the SOS cascade, state (w1_q, w2_q) at
// st[2q], st[2q+1] (the fused form of sos_step_f).  ND > 0: Normal DF-II
// (src/filter/iir/mod.rs:272-279) with ND states hh[i] = v[n-1-i]; coefficients
// num[0..ND] then den[0..ND) (a[1..] / a0), zero padded to those lengths:
//   v = x - den . hh,   y = num[0] v + num[1..] . hh,   hh <- (v, hh[0..ND-2])
//
// SOS cascades run in b0-factored coordinates (runtime_iir.cpp wscan_coefs): the
// wave-scan coefficient set of a group holds, for every section but the last, (1, b1/b0, b2/b0,
// a1, a2), so the section's output is w + b1' w1 + b2' w2 (two fused multiply-adds instead of a
// multiply and two), and the last section carries the product G of the b0 before it: (G b0, G b1,
// G b2, a1, a2).  Section q's state is then the reference's divided by G_q = prod_{j<q} b0_j:
// the D scales G_q and their inverses follow the 5 S coefficients (wscan_scale / _inv), applied
// where a call's state enters (st_in) and leaves (st_out), so the handle's state buffer stays in
// the reference's units.
template <int S, int ND, typename C, typename I>
__device__ __forceinline__ I sys_step(const C* __restrict__ c, I v, I (&st)[ND ? ND : 2 * S]) {
    if constexpr (ND == 0) {
#pragma unroll
        for (int q = 0; q < S; ++q) {
            const I w = fmac_(fmac_(v, -c[5 * q + 4], st[2 * q + 1]), -c[5 * q + 3], st[2 * q]);
            if (q + 1 < S) v = fmac_(fmac_(w, c[5 * q + 1], st[2 * q]), c[5 * q + 2], st[2 * q + 1]);
            else v = fmac_(fmac_(mul_(c[5 * q + 2], st[2 * q + 1]), c[5 * q + 1], st[2 * q]), c[5 * q + 0], w);
            st[2 * q + 1] = st[2 * q];
            st[2 * q] = w;
        }
        return v;
    } else {
        I d = mul_(c[ND + 1], st[0]);
#pragma unroll
        for (int i = 1; i < ND; ++i) d = fmac_(d, c[ND + 1 + i], st[i]);
        const I w = sub_(v, d);
        I out = mul_(c[0], w);
#pragma unroll
        for (int i = 1; i <= ND; ++i) out = fmac_(out, c[i], st[i - 1]);
#pragma unroll
        for (int i = ND - 1; i > 0; --i) st[i] = st[i - 1];
        st[0] = w;
        return out;
    }
}

// y = P x: lower block-triangular for SOS cascades, dense for Normal DF-II
template <int ND, int D, typename C, typename I>
__device__ __forceinline__ void sys_matvec(const C* __restrict__ P, const I (&x)[D], I (&y)[D]) {
    if constexpr (ND == 0) matvec_lt<D>(P, x, y);
    else matvec_full<D>(P, x, y);
}

using v4u = unsigned __attribute__((ext_vector_type(4)));
typedef float ws_f2 __attribute__((ext_vector_type(2)));

// {acc.x + s.x v[HI], acc.y + s.y v[HI]}: one v_pk_fma_f32, s an SGPR pair, v[HI] broadcast to
// both lanes by op_sel; per lane the fused multiply-add of fmac_
template <int HI> __device__ __forceinline__ ws_f2 pk_fma_sb(ws_f2 s, ws_f2 v, ws_f2 acc) {
    ws_f2 r;
    if constexpr (HI == 0) asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[0,0,0] op_sel_hi:[1,0,1]" : "=v"(r) : "s"(s), "v"(v), "v"(acc));
    else asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[0,1,0] op_sel_hi:[1,1,1]" : "=v"(r) : "s"(s), "v"(v), "v"(acc));
    return r;
}

template <typename I> __device__ __forceinline__ v4u to_v4(const I (&e)[16 / sizeof(I)]) {
    v4u v;
    __builtin_memcpy(&v, e, 16);
    return v;
}

// Rate changes (DecimatingIIRFilter decim.rs:221-231, InterpolatingIIRFilter
// interp.rs:204-210): the scan runs at the domain rate (nd = n Mi samples).  With
// Mi > 1 the staged domain sample k is x[k / Mi] at k % Mi == 0, else zero; with
// Md > 1 only domain samples k = j0 + o Md are stored, as y[o] (gathered from the
// slab so that 64 consecutive outputs leave per store instruction).
// FORM: 0 correction by the state response, next tile prefetched into registers; 1 a
// rerun from the true state instead of the correction; 2 the correction without the
// register prefetch (fewer registers: more waves per SIMD hide the tile loads instead)
// LAB selects compile-time variants for in-process A/B runs (tools/lab/iir_lab.hip; the product
// kernels are LAB = 0): ablations 1 no zero-state run, 2 no scan, 4 no correction, 8 no HBM
// loads, 16 no HBM stores; variants 32 plain (not nontemporal) loads, 64 plain stores, 128
// nontemporal stores (the round-3 product; the product's interior stores are write-through), 256
// the scalar correction (the round-3 arithmetic; real f32), 512 every scan level (the round-4 scan),
// 1024 compiled for one rate without exact carries, 2048 the lane shifts by one as DPP wave_shr
// moves (real f32, D = 8), 4096 the carry as the lane scan's element -1 (no separate fold), 8192
// compiled for 4 workgroups per CU (<= 128 VGPRs), 16384 blocks in launch order (not XCD-ordered),
// 32768 four-wave workgroups (the form before one-wave workgroups), 65536 a segment's first tile
// stored element by element (the form before round 6)
template <int S, int ND, typename C, typename I, int CB, int FORM, int LAB = 0>
__global__ void __launch_bounds__((LAB & 32768) ? kWsThreads : 64, (LAB & 8192) ? 4 : 1)
sos_wscan_kernel(const I* __restrict__ x, I* __restrict__ y, const C* __restrict__ coefs,
                 const C* __restrict__ P /* [6][D][D] */, const C* __restrict__ Cr /* [B][D] */,
                 const I* __restrict__ st_in, I* __restrict__ st_out, long long nd, int wc, int tpw, bool vec_ok,
                 int Mi, int Md, long long j0, long long nout, const I* __restrict__ cin, I* __restrict__ gagg,
                 long long nwaves) {
    constexpr int D = ND ? ND : 2 * S;
    constexpr int B = ws_chunk<I, CB>::B;
    constexpr bool RERUN = FORM == 1, PF = FORM != 2;
    // LAB 1024: the warm-up scan at one rate only (Mi = Md = 1, no exact-carry passes) compiled
    // without the other paths (lab: what their code costs when it never runs)
    if constexpr ((LAB & 1024) != 0) {
        Mi = 1, Md = 1, cin = nullptr, gagg = nullptr;
    }
    // real f32: the correction in packed math over sample pairs (Cr in the [B/2][D][2] layout,
    // runtime_iir.cpp scan_tables); LAB 256: the scalar form over the same layout
    constexpr bool kPairCr = std::is_same<I, float>::value && std::is_same<C, float>::value;  // the layout
    constexpr bool kPackedCr = kPairCr && D % 2 == 0 && (LAB & 256) == 0;
    constexpr int E = 16 / (int)sizeof(I);  // samples per 16-byte vector
    constexpr int kRowBytes = WsGeom<CB>::kRowBytes, kVecPerRow = WsGeom<CB>::kVecPerRow;
    constexpr int kSlabBytes = WsGeom<CB>::kSlabBytes;
    extern __shared__ __attribute__((aligned(16))) char lds_raw[];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    char* slab = lds_raw + wave * kSlabBytes;
    char* row = slab + lane * kRowBytes;
    // one-wave workgroups: a wave's slab and registers return to the CU when its own segment ends
    // (cfg3 1.565 -> 1.546 ms, bit-identical, profiles/r05/lab/r05zq_iirburst_onewave.log); LAB 32768:
    // the four-wave workgroups of rounds 2-5 (lab)
    constexpr int kWaves = (LAB & 32768) ? kWsWaves : 1;
    C* sP = reinterpret_cast<C*>(lds_raw + kWaves * kSlabBytes);
    for (int i = threadIdx.x; i < 6 * D * D; i += 64 * kWaves) sP[i] = P[i];
    __syncthreads();

    const int ch = blockIdx.y;
    x += (long long)ch * (nd / Mi);
    y += (long long)ch * nout;
    st_in += (long long)ch * D;
    st_out += (long long)ch * D;
    // domain sample k (zero outside the call)
    auto dom = [&](long long k) -> I {
        if (k < 0 || k >= nd) return zero_v<I>();
        if (Mi == 1) return x[k];
        return k % Mi == 0 ? x[k / Mi] : zero_v<I>();
    };

    constexpr int lab = LAB;
    // XCD-ordered blocks (gridDim.x is a multiple of 8): block b runs on XCD b % 8 and
    // takes the (b / 8)-th block of that XCD's contiguous eighth, so each XCD streams
    // one window of neighbouring segments (cfg3: -1.6 %, the HBM-only pattern -2 %)
    const long long bx = (LAB & 16384) ? (long long)blockIdx.x  // lab: launch order
                                       : (long long)(blockIdx.x & 7) * (gridDim.x / 8) + (blockIdx.x >> 3);
    const long long gw = bx * kWaves + wave;          // wave's segment
    const long long segc = (long long)tpw * 64 - wc;  // chunks per segment
    const long long c_lo = gw * segc;                 // first chunk of the segment
    const long long k_lo = c_lo * B;
    if (k_lo >= nd) return;

    // carry entering the wave's first tile: zero (warm-up lanes settle it, wave 0 injects
    // st_in), or the exact carry of the aggregate pass + carry scan (cin)
    I carry[D];
#pragma unroll
    for (int d = 0; d < D; ++d) carry[d] = cin ? cin[((long long)ch * nwaves + gw) * D + d] : zero_v<I>();
    const bool agg = gagg != nullptr;  // aggregate pass: the wave's zero-carry end state only
    // scan levels: with warm-up (wc > 0) the state response has decayed below the warm-up
    // tolerance after wc chunks (||A^(wc B)|| < 1e-9 f32 / 1e-17 f64, the criterion that admits the
    // scan), so a lane needs the states of the 2^nlev - 1 >= wc - 1 lanes before it only: the
    // levels with offsets >= wc add terms below that tolerance and are skipped (cfg3: wc = 6, 3
    // levels of 6).  The exact-carry form (wc = 0) keeps every level.
    const int nlev = (wc > 0 && !(LAB & 512)) ? (wc > 1 ? 32 - __builtin_clz((unsigned)(wc - 1)) : 0) : 6;

    // interior tiles are read with straight-line 16-byte loads, one tile ahead of
    // the compute (a per-vector branch would serialise the HBM round trips)
    auto interior_at = [&](long long k0) { return vec_ok && Mi == 1 && k0 >= 0 && k0 + 64LL * B <= nd; };
    v4u pre[kVecPerRow];
    if constexpr (PF) {
        const long long k0 = (c_lo - wc) * B;
        if (interior_at(k0)) {
#pragma unroll
            for (int j = 0; j < kVecPerRow; ++j)
                pre[j] = (lab & 8)    ? v4u{(unsigned)lane, 0u, 0u, (unsigned)j}
                         : (lab & 32) ? reinterpret_cast<const v4u*>(x + k0)[lane + 64 * j]
                                      : __builtin_nontemporal_load(reinterpret_cast<const v4u*>(x + k0) + lane + 64 * j);
        }
    }

    for (int t = 0; t < tpw; ++t) {
        const long long k0 = (c_lo - wc + (long long)t * 64) * B;  // first sample of the tile
        if (k0 >= nd) break;

        // 1. stage the tile: vector v of the tile -> row v / kVecPerRow, slot v % kVecPerRow
        const bool interior = interior_at(k0);
        if (interior) {
            if constexpr (!PF) {
#pragma unroll
                for (int j = 0; j < kVecPerRow; ++j)
                    pre[j] = (lab & 8)    ? v4u{(unsigned)lane, (unsigned)t, 0u, (unsigned)j}
                             : (lab & 32) ? reinterpret_cast<const v4u*>(x + k0)[lane + 64 * j]
                                          : __builtin_nontemporal_load(reinterpret_cast<const v4u*>(x + k0) + lane + 64 * j);
            }
#pragma unroll
            for (int j = 0; j < kVecPerRow; ++j) {
                const int v = lane + 64 * j;
                *reinterpret_cast<v4u*>(slab + (v / kVecPerRow) * kRowBytes + (v % kVecPerRow) * 16) = pre[j];
            }
        } else {
            for (int j = 0; j < kVecPerRow; ++j) {
                const int v = lane + 64 * j;
                const long long kv = k0 + (long long)v * E;
                I tmp[E];
#pragma unroll
                for (int e = 0; e < E; ++e) tmp[e] = dom(kv + e);
                *reinterpret_cast<v4u*>(slab + (v / kVecPerRow) * kRowBytes + (v % kVecPerRow) * 16) = to_v4<I>(tmp);
            }
        }
        if constexpr (PF) {  // prefetch the next tile (whatever path this one took)
            const long long kn = k0 + 64LL * B;
            if (t + 1 < tpw && interior_at(kn)) {
#pragma unroll
                for (int j = 0; j < kVecPerRow; ++j)
                    pre[j] = (lab & 8)    ? v4u{(unsigned)lane, (unsigned)t, 0u, (unsigned)j}
                             : (lab & 32) ? reinterpret_cast<const v4u*>(x + kn)[lane + 64 * j]
                                          : __builtin_nontemporal_load(reinterpret_cast<const v4u*>(x + kn) + lane + 64 * j);
            }
        }
        wave_sync();

        // 2. zero-state run over my row, y0 in place
        I s[D];
        {
#pragma unroll
            for (int d = 0; d < D; ++d) s[d] = zero_v<I>();
#pragma unroll 2
            for (int o = 0; o < kVecPerRow && !(lab & 1); ++o) {
                I e[E];
                const v4u val = *reinterpret_cast<const v4u*>(row + o * 16);
                __builtin_memcpy(e, &val, 16);
#pragma unroll
                for (int i = 0; i < E; ++i) e[i] = sys_step<S, ND>(coefs, e[i], s);
                if constexpr (!RERUN) *reinterpret_cast<v4u*>(row + o * 16) = to_v4<I>(e);
            }
        }
        if (!cin && !agg && gw == 0 && t == 0 && lane == wc - 1) {  // the call's exact carried state enters here
#pragma unroll
            for (int d = 0; d < D; ++d) {
                if constexpr (ND == 0) s[d] = mul_(wscan_inv<S>(coefs, d), st_in[d]);
                else s[d] = st_in[d];
            }
        }
        // 3. fold the carry into lane 0, then the inclusive scan over lanes.  carry_lane (LAB 4096,
        //    warm-up scans only): the carry is the scan's element -1 instead -- at level k lane
        //    2^k - 1 takes it as its predecessor (element -1 is never updated), so no separate fold;
        //    its window [l - 2^nlev + 1, l] holds element -1 for l <= 2^nlev - 2, which covers the
        //    lanes l <= wc - 2 whose carry term A^(B (l + 1)) carry is above the warm-up tolerance
        const bool carry_lane = (LAB & 4096) != 0 && wc > 0;
        if (!(lab & 2) && !carry_lane) {
            I a[D];
            sys_matvec<ND>(sP, carry, a);
            if (lane == 0) {
#pragma unroll
                for (int d = 0; d < D; ++d) s[d] = add_(s[d], a[d]);
            }
        }
        const int nlev_t = carry_lane && nlev < 1 ? 1 : nlev;
#pragma unroll
        for (int k = 0; k < 6 && !(lab & 2); ++k) {
            if (k >= nlev_t) break;  // the terms of lanes >= 2^nlev back have decayed (see nlev)
            const int off = 1 << k;
            I prev[D], a[D];
            if (k == 0) {
                shfl_up1_state<(LAB & 2048) != 0>(s, prev);
            } else {
#pragma unroll
                for (int d = 0; d < D; ++d) prev[d] = shfl_up_v(s[d], off);
            }
            if constexpr ((LAB & 4096) != 0) {
                if (carry_lane) {
#pragma unroll
                    for (int d = 0; d < D; ++d) prev[d] = lane == off - 1 ? carry[d] : prev[d];
                }
            }
            sys_matvec<ND>(sP + k * D * D, prev, a);
            if (lane >= off - (carry_lane ? 1 : 0)) {
#pragma unroll
                for (int d = 0; d < D; ++d) s[d] = add_(s[d], a[d]);
            }
        }
        I init[D];
        {
            I up[D];
            shfl_up1_state<(LAB & 2048) != 0>(s, up);
#pragma unroll
            for (int d = 0; d < D; ++d) init[d] = lane == 0 ? carry[d] : up[d];
        }
#pragma unroll
        for (int d = 0; d < D; ++d) carry[d] = readlane_v(s[d], 63);
        if (agg) {
            wave_sync();
            continue;
        }

        // 4. outputs: correction by the state response (y0 in place), or (RERUN) the
        //    chunk rerun from its true initial state over the staged input
        if constexpr (RERUN) {
            I st[D];
#pragma unroll
            for (int d = 0; d < D; ++d) st[d] = init[d];
#pragma unroll 2
            for (int o = 0; o < kVecPerRow; ++o) {
                I e[E];
                const v4u val = *reinterpret_cast<const v4u*>(row + o * 16);
                __builtin_memcpy(e, &val, 16);
#pragma unroll
                for (int i = 0; i < E; ++i) e[i] = sys_step<S, ND>(coefs, e[i], st);
                *reinterpret_cast<v4u*>(row + o * 16) = to_v4<I>(e);
            }
        } else {
            [[maybe_unused]] ws_f2 initp[kPackedCr ? D / 2 : 1];
            if constexpr (kPackedCr) {
#pragma unroll
                for (int d = 0; d < D; d += 2) initp[d / 2] = ws_f2{init[d], init[d + 1]};
            }
#pragma unroll 2
            for (int o = 0; o < kVecPerRow && !(lab & 4); ++o) {
                I e[E];
                const v4u val = *reinterpret_cast<const v4u*>(row + o * 16);
                __builtin_memcpy(e, &val, 16);
                if constexpr (kPackedCr) {
                    // real f32: samples (2q, 2q + 1) of the chunk in one v_pk_fma_f32 per state, the
                    // pair {Cr[2q][d], Cr[2q+1][d]} an SGPR operand (host layout [B/2][D][2]) and
                    // init[d] broadcast by op_sel -- per sample the fmas below, bit for bit, in half
                    // the instructions (cfg3 sustained 1.664 -> 1.643 ms; the same packing of the
                    // lane scan and a skewed packed zero-state run measured slower)
                    const ws_f2* crp = reinterpret_cast<const ws_f2*>(Cr) + (o * (E / 2)) * D;
#pragma unroll
                    for (int q = 0; q < E / 2; ++q) {
                        ws_f2 acc = {e[2 * q], e[2 * q + 1]};
#pragma unroll
                        for (int d = 0; d < D; d += 2) {
                            acc = pk_fma_sb<0>(crp[q * D + d], initp[d / 2], acc);
                            acc = pk_fma_sb<1>(crp[q * D + d + 1], initp[d / 2], acc);
                        }
                        e[2 * q] = acc.x;
                        e[2 * q + 1] = acc.y;
                    }
                } else {
#pragma unroll
                    for (int i = 0; i < E; ++i) {
                        // Cr row of sample o E + i: wave-uniform, read through the scalar cache into
                        // SGPR operands (an LDS broadcast read costs a full ds_read_b128 per 4 values)
                        const C* cr = Cr + (o * E + i) * D;
                        if constexpr (kPairCr) cr = Cr + ((o * E + i) / 2) * 2 * D + ((o * E + i) & 1);
#pragma unroll
                        for (int d = 0; d < D; ++d) e[i] = fmac_(e[i], cr[kPairCr ? 2 * d : d], init[d]);
                    }
                }
                *reinterpret_cast<v4u*>(row + o * 16) = to_v4<I>(e);
            }
        }

        // exact final state: the lane of this segment holding sample nd-1 reruns its chunk
        const long long kc = k0 + (long long)lane * B;
        if (kc >= k_lo && kc <= nd - 1 && nd - 1 < kc + B) {
            I st[D];
#pragma unroll
            for (int d = 0; d < D; ++d) st[d] = init[d];
            for (long long k = kc; k < nd; ++k) (void)sys_step<S, ND>(coefs, dom(k), st);
#pragma unroll
            for (int d = 0; d < D; ++d) {
                if constexpr (ND == 0) st_out[d] = mul_(wscan_scale<S>(coefs, d), st[d]);
                else st_out[d] = st[d];
            }
        }
        wave_sync();

        // 5. coalesced store of the segment's samples
        if (Md > 1) {  // decimated: outputs o with domain index j0 + o Md inside this tile's share
            const long long ka = k0 > k_lo ? k0 : k_lo;
            const long long kb = k0 + 64LL * B < nd ? k0 + 64LL * B : nd;
            if (kb > ka && kb > j0) {
                const long long oa = ka <= j0 ? 0 : (ka - j0 + Md - 1) / Md;
                const long long ob = (kb - 1 - j0) / Md + 1;  // exclusive
                for (long long o = oa + lane; o < ob; o += 64) {
                    const int pos = (int)(j0 + o * Md - k0), v = pos / E;
                    y[o] = *reinterpret_cast<const I*>(slab + (v / kVecPerRow) * kRowBytes + (v % kVecPerRow) * 16 +
                                                       (pos % E) * (int)sizeof(I));
                }
            }
        } else if (interior && (k0 >= k_lo || (LAB & (65536 | 128 | 64)) == 0)) {
            // a segment's first tile too (it starts wc chunks early: vectors before k_lo are the
            // warm-up's), as 16-byte stores rather than element by element (LAB 65536: the
            // element-wise form of rounds 2-5).  The descriptor starts at max(k0, k_lo): the
            // warm-up vectors' offsets go negative, i.e. past the descriptor's range, and the
            // hardware drops them (chunk boundaries are 16-byte aligned) -- no branch per vector
            const long long kb = k0 >= k_lo ? k0 : k_lo;
            const int sh = (int)((kb - k0) * (long long)sizeof(I));
            const auto ry = __builtin_amdgcn_make_buffer_rsrc((void*)(y + kb), (short)0, 0x7fffffff, 0x00020000);
#pragma unroll
            for (int j = 0; j < kVecPerRow; ++j) {
                const int v = lane + 64 * j;
                const v4u val = *reinterpret_cast<const v4u*>(slab + (v / kVecPerRow) * kRowBytes + (v % kVecPerRow) * 16);
                if ((lab & 16) && val.x != 0x7fc01234u) continue;  // ablation: stores dropped
                // write-through (sc1) stores: cfg3 1.736 -> 1.707 ms against nontemporal ones (two
                // boxes, in-process A/B, profiles/r04/lab/r04b_iirab.log, r04c_iirab.log)
                if constexpr ((lab & 128) != 0) __builtin_nontemporal_store(val, reinterpret_cast<v4u*>(y + k0) + v);
                else if constexpr ((lab & 64) != 0) reinterpret_cast<v4u*>(y + k0)[v] = val;  // lab: plain store
                else __builtin_amdgcn_raw_buffer_store_b128(val, ry, v * 16 - sh, 0, 16);
            }
        } else {
            for (int j = 0; j < kVecPerRow; ++j) {
                const int v = lane + 64 * j;
                const long long kv = k0 + (long long)v * E;
                const v4u val =
                    *reinterpret_cast<const v4u*>(slab + (v / kVecPerRow) * kRowBytes + (v % kVecPerRow) * 16);
                I tmp[E];
                __builtin_memcpy(tmp, &val, 16);
#pragma unroll
                for (int e = 0; e < E; ++e)
                    if (kv + e >= k_lo && kv + e < nd) y[kv + e] = tmp[e];
            }
        }
        wave_sync();
    }
    if (agg && lane == 0) {
#pragma unroll
        for (int d = 0; d < D; ++d) gagg[((long long)ch * nwaves + gw) * D + d] = carry[d];
    }
}

// Exact carries between the waves of one channel (one workgroup per channel):
// cin[0] = st_in, cin[w + 1] = Phi cin[w] + G[w].  Each of the 256 lanes folds a
// contiguous run of R waves (Horner with Phi), lane 0 chains the 256 run
// aggregates with Phi^R, then every lane replays its run from its exact prefix.

template <int D, int S, typename C, typename I>
__global__ void __launch_bounds__(256)
wscan_carry_kernel(const I* __restrict__ G, I* __restrict__ cin, const C* __restrict__ Phi, const I* __restrict__ st_in,
                   long long W, const C* __restrict__ coefs) {
    __shared__ C sPhi[D * D], sPhiR[D * D];
    __shared__ I agg[256][D];
    const int t = threadIdx.x, ch = blockIdx.x;
    G += (long long)ch * W * D;
    cin += (long long)ch * W * D;
    st_in += (long long)ch * D;
    const long long R = (W + 255) / 256;
    if (t < D * D) sPhi[t] = Phi[t];
    __syncthreads();
    if (t == 0) {  // Phi^R by repeated squaring (R >= 1), in the Coef type
        C acc[D * D], base[D * D], tmp[D * D];
        for (int i = 0; i < D * D; ++i) { acc[i] = (i % (D + 1) == 0) ? C(1) : C(0); base[i] = sPhi[i]; }
        for (long long e = R; e > 0; e >>= 1) {
            if (e & 1) {
                for (int i = 0; i < D; ++i)
                    for (int j = 0; j < D; ++j) {
                        C v = C(0);
                        for (int k = 0; k < D; ++k) v = fmac_(v, acc[i * D + k], base[k * D + j]);
                        tmp[i * D + j] = v;
                    }
                for (int i = 0; i < D * D; ++i) acc[i] = tmp[i];
            }
            for (int i = 0; i < D; ++i)
                for (int j = 0; j < D; ++j) {
                    C v = C(0);
                    for (int k = 0; k < D; ++k) v = fmac_(v, base[i * D + k], base[k * D + j]);
                    tmp[i * D + j] = v;
                }
            for (int i = 0; i < D * D; ++i) base[i] = tmp[i];
        }
        for (int i = 0; i < D * D; ++i) sPhiR[i] = acc[i];
    }
    const long long w0 = (long long)t * R, w1 = w0 + R < W ? w0 + R : W;
    I a[D];
#pragma unroll
    for (int d = 0; d < D; ++d) a[d] = zero_v<I>();
    for (long long w = w0; w < w1; ++w) {  // a = Phi a + G[w]
        I b[D];
        matvec_full<D>(sPhi, a, b);
#pragma unroll
        for (int d = 0; d < D; ++d) a[d] = add_(b[d], G[w * D + d]);
    }
    // a run shorter than R (the tail) is padded with zero aggregates at its front so
    // that every run spans R waves: only the last non-empty run can be short, and its
    // aggregate is not needed by any later run
#pragma unroll
    for (int d = 0; d < D; ++d) agg[t][d] = a[d];
    __syncthreads();
    if (t == 0) {  // exclusive prefixes over runs: p_{j+1} = Phi^R p_j + agg_j
        I p[D];
#pragma unroll
        for (int d = 0; d < D; ++d) {  // S > 0: an SOS group in b0-factored coordinates (sys_step)
            if constexpr (S > 0) p[d] = mul_(wscan_inv<S>(coefs, d), st_in[d]);
            else p[d] = st_in[d];
        }
        for (int j = 0; j < 256; ++j) {
            I q[D];
#pragma unroll
            for (int d = 0; d < D; ++d) q[d] = agg[j][d];
#pragma unroll
            for (int d = 0; d < D; ++d) agg[j][d] = p[d];
            I b[D];
            matvec_full<D>(sPhiR, p, b);
#pragma unroll
            for (int d = 0; d < D; ++d) p[d] = add_(b[d], q[d]);
        }
    }
    __syncthreads();
    I c[D];
#pragma unroll
    for (int d = 0; d < D; ++d) c[d] = agg[t][d];
    for (long long w = w0; w < w1; ++w) {
#pragma unroll
        for (int d = 0; d < D; ++d) cin[w * D + d] = c[d];
        I b[D];
        matvec_full<D>(sPhi, c, b);
#pragma unroll
        for (int d = 0; d < D; ++d) c[d] = add_(b[d], G[w * D + d]);
    }
}

// ---------------------------------------------------------------- paired chunks (real f32)
// Same algorithm with two chunks per lane: lane l owns virtual lanes l and
// 64 + l of a 128-chunk tile, so the recurrence, the scan's matrix products and
// the correction run as packed (v_pk_fma_f32) pairs.  The scan spans 128
// virtual lanes: shifts below 64 take the high half's predecessor from the
// low half of lane l - d + 64; the shift by 64 is the lane's own low half.
typedef float f2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ f2 splat(float c) { return f2{c, c}; }
__device__ __forceinline__ f2 pfma(f2 a, f2 b, f2 c) { return __builtin_elementwise_fma(a, b, c); }

template <int S>
__device__ __forceinline__ f2 sos_step_p(const float* __restrict__ c, f2 v, f2 (&w1)[S], f2 (&w2)[S]) {
#pragma unroll
    for (int s = 0; s < S; ++s) {
        const f2 w = pfma(splat(-c[5 * s + 3]), w1[s], pfma(splat(-c[5 * s + 4]), w2[s], v));
        v = pfma(splat(c[5 * s + 0]), w, pfma(splat(c[5 * s + 1]), w1[s], splat(c[5 * s + 2]) * w2[s]));
        w2[s] = w1[s];
        w1[s] = w;
    }
    return v;
}

template <int D>
__device__ __forceinline__ void matvec_lt_p(const float* __restrict__ P, const f2 (&x)[D], f2 (&y)[D]) {
#pragma unroll
    for (int r = 0; r < D; ++r) {
        const int cmax = (r / 2) * 2 + 2;
        f2 acc = splat(P[r * D]) * x[0];
#pragma unroll
        for (int c = 1; c < cmax; ++c) acc = pfma(splat(P[r * D + c]), x[c], acc);
        y[r] = acc;
    }
}

template <int S, int CB>
__global__ void __launch_bounds__(kWsThreads)
sos_wscan2_kernel(const float* __restrict__ x, float* __restrict__ y, const float* __restrict__ coefs,
                  const float* __restrict__ P /* [7][D][D] */, const float* __restrict__ Cr /* [B][D] */,
                  const float* __restrict__ st_in, float* __restrict__ st_out, long long nd, int wc, int tpw,
                  bool vec_ok) {
    constexpr int D = 2 * S;
    constexpr int B = CB / 4;
    constexpr int E = 4;
    constexpr int kRowBytes = CB + 16, kVecPerRow = CB / 16;
    constexpr int kSlabBytes = 128 * kRowBytes;
    constexpr int TC = 128;  // chunks per tile
    extern __shared__ __attribute__((aligned(16))) char lds_raw[];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    char* slab = lds_raw + wave * kSlabBytes;
    char* row_a = slab + lane * kRowBytes;
    char* row_b = slab + (64 + lane) * kRowBytes;
    float* sP = reinterpret_cast<float*>(lds_raw + kWsWaves * kSlabBytes);
    float* sCr = sP + 7 * D * D;
    for (int i = threadIdx.x; i < 7 * D * D; i += kWsThreads) sP[i] = P[i];
    // Cr arrives in the [B/2][D][2] layout of the real-f32 tables (scan_tables)
    for (int j = threadIdx.x; j < B * D; j += kWsThreads) {
        const int i = j / D, d = j % D;
        sCr[j] = Cr[((i / 2) * D + d) * 2 + (i & 1)];
    }
    __syncthreads();

    const int ch = blockIdx.y;
    x += (long long)ch * nd;
    y += (long long)ch * nd;
    st_in += (long long)ch * D;
    st_out += (long long)ch * D;

    const long long gw = (long long)blockIdx.x * kWsWaves + wave;
    const long long segc = (long long)tpw * TC - wc;
    const long long c_lo = gw * segc;
    const long long k_lo = c_lo * B;
    if (k_lo >= nd) return;

    float carry[D];
#pragma unroll
    for (int d = 0; d < D; ++d) carry[d] = 0.0f;

    for (int t = 0; t < tpw; ++t) {
        const long long k0 = (c_lo - wc + (long long)t * TC) * B;
        if (k0 >= nd) break;

        const bool interior = vec_ok && k0 >= 0 && k0 + (long long)TC * B <= nd;
        if (interior) {
            v4u val[2 * kVecPerRow];
#pragma unroll
            for (int j = 0; j < 2 * kVecPerRow; ++j)
                val[j] = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(x + k0) + lane + 64 * j);
#pragma unroll
            for (int j = 0; j < 2 * kVecPerRow; ++j) {
                const int v = lane + 64 * j;
                *reinterpret_cast<v4u*>(slab + (v / kVecPerRow) * kRowBytes + (v % kVecPerRow) * 16) = val[j];
            }
        } else {
            for (int j = 0; j < 2 * kVecPerRow; ++j) {
                const int v = lane + 64 * j;
                const long long kv = k0 + (long long)v * E;
                float tmp[E];
#pragma unroll
                for (int e = 0; e < E; ++e) tmp[e] = (kv + e >= 0 && kv + e < nd) ? x[kv + e] : 0.0f;
                v4u val;
                __builtin_memcpy(&val, tmp, 16);
                *reinterpret_cast<v4u*>(slab + (v / kVecPerRow) * kRowBytes + (v % kVecPerRow) * 16) = val;
            }
        }
        wave_sync();

        // zero-state run of both chunks, packed
        f2 s[D];
        {
            f2 w1[S], w2[S];
#pragma unroll
            for (int q = 0; q < S; ++q) { w1[q] = splat(0.0f); w2[q] = splat(0.0f); }
#pragma unroll 2
            for (int o = 0; o < kVecPerRow; ++o) {
                float ea[E], eb[E];
                const v4u va = *reinterpret_cast<const v4u*>(row_a + o * 16);
                const v4u vb = *reinterpret_cast<const v4u*>(row_b + o * 16);
                __builtin_memcpy(ea, &va, 16);
                __builtin_memcpy(eb, &vb, 16);
#pragma unroll
                for (int i = 0; i < E; ++i) {
                    const f2 r = sos_step_p<S>(coefs, f2{ea[i], eb[i]}, w1, w2);
                    ea[i] = r.x;
                    eb[i] = r.y;
                }
                v4u oa, ob;
                __builtin_memcpy(&oa, ea, 16);
                __builtin_memcpy(&ob, eb, 16);
                *reinterpret_cast<v4u*>(row_a + o * 16) = oa;
                *reinterpret_cast<v4u*>(row_b + o * 16) = ob;
            }
#pragma unroll
            for (int q = 0; q < S; ++q) { s[2 * q] = w1[q]; s[2 * q + 1] = w2[q]; }
        }
        if (gw == 0 && t == 0) {  // the call's exact carried state enters at virtual lane wc-1
            const int vl = wc - 1;
            if (vl < 64 && lane == vl) {
#pragma unroll
                for (int d = 0; d < D; ++d) s[d].x = wscan_inv<S>(coefs, d) * st_in[d];
            } else if (vl >= 64 && lane == vl - 64) {
#pragma unroll
                for (int d = 0; d < D; ++d) s[d].y = wscan_inv<S>(coefs, d) * st_in[d];
            }
        }
        // carry into virtual lane 0
        {
            f2 cin[D], a[D];
#pragma unroll
            for (int d = 0; d < D; ++d) cin[d] = splat(carry[d]);
            matvec_lt_p<D>(sP, cin, a);
            if (lane == 0) {
#pragma unroll
                for (int d = 0; d < D; ++d) s[d].x += a[d].x;
            }
        }
        // inclusive scan over 128 virtual lanes
#pragma unroll
        for (int k = 0; k < 6; ++k) {
            const int off = 1 << k;
            const int src = (lane - off) & 63;
            const bool in = lane >= off;
            f2 prev[D], a[D];
#pragma unroll
            for (int d = 0; d < D; ++d) {
                const float pa = __shfl(s[d].x, src);
                const float pb = __shfl(s[d].y, src);
                prev[d] = f2{pa, in ? pb : pa};
            }
            matvec_lt_p<D>(sP + k * D * D, prev, a);
#pragma unroll
            for (int d = 0; d < D; ++d) {
                if (in) s[d].x += a[d].x;
                s[d].y += a[d].y;
            }
        }
        {  // shift by 64: high half += A^(64B) * own low half
            float lo[D], a[D];
#pragma unroll
            for (int d = 0; d < D; ++d) lo[d] = s[d].x;
            matvec_lt<D>(sP + 6 * D * D, lo, a);
#pragma unroll
            for (int d = 0; d < D; ++d) s[d].y += a[d];
        }
        f2 init[D];
#pragma unroll
        for (int d = 0; d < D; ++d) {
            const float ua = __shfl(s[d].x, (lane - 1) & 63);  // lane 0 reads lane 63's low half
            const float ub = __shfl(s[d].y, (lane - 1) & 63);
            init[d] = f2{lane == 0 ? carry[d] : ua, lane == 0 ? ua : ub};
        }
#pragma unroll
        for (int d = 0; d < D; ++d) carry[d] = __shfl(s[d].y, 63);

        // correction, packed
#pragma unroll 2
        for (int o = 0; o < kVecPerRow; ++o) {
            float ea[E], eb[E];
            const v4u va = *reinterpret_cast<const v4u*>(row_a + o * 16);
            const v4u vb = *reinterpret_cast<const v4u*>(row_b + o * 16);
            __builtin_memcpy(ea, &va, 16);
            __builtin_memcpy(eb, &vb, 16);
#pragma unroll
            for (int i = 0; i < E; ++i) {
                const float* cr = sCr + (o * E + i) * D;
                f2 acc = f2{ea[i], eb[i]};
#pragma unroll
                for (int d = 0; d < D; ++d) acc = pfma(splat(cr[d]), init[d], acc);
                ea[i] = acc.x;
                eb[i] = acc.y;
            }
            v4u oa, ob;
            __builtin_memcpy(&oa, ea, 16);
            __builtin_memcpy(&ob, eb, 16);
            *reinterpret_cast<v4u*>(row_a + o * 16) = oa;
            *reinterpret_cast<v4u*>(row_b + o * 16) = ob;
        }

        // exact final state from the virtual lane of this segment holding sample nd-1
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const long long kc = k0 + (long long)(lane + 64 * h) * B;
            if (kc >= k_lo && kc <= nd - 1 && nd - 1 < kc + B) {
                float w1[S], w2[S];
#pragma unroll
                for (int q = 0; q < S; ++q) {
                    w1[q] = h ? init[2 * q].y : init[2 * q].x;
                    w2[q] = h ? init[2 * q + 1].y : init[2 * q + 1].x;
                }
                for (long long k = kc; k < nd; ++k) (void)sos_step_f<S>(coefs, x[k], w1, w2);
#pragma unroll
                for (int q = 0; q < S; ++q) {
                    st_out[2 * q] = wscan_scale<S>(coefs, 2 * q) * w1[q];
                    st_out[2 * q + 1] = wscan_scale<S>(coefs, 2 * q + 1) * w2[q];
                }
            }
        }
        wave_sync();

        if (interior && k0 >= k_lo) {
#pragma unroll
            for (int j = 0; j < 2 * kVecPerRow; ++j) {
                const int v = lane + 64 * j;
                const v4u val = *reinterpret_cast<const v4u*>(slab + (v / kVecPerRow) * kRowBytes + (v % kVecPerRow) * 16);
                __builtin_nontemporal_store(val, reinterpret_cast<v4u*>(y + k0) + v);
            }
        } else {
            for (int j = 0; j < 2 * kVecPerRow; ++j) {
                const int v = lane + 64 * j;
                const long long kv = k0 + (long long)v * E;
                const v4u val =
                    *reinterpret_cast<const v4u*>(slab + (v / kVecPerRow) * kRowBytes + (v % kVecPerRow) * 16);
                float tmp[E];
                __builtin_memcpy(tmp, &val, 16);
#pragma unroll
                for (int e = 0; e < E; ++e)
                    if (kv + e >= k_lo && kv + e < nd) y[kv + e] = tmp[e];
            }
        }
        wave_sync();
    }
}

template <int S, int CB>
hipError_t launch_wscan2_t(const IirArgs& a, hipStream_t st) {
    constexpr int B = CB / 4;
    const long long nd = (long long)a.n;
    const long long nch = (nd + B - 1) / B;
    int tpw = (int)(nch / (128LL * 4096));
    tpw = tpw < 1 ? 1 : (tpw > 8 ? 8 : tpw);
    const long long segc = (long long)tpw * 128 - a.wc;
    const long long waves = (nch + segc - 1) / segc;
    dim3 grid((unsigned)((waves + kWsWaves - 1) / kWsWaves), (unsigned)a.channels);
    const bool vec_ok = reinterpret_cast<uintptr_t>(a.x) % 16 == 0 && reinterpret_cast<uintptr_t>(a.y) % 16 == 0 &&
                        (a.channels == 1 || (nd * 4) % 16 == 0);
    const size_t lds = (size_t)kWsWaves * 128 * (CB + 16) + sizeof(float) * (7 * 4 * S * S + B * 2 * S);
    hipLaunchKernelGGL((sos_wscan2_kernel<S, CB>), grid, dim3(kWsThreads), lds, st, (const float*)a.x, (float*)a.y,
                       (const float*)a.coefs, (const float*)a.P, (const float*)a.Cr, (const float*)a.st_in,
                       (float*)a.st_out, nd, a.wc, tpw, vec_ok);
    return hipGetLastError();
}

template <int CB>
hipError_t launch_wscan2_s(const IirArgs& a, hipStream_t st) {
    switch (a.sections) {
        case 1: return launch_wscan2_t<1, CB>(a, st);
        case 2: return launch_wscan2_t<2, CB>(a, st);
        case 3: return launch_wscan2_t<3, CB>(a, st);
        case 4: return launch_wscan2_t<4, CB>(a, st);
        case 5: return launch_wscan2_t<5, CB>(a, st);
        case 6: return launch_wscan2_t<6, CB>(a, st);
        case 7: return launch_wscan2_t<7, CB>(a, st);
        case 8: return launch_wscan2_t<8, CB>(a, st);
    }
    return hipErrorInvalidValue;
}

template <int CB> int wscan_tpw(long long nch) {
    // tiles per wave: long segments amortise the wc warm-up chunks; keep >= ~4k waves when possible.
    // At most 5 tiles: cfg3 (2^30 real f32, 128-byte chunks, 20 back-to-back calls, 16 interleaved
    // rounds) ran 1.653 / 1.650 / 1.627 / 1.615 / 1.640 ms at 8 / 7 / 6 / 5 / 4 tiles, outputs within
    // 1.1e-8 rel-RMS of each other (the warm-up boundaries move; profiles/r05/lab/r05ze_iirburst.log);
    // cfg12 (256-byte chunks) 1.670 -> 1.643 ms at 5 instead of 8 (alternating bench lines,
    // profiles/r05/lab/r05zh_libab_cfg12.log)
    constexpr int kMax = 5;
    int tpw = (int)(nch / (64LL * 4096));
    return tpw < 1 ? 1 : (tpw > kMax ? kMax : tpw);
}

// LAB: sos_wscan_kernel (0 = the product kernel); tpw_force > 0 sets the tiles per wave of a
// warm-up scan (lab runs)
template <typename C, typename I, int S, int CB, int FORM, int ND = 0, int LAB = 0>
hipError_t launch_wscan_t(const IirArgs& a, hipStream_t st, int tpw_force = 0) {
    constexpr int B = ws_chunk<I, CB>::B;
    constexpr int D = ND ? ND : 2 * S;
    const long long nd = (long long)a.n * a.Mi;  // domain samples
    const long long nch = (nd + B - 1) / B;
    int tpw = wscan_tpw<CB>(nch);
    if (a.wc > 0 && tpw_force > 0) tpw = tpw_force;
    const long long segc = (long long)tpw * 64 - a.wc;
    const long long waves = (nch + segc - 1) / segc;
    const bool exact = a.wc == 0;  // exact inter-wave carries: aggregate pass + carry scan first
    if (exact && (!a.Phi || !a.G || !a.Cin || (size_t)waves > a.scratch_waves)) return hipErrorInvalidValue;
    // whole eighths for the XCD-ordered block map (surplus blocks find no segment and return)
    constexpr int kWaves = (LAB & 32768) ? kWsWaves : 1;  // waves per workgroup (see sos_wscan_kernel)
    dim3 grid((unsigned)((waves + 8 * kWaves - 1) / (8 * kWaves) * 8), (unsigned)a.channels);
    // 16-byte vector path: aligned bases and channel strides
    const bool vec_ok = reinterpret_cast<uintptr_t>(a.x) % 16 == 0 && reinterpret_cast<uintptr_t>(a.y) % 16 == 0 &&
                        (a.channels == 1 || (nd * (long long)sizeof(I)) % 16 == 0);
    const size_t lds = (size_t)kWaves * WsGeom<CB>::kSlabBytes + sizeof(C) * (6 * D * D);
    const long long j0 = a.Md > 1 ? (long long)((a.Md - 1 - a.phase) % a.Md) : 0;  // first emitting domain index
    const long long ny = a.Md > 1 ? (long long)a.nout : nd;
    if (exact) {
        hipLaunchKernelGGL((sos_wscan_kernel<S, ND, C, I, CB, FORM, LAB>), grid, dim3(64 * kWaves), lds, st, (const I*)a.x,
                           (I*)a.y, (const C*)a.coefs, (const C*)a.P, (const C*)a.Cr, (const I*)a.st_in, (I*)a.st_out,
                           nd, 0, tpw, vec_ok, a.Mi, a.Md, j0, ny, (const I*)nullptr, (I*)a.G, waves);
        hipLaunchKernelGGL((wscan_carry_kernel<D, ND ? 0 : S, C, I>), dim3((unsigned)a.channels), dim3(256), 0, st,
                           (const I*)a.G, (I*)a.Cin, (const C*)a.Phi + (size_t)(tpw - 1) * D * D, (const I*)a.st_in,
                           waves, (const C*)a.coefs);
    }
    hipLaunchKernelGGL((sos_wscan_kernel<S, ND, C, I, CB, FORM, LAB>), grid, dim3(64 * kWaves), lds, st, (const I*)a.x, (I*)a.y,
                       (const C*)a.coefs, (const C*)a.P, (const C*)a.Cr, (const I*)a.st_in, (I*)a.st_out, nd, a.wc,
                       tpw, vec_ok, a.Mi, a.Md, j0, ny, exact ? (const I*)a.Cin : (const I*)nullptr, (I*)nullptr,
                       waves);
    return hipGetLastError();
}

template <typename C, typename I, int CB, int FORM = 0>
hipError_t launch_wscan_s(const IirArgs& a, hipStream_t st) {
    switch (a.sections) {
        case 1: return launch_wscan_t<C, I, 1, CB, FORM>(a, st);
        case 2: return launch_wscan_t<C, I, 2, CB, FORM>(a, st);
        case 3: return launch_wscan_t<C, I, 3, CB, FORM>(a, st);
        case 4: return launch_wscan_t<C, I, 4, CB, FORM>(a, st);
        case 5: return launch_wscan_t<C, I, 5, CB, FORM>(a, st);
        case 6: return launch_wscan_t<C, I, 6, CB, FORM>(a, st);
        case 7: return launch_wscan_t<C, I, 7, CB, FORM>(a, st);
        case 8: return launch_wscan_t<C, I, 8, CB, FORM>(a, st);
    }
    return hipErrorInvalidValue;
}

// Normal DF-II with D = cap - 1 states (D <= 8), CB-byte chunks
template <typename C, typename I, int CB>
hipError_t launch_wscan_normal_cb(const IirArgs& a, hipStream_t st) {
    switch (a.cap - 1) {
        case 1: return launch_wscan_t<C, I, 0, CB, 0, 1>(a, st);
        case 2: return launch_wscan_t<C, I, 0, CB, 0, 2>(a, st);
        case 3: return launch_wscan_t<C, I, 0, CB, 0, 3>(a, st);
        case 4: return launch_wscan_t<C, I, 0, CB, 0, 4>(a, st);
        case 5: return launch_wscan_t<C, I, 0, CB, 0, 5>(a, st);
        case 6: return launch_wscan_t<C, I, 0, CB, 0, 6>(a, st);
        case 7: return launch_wscan_t<C, I, 0, CB, 0, 7>(a, st);
        case 8: return launch_wscan_t<C, I, 0, CB, 0, 8>(a, st);
    }
    return hipErrorInvalidValue;
}
// 256-byte chunks; real f32 takes 128-byte chunks for variant 1 (its default, as for the cascades)
template <typename C, typename I>
hipError_t launch_wscan_normal(const IirArgs& a, hipStream_t st) {
    if constexpr (std::is_same<I, float>::value && std::is_same<C, float>::value)
        if (a.ws_variant == 1) return launch_wscan_normal_cb<C, I, 128>(a, st);
    return launch_wscan_normal_cb<C, I, 256>(a, st);
}

template <typename C, typename I>
hipError_t launch_wscan_dt(const IirArgs& a, hipStream_t st) {
    if (a.sections == 0) return launch_wscan_normal<C, I>(a, st);
    if (a.Mi != 1 || a.Md != 1 || a.wc == 0)  // rate changes / exact carries: the single-chunk kernels only
        return a.ws_variant == 5   ? launch_wscan_s<C, I, 128, 2>(a, st)
               : a.ws_variant == 1 ? launch_wscan_s<C, I, 128>(a, st)
                                   : launch_wscan_s<C, I, 256>(a, st);
    if constexpr (std::is_same<I, float>::value) {
        if (a.ws_variant == 2) return launch_wscan2_s<128>(a, st);
        if (a.ws_variant == 3) return launch_wscan2_s<64>(a, st);
    }
    if (a.ws_variant == 4) return launch_wscan_s<C, I, 256, 1>(a, st);  // rerun instead of correction
    if (a.ws_variant == 5) return launch_wscan_s<C, I, 128, 2>(a, st);  // 128-byte chunks, no register prefetch
    return a.ws_variant == 1 ? launch_wscan_s<C, I, 128>(a, st) : launch_wscan_s<C, I, 256>(a, st);
}

}  // namespace


size_t iir_wscan_waves(int dtype, const IirArgs& a, int* tpw_out) {
    const bool c128 = a.ws_variant == 1 || a.ws_variant == 5;
    const int B = iir_wscan_chunk(dtype, c128 ? 1 : 0);
    if (B == 0) return 0;
    const long long nch = ((long long)a.n * a.Mi + B - 1) / B;
    const int tpw = c128 ? wscan_tpw<128>(nch) : wscan_tpw<256>(nch);
    if (tpw_out) *tpw_out = tpw;
    const long long segc = (long long)tpw * 64 - a.wc;
    return (size_t)((nch + segc - 1) / segc);
}

int iir_wscan_chunk(int dtype, int variant) {
    // variants: 0 = 256-byte chunks, 1 = 128-byte, 2/3 = paired 128/64-byte chunks (real f32 only),
    // 4 = 256-byte chunks with a rerun instead of the state-response correction, 5 = 128-byte
    // chunks without the register prefetch
    if ((variant == 2 || variant == 3) && dtype != 0) return 0;
    const int cb = (variant == 0 || variant == 4) ? 256 : (variant == 3 ? 64 : 128);
    switch (dtype) {
        case 0: return cb / (int)sizeof(float);
        case 1: return cb / (int)sizeof(c32);
        case 3: return cb / (int)sizeof(double);
        case 4: return cb / (int)sizeof(c64);
    }
    return 0;
}

hipError_t launch_iir_wscan(int dtype, const IirArgs& a, hipStream_t st) {
    if (a.n == 0) return hipSuccess;
    switch (dtype) {
        case 0: return launch_wscan_dt<float, float>(a, st);
        case 1: return launch_wscan_dt<float, c32>(a, st);
        case 3: return launch_wscan_dt<double, double>(a, st);
        case 4: return launch_wscan_dt<double, c64>(a, st);
    }
    return hipErrorInvalidValue;
}

}  // namespace sdsp
