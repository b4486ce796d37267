// Overlap-save FIR, N = 4096, in packed FP32 arithmetic (gfx950).
//
// Same transform, data flow and LDS images as fir_ols4096_kernel in
// kern_fir_ols.hip (P1..P5, three radix-16 passes each way, spectrum in
// registers, two LDS regions, four barriers per segment), but every complex
// value is a float pair and every complex add/sub/multiply is a
// v_pk_add/v_pk_mul/v_pk_fma_f32: on gfx950 a packed op issues in about the
// time of one scalar FMA and does two lanes' worth of work (measured with
// tools/valu_probe.hip and tools/fft_occ_probe.hip: a register DFT16 loop runs
// 1.6x faster packed).  Each component goes through the same IEEE operation
// sequence as the scalar kernel, so the two kernels agree bit for bit.
//
// To keep the register allocator from adding moves and spills around the
// pair-aligned operands:
//   * the workgroup only runs interior segments; the (at most two) boundary
//     segments of a call go through the scalar kernel's code in a separate
//     launch (fir_ols4096_edge_kernel);
//   * DFT16 leaves its output in the stage order X[ka + 4 kb] -> v[4 ka + kb];
//     callers index through kout() instead of copying into natural order;
//   * the twiddle and spectrum registers are made opaque once per segment so
//     swizzled copies of them are not hoisted out of the loop.
//
// The file is compiled once per scheduling strategy (Makefile: SDSP_PK_NS names
// the namespace, e.g. -mllvm -amdgpu-sched-strategy=max-ilp for pk_ilp), so the
// strategies can be A/B'd in one process through SDSP_TUNE_OLS_PACKED.
#include "sdsp_device.hpp"
#include "sdsp_kernels.hpp"

#ifndef SDSP_PK_NS
#define SDSP_PK_NS pk_default
#endif

namespace sdsp {
namespace SDSP_PK_NS {

namespace {

typedef float f2 __attribute__((ext_vector_type(2)));
typedef float f4v __attribute__((ext_vector_type(4)));

// Complex helpers.  Per component each performs the operation sequence of its
// scalar counterpart in kern_fir_ols.hip (cmul, cmulc, dft4, tw16), so results
// are bit-identical.  A swapped, half-negated operand ({b.y, -b.x}) is written
// as a product or fma with a +-1 pair (exact; the pair lives in an SGPR pair and
// the swap becomes op_sel): the backend does not fold a one-lane negation into
// neg_lo / neg_hi and would emit v_xor + v_mov pairs instead.
//
// The table products a * w (two per complex multiply) exist in two builds:
// ASM = true issues them as two VOP3P instructions with op_sel / neg modifiers
// (inline asm: the scheduler sees no latency for them); ASM = false uses three
// compiler-visible instructions.
constexpr f2 kPM = {1.0f, -1.0f};
constexpr f2 kMP = {-1.0f, 1.0f};

// a * b = {fma(a.x, b.x, -(a.y b.y)), fma(a.x, b.y, a.y b.x)}
template <bool ASM> __device__ __forceinline__ f2 pmul(f2 a, f2 b) {
    if constexpr (ASM) {
        f2 t, r;
        asm("v_pk_mul_f32 %0, %1, %2 op_sel:[1,1] op_sel_hi:[1,0] neg_lo:[0,1]" : "=v"(t) : "v"(a), "v"(b));
        asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel_hi:[0,1,1]" : "=v"(r) : "v"(a), "v"(b), "v"(t));
        return r;
    } else {
        return __builtin_elementwise_fma(a.xx, b, (a.yy * b.yx) * kMP);
    }
}
// a * conj(b) = {fma(a.x, b.x, a.y b.y), fma(a.y, b.x, -(a.x b.y))}
template <bool ASM> __device__ __forceinline__ f2 pmulc(f2 a, f2 b) {
    if constexpr (ASM) {
        f2 t, r;
        asm("v_pk_mul_f32 %0, %1, %2 op_sel:[1,1] op_sel_hi:[0,1] neg_hi:[0,1]" : "=v"(t) : "v"(a), "v"(b));
        asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel_hi:[1,0,1]" : "=v"(r) : "v"(a), "v"(b), "v"(t));
        return r;
    } else {
        return __builtin_elementwise_fma(a, b.xx, (a.yx * b.yy) * kPM);
    }
}
// b + (-j) e = {b.x + e.y, b.y - e.x}
__device__ __forceinline__ f2 padd_mj(f2 b, f2 e) { return __builtin_elementwise_fma(e.yx, kPM, b); }
// b + (+j) e = {b.x - e.y, b.y + e.x}
__device__ __forceinline__ f2 padd_pj(f2 b, f2 e) { return __builtin_elementwise_fma(e.yx, kMP, b); }
// (-j) v = {v.y, -v.x} (forward) / (+j) v = {-v.y, v.x} (inverse)
template <bool INV> __device__ __forceinline__ f2 prot(f2 v) { return v.yx * (INV ? kMP : kPM); }
template <bool INV> __device__ __forceinline__ void pdft4(f2& x0, f2& x1, f2& x2, f2& x3) {
    const f2 a = x0 + x2, b = x0 - x2, c = x1 + x3, e = x1 - x3;
    x0 = a + c;
    x2 = a - c;
    if constexpr (INV) {
        x1 = padd_pj(b, e);
        x3 = padd_mj(b, e);
    } else {
        x1 = padd_mj(b, e);
        x3 = padd_pj(b, e);
    }
}

constexpr float kC1 = 0.92387953251128674f;  // cos(pi/8)
constexpr float kS1 = 0.38268343236508978f;  // sin(pi/8)
constexpr float kR2 = 0.70710678118654752f;  // sqrt(1/2)

// v * (cr + j ci) for compile-time cr, ci
__device__ __forceinline__ f2 pmulk(f2 v, float cr, float ci) {
    return __builtin_elementwise_fma(v.xx, f2{cr, ci}, v.yy * f2{-ci, cr});
}
// tw16 m = 2: kR2 * (v.x + s v.y, v.y - s v.x)
template <bool INV> __device__ __forceinline__ f2 ptw2(f2 v) {
    return (INV ? padd_pj(v, v) : padd_mj(v, v)) * kR2;
}
// tw16 m = 6: kR2 * (-v.x + s v.y, -v.y - s v.x)
template <bool INV> __device__ __forceinline__ f2 ptw6(f2 v) {
    if constexpr (INV) return __builtin_elementwise_fma(v.xx, kMP, -v.yy) * kR2;  // {-v.x - v.y, v.x - v.y}
    else return __builtin_elementwise_fma(v.yy, kPM, -v.xx) * kR2;                 // {v.y - v.x, -v.y - v.x}
}
template <bool INV, int m> __device__ __forceinline__ f2 ptw16(f2 v) {
    constexpr float s = INV ? -1.0f : 1.0f;
    if constexpr (m == 0) return v;
    else if constexpr (m == 1) return pmulk(v, kC1, -s * kS1);
    else if constexpr (m == 2) return ptw2<INV>(v);
    else if constexpr (m == 3) return pmulk(v, kS1, -s * kC1);
    else if constexpr (m == 4) return prot<INV>(v);
    else if constexpr (m == 6) return ptw6<INV>(v);
    else if constexpr (m == 9) return pmulk(v, -kC1, s * kS1);
    else return v;
}

// lanes 16..31 of a <-> lanes 0..15 of b, in each half wave (v_permlane16_swap_b32)
__device__ __forceinline__ void swap16(float& a, float& b) {
    const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(a), __float_as_uint(b), false, false);
    a = __uint_as_float(r[0]);
    b = __uint_as_float(r[1]);
}

// X[k] of a DFT16 lives at v[kout(k)] (stage order, no reordering copy)
constexpr int kout(int k) { return 4 * (k & 3) + (k >> 2); }

// in-place 16-point DFT: natural order in, stage order out (X[ka + 4 kb] at v[4 ka + kb])
template <bool INV> __device__ __forceinline__ void pdft16(f2 (&v)[16]) {
#pragma unroll
    for (int nb = 0; nb < 4; ++nb) pdft4<INV>(v[nb], v[4 + nb], v[8 + nb], v[12 + nb]);
    v[5] = ptw16<INV, 1>(v[5]);
    v[6] = ptw16<INV, 2>(v[6]);
    v[7] = ptw16<INV, 3>(v[7]);
    v[9] = ptw16<INV, 2>(v[9]);
    v[10] = ptw16<INV, 4>(v[10]);
    v[11] = ptw16<INV, 6>(v[11]);
    v[13] = ptw16<INV, 3>(v[13]);
    v[14] = ptw16<INV, 6>(v[14]);
    v[15] = ptw16<INV, 9>(v[15]);
#pragma unroll
    for (int ka = 0; ka < 4; ++ka) pdft4<INV>(v[4 * ka + 0], v[4 * ka + 1], v[4 * ka + 2], v[4 * ka + 3]);
}

constexpr int kRowA = 272;           // A image: 16 rows of 256 (+16 pad) samples
constexpr int kRegion = 16 * kRowA;  // samples per LDS region
// LDS images, bank-conflict free for every access of P1..P5 (MI355X_MICROARCH.md §LDS
// lane groups):
// A image: 16 rows of 256 (+16 pad) samples; column c sits at acol(c) = c ^ bit 4 of c,
//   so P1's 16-lane ds_write_b64 groups (columns 0, 2, .., 30 of the W16 lane order)
//   cover all 32 write banks
// B image: 256 rows x 16 samples; row r sits at physical row r ^ bit 4 of r (rows r and
//   r + 16, read by one 32-lane half in P4, land in opposite halves of the 64 banks) and its
//   16-byte pairs are XOR-swizzled by r & 7 (P3's 8-lane ds_write_b128 groups hit 8 slots)
__device__ __forceinline__ int acol(int c) { return c ^ ((c >> 4) & 1); }
__device__ __forceinline__ int brow(int r) { return r ^ ((r >> 4) & 1); }
__device__ __forceinline__ int bidx(int r, int c) { return brow(r) * 16 + ((((c >> 1) ^ r) & 7) << 1) + (c & 1); }

}  // namespace

// ABL: profiling ablations (outputs invalid), same arithmetic.  Bit 0: no HBM loads
// or stores; bit 1: no workgroup barriers; bit 2: no LDS (transposes become
// register renames).  ABL = 8: HBM traffic only (no arithmetic, LDS or barriers)
//
// W16: 16-byte global accesses.  Lane t then owns column
//     col(t) = 32 (t >> 5) + 2 (t & 15) + ((t >> 4) & 1)
// instead of t: a lane loads two adjacent columns (X, X + 1), X = col - (t>>4 & 1),
// of one row (rows 2i and 2i + 1 for the lower / upper 16 lanes of each 32), and
// one v_permlane16_swap per dword (lanes 16..31 of the first operand <-> lanes
// 0..15 of the second) turns the pair into column X (lower lane) and X + 1 (upper
// lane) over rows 2i, 2i + 1.  The same swap turns P5's columns back into row
// pairs for dwordx4 stores.  P1 writes and P5 reads LDS column col(t) (a
// permutation of the columns inside each wave, still conflict-free) and w1 is the
// table row of col(t); P2..P4 are unchanged.
template <int B> struct Buf { static constexpr int value = B; };

// HBM issue schedules of the packed kernel (SCH): hook point of each row-pair chunk.
// Points: 0 loop head, 1 after P1's LDS writes, 2 after P2's DFT, 3 after P2's LDS
// writes, 4 after P3's forward DFT and spectrum product, 5 after P3's LDS writes,
// 6 after P4's DFT, 7 after P4's LDS writes, 8 after P5's LDS reads.
constexpr int kNumSch = 10;
constexpr int kLoadAt[kNumSch][8] = {
    {1, 1, 1, 1, 1, 1, 1, 1}, {0, 0, 1, 1, 3, 3, 5, 5}, {0, 0, 1, 2, 3, 4, 5, 6},
    {0, 1, 2, 3, 4, 5, 6, 7}, {0, 0, 1, 1, 2, 2, 3, 3}, {0, 0, 0, 0, 1, 1, 1, 1},
    {0, 0, 0, 0, 1, 1, 3, 3}, {0, 0, 1, 1, 3, 3, 5, 5}, {0, 0, 1, 1, 3, 3, 5, 5},
    {0, 0, 1, 1, 3, 3, 5, 5}};
constexpr int kStoreAt[kNumSch][8] = {
    {1, 1, 1, 1, 1, 1, 1, 1}, {1, 1, 3, 3, 5, 5, 7, 7}, {1, 2, 3, 4, 5, 6, 7, 8},
    {1, 2, 3, 4, 5, 6, 7, 8}, {1, 2, 3, 4, 5, 6, 7, 8}, {1, 2, 3, 4, 5, 6, 7, 8},
    {1, 1, 3, 3, 5, 5, 7, 7}, {3, 3, 5, 5, 7, 7, 8, 8}, {1, 1, 1, 1, 5, 5, 5, 5},
    {2, 2, 4, 4, 6, 6, 8, 8}};

template <int H2, int ABL, bool ASM, bool W16, int NT = 0, int D = 1, int SCH = 0>
__global__ void __launch_bounds__(256, 2)
fir_ols4096_pk_kernel(const f2* __restrict__ x, const f2* __restrict__ Hs, const f2* __restrict__ tw1,
                      const f2* __restrict__ tw2, f2* __restrict__ y, long long n, long long seg_lo,
                      long long seg_hi, long long per, long long xm) {
    static_assert(D == 1 || (D == 2 && W16), "two segments in flight need the 16-byte path");
    // SCH: issue schedule of the HBM traffic over a segment (tables kLoadAt / kStoreAt:
    // hook point of each row-pair chunk i of the next segment's loads / the previous
    // segment's deferred stores).  SCH 0: everything at point 1 (D = 2: stores at the end
    // of P5 instead).
    static_assert(SCH == 0 || (W16 && D == 1), "spread schedules: 16-byte path, one segment ahead");
    __shared__ __attribute__((aligned(16))) f2 lds[2 * kRegion];
    f2* const rA = lds;
    f2* const rB = lds + kRegion;
    const int ch = blockIdx.y;
    x += (long long)ch * n;
    y += (long long)ch * n;
    const int t = threadIdx.x;
    const int hi4 = t >> 4, lo4 = t & 15;
    const int up = (t >> 4) & 1;                   // W16: upper 16 lanes of a 32
    const int colX = 32 * (t >> 5) + 2 * (t & 15);  // W16: first column of the lane pair
    const int col = W16 ? colX + up : t;
    f2 w1[16], w2[16], Hr[16];
    // issued after the first segment's loads: a one-shot workgroup (per = 1) then waits
    // for the tables only where P1 first needs them, not ahead of its HBM stream
    auto load_tables = [&] {
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            if constexpr (ABL & 16) {  // ablation: no table loads
                w1[k] = w2[k] = Hr[k] = f2{(float)k, (float)t};
            } else if constexpr (ABL & 32) {  // ablation: the spectrum table only
                w1[k] = w2[k] = f2{(float)k, (float)t};
                const float4 e = reinterpret_cast<const float4*>(Hs)[(k / 2) * 256 + t];
                Hr[k] = k % 2 ? f2{e.z, e.w} : f2{e.x, e.y};
            } else if (k % 2 == 0) {  // k-pair major tables (OlsPlan::d_pkt): coalesced 16-byte loads
                const float4 a = reinterpret_cast<const float4*>(tw1)[(k / 2) * 256 + col];
                const float4 c = reinterpret_cast<const float4*>(tw2)[(k / 2) * 16 + lo4];
                const float4 e = reinterpret_cast<const float4*>(Hs)[(k / 2) * 256 + t];
                w1[k] = f2{a.x, a.y};
                w1[k + 1] = f2{a.z, a.w};
                w2[k] = f2{c.x, c.y};
                w2[k + 1] = f2{c.z, c.w};
                Hr[k] = f2{e.x, e.y};
                Hr[k + 1] = f2{e.z, e.w};
            }
        }
    };
    constexpr int V = 4096 - 256 * H2;
    // interior segments [seg_lo, seg_hi): per == 0, interleaved over a persistent
    // grid; per > 0, `per` consecutive segments per workgroup (the dispatcher then
    // keeps the resident workgroups on one compact window of the stream)
    long long sstep, seg;
    if (per == 0) {
        sstep = gridDim.x;
        seg = seg_lo + blockIdx.x;
    } else if (per < 0) {
        // XCD-local interleave: XCD b % 8 owns one contiguous eighth of the segments and its
        // resident workgroups b / 8 walk it interleaved (a compact window per XCD; the halo
        // row of a segment was read by a neighbour on the same XCD, i.e. through its L2)
        const long long x8 = blockIdx.x % 8, nj = gridDim.x / 8;
        const long long s8 = (seg_hi - seg_lo + 7) / 8;
        const long long a = seg_lo + x8 * s8;
        if (a + s8 < seg_hi) seg_hi = a + s8;
        seg = a + blockIdx.x / 8;
        sstep = nj;
    } else {
        sstep = 1;
        // xm > 0: the dispatcher places workgroup b on XCD b % 8; chunk (b % 8) xm + b / 8
        // keeps each XCD on one contiguous part of the stream
        const long long b = xm > 0 ? (long long)(blockIdx.x % 8) * xm + blockIdx.x / 8 : (long long)blockIdx.x;
        seg = seg_lo + b * per;
        const long long e = seg + per;
        if (e < seg_hi) seg_hi = e;
    }
    f2 nv[16];         // 8-byte path: lane's column over rows
    float4 nq[D][8];   // W16 path: row 2i + up, columns colX, colX + 1 (D segments in flight)
    // rows 2i, 2i + 1 for the i with sel(i)
    auto load = [&](long long sg, auto bt, auto sel) {
        constexpr int b = decltype(bt)::value;
        if constexpr (ABL & 1) {
            if constexpr (W16) {
#pragma unroll
                for (int i = 0; i < 8; ++i)
                    if (sel(i)) nq[b][i] = make_float4((float)(t + i), (float)(sg & 1023), 0.f, 1.f);
            } else {
#pragma unroll
                for (int r = 0; r < 16; ++r) nv[r] = f2{(float)(t + r), (float)(sg & 1023)};
            }
        } else if constexpr (W16) {
            const float4* xb = reinterpret_cast<const float4*>(x + sg * V - 256 * H2 + 256 * up + colX);
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                if (!sel(i)) continue;
                if constexpr (NT & 1) {
                    const f4v q = __builtin_nontemporal_load(reinterpret_cast<const f4v*>(xb + 256 * i));
                    nq[b][i] = make_float4(q.x, q.y, q.z, q.w);
                } else {
                    nq[b][i] = xb[256 * i];
                }
            }
        } else {
            const f2* xb = x + sg * V - 256 * H2 + t;
#pragma unroll
            for (int r = 0; r < 16; ++r) nv[r] = xb[256 * r];
        }
    };
    // D = 1: stores are deferred by one segment: segment s's outputs go out after P1
    // of segment s + 1, ahead of the loads for segment s + 2, so the wait for those
    // loads at the loop head never covers freshly issued stores.  D = 2: the loads
    // consumed at a loop head were issued two segments earlier, ahead of every
    // store still in flight, so stores go out at the end of P5 (ov is not kept live
    // across the next segment).
    constexpr bool DEFER = D == 1;
    f2 ov[16];
    long long oseg = -1;
    auto store_out = [&](auto sel) {
        if constexpr (W16 && !(ABL & 1)) {
            float4* yb = reinterpret_cast<float4*>(y + oseg * V - 256 * H2 + 256 * up + colX);
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                if (!sel(i)) continue;
                if (2 * i + 1 < H2) continue;  // both rows are halo
                float4 q = make_float4(ov[2 * i].x, ov[2 * i].y, ov[2 * i + 1].x, ov[2 * i + 1].y);
                swap16(q.x, q.z);
                swap16(q.y, q.w);
                if (2 * i >= H2 || up) {  // row 2i is halo when 2i < H2: only the upper lanes (row 2i + 1) store
                    if constexpr (NT & 2) __builtin_nontemporal_store(f4v{q.x, q.y, q.z, q.w}, reinterpret_cast<f4v*>(yb + 256 * i));
                    else yb[256 * i] = q;
                }
            }
        } else {
            f2* yb = y + oseg * V - 256 * H2 + t;
#pragma unroll
            for (int k = H2; k < 16; ++k) {
                if constexpr (ABL & 1) {  // keep the outputs live, no stores
                    if (sel(k >> 1)) { const f2 tv = ov[k]; asm volatile("" : : "v"(tv)); }
                } else {
                    yb[256 * k] = ov[k];
                }
            }
        }
    };
    auto bar = [] {
        if constexpr (ABL & 2) __builtin_amdgcn_wave_barrier();
        else __syncthreads();
    };
    f2 tmp[16];
    auto sto = [&](f2* r, int i, int k, f2 val) {
        if constexpr (ABL & 4) {
            tmp[k] = val;
            asm volatile("" : "+v"(tmp[k]));
        } else {
            r[i] = val;
        }
    };
    auto ldo = [&](const f2* r, int i, int k) -> f2 {
        if constexpr (ABL & 4) return tmp[k];
        else return r[i];
    };
    // one segment; its input sits in buffer b (nq[b] / nv), the load it issues
    // (segment seg + D * sstep, clamped) refills the same buffer
    auto segment = [&](auto bt) {
        constexpr int b = decltype(bt)::value;
        f2 v[16];
        if constexpr (W16) {
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                float4 q = nq[b][i];
                swap16(q.x, q.z);
                swap16(q.y, q.w);
                v[2 * i] = f2{q.x, q.y};
                v[2 * i + 1] = f2{q.z, q.w};
            }
        } else {
#pragma unroll
            for (int r = 0; r < 16; ++r) v[r] = nv[r];
        }
        const long long ahead = seg + D * sstep;
        const long long nxt = ahead < seg_hi ? ahead : seg;
        // HBM traffic issued at hook point P (SCH tables)
        auto hook = [&](auto pt) {
            constexpr int P = decltype(pt)::value;
            if constexpr (DEFER) {
                if (oseg >= 0) store_out([](int i) { return kStoreAt[SCH][i] == P; });
            }
            load(nxt, bt, [](int i) { return kLoadAt[SCH][i] == P; });
        };
        if constexpr ((ABL & ~48) == 8) {  // the kernel's HBM traffic alone: same grid, loads and deferred stores
#pragma unroll
            for (int k = 0; k < 16; ++k) asm volatile("" : "+v"(v[k]));
#pragma unroll
            for (int k = 0; k < 16; ++k) asm volatile("" : : "v"(w1[k]), "v"(w2[k]), "v"(Hr[k]));
            if (DEFER && oseg >= 0) store_out([](int) { return true; });
            load(nxt, bt, [](int) { return true; });
#pragma unroll
            for (int k = 0; k < 16; ++k) ov[k] = v[k];
            oseg = seg;
            if constexpr (!DEFER) store_out([](int) { return true; });
            return;
        }
        hook(Buf<0>{});
        // P1: DFT over n2 -> k0, twiddle, A[k0][t]
        pdft16<false>(v);
#pragma unroll
        for (int k = 0; k < 16; ++k) sto(rA, k * kRowA + acol(col), k, pmul<ASM>(v[kout(k)], w1[k]));
        hook(Buf<1>{});
        bar();
        // P2: lane (k0=hi4, n0=lo4) reads n1
#pragma unroll
        for (int k = 0; k < 16; ++k) v[k] = ldo(rA, hi4 * kRowA + 16 * k + (lo4 ^ (k & 1)), k);
        pdft16<false>(v);
        hook(Buf<2>{});
#pragma unroll
        for (int k = 0; k < 16; ++k) sto(rB, bidx(16 * hi4 + k, lo4), k, pmul<ASM>(v[kout(k)], w2[k]));
        hook(Buf<3>{});
        bar();
        // P3: lane (k0=hi4, k1=lo4) reads its row over n0
        {
            const float4* row = reinterpret_cast<const float4*>(rB + brow(t) * 16);
#pragma unroll
            for (int p = 0; p < 8; ++p) {
                if constexpr (ABL & 4) {
                    v[2 * p] = tmp[2 * p];
                    v[2 * p + 1] = tmp[2 * p + 1];
                } else {
                    const float4 q = row[(p ^ t) & 7];
                    v[2 * p] = f2{q.x, q.y};
                    v[2 * p + 1] = f2{q.z, q.w};
                }
            }
        }
        pdft16<false>(v);
        f2 u[16];
#pragma unroll
        for (int k = 0; k < 16; ++k) u[k] = pmul<ASM>(v[kout(k)], Hr[k]);
        hook(Buf<4>{});
        pdft16<true>(u);
        {
            float4* row = reinterpret_cast<float4*>(rA + brow(t) * 16);
#pragma unroll
            for (int p = 0; p < 8; ++p) {
                const f2 a = pmulc<ASM>(u[kout(2 * p)], w2[2 * p]);
                const f2 c = pmulc<ASM>(u[kout(2 * p + 1)], w2[2 * p + 1]);
                if constexpr (ABL & 4) {
                    tmp[2 * p] = a;
                    tmp[2 * p + 1] = c;
                } else {
                    row[(p ^ t) & 7] = make_float4(a.x, a.y, c.x, c.y);
                }
            }
        }
        hook(Buf<5>{});
        bar();
        // P4: lane (k0=hi4, n0=lo4) reads k1
#pragma unroll
        for (int k = 0; k < 16; ++k) v[k] = ldo(rA, bidx(16 * hi4 + k, lo4), k);
        pdft16<true>(v);
        hook(Buf<6>{});
#pragma unroll
        for (int k = 0; k < 16; ++k) sto(rB, hi4 * kRowA + 16 * k + (lo4 ^ (k & 1)), k, v[kout(k)]);
        hook(Buf<7>{});
        bar();
        // P5: lane t=(n1,n0) reads k0
#pragma unroll
        for (int k = 0; k < 16; ++k) v[k] = pmulc<ASM>(ldo(rB, k * kRowA + acol(col), k), w1[k]);
        hook(Buf<8>{});
        pdft16<true>(v);
#pragma unroll
        for (int k = 0; k < 16; ++k) ov[k] = v[kout(k)];
        oseg = seg;
        if constexpr (!DEFER) store_out([](int) { return true; });
        // tables opaque once per segment: swizzled copies of them are not hoisted out of the loop
#pragma unroll
        for (int k = 0; k < 16; ++k) asm volatile("" : "+v"(w1[k]), "+v"(w2[k]), "+v"(Hr[k]));
        // the next segment's P1 writes region A: every lane has finished reading
        // region A (P4) before the barrier that precedes P5.
    };
    if constexpr (D == 1) {
        if (seg < seg_hi)
            load(seg, Buf<0>{}, [](int) { return true; });
        load_tables();
        for (; seg < seg_hi; seg += sstep) segment(Buf<0>{});
    } else {
        // two buffers: the loop body is unrolled so each buffer index is static
        if (seg < seg_hi) {
            load(seg, Buf<0>{}, [](int) { return true; });
            load(seg + sstep < seg_hi ? seg + sstep : seg, Buf<1>{}, [](int) { return true; });
        }
        load_tables();
        while (seg < seg_hi) {
            segment(Buf<0>{});
            seg += sstep;
            if (seg >= seg_hi) break;
            segment(Buf<1>{});
            seg += sstep;
        }
    }
    if (DEFER && oseg >= 0) store_out([](int) { return true; });
}

hipError_t launch_fir_ols_pk(const OlsPlan& p, const void* x, void* y, size_t n, size_t channels, int num_cus,
                             hipStream_t s, long long lo, long long hi, int ablate) {
    // k-pair-major tables (OlsPlan::d_pkt): spectrum, tw1, tw2 parts
    const float4* const pkt = reinterpret_cast<const float4*>(p.d_pkt);
#define PK_TABLES (const f2*)pkt, (const f2*)(pkt + 2048), (const f2*)(pkt + 4096)
    if (hi <= lo) return hipSuccess;
    const long long per = p.segs_per_block;
    // 16-byte accesses need 16-byte aligned rows in every channel
    const bool w16 = p.wide && ((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(y)) & 15) == 0 &&
                     (channels == 1 || n % 2 == 0);
    long long blocks = (long long)num_cus * 2;
    long long xm = 0;
    if (per > 0) {
        blocks = (hi - lo + per - 1) / per;
        if (p.xcd) {
            xm = (blocks + 7) / 8;
            blocks = 8 * xm;
        }
    }
    else if (per < 0) blocks = blocks / 8 * 8;  // grid must be a multiple of the 8 XCDs
    else if (blocks > hi - lo) blocks = hi - lo;
    dim3 grid((unsigned)blocks, (unsigned)channels);
#define SDSP_OLS_PK_W(HV, A, M, W)                                                                               \
    hipLaunchKernelGGL((fir_ols4096_pk_kernel<HV, A, M, W>), grid, dim3(256), 0, s, (const f2*)x, PK_TABLES,      \
                       (f2*)y, (long long)n, lo, hi, per, xm)
#define SDSP_OLS_PK_L(HV, A)                                                                                     \
    do {                                                                                                         \
        if (p.packed % 2 == 0) {                                                                                 \
            if (w16) SDSP_OLS_PK_W(HV, A, false, true); else SDSP_OLS_PK_W(HV, A, false, false);                 \
        } else {                                                                                                 \
            if (w16) SDSP_OLS_PK_W(HV, A, true, true); else SDSP_OLS_PK_W(HV, A, true, false);                   \
        }                                                                                                        \
    } while (0)
#define SDSP_OLS_PK(HV) SDSP_OLS_PK_L(HV, 0)
    if (w16 && p.depth2 && p.halo_rows == 1) {  // loads two segments ahead and / or spread over the phases
#define SDSP_OLS_PK_D2(M, A, DV, SPV, NTV)                                                                       \
    hipLaunchKernelGGL((fir_ols4096_pk_kernel<1, A, M, true, NTV, DV, SPV>), grid, dim3(256), 0, s, (const f2*)x, \
                       PK_TABLES, (f2*)y, (long long)n, lo, hi, per, xm)
#define SDSP_OLS_PK_D2A(A, DV, SPV)                                                                              \
    do {                                                                                                         \
        if (DV == 1 && SPV == 1 && (p.nt & 3) == 2 && !A) SDSP_OLS_PK_D2(true, 0, 1, 1, 2);                      \
        else if (DV == 1 && SPV == 1 && (p.nt & 3) == 3 && !A) SDSP_OLS_PK_D2(true, 0, 1, 1, 3);                 \
        else if (DV == 1 && SPV == 1 && (p.nt & 3) == 1 && !A) SDSP_OLS_PK_D2(true, 0, 1, 1, 1);                 \
        else if (p.packed % 2 != 0) SDSP_OLS_PK_D2(true, A, DV, SPV, 0);                                         \
        else SDSP_OLS_PK_D2(false, A, DV, SPV, 0);                                                               \
    } while (0)
#define SDSP_OLS_PK_D2V(A)                                                                                       \
    do {                                                                                                         \
        switch (p.depth2) {                                                                                      \
            case 1: SDSP_OLS_PK_D2A(A, 2, 0); break;                                                             \
            case 2: SDSP_OLS_PK_D2A(A, 1, 1); break;                                                             \
            case 3: SDSP_OLS_PK_D2A(A, 1, 2); break;                                                             \
            case 4: SDSP_OLS_PK_D2A(A, 1, 3); break;                                                             \
            case 5: SDSP_OLS_PK_D2A(A, 1, 4); break;                                                             \
            case 6: SDSP_OLS_PK_D2A(A, 1, 5); break;                                                             \
            case 7: SDSP_OLS_PK_D2A(A, 1, 6); break;                                                             \
            case 8: SDSP_OLS_PK_D2A(A, 1, 7); break;                                                             \
            case 9: SDSP_OLS_PK_D2A(A, 1, 8); break;                                                             \
            default: SDSP_OLS_PK_D2A(A, 1, 9); break;                                                            \
        }                                                                                                        \
    } while (0)
        switch (ablate) {
            case 0: SDSP_OLS_PK_D2V(0); break;
            case 1: SDSP_OLS_PK_D2V(1); break;
            case 8: SDSP_OLS_PK_D2V(8); break;
            case 24: SDSP_OLS_PK_D2V(24); break;
            case 40: SDSP_OLS_PK_D2V(40); break;
            case 16: SDSP_OLS_PK_D2V(16); break;
            default: return hipErrorInvalidValue;
        }
#undef SDSP_OLS_PK_D2V
#undef SDSP_OLS_PK_D2A
#undef SDSP_OLS_PK_D2
        return hipGetLastError();
    }
    if (w16 && p.nt && p.halo_rows == 1 && !ablate) {  // nontemporal hints (bit 0 loads, bit 1 stores), h2 = 1
#define SDSP_OLS_PK_NT(M, NTV)                                                                                   \
    hipLaunchKernelGGL((fir_ols4096_pk_kernel<1, 0, M, true, NTV>), grid, dim3(256), 0, s, (const f2*)x,         \
                       PK_TABLES, (f2*)y, (long long)n, lo, hi, per, xm)
        const int ntv = p.nt & 3;
        if (p.packed % 2 == 0) {
            if (ntv == 1) SDSP_OLS_PK_NT(false, 1); else if (ntv == 2) SDSP_OLS_PK_NT(false, 2); else SDSP_OLS_PK_NT(false, 3);
        } else {
            if (ntv == 1) SDSP_OLS_PK_NT(true, 1); else if (ntv == 2) SDSP_OLS_PK_NT(true, 2); else SDSP_OLS_PK_NT(true, 3);
        }
#undef SDSP_OLS_PK_NT
        return hipGetLastError();
    }
    if (ablate) {  // profiling ablations, h2 = 1 only
        if (p.halo_rows != 1) return hipErrorInvalidValue;
        if (ablate == 1) SDSP_OLS_PK_L(1, 1);
        else if (ablate == 3) SDSP_OLS_PK_L(1, 3);
        else if (ablate == 7) SDSP_OLS_PK_L(1, 7);
        else if (ablate == 8) SDSP_OLS_PK_L(1, 8);
        else if (ablate == 24) SDSP_OLS_PK_L(1, 24);
        else return hipErrorInvalidValue;
        return hipGetLastError();
    }
    switch (p.halo_rows) {
        case 1: SDSP_OLS_PK(1); break;
        case 2: SDSP_OLS_PK(2); break;
        case 3: SDSP_OLS_PK(3); break;
        case 4: SDSP_OLS_PK(4); break;
        default: return hipErrorInvalidValue;
    }
#undef SDSP_OLS_PK
#undef SDSP_OLS_PK_L
#undef SDSP_OLS_PK_W
#undef PK_TABLES
    return hipGetLastError();
}

}  // namespace SDSP_PK_NS
}  // namespace sdsp
