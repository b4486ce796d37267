// Packed-FP32 complex arithmetic and the register DFT16 shared by the
// overlap-save kernels (kern_fir_ols_pk.hip, kern_fir_ols_os.hip).
//
// A complex value is a float pair; every complex add/sub/multiply is a
// v_pk_add/v_pk_mul/v_pk_fma_f32.  Per component each helper performs the
// operation sequence of its scalar counterpart in kern_fir_ols.hip (cmul,
// cmulc, dft4, tw16), so the packed and scalar transforms agree bit for bit.
// A swapped, half-negated operand ({b.y, -b.x}) is written as a product or fma
// with a +-1 pair (exact; the swap becomes op_sel): the backend does not fold a
// one-lane negation into neg_lo / neg_hi and would emit v_xor + v_mov pairs.
#pragma once
#include <hip/hip_runtime.h>

namespace sdsp {
namespace pk {

typedef float f2 __attribute__((ext_vector_type(2)));
typedef float f4v __attribute__((ext_vector_type(4)));

constexpr f2 kPM = {1.0f, -1.0f};
constexpr f2 kMP = {-1.0f, 1.0f};

// a * b = {fma(a.x, b.x, -(a.y b.y)), fma(a.x, b.y, a.y b.x)}: two VOP3P
// instructions with op_sel / neg modifiers
__device__ __forceinline__ f2 pmul(f2 a, f2 b) {
    f2 t, r;
    asm("v_pk_mul_f32 %0, %1, %2 op_sel:[1,1] op_sel_hi:[1,0] neg_lo:[0,1]" : "=v"(t) : "v"(a), "v"(b));
    asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel_hi:[0,1,1]" : "=v"(r) : "v"(a), "v"(b), "v"(t));
    return r;
}
// a * conj(b) = {fma(a.x, b.x, a.y b.y), fma(a.y, b.x, -(a.x b.y))}
__device__ __forceinline__ f2 pmulc(f2 a, f2 b) {
    f2 t, r;
    asm("v_pk_mul_f32 %0, %1, %2 op_sel:[1,1] op_sel_hi:[0,1] neg_hi:[0,1]" : "=v"(t) : "v"(a), "v"(b));
    asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel_hi:[1,0,1]" : "=v"(r) : "v"(a), "v"(b), "v"(t));
    return r;
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
template <bool INV> __device__ __forceinline__ f2 ptw2(f2 v) { return (INV ? padd_pj(v, v) : padd_mj(v, v)) * kR2; }
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

// ---- the fused DFT16 of the one-shot overlap-save kernel (kern_fir_ols_os.hip) ----
// R = -j (forward) / +j (inverse), the DFT4 rotation.  x + k R y as one v_pk_fma_f32.
template <bool INV> __device__ __forceinline__ f2 rfma(f2 y, float k, f2 x) {
    return __builtin_elementwise_fma(y.yx, INV ? f2{-k, k} : f2{k, -k}, x);
}
constexpr float kT1 = 0.41421356237309505f;  // tan(pi/8)

// the same DFT16 as pdft16 (natural order in, stage order out) in 72 instead of 81 packed
// instructions: the second-stage twiddles are written W1 = c1 (1 + t R), W3 = c1 R (1 - t R),
// W2 = r2 (1 + R), W6 = r2 R (1 + R), W9 = -W1 (c1 = cos pi/8, t = tan pi/8, r2 = sqrt 1/2),
// so each twiddled input costs one fma and its real scale folds into the DFT4's sums.  Equal to
// pdft16 within rounding (not bit for bit).
template <bool INV> __device__ __forceinline__ void pdft16f(f2 (&v)[16]) {
#pragma unroll
    for (int nb = 0; nb < 4; ++nb) pdft4<INV>(v[nb], v[4 + nb], v[8 + nb], v[12 + nb]);
    pdft4<INV>(v[0], v[1], v[2], v[3]);
    const f2 c1 = {kC1, kC1}, nc1 = {-kC1, -kC1}, r2 = {kR2, kR2}, nr2 = {-kR2, -kR2};
    {  // ka = 1: W1, W2, W3
        const f2 g1 = rfma<INV>(v[5], kT1, v[5]), g3 = rfma<INV>(v[7], -kT1, v[7]);
        const f2 cc = rfma<INV>(g3, 1.0f, g1), ee = rfma<INV>(g3, -1.0f, g1);
        const f2 u2 = rfma<INV>(v[6], 1.0f, v[6]);
        const f2 a = __builtin_elementwise_fma(u2, r2, v[4]), b = __builtin_elementwise_fma(u2, nr2, v[4]);
        v[4] = __builtin_elementwise_fma(cc, c1, a);
        v[6] = __builtin_elementwise_fma(cc, nc1, a);
        v[5] = rfma<INV>(ee, kC1, b);
        v[7] = rfma<INV>(ee, -kC1, b);
    }
    {  // ka = 2: W2, W4 = R, W6
        const f2 a = rfma<INV>(v[10], 1.0f, v[8]), b = rfma<INV>(v[10], -1.0f, v[8]);
        const f2 p = rfma<INV>(v[11], 1.0f, v[9]), q = rfma<INV>(v[11], -1.0f, v[9]);
        const f2 u = rfma<INV>(p, 1.0f, p), s = rfma<INV>(q, 1.0f, q);
        v[8] = __builtin_elementwise_fma(u, r2, a);
        v[10] = __builtin_elementwise_fma(u, nr2, a);
        v[9] = rfma<INV>(s, kR2, b);
        v[11] = rfma<INV>(s, -kR2, b);
    }
    {  // ka = 3: W3, W6, W9
        const f2 h1 = rfma<INV>(v[13], -kT1, v[13]), h3 = rfma<INV>(v[15], kT1, v[15]);
        const f2 cc = rfma<INV>(h1, 1.0f, -h3), ee = rfma<INV>(h1, 1.0f, h3);
        const f2 u2 = rfma<INV>(v[14], 1.0f, v[14]);
        const f2 a = rfma<INV>(u2, kR2, v[12]), b = rfma<INV>(u2, -kR2, v[12]);
        v[12] = __builtin_elementwise_fma(cc, c1, a);
        v[14] = __builtin_elementwise_fma(cc, nc1, a);
        v[13] = rfma<INV>(ee, kC1, b);
        v[15] = rfma<INV>(ee, -kC1, b);
    }
}

}  // namespace pk
}  // namespace sdsp
