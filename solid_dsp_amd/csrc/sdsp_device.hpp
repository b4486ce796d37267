// Device-side arithmetic for the sdsp kernels (gfx950).
//
// Every kernel TU is compiled with -ffp-contract=off, so `a * b + c` is a
// rounded multiply followed by a rounded add — the arithmetic the reference's
// Rust code performs (num-complex 0.4 Mul/Add, src/dot_product/mod.rs:159-170).
// Fused multiply-add is only ever requested explicitly (fmac below).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace sdsp {

template <typename T> struct cpx {
    T re, im;
};
using c32 = cpx<float>;
using c64 = cpx<double>;

template <typename T> struct is_cpx { static constexpr bool value = false; };
template <typename T> struct is_cpx<cpx<T>> { static constexpr bool value = true; };
template <typename T> struct real_of { using type = T; };
template <typename T> struct real_of<cpx<T>> { using type = T; };

template <typename T> __host__ __device__ inline T zero_v() { return T(0); }
template <> __host__ __device__ inline c32 zero_v<c32>() { return {0.0f, 0.0f}; }
template <> __host__ __device__ inline c64 zero_v<c64>() { return {0.0, 0.0}; }

// ---- num-complex semantics (no contraction: TU built with -ffp-contract=off)
__device__ inline float mul_(float a, float b) { return a * b; }
__device__ inline double mul_(double a, double b) { return a * b; }
template <typename T> __device__ inline cpx<T> mul_(T a, cpx<T> b) { return {a * b.re, a * b.im}; }
template <typename T> __device__ inline cpx<T> mul_(cpx<T> a, T b) { return {a.re * b, a.im * b}; }
template <typename T> __device__ inline cpx<T> mul_(cpx<T> a, cpx<T> b) {
    T re = a.re * b.re - a.im * b.im;
    T im = a.re * b.im + a.im * b.re;
    return {re, im};
}
__device__ inline float add_(float a, float b) { return a + b; }
__device__ inline double add_(double a, double b) { return a + b; }
template <typename T> __device__ inline cpx<T> add_(cpx<T> a, cpx<T> b) { return {a.re + b.re, a.im + b.im}; }
__device__ inline float sub_(float a, float b) { return a - b; }
__device__ inline double sub_(double a, double b) { return a - b; }
template <typename T> __device__ inline cpx<T> sub_(cpx<T> a, cpx<T> b) { return {a.re - b.re, a.im - b.im}; }

// ---- fused variants: acc + c * s with one rounding per fma
__device__ inline float fmac_(float acc, float c, float s) { return __builtin_fmaf(c, s, acc); }
__device__ inline double fmac_(double acc, double c, double s) { return __builtin_fma(c, s, acc); }
template <typename T> __device__ inline cpx<T> fmac_(cpx<T> acc, T c, cpx<T> s) {
    return {fmac_(acc.re, c, s.re), fmac_(acc.im, c, s.im)};
}
template <typename T> __device__ inline cpx<T> fmac_(cpx<T> acc, cpx<T> c, cpx<T> s) {
    T re = fmac_(fmac_(acc.re, c.re, s.re), -c.im, s.im);
    T im = fmac_(fmac_(acc.im, c.re, s.im), c.im, s.re);
    return {re, im};
}

// acc += c * s   in the reference order (EXACT) or fused
template <bool EXACT, typename C, typename I, typename O>
__device__ inline O mac(O acc, C c, I s) {
    if constexpr (EXACT) return add_(acc, mul_(c, s));
    else return fmac_(acc, c, s);
}

// Out type of Coef * In
template <typename C, typename I> struct out_of { using type = I; };

// Workgroups are dealt round-robin over the 8 XCDs (blockIdx % 8 share one);
// remap so each XCD streams its own contiguous eighth of the workgroups' data --
// the one-shot order that ran at copy speed in tools/pattern_probe.hip (ORD 2).
// A bijection on [0, nb): blocks past the last whole eighth keep their index.
__device__ __forceinline__ unsigned xcd_order(unsigned b, unsigned nb) {
    const unsigned q = nb / 8;
    return b < 8 * q ? (b % 8) * q + b / 8 : b;
}

// A streaming store that bypasses the caches' normal retention (nontemporal):
// T is copied out as 16-, 8- or 4-byte stores (by its size and alignment).  Outputs that no kernel
// of the same call reads again (cfg2 OLS: 3.14 -> 3.08 ms, in-process A/B).
template <typename T> __device__ __forceinline__ void store_nt(T* p, const T& v) {
    static_assert(sizeof(T) % 4 == 0, "store_nt: 4-byte multiples");
    if constexpr (sizeof(T) % 8 != 0 || alignof(T) < 8) {
        unsigned w[sizeof(T) / 4];
        __builtin_memcpy(w, &v, sizeof(T));
#pragma unroll
        for (unsigned i = 0; i < sizeof(T) / 4; ++i) __builtin_nontemporal_store(w[i], reinterpret_cast<unsigned*>(p) + i);
    } else if constexpr (sizeof(T) % 16 == 0 && alignof(T) >= 16) {
        typedef unsigned u4 __attribute__((ext_vector_type(4)));
        u4 w[sizeof(T) / 16];
        __builtin_memcpy(w, &v, sizeof(T));
#pragma unroll
        for (unsigned i = 0; i < sizeof(T) / 16; ++i) __builtin_nontemporal_store(w[i], reinterpret_cast<u4*>(p) + i);
    } else {
        typedef unsigned u2 __attribute__((ext_vector_type(2)));
        u2 w[sizeof(T) / 8];
        __builtin_memcpy(w, &v, sizeof(T));
#pragma unroll
        for (unsigned i = 0; i < sizeof(T) / 8; ++i) __builtin_nontemporal_store(w[i], reinterpret_cast<u2*>(p) + i);
    }
}

}  // namespace sdsp
