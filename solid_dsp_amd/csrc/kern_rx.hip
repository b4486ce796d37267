// Receive-chain kernels next to the filter path:
//   * AutoCorrelator  src/filter/auto_correlator/mod.rs:26-214
//   * NCO mixing      src/nco/mod.rs:94-172
//
// AutoCorrelator.  After pushing x[n] the reference returns
//     execute() = sum_{j < W} window[j] * delayed[j]     (:156-163)
// with window[j] = x[n - j] and delayed[j] = conj(x[n - j - d]) for j + d < W and
// 0 otherwise: the delayed Window keeps W + d zeroed slots but shifts only the
// first W - 1 (src/window/mod.rs:63-71), so its tail slots [W, W + d) stay zero.
// With K = max(W - d, 0) the sum is
//     y[n] = (((0 + p[n]) + p[n-1]) + ...) + p[n-K+1],   p[m] = x[m] * conj(x[m-d]),
// the zero-product terms j >= K leave the sum unchanged (it starts at +0 and is
// never -0).  Each one-wave workgroup owns 512 consecutive outputs (8 per lane); p over the window the
// outputs need is built once in LDS (one num-complex product per input, the
// reference's rounding) and every lane adds its K terms newest first, in chunks
// of kChunk so W is unbounded.  Bit-identical to the restatement at the handle's
// precision; HBM traffic is one read of x and one write of y per sample.
//
// energy (:106-111, :212-214) is the sum of |x|^2 over the last W inputs; the
// reference keeps it as a running f64 sum (add the new e2, subtract the one
// leaving).  One workgroup per channel re-sums the last W e2 values in f64.
//
// NCO.  theta_i = theta_0 + i * dtheta (u32, wrapping, :94-96); the phasor is
// (table[(idx + 256) & 1023], table[idx]), idx = ((theta + 2^21) >> 22) & 1023
// (:99-121) from the handle's 1024-entry f64 sine table, staged in LDS;
// mix_up = phasor * x, mix_down = conj(phasor) * x (num-complex Mul).
//
// AGC (src/auto_gain_control/mod.rs:214-246, :631-677).  A serial non-linear
// recurrence per channel (gain depends on every earlier sample through exp/ln),
// so one lane runs one channel; a 64-lane workgroup serves 64 channels and
// stages kAgcS samples of each through LDS so that HBM sees 16 * kAgcS-byte
// runs per channel instead of one sample per lane per row.
#include "sdsp.h"
#include <map>
#include <mutex>
#include <tuple>
#include "sdsp_device.hpp"
#include "sdsp_kernels.hpp"

namespace sdsp {

namespace {

constexpr int kTile = 64;            // lanes per workgroup (one wave)
constexpr int kR = 8;                // consecutive outputs per lane
constexpr int kOut = kTile * kR;     // outputs per workgroup
constexpr int kChunk = 256;          // j-terms staged per pass
// one spare slot per 8: lane t reads slot 8t + o, i.e. LDS element 9t + ..., so the
// 32 (c32) or 16 (c64) lanes of one LDS cycle hit distinct banks
__host__ __device__ constexpr int pad8(int s) { return s + (s >> 3); }

template <typename T> __device__ inline cpx<T> conj_(cpx<T> a) { return {a.re, -a.im}; }

// a * conj(c) with num-complex rounding (mul_(a, conj_(c)): re = a.re c.re - a.im (-c.im), im =
// a.re (-c.im) + a.im c.re, every product rounded, no fma) in three packed instructions for c32:
// m0 = {a.re c.re, a.re c.im}, m1 = {a.im c.im, a.im c.re}, {m0.x + m1.x, -m0.y + m1.y} -- the same
// roundings (negation is exact, x - (-y) == x + y, the sums commute)
template <typename T> __device__ __forceinline__ cpx<T> mul_conj_(cpx<T> a, cpx<T> c) { return mul_(a, conj_(c)); }
template <> __device__ __forceinline__ cpx<float> mul_conj_(cpx<float> a, cpx<float> c) {
    typedef float f2v __attribute__((ext_vector_type(2)));
    const f2v av = {a.re, a.im}, cv = {c.re, c.im};
    f2v m0, m1, r;
    asm("v_pk_mul_f32 %0, %1, %2 op_sel:[0,0] op_sel_hi:[0,1]" : "=v"(m0) : "v"(av), "v"(cv));
    asm("v_pk_mul_f32 %0, %1, %2 op_sel:[1,1] op_sel_hi:[1,0]" : "=v"(m1) : "v"(av), "v"(cv));
    asm("v_pk_add_f32 %0, %1, %2 neg_hi:[1,0]" : "=v"(r) : "v"(m0), "v"(m1));
    return {r.x, r.y};
}


template <typename T>
__device__ inline cpx<T> ext_at(const cpx<T>* __restrict__ x, const cpx<T>* __restrict__ hist, long long j, int H) {
    if (j >= 0) return x[j];
    if (j >= -(long long)H) return hist[H + j];
    return zero_v<cpx<T>>();
}

// Lane t owns outputs o_r = n0 + kR t + r (r < kR).  Within a chunk of terms
// [j0, j0 + cj), output o_r adds p[o_r - j0 - jj] for jj = 0, 1, ... newest first;
// p[n0 + kR t + q - j0] (q = r - jj) is shared by all r, so the lane walks q
// downward, reads each p once from LDS and adds it to every accumulator whose
// jj = r - q lies in [0, cj) — the same additions in the same order as the
// one-output-per-lane form, with kR-fold fewer LDS reads.
// STAGE (delays d <= kDmax): the chunk's input x[base - d, base + cnt) is staged in LDS
// once and each product reads both of its factors there (one load per input sample
// instead of two, 16 fewer VGPRs per load slot); otherwise both factors are loaded.
constexpr int kDmax = 256;
template <typename T, bool STAGE>
__global__ void __launch_bounds__(kTile) acorr_kernel(const cpx<T>* __restrict__ x, const cpx<T>* __restrict__ hist,
                                                      cpx<T>* __restrict__ y, long long n, int H, int d, int K,
                                                      long long tile0) {
    // LDS sized by the launch (acorr_lds_bytes): p for the widest chunk, then (STAGE) the staged input
    extern __shared__ __attribute__((aligned(16))) char acorr_lds[];
    cpx<T>* p = reinterpret_cast<cpx<T>*>(acorr_lds);
    cpx<T>* xs = p + pad8(kOut + (K < kChunk ? K : kChunk) - 1) + 1;
    const int ch = blockIdx.y;
    x += (long long)ch * n;
    y += (long long)ch * n;
    hist += (long long)ch * H;
    const int t = threadIdx.x;
    const long long n0 = (tile0 + (long long)xcd_order(blockIdx.x, gridDim.x)) * kOut;
    cpx<T> acc[kR];
#pragma unroll
    for (int r = 0; r < kR; ++r) acc[r] = zero_v<cpx<T>>();
    for (int j0 = 0; j0 < K; j0 += kChunk) {
        const int cj = K - j0 < kChunk ? K - j0 : kChunk;
        // p[m] for m in [n0 - j0 - cj + 1, n0 + kOut - 1 - j0]: slot s <-> m = base + s
        const long long base = n0 - j0 - cj + 1;
        const int cnt = kOut + cj - 1;
        __syncthreads();  // previous chunk's readers are done
        // every load of the chunk is issued before the first product: the loads of
        // one lane are independent, so the wave keeps kLd x 2 requests in flight
        constexpr int kLd = (kOut + kChunk - 1 + kTile - 1) / kTile;
        if constexpr (STAGE) {
            constexpr int kLs = (kOut + kChunk - 1 + kDmax + kTile - 1) / kTile;
            const long long b0 = base - d;  // xs[i] = x[b0 + i], i < cnt + d
            const int ns = cnt + d;
            cpx<T> v[kLs];
            if (b0 >= 0 && base + cnt <= n) {  // interior tile: plain loads
#pragma unroll
                for (int k = 0; k < kLs; ++k) {
                    const int i = t + k * kTile;
                    if (i < ns) v[k] = x[b0 + i];
                }
            } else {
#pragma unroll
                for (int k = 0; k < kLs; ++k) {
                    const int i = t + k * kTile;
                    if (i < ns) v[k] = ext_at(x, hist, b0 + i, H);
                }
            }
#pragma unroll
            for (int k = 0; k < kLs; ++k) {
                const int i = t + k * kTile;
                if (i < ns) xs[i] = v[k];
            }
            __syncthreads();
#pragma unroll
            for (int k = 0; k < kLd; ++k) {
                const int s = t + k * kTile;
                if (s < cnt) p[pad8(s)] = mul_(xs[s + d], conj_(xs[s]));
            }
        } else {
        cpx<T> va[kLd], vb[kLd];
        if (base - d >= 0 && base + cnt <= n) {  // interior tile: plain loads
#pragma unroll
            for (int k = 0; k < kLd; ++k) {
                const int s = t + k * kTile;
                if (s < cnt) {
                    va[k] = x[base + s];
                    vb[k] = x[base + s - d];
                }
            }
        } else {
#pragma unroll
            for (int k = 0; k < kLd; ++k) {
                const int s = t + k * kTile;
                if (s < cnt) {
                    va[k] = ext_at(x, hist, base + s, H);
                    vb[k] = ext_at(x, hist, base + s - d, H);
                }
            }
        }
#pragma unroll
        for (int k = 0; k < kLd; ++k) {
            const int s = t + k * kTile;
            if (s < cnt) p[pad8(s)] = mul_(va[k], conj_(vb[k]));
        }
        }
        __syncthreads();
        // slot of p[n0 + kR t + q - j0] is kR t + q + cj - 1
        const int s0 = kR * t + cj - 1;
        auto edge = [&](int q) {
            const cpx<T> v = p[pad8(s0 + q)];
#pragma unroll
            for (int r = 0; r < kR; ++r)
                if (r - q >= 0 && r - q < cj) acc[r] = add_(acc[r], v);
        };
        if (cj >= kR) {
            // head q = kR-1 .. 0: accumulators r >= q (compile-time masks)
#pragma unroll
            for (int q = kR - 1; q >= 0; --q) {
                const cpx<T> v = p[pad8(s0 + q)];
#pragma unroll
                for (int r = q; r < kR; ++r) acc[r] = add_(acc[r], v);
            }
#pragma unroll 4
            for (int q = -1; q > kR - 1 - cj; --q) {              // body: every r
                const cpx<T> v = p[pad8(s0 + q)];
#pragma unroll
                for (int r = 0; r < kR; ++r) acc[r] = add_(acc[r], v);
            }
            // tail q = kR-1-cj-u (u = 0 .. kR-2): accumulators r < kR-1-u
#pragma unroll
            for (int u = 0; u < kR - 1; ++u) {
                const cpx<T> v = p[pad8(s0 + kR - 1 - cj - u)];
#pragma unroll
                for (int r = 0; r < kR - 1 - u; ++r) acc[r] = add_(acc[r], v);
            }
        } else {
            for (int q = kR - 1; q > -cj; --q) edge(q);
        }
    }
    // stage through LDS for coalesced stores
    __syncthreads();
#pragma unroll
    for (int r = 0; r < kR; ++r) p[pad8(kR * t + r)] = acc[r];
    __syncthreads();
    for (int s = t; s < kOut; s += kTile)
        if (n0 + s < n) store_nt(y + n0 + s, p[pad8(s)]);
}

// Persistent, software-pipelined form (K <= kPipeK, d <= kPipeD; c32 / c64): one
// wave walks tiles b, b + G, ... of its channel; the next tile's inputs are loaded
// into registers before this tile's products, sums and stores, so the loads' latency
// overlaps the 48-add chains instead of stalling each one-shot wave.  Same products,
// same summation order per output as acorr_kernel (bit-identical).
constexpr int kPipeK = 128, kPipeD = 128;
template <typename T>
__global__ void __launch_bounds__(kTile) acorr_pipe_kernel(const cpx<T>* __restrict__ x, cpx<T>* __restrict__ y,
                                                           long long n, int d, int K, long long t_lo, long long t_hi) {
    extern __shared__ __attribute__((aligned(16))) char acorr_lds[];
    cpx<T>* p = reinterpret_cast<cpx<T>*>(acorr_lds);
    cpx<T>* xs = p + pad8(kOut + K - 1) + 1;
    constexpr int kLp = (kOut + kPipeK - 1 + kPipeD + kTile - 1) / kTile;
    constexpr int kE = (int)sizeof(cpx<T>);
    typedef unsigned u2 __attribute__((ext_vector_type(2)));
    typedef unsigned u4 __attribute__((ext_vector_type(4)));
    const int ch = blockIdx.y;
    x += (long long)ch * n;
    y += (long long)ch * n;
    const int t = threadIdx.x;
    const int cnt = kOut + K - 1, ns = cnt + d;  // products and staged inputs per tile
    // one wave per workgroup: LDS hand-offs need only this wave's LDS operations done
    auto lds_sync = [] { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); };
    // XCD-ordered walk (gridDim.x a multiple of 8): workgroup b on XCD b % 8 takes tiles
    // (b / 8) + i G/8 of that XCD's contiguous eighth, so the tiles an XCD has in flight are
    // neighbours and each tile's K - 1 + d halo samples were just read into the same L2
    const long long nt = t_hi - t_lo, Q = (nt + 7) / 8, Gx = gridDim.x / 8;
    const long long e_lo = t_lo + (long long)(blockIdx.x & 7) * Q, e_hi0 = e_lo + Q;
    const long long e_hi = e_hi0 < t_hi ? e_hi0 : t_hi;
    long long tile = e_lo + (blockIdx.x >> 3);
    if (tile >= e_hi) return;
    cpx<T> v[kLp];
    // interior tiles only (t_lo..t_hi): x[b0, b0 + ns) lies inside the call; the descriptor's
    // bound returns zeros past ns, so every lane issues the same kLp loads (no branches)
    // past the eighth's last tile (ok false): an empty descriptor, so the loads return zeros without
    // touching memory and no branch sits around them
    auto load = [&](long long tl, bool ok) {
        const auto rx = __builtin_amdgcn_make_buffer_rsrc((void*)(x + (ok ? tl : tile) * kOut - (K - 1) - d), (short)0,
                                                          ok ? ns * kE : 0, 0x00020000);
#pragma unroll
        for (int k = 0; k < kLp; ++k) {
            if constexpr (kE == 8)
                v[k] = __builtin_bit_cast(cpx<T>, __builtin_amdgcn_raw_buffer_load_b64(rx, (t + k * kTile) * kE, 0, 0));
            else
                v[k] = __builtin_bit_cast(cpx<T>, __builtin_amdgcn_raw_buffer_load_b128(rx, (t + k * kTile) * kE, 0, 0));
        }
    };
    // rows k < kOut / kTile lie inside every tile's ns = kOut + K - 1 + d staged samples: no test
    auto stage = [&] {
#pragma unroll
        for (int k = 0; k < kLp; ++k) {
            const int i = t + k * kTile;
            if (k < kOut / kTile || i < ns) xs[i] = v[k];
        }
    };
    load(tile, true);
    stage();
    // rotated: each tile is staged at the end of the previous iteration, in the same iteration as
    // its loads, so the compiler's wait for them sits behind only that iteration's stores (at the
    // loop header it merged with the prologue's state and waited for the stores too)
    for (;;) {
        const long long n0 = tile * kOut;
        lds_sync();
        const long long nxt = tile + Gx;
        load(nxt, nxt < e_hi);  // in flight across this tile's products, sums and stores
        // products: the kOut / kTile full rows with all their LDS reads issued first, then the
        // ragged rest (cnt = kOut + K - 1)
        {
            constexpr int kF = kOut / kTile;
            cpx<T> pa[kF], pc[kF];
#pragma unroll
            for (int k = 0; k < kF; ++k) {
                const int s = t + k * kTile;
                pa[k] = xs[s + d];
                pc[k] = xs[s];
            }
#pragma unroll
            for (int k = 0; k < kF; ++k) p[pad8(t + k * kTile)] = mul_conj_(pa[k], pc[k]);
#pragma unroll
            for (int k = kF; k < (kOut + kPipeK - 1 + kTile - 1) / kTile; ++k) {
                const int s = t + k * kTile;
                if (s < cnt) p[pad8(s)] = mul_conj_(xs[s + d], xs[s]);
            }
        }
        lds_sync();
        cpx<T> acc[kR];
#pragma unroll
        for (int r = 0; r < kR; ++r) acc[r] = zero_v<cpx<T>>();
        // slot of p[n0 + kR t + q] is kR t + q + K - 1 (the one-shot kernel's single chunk)
        const int s0 = kR * t + K - 1;
        if (K >= kR) {
            // term m = K - 1 + q of this lane sits at pad8(8 t + m) = 9 t + m + (m >> 3): a lane base
            // plus a wave-uniform offset, so whole blocks of eight m (m = 8 j .. 8 j + 7) read at
            // compile-time offsets from one address (the per-read pad8 arithmetic cost ~0.4 VALU
            // per add).  Same terms, same order: m from K + 6 down to 0.
            const cpx<T>* pl = p + (kR + 1) * t;
            auto term = [&](int m) { return pl[m + (m >> 3)]; };
#pragma unroll
            for (int q = kR - 1; q >= 0; --q) {  // head: m = K - 1 + q, accumulators r >= q
                const cpx<T> pv = term(K - 1 + q);
#pragma unroll
                for (int r = q; r < kR; ++r) acc[r] = add_(acc[r], pv);
            }
            int m = K - 2;  // body: m = K - 2 .. 7, every accumulator
            for (; m >= kR - 1 && (m & 7) != 7; --m) {
                const cpx<T> pv = term(m);
#pragma unroll
                for (int r = 0; r < kR; ++r) acc[r] = add_(acc[r], pv);
            }
            for (; m >= 15; m -= 8) {
                const cpx<T>* b = pl + 9 * (m >> 3);  // terms 8 (m >> 3) + i at b[i]
#pragma unroll
                for (int i = 7; i >= 0; --i) {
                    const cpx<T> pv = b[i];
#pragma unroll
                    for (int r = 0; r < kR; ++r) acc[r] = add_(acc[r], pv);
                }
            }
            if (m == kR - 1) {
                const cpx<T> pv = pl[kR - 1];
#pragma unroll
                for (int r = 0; r < kR; ++r) acc[r] = add_(acc[r], pv);
            }
#pragma unroll
            for (int u = 0; u < kR - 1; ++u) {  // tail: m = 6 - u, accumulators r < 7 - u
                const cpx<T> pv = pl[kR - 2 - u];
#pragma unroll
                for (int r = 0; r < kR - 1 - u; ++r) acc[r] = add_(acc[r], pv);
            }
        } else {
            for (int q = kR - 1; q > -K; --q) {
                const cpx<T> pv = p[pad8(s0 + q)];
#pragma unroll
                for (int r = 0; r < kR; ++r)
                    if (r - q >= 0 && r - q < K) acc[r] = add_(acc[r], pv);
            }
        }
        lds_sync();
#pragma unroll
        for (int r = 0; r < kR; ++r) p[pad8(kR * t + r)] = acc[r];
        lds_sync();
        const auto ry = __builtin_amdgcn_make_buffer_rsrc((void*)(y + n0), (short)0, kOut * kE, 0x00020000);
#pragma unroll
        for (int k = 0; k < kOut / kTile; ++k) {
            const cpx<T> o = p[pad8(t + k * kTile)];
            if constexpr (kE == 8)
                __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u2, o), ry, (t + k * kTile) * kE, 0, 2);
            else
                __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4, o), ry, (t + k * kTile) * kE, 0, 2);
        }
        if (nxt >= e_hi) break;
        tile = nxt;
        lds_sync();  // every read of xs and p done before the next tile is staged
        stage();
    }
}

// execute() on the current window (no push): the output for the newest history sample
template <typename T>
__global__ void acorr_current_kernel(const cpx<T>* __restrict__ hist, cpx<T>* __restrict__ out, int H, int d, int K) {
    const int ch = blockIdx.x;
    hist += (long long)ch * H;
    if (threadIdx.x != 0) return;
    cpx<T> acc = zero_v<cpx<T>>();
    for (int j = 0; j < K; ++j) {
        const long long m = -1 - j;
        acc = add_(acc, mul_(ext_at<T>(nullptr, hist, m, H), conj_(ext_at<T>(nullptr, hist, m - d, H))));
    }
    out[ch] = acc;
}

// sum of e2 = (x * conj(x)).re over the W newest samples of (hist ++ x), in f64
template <typename T>
__global__ void __launch_bounds__(256) acorr_energy_kernel(const cpx<T>* __restrict__ x, const cpx<T>* __restrict__ hist,
                                                           long long n, int H, int W, double* __restrict__ energy) {
    __shared__ double part[256];
    const int ch = blockIdx.x;
    x += (long long)ch * n;
    hist += (long long)ch * H;
    double s = 0.0;
    for (int i = threadIdx.x; i < W; i += 256) {
        const cpx<T> v = ext_at(x, hist, n - W + i, H);
        s += (double)mul_(v, conj_(v)).re;
    }
    part[threadIdx.x] = s;
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
        if (threadIdx.x < w) part[threadIdx.x] += part[threadIdx.x + w];
        __syncthreads();
    }
    if (threadIdx.x == 0) energy[ch] = part[0];
}

template <typename T, bool DOWN>
__device__ __forceinline__ cpx<T> nco_one(const T* lut, cpx<T> v, long long i, uint32_t theta0, uint32_t dtheta) {
    const uint32_t th = theta0 + (uint32_t)i * dtheta;  // wrapping u32: theta_0 + i dtheta mod 2^32
    const uint32_t idx = ((th + (1u << 21)) >> 22) & 0x3ffu;
    cpx<T> ph = {lut[(idx + 256) & 0x3ffu], lut[idx]};
    if constexpr (DOWN) ph = conj_(ph);
    return mul_(ph, v);
}

// One-shot, XCD-ordered: a workgroup mixes kU x 256 consecutive V-sample vectors
// (32 KB of c32 input), issuing all its loads before staging the f32/f64 copy of
// the sine table in LDS.
constexpr int kNcoU = 8;
#ifndef SDSP_NCO_WT
#define SDSP_NCO_WT 1
#endif
template <typename T, bool DOWN, int V>
__global__ void __launch_bounds__(256) nco_mix_kernel(const cpx<T>* __restrict__ x, cpx<T>* __restrict__ y, long long n,
                                                      const double* __restrict__ table, uint32_t theta0,
                                                      uint32_t dtheta) {
    struct alignas(V * sizeof(cpx<T>)) Vec { cpx<T> s[V]; };
    __shared__ T lut[1024];
    const long long nv = n / V;
    const Vec* xv = reinterpret_cast<const Vec*>(x);
    Vec* yv = reinterpret_cast<Vec*>(y);
    const long long base = (long long)xcd_order(blockIdx.x, gridDim.x) * 256 * kNcoU + threadIdx.x;
    Vec r[kNcoU];
    // 16-byte vectors (SDSP_NCO_WT): nontemporal loads and write-through (sc1) stores, the copy
    // probe's fastest policy pair (profiles/LABLOG.md "Copy ceilings"); stores through a descriptor
    // bounded by the call, so vectors past its end are dropped
    constexpr bool kWt = SDSP_NCO_WT && sizeof(Vec) == 16;
    typedef unsigned nco_u4 __attribute__((ext_vector_type(4)));
#pragma unroll
    for (int u = 0; u < kNcoU; ++u)
        if (base + 256 * u < nv) {
            if constexpr (kWt) {
                const nco_u4 w = __builtin_nontemporal_load(reinterpret_cast<const nco_u4*>(xv + base + 256 * u));
                __builtin_memcpy(&r[u], &w, 16);
            } else {
                r[u] = xv[base + 256 * u];
            }
        }
    for (int i = threadIdx.x; i < 1024; i += 256) lut[i] = (T)table[i];
    __syncthreads();
    const long long vb = base - threadIdx.x;  // the block's first vector
    const long long vrem = nv - vb;
    const auto ry = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(yv + (vrem > 0 ? vb : 0)), (short)0,
        vrem <= 0 ? 0u : (unsigned)((vrem < 256LL * kNcoU ? vrem : 256LL * kNcoU) * 16), 0x00020000);
#pragma unroll
    for (int u = 0; u < kNcoU; ++u) {
        const long long v = base + 256 * u;
        if (v < nv) {
#pragma unroll
            for (int k = 0; k < V; ++k) r[u].s[k] = nco_one<T, DOWN>(lut, r[u].s[k], v * V + k, theta0, dtheta);
            if constexpr (kWt) {
                nco_u4 w;
                __builtin_memcpy(&w, &r[u], 16);
                __builtin_amdgcn_raw_buffer_store_b128(w, ry, (unsigned)(threadIdx.x + 256 * u) * 16u, 0, 16);
            } else {
                store_nt(yv + v, r[u]);
            }
        }
    }
    if (blockIdx.x == 0 && threadIdx.x < n - nv * V) {  // ragged tail (c32, odd n)
        const long long i = nv * V + threadIdx.x;
        y[i] = nco_one<T, DOWN>(lut, x[i], i, theta0, dtheta);
    }
}

// ---------------------------------------------------------------- AGC
constexpr int kAgcS = 8;  // samples per channel per LDS chunk

template <bool CPLX> struct AgcSample;
template <> struct AgcSample<false> {
    double v;
    __device__ double energy() const { return v * v; }  // (out.conj() * out).real() for f64
    __device__ AgcSample scaled(double g) const { return {v * g}; }
};
template <> struct AgcSample<true> {
    double re, im;
    // (conj(out) * out).re = re * re - (-im) * im  (num-complex Mul, no FMA)
    __device__ double energy() const { return re * re - (-im) * im; }
    __device__ AgcSample scaled(double g) const { return {re * g, im * g}; }
};

// get_rssi() > squelch_threshold  (:442-444, :632).  -20 log10(g) is decreasing
// in g, so away from the threshold gain gthr = 10^(-threshold/20) the answer is
// g < gthr; within 1e-6 relative of it (a log10 margin of 4e-7, far above the
// rounding of either side) the reference expression decides.  NaN and infinite
// operands fail both strict tests and take the reference expression too.
__device__ __forceinline__ bool agc_rssi_exceeds(const sdsp_agc_state& s, double gthr) {
    if (s.gain < gthr * (1.0 - 1e-6)) return true;
    if (s.gain > gthr * (1.0 + 1e-6)) return false;
    return log10(s.gain) * -20.0 > s.squelch_threshold;
}

// update_squelch_mode  :631-677 (usize timer wraps, as a release build does)
__device__ __forceinline__ void agc_squelch(sdsp_agc_state& s, double gthr) {
    if (s.squelch_mode == SDSP_SQUELCH_DISABLED || s.squelch_mode == SDSP_SQUELCH_UNKNOWN) {
        s.squelch_mode = SDSP_SQUELCH_DISABLED;  // `_ => DISABLED`; the rssi it computes is unused
        return;
    }
    const bool exceeded = agc_rssi_exceeds(s, gthr);
    switch (s.squelch_mode) {
        case SDSP_SQUELCH_ENABLED: s.squelch_mode = exceeded ? SDSP_SQUELCH_RISE : SDSP_SQUELCH_ENABLED; break;
        case SDSP_SQUELCH_RISE: s.squelch_mode = exceeded ? SDSP_SQUELCH_SIGNALHI : SDSP_SQUELCH_FALL; break;
        case SDSP_SQUELCH_SIGNALHI: s.squelch_mode = exceeded ? SDSP_SQUELCH_SIGNALHI : SDSP_SQUELCH_FALL; break;
        case SDSP_SQUELCH_FALL:
            s.squelch_timer = s.squelch_timeout;
            s.squelch_mode = exceeded ? SDSP_SQUELCH_SIGNALHI : SDSP_SQUELCH_SIGNALLO;
            break;
        case SDSP_SQUELCH_SIGNALLO:
            s.squelch_timer -= 1;
            s.squelch_mode = s.squelch_timer == 0 ? SDSP_SQUELCH_TIMEOUT
                             : exceeded            ? SDSP_SQUELCH_SIGNALHI
                                                   : SDSP_SQUELCH_SIGNALLO;
            break;
        default: s.squelch_mode = SDSP_SQUELCH_ENABLED;  // TIMEOUT
    }
}

// execute  :214-246
template <bool CPLX>
__device__ __forceinline__ AgcSample<CPLX> agc_execute(sdsp_agc_state& s, AgcSample<CPLX> in, double gthr) {
    const AgcSample<CPLX> out = in.scaled(s.gain);
    s.energy_estimate = (1.0 - s.alpha) * s.energy_estimate + out.energy() * s.alpha;
    if (s.lock) return out;
    if (s.energy_estimate > 0.000001) s.gain *= exp(-0.5 * s.alpha * log(s.energy_estimate));
    if (s.gain > 1000000.0) s.gain = 1000000.0;
    agc_squelch(s, gthr);
    if (s.squelch_mode == SDSP_SQUELCH_ENABLED) return in;
    return out.scaled(s.scale);
}

template <bool CPLX>
__global__ void __launch_bounds__(64, 4) agc_kernel(const AgcSample<CPLX>* __restrict__ x, AgcSample<CPLX>* __restrict__ y,
                                                 long long n, sdsp_agc_state* __restrict__ state, long long channels) {
    __shared__ AgcSample<CPLX> buf[64 * (kAgcS + 1)];  // row per channel, one spare slot
    const int t = threadIdx.x;
    const long long ch0 = (long long)blockIdx.x * 64;
    const long long me = ch0 + t;
    sdsp_agc_state s;
    double gthr = 0.0;
    if (me < channels) {
        s = state[me];
        gthr = pow(10.0, -s.squelch_threshold / 20.0);  // fixed for the launch (setters run between launches)
    }
    for (long long i0 = 0; i0 < n; i0 += kAgcS) {
        const int cnt = n - i0 < kAgcS ? (int)(n - i0) : kAgcS;
#pragma unroll
        for (int k = 0; k < kAgcS; ++k) {  // lane e of a row group reads consecutive samples of one channel
            const int e = t + 64 * k, c = e / kAgcS, j = e % kAgcS;
            if (j < cnt && ch0 + c < channels) buf[c * (kAgcS + 1) + j] = x[(ch0 + c) * n + i0 + j];
        }
        __syncthreads();
        if (me < channels)
            for (int j = 0; j < cnt; ++j) {
                AgcSample<CPLX>& v = buf[t * (kAgcS + 1) + j];
                v = agc_execute<CPLX>(s, v, gthr);
            }
        __syncthreads();
#pragma unroll
        for (int k = 0; k < kAgcS; ++k) {
            const int e = t + 64 * k, c = e / kAgcS, j = e % kAgcS;
            if (j < cnt && ch0 + c < channels) y[(ch0 + c) * n + i0 + j] = buf[c * (kAgcS + 1) + j];  // plain: nontemporal +7 %
        }
        __syncthreads();
    }
    if (me < channels) state[me] = s;
}

// agc_kernel with the next chunk's loads in flight across this chunk's gain chain: whole chunks
// through buffer loads / stores bounded by the workgroup's channels (rows past the last channel
// read zeros and drop their stores, so no branch sits around a memory op and the loads of chunk
// i + 1, issued before the stores of chunk i, are waited for alone), the ragged last chunk as in
// agc_kernel.  Offsets are 32-bit: n < 2^22 (the launcher routes larger n to agc_kernel).
template <bool CPLX> struct AgcRaw;
template <> struct AgcRaw<true> { typedef unsigned T __attribute__((ext_vector_type(4))); };
template <> struct AgcRaw<false> { typedef unsigned T __attribute__((ext_vector_type(2))); };
constexpr long long kAgcPipeMaxN = 1LL << 22;
#ifndef SDSP_AGC_PIPE_S
#define SDSP_AGC_PIPE_S 16
#endif
constexpr int kAgcPipeS = SDSP_AGC_PIPE_S;  // samples per channel per chunk

template <bool CPLX, int S>
__global__ void __launch_bounds__(64) agc_pipe_kernel(const AgcSample<CPLX>* __restrict__ x, AgcSample<CPLX>* __restrict__ y,
                                                      long long n, sdsp_agc_state* __restrict__ state, long long channels) {
    typedef typename AgcRaw<CPLX>::T V;
    constexpr unsigned SZ = sizeof(AgcSample<CPLX>);
    __shared__ AgcSample<CPLX> buf[64 * (S + 1)];
    const int t = threadIdx.x;
    const long long ch0 = (long long)blockIdx.x * 64;
    const long long me = ch0 + t, nch = channels - ch0 < 64 ? channels - ch0 : 64;
    sdsp_agc_state s;
    double gthr = 0.0;
    if (me < channels) {
        s = state[me];
        gthr = pow(10.0, -s.squelch_threshold / 20.0);
    }
    const long long nfull = n / S * S;
    // lane e = t + 64 k of a row group: channel e / S, sample e % S of the chunk
    unsigned off[S];
#pragma unroll
    for (int k = 0; k < S; ++k) {
        const int e = t + 64 * k;
        off[k] = (unsigned)(((long long)(e / S) * n + e % S) * SZ);
    }
    V r[S];
    // chunk at i0 (whole chunks only; past nfull: an empty descriptor, no traffic)
    auto rsrc = [&](const void* base, long long i0) {
        const bool ok = i0 < nfull;
        const unsigned nrec = ok ? (unsigned)((nch * n - i0) * SZ) : 0u;
        return __builtin_amdgcn_make_buffer_rsrc((void*)((const AgcSample<CPLX>*)base + ch0 * n + (ok ? i0 : 0)), (short)0,
                                                 nrec, 0x00020000);
    };
    auto load_chunk = [&](long long i0) {
        const auto rx = rsrc(x, i0);
#pragma unroll
        for (int k = 0; k < S; ++k) {
            if constexpr (CPLX) r[k] = __builtin_bit_cast(V, __builtin_amdgcn_raw_buffer_load_b128(rx, off[k], 0, 0));
            else r[k] = __builtin_bit_cast(V, __builtin_amdgcn_raw_buffer_load_b64(rx, off[k], 0, 0));
        }
    };
    auto stage = [&] {  // the loaded chunk into the LDS rows
#pragma unroll
        for (int k = 0; k < S; ++k) {
            const int e = t + 64 * k;
            buf[(e / S) * (S + 1) + e % S] = __builtin_bit_cast(AgcSample<CPLX>, r[k]);
        }
    };
    load_chunk(0);
    stage();
    __syncthreads();
    // rotated so that each wait for a chunk's loads sits in the same iteration as the loads,
    // behind only that iteration's stores
    for (long long i0 = 0; i0 < nfull; i0 += S) {
        load_chunk(i0 + S);
        if (me < channels)
            for (int j = 0; j < S; ++j) {
                AgcSample<CPLX>& v = buf[t * (S + 1) + j];
                v = agc_execute<CPLX>(s, v, gthr);
            }
        __syncthreads();
        const auto ry = rsrc(y, i0);
#pragma unroll
        for (int k = 0; k < S; ++k) {
            const int e = t + 64 * k;
            const V v = __builtin_bit_cast(V, buf[(e / S) * (S + 1) + e % S]);
            if constexpr (CPLX) __builtin_amdgcn_raw_buffer_store_b128(v, ry, off[k], 0, 0);
            else __builtin_amdgcn_raw_buffer_store_b64(v, ry, off[k], 0, 0);
        }
        __syncthreads();
        stage();
        __syncthreads();
    }
    if (nfull < n) {  // the ragged last chunk
        const long long i0 = nfull;
        const int cnt = (int)(n - i0);
#pragma unroll
        for (int k = 0; k < S; ++k) {
            const int e = t + 64 * k, c = e / S, j = e % S;
            if (j < cnt && ch0 + c < channels) buf[c * (S + 1) + j] = x[(ch0 + c) * n + i0 + j];
        }
        __syncthreads();
        if (me < channels)
            for (int j = 0; j < cnt; ++j) {
                AgcSample<CPLX>& v = buf[t * (S + 1) + j];
                v = agc_execute<CPLX>(s, v, gthr);
            }
        __syncthreads();
#pragma unroll
        for (int k = 0; k < S; ++k) {
            const int e = t + 64 * k, c = e / S, j = e % S;
            if (j < cnt && ch0 + c < channels) y[(ch0 + c) * n + i0 + j] = buf[c * (S + 1) + j];
        }
    }
    if (me < channels) state[me] = s;
}

// init  :568-586 then set_signal_level  :416-428
template <bool CPLX>
__global__ void __launch_bounds__(64) agc_init_kernel(const AgcSample<CPLX>* __restrict__ x, long long n,
                                                      sdsp_agc_state* __restrict__ state, double* __restrict__ levels,
                                                      long long channels) {
    const long long ch = (long long)blockIdx.x * 64 + threadIdx.x;
    if (ch >= channels) return;
    double x2 = 0.0;
    for (long long i = 0; i < n; ++i) x2 += x[ch * n + i].energy();  // (i * i.conj()).real(), in order
    x2 = sqrt(x2 / (double)n) + 1e-16;  // 10f64.powi(-16)
    levels[ch] = x2;
    if (x2 <= 0.0) return;  // SignalLevelOutOfRange: the host reports it
    state[ch].gain = 1.0 / x2;
    state[ch].energy_estimate = 1.0;
}

}  // namespace

// dynamic LDS of acorr_kernel: the product tile of the widest chunk, plus the staged input
static size_t acorr_lds_bytes(size_t elem, int d, int K, bool stage) {
    const int cj = K < kChunk ? K : kChunk;
    const size_t np = (size_t)pad8(kOut + cj - 1) + 1, nx = stage ? (size_t)(kOut + cj - 1 + d) : 0;
    return (np + nx) * elem;
}

// resident one-wave workgroups of acorr_pipe_kernel on the current device (CU count x occupancy
// at `lds` bytes), looked up once per (device, precision, LDS size)
static long long acorr_pipe_slots(int prec, size_t lds) {
    static std::mutex mu;
    static std::map<std::tuple<int, int, size_t>, long long> cache;
    int dev = 0;
    (void)hipGetDevice(&dev);
    const auto key = std::make_tuple(dev, prec, lds);
    std::lock_guard<std::mutex> g(mu);
    const auto it = cache.find(key);
    if (it != cache.end()) return it->second;
    int cus = 256, per_cu = 0;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (prec == 0)
        (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, acorr_pipe_kernel<float>, kTile, lds);
    else
        (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, acorr_pipe_kernel<double>, kTile, lds);
    const long long res = (long long)(per_cu > 0 ? per_cu : 8) * cus;
    cache.emplace(key, res);
    return res;
}

hipError_t launch_acorr(int prec, const void* x, const void* hist, void* y, size_t n, int H, int d, int K,
                        size_t channels, hipStream_t s, int kernel) {
    if (n == 0) return hipSuccess;
    dim3 grid((unsigned)((n + kOut - 1) / kOut), (unsigned)channels);
    const bool nostage = kernel == 2, pipe = kernel == 0;
    if (pipe && K >= 1 && K <= kPipeK && d <= kPipeD) {
        // interior tiles (whole input window and all outputs inside the call) on the pipelined
        // kernel; the edge tiles on the one-shot kernel
        const long long ntiles = (long long)((n + kOut - 1) / kOut);
        const long long t_lo = (K - 1 + d + kOut - 1) / kOut, t_hi = (long long)(n / kOut);
        if (t_hi > t_lo) {
            const size_t elem = prec == 0 ? sizeof(c32) : sizeof(c64);
            const size_t lds2 = ((size_t)pad8(kOut + K - 1) + 1 + (size_t)(kOut + K - 1 + d)) * elem;
            // one persistent wave per resident slot (registers / LDS decide how many per CU): the
            // current device's CU count and the kernel's occupancy at this LDS size, cached
            const long long res = acorr_pipe_slots(prec, lds2);
            const long long nt = t_hi - t_lo;
            long long G = nt < res ? nt : res;
            G = (G + 7) / 8 * 8;  // whole workgroups per XCD (surplus ones find no tile and return)
            const dim3 g2((unsigned)G, (unsigned)channels);
            if (prec == 0)
                hipLaunchKernelGGL((acorr_pipe_kernel<float>), g2, dim3(kTile), lds2, s, (const c32*)x, (c32*)y,
                                   (long long)n, d, K, t_lo, t_hi);
            else
                hipLaunchKernelGGL((acorr_pipe_kernel<double>), g2, dim3(kTile), lds2, s, (const c64*)x, (c64*)y,
                                   (long long)n, d, K, t_lo, t_hi);
            const size_t lds = acorr_lds_bytes(prec == 0 ? sizeof(c32) : sizeof(c64), d, K, true);
            auto edge = [&](long long a, long long b) {
                if (b <= a) return;
                const dim3 ge((unsigned)(b - a), (unsigned)channels);
                if (prec == 0)
                    hipLaunchKernelGGL((acorr_kernel<float, true>), ge, dim3(kTile), lds, s, (const c32*)x,
                                       (const c32*)hist, (c32*)y, (long long)n, H, d, K, a);
                else
                    hipLaunchKernelGGL((acorr_kernel<double, true>), ge, dim3(kTile), lds, s, (const c64*)x,
                                       (const c64*)hist, (c64*)y, (long long)n, H, d, K, a);
            };
            edge(0, t_lo);
            edge(t_hi, ntiles);
            return hipGetLastError();
        }
    }
    const bool stage = d <= kDmax && !nostage;
    const size_t lds = acorr_lds_bytes(prec == 0 ? sizeof(c32) : sizeof(c64), d, K, stage);
    if (prec == 0) {
        if (stage)
            hipLaunchKernelGGL((acorr_kernel<float, true>), grid, dim3(kTile), lds, s, (const c32*)x, (const c32*)hist,
                               (c32*)y, (long long)n, H, d, K, 0LL);
        else
            hipLaunchKernelGGL((acorr_kernel<float, false>), grid, dim3(kTile), lds, s, (const c32*)x, (const c32*)hist,
                               (c32*)y, (long long)n, H, d, K, 0LL);
    } else {
        if (stage)
            hipLaunchKernelGGL((acorr_kernel<double, true>), grid, dim3(kTile), lds, s, (const c64*)x, (const c64*)hist,
                               (c64*)y, (long long)n, H, d, K, 0LL);
        else
            hipLaunchKernelGGL((acorr_kernel<double, false>), grid, dim3(kTile), lds, s, (const c64*)x, (const c64*)hist,
                               (c64*)y, (long long)n, H, d, K, 0LL);
    }
    return hipGetLastError();
}

hipError_t launch_acorr_current(int prec, const void* hist, void* out, int H, int d, int K, size_t channels,
                                hipStream_t s) {
    if (prec == 0)
        hipLaunchKernelGGL(acorr_current_kernel<float>, dim3((unsigned)channels), dim3(64), 0, s, (const c32*)hist,
                           (c32*)out, H, d, K);
    else
        hipLaunchKernelGGL(acorr_current_kernel<double>, dim3((unsigned)channels), dim3(64), 0, s, (const c64*)hist,
                           (c64*)out, H, d, K);
    return hipGetLastError();
}

hipError_t launch_acorr_energy(int prec, const void* x, const void* hist, size_t n, int H, int W, size_t channels,
                               double* energy, hipStream_t s) {
    if (prec == 0)
        hipLaunchKernelGGL(acorr_energy_kernel<float>, dim3((unsigned)channels), dim3(256), 0, s, (const c32*)x,
                           (const c32*)hist, (long long)n, H, W, energy);
    else
        hipLaunchKernelGGL(acorr_energy_kernel<double>, dim3((unsigned)channels), dim3(256), 0, s, (const c64*)x,
                           (const c64*)hist, (long long)n, H, W, energy);
    return hipGetLastError();
}

hipError_t launch_nco_mix(int prec, bool down, const void* x, void* y, size_t n, const double* table, uint32_t theta0,
                          uint32_t dtheta, int num_cus, hipStream_t s) {
    if (n == 0) return hipSuccess;
    const bool a16 = (((uintptr_t)x | (uintptr_t)y) & 15) == 0;
    const int V = prec == 0 && a16 ? 2 : 1;
    (void)num_cus;
    long long blocks = ((long long)n / V + 256 * kNcoU - 1) / (256 * kNcoU);
    if (blocks < 1) blocks = 1;
    if (blocks > 0x7fffffffLL) return hipErrorInvalidValue;
    dim3 grid((unsigned)blocks);
#define SDSP_NCO(T, D, V)                                                                                        \
    hipLaunchKernelGGL((nco_mix_kernel<T, D, V>), grid, dim3(256), 0, s, (const cpx<T>*)x, (cpx<T>*)y, (long long)n, \
                       table, theta0, dtheta)
    if (prec == 0 && V == 2) {
        if (down) SDSP_NCO(float, true, 2); else SDSP_NCO(float, false, 2);
    } else if (prec == 0) {
        if (down) SDSP_NCO(float, true, 1); else SDSP_NCO(float, false, 1);
    } else {
        if (down) SDSP_NCO(double, true, 1); else SDSP_NCO(double, false, 1);
    }
#undef SDSP_NCO
    return hipGetLastError();
}

hipError_t launch_agc(bool cplx, const void* x, void* y, size_t n, void* state, size_t channels, hipStream_t s,
                      bool pipe) {
    if (n == 0 || channels == 0) return hipSuccess;
    dim3 grid((unsigned)((channels + 63) / 64));
    if (pipe && (long long)n < kAgcPipeMaxN) {
        if (cplx)
            hipLaunchKernelGGL((agc_pipe_kernel<true, kAgcPipeS>), grid, dim3(64), 0, s, (const AgcSample<true>*)x,
                               (AgcSample<true>*)y, (long long)n, (sdsp_agc_state*)state, (long long)channels);
        else
            hipLaunchKernelGGL((agc_pipe_kernel<false, kAgcPipeS>), grid, dim3(64), 0, s, (const AgcSample<false>*)x,
                               (AgcSample<false>*)y, (long long)n, (sdsp_agc_state*)state, (long long)channels);
        return hipGetLastError();
    }
    if (cplx)
        hipLaunchKernelGGL(agc_kernel<true>, grid, dim3(64), 0, s, (const AgcSample<true>*)x, (AgcSample<true>*)y,
                           (long long)n, (sdsp_agc_state*)state, (long long)channels);
    else
        hipLaunchKernelGGL(agc_kernel<false>, grid, dim3(64), 0, s, (const AgcSample<false>*)x, (AgcSample<false>*)y,
                           (long long)n, (sdsp_agc_state*)state, (long long)channels);
    return hipGetLastError();
}

hipError_t launch_agc_init(bool cplx, const void* x, size_t n, void* state, double* levels, size_t channels,
                           hipStream_t s) {
    dim3 grid((unsigned)((channels + 63) / 64));
    if (cplx)
        hipLaunchKernelGGL(agc_init_kernel<true>, grid, dim3(64), 0, s, (const AgcSample<true>*)x, (long long)n,
                           (sdsp_agc_state*)state, levels, (long long)channels);
    else
        hipLaunchKernelGGL(agc_init_kernel<false>, grid, dim3(64), 0, s, (const AgcSample<false>*)x, (long long)n,
                           (sdsp_agc_state*)state, levels, (long long)channels);
    return hipGetLastError();
}

}  // namespace sdsp
