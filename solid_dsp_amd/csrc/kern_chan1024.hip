// 1024-channel PFB + FFT channeliser for complex-f32 streams (gfx950).
//
// Same composition as chan_kernel in kern_fft.hip (PolyPhaseFilterBank
// branch sums, src/filter/fir/pfb.rs:81-90, feeding a forward FFT,
// src/fft/mod.rs:175-215):
//     v_p[m] = sum_{i<K} cb[p][i] * x[(m-i)M + (M-1-p)],   X_m = FFT_1024(v[m])
// One 1024-thread workgroup walks F consecutive frames of one stream, sixteen
// frames per round:
//   * PFB: thread t owns branch p = t; its taps and the last 8 input samples of
//     the branch live in registers (a ring indexed by frame mod 8, static in the
//     unrolled round), so every input sample is read from HBM once (plus K-1
//     warm-up frames per workgroup) and costs K fused multiply-adds.  The
//     round's sixteen frames of branch outputs go to sixteen LDS buffers.
//   * FFT: wave w transforms buffer w, 1024 = 16 x 16 x 4 with the
//     decomposition n = n0 + 4 n1 + 64 n2, k = k2 + 16 k1 + 256 k0:
//       P1 lane L = n0 + 4 n1: DFT16 over n2, * W1024^(L k2)
//       P2 lane k2 + 16 n0:    DFT16 over n1, * W1024^(16 n0 k1)
//       P3 lanes (k2 + 16 n0), row-swap transposed: DFT4 over n0 -> X[k2 + 16 k1 + 256 k0]
//     with one wave-local LDS transpose (swizzled, conflict-free; see
//     fft1024_chan), so the FFTs need no workgroup barrier.  Outputs: natural
//     channel order, as kern_fft.hip.
// Arithmetic: fused multiply-add, f32; parity is the §8d tolerance against the
// f64 restatement (tests/test_gpu_fft.py).
#include "sdsp_device.hpp"
#include <cstdlib>

#include "sdsp_kernels.hpp"
#include "sdsp_pk.hpp"

namespace sdsp {

namespace {

struct alignas(8) cf { float re, im; };  // 8-byte aligned: b64 LDS / global accesses
__device__ __forceinline__ cf cadd(cf a, cf b) { return {a.re + b.re, a.im + b.im}; }
__device__ __forceinline__ cf csub(cf a, cf b) { return {a.re - b.re, a.im - b.im}; }
__device__ __forceinline__ cf cmul(cf a, cf b) {
    return {__builtin_fmaf(a.re, b.re, -(a.im * b.im)), __builtin_fmaf(a.re, b.im, a.im * b.re)};
}
__device__ __forceinline__ cf rotj(cf a) { return {a.im, -a.re}; }  // * (-j)

__device__ __forceinline__ void dft4(cf& x0, cf& x1, cf& x2, cf& x3) {
    const cf a = cadd(x0, x2), b = csub(x0, x2), c = cadd(x1, x3), d = rotj(csub(x1, x3));
    x0 = cadd(a, c);
    x2 = csub(a, c);
    x1 = cadd(b, d);
    x3 = csub(b, d);
}

constexpr float kC1 = 0.92387953251128674f;  // cos(pi/8)
constexpr float kS1 = 0.38268343236508978f;  // sin(pi/8)
constexpr float kR2 = 0.70710678118654752f;  // sqrt(1/2)

template <int m> __device__ __forceinline__ cf tw16(cf v) {  // v * e^{-j 2 pi m / 16}
    if constexpr (m == 0) return v;
    else if constexpr (m == 1) return cmul(v, cf{kC1, -kS1});
    else if constexpr (m == 2) return cf{kR2 * (v.re + v.im), kR2 * (v.im - v.re)};
    else if constexpr (m == 3) return cmul(v, cf{kS1, -kC1});
    else if constexpr (m == 4) return rotj(v);
    else if constexpr (m == 6) return cf{kR2 * (-v.re + v.im), kR2 * (-v.im - v.re)};
    else if constexpr (m == 9) return cmul(v, cf{-kC1, kS1});
    else return v;
}

// in-place forward 16-point DFT, natural order in and out
__device__ __forceinline__ void dft16(cf (&v)[16]) {
#pragma unroll
    for (int nb = 0; nb < 4; ++nb) dft4(v[nb], v[4 + nb], v[8 + nb], v[12 + nb]);
    v[5] = tw16<1>(v[5]);
    v[6] = tw16<2>(v[6]);
    v[7] = tw16<3>(v[7]);
    v[9] = tw16<2>(v[9]);
    v[10] = tw16<4>(v[10]);
    v[11] = tw16<6>(v[11]);
    v[13] = tw16<3>(v[13]);
    v[14] = tw16<6>(v[14]);
    v[15] = tw16<9>(v[15]);
#pragma unroll
    for (int ka = 0; ka < 4; ++ka) dft4(v[4 * ka + 0], v[4 * ka + 1], v[4 * ka + 2], v[4 * ka + 3]);
    cf t[16];
#pragma unroll
    for (int ka = 0; ka < 4; ++ka)
#pragma unroll
        for (int kb = 0; kb < 4; ++kb) t[ka + 4 * kb] = v[4 * ka + kb];
#pragma unroll
    for (int i = 0; i < 16; ++i) v[i] = t[i];
}

// LDS hand-off between the lanes of one wave (LDS counter only; global
// loads and stores stay in flight)
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_s_waitcnt(0xC07F);
    __builtin_amdgcn_wave_barrier();
}

constexpr int kM = 1024;

// Wave buffer: 64 rows of 18 complex (16 + 2 pad): every LDS address below is
// a lane base plus a compile-time offset, and 16 lanes reading the same slot
// of 16 consecutive rows hit distinct banks.
constexpr int kRow = 18;
constexpr int kBuf = 64 * kRow;

// W1024^j from the table: the whole table (QTW false), or its first quarter rotated by
// W1024^(256 q) = (-j)^q (QTW, the 8-transform lab form: 2 KB of LDS instead of 8)
template <bool QTW> __device__ __forceinline__ cf tw1024(const cf* __restrict__ stw, int j) {
    if constexpr (!QTW) {
        return stw[j & (kM - 1)];
    } else {
        const cf b = stw[j & 255];
        const int q = (j >> 8) & 3;
        cf r = (q & 1) ? cf{b.im, -b.re} : b;
        return (q & 2) ? cf{-r.re, -r.im} : r;
    }
}

// P1 and P2 of one wave's 1024-point FFT: buffer holds v[p] at index p on
// entry; on exit the P3 inputs of column c = (k2 + 16 k1) sit at buf[4 c + n0]
template <bool QTW = false>
__device__ __forceinline__ void fft1024_p12(cf* __restrict__ buf, const cf* __restrict__ stw, int L) {
    cf v[16];
#pragma unroll
    for (int n2 = 0; n2 < 16; ++n2) v[n2] = buf[L + 64 * n2];
    dft16(v);
#pragma unroll
    for (int k2 = 1; k2 < 16; ++k2) v[k2] = cmul(v[k2], tw1024<QTW>(stw, L * k2));
    wave_sync();
    const int n0 = L & 3, n1 = L >> 2;
#pragma unroll
    for (int k2 = 0; k2 < 16; ++k2) buf[(n0 + 4 * k2) * kRow + n1] = v[k2];
    wave_sync();
    // lane L = (n0, k2) with n0 = L & 3, k2 = L >> 2: row L holds n1 = 0..15
#pragma unroll
    for (int i = 0; i < 16; ++i) v[i] = buf[L * kRow + i];
    dft16(v);
#pragma unroll
    for (int k1 = 1; k1 < 16; ++k1) v[k1] = cmul(v[k1], tw1024<QTW>(stw, 16 * n0 * k1));
    wave_sync();
    const int k2 = L >> 2;
#pragma unroll
    for (int k1 = 0; k1 < 16; ++k1) buf[(k2 + 16 * k1) * 4 + n0] = v[k1];
    wave_sync();
}

// the same FFT leaving natural-order X in buf[0, 1024)
template <bool QTW = false>
__device__ __forceinline__ void fft1024_wave_lds(cf* __restrict__ buf, const cf* __restrict__ stw, int L) {
    fft1024_p12<QTW>(buf, stw, L);
    cf o[4][4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int c = L + 64 * j;
        o[j][0] = buf[c * 4 + 0];
        o[j][1] = buf[c * 4 + 1];
        o[j][2] = buf[c * 4 + 2];
        o[j][3] = buf[c * 4 + 3];
        dft4(o[j][0], o[j][1], o[j][2], o[j][3]);
    }
    wave_sync();
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int k0 = 0; k0 < 4; ++k0) buf[L + 64 * j + 256 * k0] = o[j][k0];
    wave_sync();
}

// ---- the channeliser's per-frame FFT --------------------------------------
// Same decomposition and arithmetic as fft1024_p12 + the DFT4 pass (bit for
// bit), with fewer LDS cycles per frame:
//   * frame buffer of 1024 complex, unpadded: the PFB writes v[p] at p (rows of
//     512 B) and P1 reads v[L + 64 n2];
//   * the P1 -> P2 transpose goes to 64 rows of 16 with column c of row r at
//     r*16 + (c ^ swz(r)), swz(r) = ((r & 3) << 2) ^ (r >> 2): conflict-free for
//     the P1 stores (16-lane groups see 16 distinct columns) and for the P2 reads
//     (lane k2 + 16 n0 reads row n0 + 4 k2: 32-lane groups, row parity x column
//     distinct);
//   * twiddles from [k2][L] and [k1][n0] tables (contiguous / broadcast reads,
//     where W^(L k2) from one 1024-entry table was up to 8-way bank-conflicted);
//   * the final DFT4 over n0: a 4 x 4 lanes x registers transpose with the
//     gfx950 row swaps (P2 puts n0 in lane bits 4-5), then in registers, instead
//     of a third LDS round trip; stores stay 512 contiguous bytes in lane order.
using pk::f2;

struct ChanTw {
    f2 p1[15 * 64];  // W^(L k2), k2 = 1..15
    f2 p2[16 * 4];   // W^(16 n0 k1)
};

__device__ __forceinline__ void chan_tw_init(ChanTw& s, const f2* __restrict__ tw, int t, int nt) {
    for (int i = t; i < 15 * 64; i += nt) s.p1[i] = tw[((i & 63) * ((i >> 6) + 1)) & (kM - 1)];
    for (int i = t; i < 64; i += nt) s.p2[i] = tw[(16 * (i & 3) * (i >> 2)) & (kM - 1)];
}

// exchange between lane rows (gfx950 v_permlane16/32_swap): with S = 16 the odd
// 16-lane rows of a trade places with the even rows of b, with S = 32 the upper
// half of a with the lower half of b -- one step of a lanes x registers transpose
template <int S> __device__ __forceinline__ void row_swap(float& a, float& b) {
    const unsigned ua = __float_as_uint(a), ub = __float_as_uint(b);
    auto r = S == 16 ? __builtin_amdgcn_permlane16_swap(ua, ub, false, false)
                     : __builtin_amdgcn_permlane32_swap(ua, ub, false, false);
    a = __uint_as_float(r[0]);
    b = __uint_as_float(r[1]);
}
template <int S> __device__ __forceinline__ void row_swap(f2& a, f2& b) {
    float ax = a.x, ay = a.y, bx = b.x, by = b.y;
    row_swap<S>(ax, bx);
    row_swap<S>(ay, by);
    a = f2{ax, ay};
    b = f2{bx, by};
}

// PLAIN: plain instead of nontemporal stores (a lab variant, LAB bit 32 below)
template <bool PLAIN> __device__ __forceinline__ void st_nt2(f2* p, f2 v) {
    if constexpr (PLAIN) *p = v;
    else __builtin_nontemporal_store(v, p);
}

// one frame by one wave: buf holds v[p] at p; natural-order X to yf.  Packed
// FP32 throughout (sdsp_pk.hpp: each complex add / multiply is one or two
// v_pk_* instructions, the same per-component operation order as cmul / dft4 /
// tw16 above); pdft16 leaves X[k] of its 16 points at v[kout(k)].
// store false: the same sixteen store instructions go to an empty buffer descriptor (dropped), so
// every wave of a round issues the same number of memory operations -- the waits the compiler
// places for the next round's loads then let this round's stores stay in flight
typedef unsigned chan_u2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void chan_dummy_stores(f2* yf) {
    const auto rz = __builtin_amdgcn_make_buffer_rsrc((void*)yf, (short)0, 0, 0x00020000);
#pragma unroll
    for (int k = 0; k < 16; ++k)  // distinct offsets: identical stores would be merged into one
        __builtin_amdgcn_raw_buffer_store_b64(chan_u2{0u, 0u}, rz, 0, 8 * k, 2);
}
// AUX: the stores' cache policy (2 nontemporal; 16 write-through sc1, a lab variant)
template <int AUX = 2>
__device__ __forceinline__ void fft1024_chan(f2* __restrict__ buf, const ChanTw& tw, int L, f2* __restrict__ yf,
                                             bool store) {
    using pk::kout;
    // the swizzled addresses depend on the lane only: keep them from being
    // hoisted out of the caller's frame loop (32 loop-invariant VGPRs spill)
    asm volatile("" : "+v"(L));
    f2 v[16];
#pragma unroll
    for (int n2 = 0; n2 < 16; ++n2) v[n2] = buf[L + 64 * n2];
    pk::pdft16<false>(v);
#pragma unroll
    for (int k2 = 1; k2 < 16; ++k2) v[kout(k2)] = pk::pmul(v[kout(k2)], tw.p1[(k2 - 1) * 64 + L]);
    wave_sync();
    {
        // P1 lane L = n0 + 4 n1 writes row r = n0 + 4 k2, column n1
        const int n0 = L & 3, n1 = L >> 2;
        const int u = n1 ^ (n0 << 2);  // swz(r) = (n0 << 2) ^ k2
        f2* row = buf + n0 * 16;
#pragma unroll
        for (int k2 = 0; k2 < 16; ++k2) row[64 * k2 + (u ^ k2)] = v[kout(k2)];
    }
    wave_sync();
    // P2 lane L = k2 + 16 n0 reads row r = n0 + 4 k2 (n1 = 0..15)
    const int n0 = L >> 4, k2 = L & 15;
    {
        const int sw = (n0 << 2) ^ k2;
        const f2* row = buf + (n0 + 4 * k2) * 16;
#pragma unroll
        for (int i = 0; i < 16; ++i) v[i] = row[i ^ sw];
    }
    pk::pdft16<false>(v);
#pragma unroll
    for (int k1 = 1; k1 < 16; ++k1) v[kout(k1)] = pk::pmul(v[kout(k1)], tw.p2[k1 * 4 + n0]);
    // P3: per block of four k1 = 4 b + i, transpose lanes n0 (lane bits 4, 5) x
    // registers i, so lane (n0, k2) holds the four n0-inputs of k1 = 4 b + n0; an
    // in-register DFT4 then gives X[k2 + 16 (4 b + n0) + 256 k0] = X[L + 64 b + 256 k0]:
    // every store instruction writes 512 bytes in lane order (8-byte and paired
    // 16-byte stores measured the same on cfg5)
    const auto ry = __builtin_amdgcn_make_buffer_rsrc((void*)yf, (short)0, store ? kM * 8 : 0, 0x00020000);
#pragma unroll
    for (int bk = 0; bk < 4; ++bk) {
        f2 r[4] = {v[kout(4 * bk)], v[kout(4 * bk + 1)], v[kout(4 * bk + 2)], v[kout(4 * bk + 3)]};
        row_swap<16>(r[0], r[1]);
        row_swap<16>(r[2], r[3]);
        row_swap<32>(r[0], r[2]);
        row_swap<32>(r[1], r[3]);
        pk::pdft4<false>(r[0], r[1], r[2], r[3]);
#pragma unroll
        for (int k0 = 0; k0 < 4; ++k0)  // nontemporal (aux 2)
            __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(chan_u2, r[k0]), ry, (L + 64 * bk + 256 * k0) * 8, 0, AUX);
    }
}

// T = 1024: one branch per thread, sixteen frames per round, 136 KB of LDS
// (one workgroup per CU).  T = 512: two branches per thread, eight frames per
// round, 72 KB (two workgroups per CU, so one's loads overlap the other's
// PFB/FFT).  Twiddle tables in LDS for both.  PF (the default with T = 1024):
// the next round's loads are issued after the PFB, before the FFT's stores --
// vmcnt counts loads and stores in issue order, so loads issued after the
// stores would make every round wait for the previous round's stores
// (cfg5: 0.423 -> 0.414 ms against the 512-thread form, 25-round A/B).
// R (frames per round) defaults to one per wave; R = 8 / 4 with T = 1024 (SDSP_TUNE_CHAN_STREAMING
// = 5 / 6) halve / quarter the bytes a CU has in flight per round (R x 8 KB of loads and as
// many of stores) and transform the round's frames on waves 0..R-1.
// LAB selects compile-time variants for in-process A/B runs (tools/lab/chan_lab.hip; the
// product kernels are LAB = 0): 1 no FFT, 2 no loads, 4 no stores (ablations; 1 and 4 issue fewer
// than the sixteen stores per round that the PF / R = 8 form's vmcnt(16) wait counts on, so with
// that form they are timing ablations only, their outputs invalid); 8 / 16 odd
// workgroups start ~6.8 / ~3.4 us late; 32 plain stores; 64 nontemporal loads (16-byte and
// guarded paths); 128 write-through (sc1) stores; 256 plain (not nontemporal) round loads (the
// asm path; the round-3 product).
template <int K, int T, bool PF, int R = T / 64, int LAB = 0>
__global__ void __launch_bounds__(T, T == 1024 ? 4 : 2)  // 1024 lanes: 4 waves per SIMD, 128 VGPRs
chan1024_kernel(const f2* __restrict__ x, const f2* __restrict__ hist, const float* __restrict__ cb,
                f2* __restrict__ y, const f2* __restrict__ tw, long long n, long long frames, int F, int cps,
                int C, int xcd) {
    constexpr int kThreads = T, kNB = kM / T, kFrames = R;
    static_assert(R <= T / 64, "one frame per wave at most");
    // branch taps resident in LDS ([tap][branch], conflict-free) when they fit beside the frame
    // buffers; otherwise re-read from L2 every round
    constexpr bool kTapsLds = (size_t)R * kM * 8 + sizeof(ChanTw) + (size_t)K * kM * 4 <= 160 * 1024;
    // the PFB ring holds the last 8 inputs of a branch, slot = frame mod 8: rounds of fewer
    // than 8 frames run as 8 / R sub-rounds of one 8-frame step (compile-time slots)
    constexpr int kStep = R < 8 ? 8 : R;
    static_assert(kStep % 8 == 0 && kStep % R == 0, "ring slots are frame mod 8");
    __shared__ ChanTw stw;
    __shared__ f2 sbuf[kFrames * kM];
    __shared__ float ctap[kTapsLds ? K * kM : 1];
    const int t = threadIdx.x, L = t & 63, w = __builtin_amdgcn_readfirstlane(t >> 6);  // wave-uniform
    // chunks of F frames, C in all (cps per stream), walked by G resident
    // workgroups.  xcd: workgroup b runs on XCD b mod 8 (dispatch order), so XCD x
    // takes the contiguous range [x Q, (x+1) Q) of chunks, Q = ceil(C / 8), and its
    // G/8 workgroups step through it side by side: at any time an XCD streams one
    // window of neighbouring chunks (DRAM row locality), and a chunk's K-1 warm-up
    // frames were just read by the workgroup on the chunk before (same L2).
    // Without xcd: chunk b + k G.
    const unsigned G = gridDim.x, bid = blockIdx.x;
    constexpr int lab = LAB & 7;
    if constexpr ((LAB & 24) != 0) {
        if ((bid >> 3) & 1) {  // stagger: desynchronise the rounds of neighbouring workgroups
            constexpr int ns = ((LAB & 8) ? 2 : 0) + ((LAB & 16) ? 1 : 0);
            for (int i = 0; i < ns; ++i) __builtin_amdgcn_s_sleep(127);
        }
    }
    const unsigned Q = xcd ? (C + 7) / 8 : C, Gx = xcd ? G / 8 : G;
    const unsigned c_lo = xcd ? (bid & 7) * Q : 0, c_hi = c_lo + Q < (unsigned)C ? c_lo + Q : C;
    const unsigned c_first = c_lo + (xcd ? bid >> 3 : bid);
    const long long H = (long long)(K - 1) * kM;
    const f2* __restrict__ xs = x;
    const f2* __restrict__ hs = hist;
    f2* __restrict__ ys = y;
    long long m0 = 0, m_end = 0;
    chan_tw_init(stw, tw, t, kThreads);

    // Branch taps are re-read (L2-resident, 32 KB)
    // each round rather than held across the FFT: that keeps the FFT phase
    // inside 128 VGPRs (four waves per SIMD).  The pointer goes through an
    // empty asm so the loads stay inside the loop.
    // branches of this thread: T = 1024: p = t; T = 512: p = 2t + j, whose samples
    // x[f M + M-1-p] are adjacent -- one 16-byte load per frame (8-byte accesses
    // stream at well under the 16-byte rate)
    constexpr bool kPair = kNB == 2;
    auto branch = [&](int j) { return kPair ? 2 * t + j : t + kThreads * j; };
    auto load_pair = [&](const f2* xf, f2 (&v)[kNB]) {
        if constexpr (kPair) {
            const pk::f4v* qp = reinterpret_cast<const pk::f4v*>(xf + kM - 2 - 2 * t);
            pk::f4v q;
            if constexpr ((LAB & 64) != 0) q = __builtin_nontemporal_load(qp);
            else q = *qp;
            v[0] = f2{q.z, q.w};  // branch 2t:   x[M-1-2t]
            v[1] = f2{q.x, q.y};  // branch 2t+1: x[M-2-2t]
        } else {
            if constexpr ((LAB & 64) != 0) v[0] = __builtin_nontemporal_load(xf + kM - 1 - t);
            else v[0] = xf[kM - 1 - t];
        }
    };
    float c[kNB][K];
    if constexpr (kTapsLds) {
        for (int e = t; e < K * kM; e += kThreads) ctap[(e % K) * kM + e / K] = cb[e];  // cb[p K + i] -> [i][p]
    }
    auto load_taps = [&]() {
        if constexpr (kTapsLds) {
#pragma unroll
            for (int j = 0; j < kNB; ++j)
#pragma unroll
                for (int i = 0; i < K; ++i) c[j][i] = ctap[i * kM + branch(j)];
        } else {
            const float* cbp = cb;
            asm volatile("" : "+s"(cbp));
#pragma unroll
            for (int j = 0; j < kNB; ++j)
#pragma unroll
                for (int i = 0; i < K; ++i) c[j][i] = cbp[branch(j) * K + i];
        }
    };

    // input sample of branch p_j at frame f: x[f*M + M-1-p_j]; before the call: history
    auto ext = [&](long long f, int j) -> f2 {
        const long long q = f * kM + (kM - 1 - branch(j));
        if (q >= 0) return q < n ? xs[q] : f2{0.0f, 0.0f};
        return H + q >= 0 ? hs[H + q] : f2{0.0f, 0.0f};
    };

    f2 ring[kNB][8];

    // a round's new samples: plain loads when those frames exist (uniform test; a
    // per-load branch would serialise the HBM round trips), else guarded
    f2 nx[kFrames][kNB];
    // a round's frames f0 >= 0 read only the call's input: buffer loads bounded by the end of the
    // chunk (and of the call), so loads past it return zeros without traffic and every round
    // issues the same loads, with no branch (a branch around them makes the compiler wait for
    // all outstanding memory operations, this round's stores included, at the merge)
    auto load_round = [&](long long f0) {
        if (lab & 2) {
#pragma unroll
            for (int f = 0; f < kFrames; ++f)
#pragma unroll
                for (int j = 0; j < kNB; ++j) nx[f][j] = ring[j][(f + 3) & 7];
        } else {
            const long long q0 = f0 * kM, qe0 = m_end * kM, qe = qe0 < n ? qe0 : n, rem = qe - q0;
            const unsigned nrec = rem <= 0 ? 0u : (unsigned)((rem < (long long)kFrames * kM ? rem : (long long)kFrames * kM) * 8);
            const auto rx = __builtin_amdgcn_make_buffer_rsrc((void*)(xs + (rem > 0 ? q0 : 0)), (short)0, nrec, 0x00020000);
#pragma unroll
            for (int f = 0; f < kFrames; ++f) {
                if constexpr (kPair) {
                    const pk::f4v q = __builtin_bit_cast(pk::f4v, __builtin_amdgcn_raw_buffer_load_b128(
                                                                    rx, (unsigned)(f * kM + kM - 2 - 2 * t) * 8, 0, 0));
                    nx[f][0] = f2{q.z, q.w};  // branch 2t:   x[M-1-2t]
                    nx[f][1] = f2{q.x, q.y};  // branch 2t+1: x[M-2-2t]
                } else if constexpr (kFrames != 8 || !PF) {
                    nx[f][0] = __builtin_bit_cast(f2, __builtin_amdgcn_raw_buffer_load_b64(
                                                          rx, (unsigned)(f * kM + kM - 1 - t) * 8, 0, 0));
                } else {
                    // untracked by the compiler (its waits, merged over the loop's paths, would cover
                    // this round's stores too): the wait is wait_round's, after those stores
                    const unsigned long long a = (unsigned long long)(xs + (rem > 0 ? q0 : 0));
                    typedef unsigned u4s __attribute__((ext_vector_type(4)));
                    const u4s rw = {(unsigned)a, (unsigned)(a >> 32) & 0xffffu, nrec, 0x00020000u};
                    f2 r;
                    // nontemporal (the round's samples are read once): cfg5 sustained 0.388 ->
                    // 0.376 ms (profiles/r04/lab/r04ab_chanburst.log, r04ac_chanburst.log)
                    if constexpr ((LAB & 256) == 0)
                        asm volatile("buffer_load_dwordx2 %0, %1, %2, 0 offen nt"
                                     : "=v"(r)
                                     : "v"((unsigned)(f * kM + kM - 1 - t) * 8), "s"(rw)
                                     : "memory");
                    else
                        asm volatile("buffer_load_dwordx2 %0, %1, %2, 0 offen"
                                     : "=v"(r)
                                     : "v"((unsigned)(f * kM + kM - 1 - t) * 8), "s"(rw)
                                     : "memory");
                    nx[f][0] = r;
                }
            }
        }
    };
    // the prefetched round has landed: every wave issued exactly sixteen stores after its loads
    // (the frame's, or sixteen dropped ones), so vmcnt(16) waits for the loads alone
    auto wait_round = [&](bool first) {
        if constexpr (!kPair && kFrames == 8 && PF) {
            if (first) asm volatile("s_waitcnt vmcnt(0)" : "+v"(nx[0][0]), "+v"(nx[1][0]), "+v"(nx[2][0]), "+v"(nx[3][0]),
                                    "+v"(nx[4][0]), "+v"(nx[5][0]), "+v"(nx[6][0]), "+v"(nx[7][0]) :: "memory");
            else asm volatile("s_waitcnt vmcnt(16)" : "+v"(nx[0][0]), "+v"(nx[1][0]), "+v"(nx[2][0]), "+v"(nx[3][0]),
                              "+v"(nx[4][0]), "+v"(nx[5][0]), "+v"(nx[6][0]), "+v"(nx[7][0]) :: "memory");
        }
    };
    __syncthreads();

    for (unsigned ck = c_first; ck < c_hi; ck += Gx) {
        const int s = (int)(ck / cps);
        xs = x + (long long)s * n;
        ys = y + (long long)s * n;
        hs = hist + (long long)s * H;
        m0 = (long long)(ck - (unsigned)s * cps) * F;
        m_end = m0 + F < frames ? m0 + F : frames;
#pragma unroll
        for (int j = 0; j < kNB; ++j)
#pragma unroll
            for (int r = 0; r < 8; ++r) ring[j][r] = f2{0.0f, 0.0f};
        // warm-up: frames m0-1 .. m0-K+1 into slots 7 .. 8-K+1 (slot = frame - m0 mod 8)
        if (m0 >= K - 1) {  // uniform: plain loads (all in flight together)
#pragma unroll
            for (int q = 1; q < K; ++q) {
                f2 v[kNB];
                load_pair(xs + (m0 - q) * kM, v);
#pragma unroll
                for (int j = 0; j < kNB; ++j) ring[j][8 - q] = v[j];
            }
        } else {
#pragma unroll
            for (int q = 1; q < K; ++q)
#pragma unroll
                for (int j = 0; j < kNB; ++j) ring[j][8 - q] = ext(m0 - q, j);
        }
        // PF: the next round's samples are requested before this round's FFT stores,
        // so waiting for them (vmcnt counts loads and stores in issue order) never
        // waits for the stores
        if (PF) {
            load_round(m0);
            wait_round(true);  // the chunk's first round: once per chunk
        }
        for (long long mb = m0; mb < m_end; mb += kStep) {
            load_taps();
#pragma unroll
            for (int sub = 0; sub < kStep / kFrames; ++sub) {
                const long long mr = mb + (long long)sub * kFrames;
                if (sub > 0 && mr >= m_end) break;  // uniform (sub 0 starts below m_end)
                if (!PF) load_round(mr);
                // PFB: frame mr + g into buffer g (ring slot (sub R + g) mod 8); per component
                // acc = fma(c_i, h, acc), one v_pk_fma_f32 per tap
#pragma unroll
                for (int g = 0; g < kFrames; ++g) {
                    const int sl = sub * kFrames + g;
                    f2 pacc[kNB];
#pragma unroll
                    for (int j = 0; j < kNB; ++j) {
                        ring[j][sl & 7] = nx[g][j];
                        f2 acc = {0.0f, 0.0f};
#pragma unroll
                        for (int i = 0; i < K; ++i)
                            acc = __builtin_elementwise_fma(f2{c[j][i], c[j][i]}, ring[j][(sl - i) & 7], acc);
                        pacc[j] = acc;
                    }
                    if constexpr (kPair) {  // branches 2t, 2t+1: one 16-byte LDS store
                        *reinterpret_cast<pk::f4v*>(sbuf + g * kM + 2 * t) = pk::f4v{pacc[0].x, pacc[0].y, pacc[1].x, pacc[1].y};
                    } else {
#pragma unroll
                        for (int j = 0; j < kNB; ++j) sbuf[g * kM + t + kThreads * j] = pacc[j];
                    }
                }
                if (PF) load_round(mr + kFrames);  // past the chunk: zeros, no traffic
                __syncthreads();
                const long long f = mr + w;
                if (w >= kFrames) {  // uniform per wave: no frame for this wave in the round
                    chan_dummy_stores(ys);
                } else if (lab & 1) {
                    if (!(lab & 4) && f < m_end)
#pragma unroll
                        for (int k = 0; k < 16; ++k) st_nt2<(LAB & 32) != 0>(ys + f * kM + L + 64 * k, sbuf[w * kM + L + 64 * k]);
                } else {
                    fft1024_chan<(LAB & 128) ? 16 : 2>(sbuf + w * kM, stw, L, ys + f * kM, f < m_end && !(lab & 4));
                }
                if (PF) wait_round(false);
                __syncthreads();
            }
        }
    }
}

// Four-step pass with L = 1024, complex f32 (kern_fft.hip's fft_pass_kernel
// semantics, FftPass in sdsp_kernels.hpp): a workgroup runs 16 transforms, one
// per wave, on the register/LDS 1024-point FFT above.  The 16 transforms are
// consecutive t, whose elements interleave with unit stride on the strided side
// (S1 == 1 on input, T1 == 1 on output), so loads and stores move 128-byte runs.
// Reverse transforms conjugate in and out.  TW: the inter-pass twiddle
// W_Ntw^m = Th[m >> 10] * Tl[m & 1023] (Ntw = 2^20, twx = [Tl | Th], f64-derived).
constexpr int kPassBuf = kBuf + 4;  // wave-buffer stride: 16 buffers spread over LDS banks

template <bool INV, bool TW, int TPB>
__global__ void __launch_bounds__(64 * TPB)
fft1024_pass_kernel(const cf* __restrict__ x, cf* __restrict__ y, const cf* __restrict__ tw,
                    const cf* __restrict__ twx, long long count, long long G, long long S0, long long S1,
                    long long Si, long long T1, long long So) {
    // TPB = 16: 156 KB of LDS, one workgroup per CU, twiddles in LDS; TPB = 8: 74 KB,
    // two workgroups per CU (one's loads overlap the other's FFT), twiddles via L1
    constexpr int kT = 64 * TPB, kLog = TPB == 16 ? 4 : 3;
    __shared__ cf stw_l[TPB == 16 ? kM : 1];
    __shared__ cf sbuf[TPB * kPassBuf];
    __shared__ cf ktab[TW ? TPB * 16 : 1];  // W^(64 (g0 + c) k), k = 0..15 (c-fast outputs)
    const cf* stw = tw;
    const int t = threadIdx.x, L = t & 63, w = t >> 6;
    const long long t0 = (long long)blockIdx.x * TPB;
    const long long g0 = t0 % G;
    const long long ib = (t0 / G) * S0 + g0 * S1, ob = (t0 / G) * S0 + g0 * T1;
    const int ntr = count - t0 < TPB ? (int)(count - t0) : TPB;
    if constexpr (TPB == 16) {
        stw_l[t] = tw[t];
        stw = stw_l;
    }
    // inter-pass twiddle of c-fast output k of this thread: i = (t >> kLog) + 64 k, so
    // W^((g0 + c) i) = W^((g0 + c) (t >> kLog)) * W^(64 (g0 + c) k): one per-thread base
    // and a 16-entry row per column, each Th * Tl from the f64-built tables
    auto twx_at = [&](long long m) -> cf {
        const unsigned u = (unsigned)(m & ((1 << 20) - 1));
        return cmul(twx[1024 + (u >> 10)], twx[u & 1023]);
    };
    cf tbase = cf{1.0f, 0.0f};
    if constexpr (TW) {
        if (t < TPB * 16) ktab[t] = twx_at(64 * (g0 + (t >> 4)) * (long long)(t & 15));
        if (T1 == 1) tbase = twx_at((g0 + (t & (TPB - 1))) * (long long)(t >> kLog));
    }
    cf v[16];
    const bool cfast = S1 == 1;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        const int e = t + kT * k;
        const int c = cfast ? (e & (TPB - 1)) : (e >> 10), i = cfast ? (e >> kLog) : (e & 1023);
        v[k] = c < ntr ? x[ib + c * S1 + i * Si] : cf{0.0f, 0.0f};
    }
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        const int e = t + kT * k;
        const int c = cfast ? (e & (TPB - 1)) : (e >> 10), i = cfast ? (e >> kLog) : (e & 1023);
        sbuf[c * kPassBuf + i] = INV ? cf{v[k].re, -v[k].im} : v[k];
    }
    __syncthreads();
    fft1024_wave_lds(sbuf + w * kPassBuf, stw, L);
    __syncthreads();
    const bool ofast = T1 == 1;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        const int e = t + kT * k;
        const int c = ofast ? (e & (TPB - 1)) : (e >> 10), i = ofast ? (e >> kLog) : (e & 1023);
        if (c >= ntr) continue;
        cf r = sbuf[c * kPassBuf + i];
        if (INV) r.im = -r.im;
        if constexpr (TW) {
            cf wv = ofast ? cmul(tbase, ktab[c * 16 + k]) : twx_at((g0 + c) * (long long)i);
            if (INV) wv.im = -wv.im;
            r = cmul(r, wv);
        }
        y[ob + c * T1 + i * So] = r;
    }
}

// Persistent, software-pipelined form of the pass above (the default): grid = one
// 1024-thread workgroup per CU, workgroup b runs groups b, b + G, b + 2G, ... of TPB = 16
// transforms (8-transform groups in two 512-thread workgroups per CU measured 2.25 against
// 1.80 ms on cfg8, profiles/r04/lab/r04b_tune8_*.log).  The loads of the next group are issued
// into registers BEFORE the current group's FFT and stores, so each CU's HBM
// queue never drains while it transforms (the one-shot kernel alternated: load,
// barrier, FFT, barrier, store, with one 141 KB workgroup per CU and nothing else
// resident).  At step k the chip's workgroups run the neighbouring groups
// kG .. kG + G - 1: on the strided (column) side the rows they read are 32 KB
// contiguous runs.  Same arithmetic, element order and twiddles as
// fft1024_pass_kernel<INV, TW, TPB> (bit-identical).  PRE: next-group loads issued before
// the FFT (the rest after it).
// LA / SA: the loads' / stores' cache policy (0 default, 2 nontemporal; lab variants), LA & 8
// the skeleton without the FFT (lab), LA / SA & 16 16-byte lanes on the strided side (LA & 16 in
// the product), LA & 32 XCD-ordered groups (lab: 953 -> 970 us on the column pass), LA & 64 (lab)
// neighbouring groups paired on one XCD (workgroups b and b + 8 start on groups 2P and 2P + 1,
// so the two halves of each 2 x TPB-column run are read through one L2).  TPB = 8 (lab,
// tools/lab/chan_lab.hip, the column pass only): 512-thread workgroups, two per CU, the W1024
// table's first quarter in LDS (tw1024<true>: the 8 padded wave buffers and the whole table do
// not fit twice in 160 KB)
template <bool INV, bool TW, bool CFAST, bool OFAST, int TPB = 16, int PRE = 8, int LA = 0, int SA = 0>
__device__ __forceinline__ void fft1024_pipe_body(const cf* __restrict__ x, cf* __restrict__ y,
                                                  const cf* __restrict__ tw, const cf* __restrict__ twx,
                                                  long long count, long long G, long long S0, long long S1,
                                                  long long Si, long long T1, long long So) {
    static_assert(TPB == 16 || (TPB == 8 && CFAST && OFAST), "16 transforms per workgroup (8: the column pass)");
    constexpr int kT = 64 * TPB, kLog = TPB == 16 ? 4 : 3;
    constexpr int kPre = PRE;
    constexpr bool kQtw = TPB != 16;
    __shared__ cf stw[kQtw ? 256 : kM];
    __shared__ cf sbuf[TPB * kPassBuf];
    __shared__ cf ktab[TW ? TPB * 16 : 1];
    const int t = threadIdx.x, L = t & 63, w = t >> 6;
    const long long ngroups = count / TPB;
    if (!kQtw || t < 256) stw[t] = tw[t];
    auto twx_at = [&](long long m) -> cf {
        const unsigned u = (unsigned)(m & ((1 << 20) - 1));
        return cmul(twx[1024 + (u >> 10)], twx[u & 1023]);
    };
    constexpr bool cfast = CFAST, ofast = OFAST;  // compile-time: LDS offsets fold into immediates
    // group -> (input base, output base, first column g0)
    auto bases = [&](long long grp, long long& ib, long long& ob, long long& g0) {
        const long long t0 = grp * TPB;
        g0 = t0 % G;
        ib = (t0 / G) * S0 + g0 * S1;
        ob = (t0 / G) * S0 + g0 * T1;
    };
    // element k of thread t sits at lane offset + k * (scalar stride): buffer loads and
    // stores with one offset VGPR (64-bit addresses per element spill the pipeline's
    // registers).  cfast: c = t & (TPB - 1), i = (t >> kLog) + 64 k; else c = k, i = t.
    const unsigned in_lane = (unsigned)(cfast ? ((t & (TPB - 1)) + (long long)(t >> kLog) * Si) : (long long)t * Si) * 8u;
    const unsigned in_k = (unsigned)(cfast ? 64 * Si : S1) * 8u;
    const unsigned out_lane = (unsigned)(ofast ? ((t & (TPB - 1)) + (long long)(t >> kLog) * So) : (long long)t * So) * 8u;
    const unsigned out_k = (unsigned)(ofast ? 64 * So : T1) * 8u;
    // LA & 16 (the product when the input allows it): the strided-side loads in 16-byte lanes, lane t
    // holding columns 2 (t & 7) and 2 (t & 7) + 1 of rows (t >> 3) + 128 m, m = k / 2: half the load
    // instructions for the same bytes, the column pass 953 -> 918 us on cfg8, bit-identical
    // (profiles/r05/lab/r05u_fftlab_lanes.log; tools/stride_probe.hip: 128-byte runs 3.4 % faster in
    // 16-byte than in 8-byte lanes).  SA & 16 (lab only): the same for the strided-side stores
    // (slower: 1042 us, the twiddle base per column pair costs more than the stores save)
    constexpr bool wide_in = (LA & 16) != 0 && cfast, wide_out = (SA & 16) != 0 && ofast;
    // (TPB = 8: lane t holds columns 2 (t & 3), 2 (t & 3) + 1 of rows (t >> 2) + 128 m)
    constexpr int kHm = TPB / 2 - 1, kHs = kLog - 1;
    const unsigned in_lane16 = (unsigned)(2 * (t & kHm) + (long long)(t >> kHs) * Si) * 8u, in_k16 = (unsigned)(128 * Si) * 8u;
    const unsigned out_lane16 = (unsigned)(2 * (t & kHm) + (long long)(t >> kHs) * So) * 8u, out_k16 = (unsigned)(128 * So) * 8u;
    typedef unsigned u2v __attribute__((ext_vector_type(2)));
    typedef unsigned u4v __attribute__((ext_vector_type(4)));
    typedef float f4v __attribute__((ext_vector_type(4)));
    cf v[16];
    // past the last group (ok false): an empty descriptor, so the loads return zeros without touching
    // memory and every path issues the same loads -- no branch around them, whose merge would make
    // the compiler wait for all of them at once
    auto load = [&](long long grp, int k0, int k1, bool ok = true) {
        long long ib, ob, g0;
        bases(ok ? grp : 0, ib, ob, g0);
        const auto rx = __builtin_amdgcn_make_buffer_rsrc((void*)(x + ib), (short)0, ok ? 0x7fffffff : 0, 0x00020000);
        if constexpr (wide_in) {
#pragma unroll
            for (int m = k0 / 2; m < k1 / 2; ++m) {
                const f4v q = __builtin_bit_cast(f4v, __builtin_amdgcn_raw_buffer_load_b128(rx, in_lane16, m * in_k16, LA & 3));
                v[2 * m] = cf{q.x, q.y}, v[2 * m + 1] = cf{q.z, q.w};
            }
        } else {
#pragma unroll
            for (int k = k0; k < k1; ++k)
                v[k] = __builtin_bit_cast(cf, __builtin_amdgcn_raw_buffer_load_b64(rx, in_lane, k * in_k, LA & 3));
        }
    };
    // LA & 32 (lab): XCD-ordered groups, workgroup b on XCD b % 8 walking that XCD's contiguous
    // eighth (when the grid is a whole number of workgroups per XCD); the product form names
    // gridDim / ngroups directly
    auto next_of = [&](long long g) -> long long {
        if constexpr ((LA & 32) != 0) return g + ((gridDim.x & 7) == 0 ? gridDim.x >> 3 : gridDim.x);
        else return g + gridDim.x;
    };
    auto last = [&]() -> long long {
        if constexpr ((LA & 32) != 0) {
            const long long e = ((ngroups + 7) / 8) * ((blockIdx.x & 7) + 1);
            return (gridDim.x & 7) == 0 && e < ngroups ? e : ngroups;
        } else {
            return ngroups;
        }
    };
    long long grp = blockIdx.x;
    if constexpr ((LA & 64) != 0)
        if ((gridDim.x & 15) == 0) grp = ((blockIdx.x >> 4) << 4) + 2 * (blockIdx.x & 7) + ((blockIdx.x >> 3) & 1);
    if constexpr ((LA & 32) != 0)
        if ((gridDim.x & 7) == 0) grp = ((ngroups + 7) / 8) * (blockIdx.x & 7) + (blockIdx.x >> 3);
    if (grp >= last()) return;  // uniform
    load(grp, 0, 16);
    for (;;) {
        // stage the group's columns (waits for its loads: the previous stores may stay in flight)
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            const int e = t + kT * k;
            int c = cfast ? (e & (TPB - 1)) : (e >> 10), i = cfast ? (e >> kLog) : (e & 1023);
            if constexpr (wide_in) c = 2 * (t & kHm) + (k & 1), i = (t >> kHs) + 128 * (k >> 1);
            sbuf[c * kPassBuf + i] = INV ? cf{v[k].re, -v[k].im} : v[k];
        }
        long long ib, ob, g0;
        bases(grp, ib, ob, g0);
        cf tbase = cf{1.0f, 0.0f}, tbase1 = cf{1.0f, 0.0f};
        if constexpr (TW) {
            if (t < TPB * 16) ktab[t] = twx_at(64 * (g0 + (t >> 4)) * (long long)(t & 15));
            if constexpr (wide_out) {
                tbase = twx_at((g0 + 2 * (t & kHm)) * (long long)(t >> kHs));
                tbase1 = twx_at((g0 + 2 * (t & kHm) + 1) * (long long)(t >> kHs));
            } else if (ofast) {
                tbase = twx_at((g0 + (t & (TPB - 1))) * (long long)(t >> kLog));
            }
        }
        asm volatile("" : "+v"(tbase.re), "+v"(tbase.im));  // formed here, before the next group's loads
        if constexpr (wide_out) asm volatile("" : "+v"(tbase1.re), "+v"(tbase1.im));
        __syncthreads();
        // the next group's loads: half in flight across this group's FFT, half across its
        // stores.  Holding more of them through the FFT makes it spill (1024 threads: 128
        // VGPRs), and every scratch reload waits for all outstanding loads (vmcnt counts
        // scratch too): cfg8 2.09 ms with all sixteen, 1.79 with eight, 1.90 with four
        const long long nxt = next_of(grp);
        load(nxt, 0, kPre, nxt < last());
        // LA & 8 (lab only): the pass's skeleton -- loads, staging, twiddle and stores, no FFT
        if constexpr ((LA & 8) == 0) fft1024_wave_lds<kQtw>(sbuf + w * kPassBuf, stw, L);
        __syncthreads();
        load(nxt, kPre, 16, nxt < last());
        const auto ry = __builtin_amdgcn_make_buffer_rsrc((void*)(y + ob), (short)0, 0x7fffffff, 0x00020000);
        if constexpr (wide_out) {
#pragma unroll
            for (int m = 0; m < 8; ++m) {
                cf r[2];
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    const int c = 2 * (t & kHm) + j, i = (t >> kHs) + 128 * m;
                    r[j] = sbuf[c * kPassBuf + i];
                    if (INV) r[j].im = -r[j].im;
                    if constexpr (TW) {
                        cf wv = cmul(j ? tbase1 : tbase, ktab[c * 16 + 2 * m]);
                        if (INV) wv.im = -wv.im;
                        r[j] = cmul(r[j], wv);
                    }
                }
                __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4v, f4v{r[0].re, r[0].im, r[1].re, r[1].im}), ry,
                                                       out_lane16, m * out_k16, SA & 3);
            }
        } else {
#pragma unroll
            for (int k = 0; k < 16; ++k) {
                const int e = t + kT * k;
                const int c = ofast ? (e & (TPB - 1)) : (e >> 10), i = ofast ? (e >> kLog) : (e & 1023);
                cf r = sbuf[c * kPassBuf + i];
                if (INV) r.im = -r.im;
                if constexpr (TW) {
                    cf wv = ofast ? cmul(tbase, ktab[c * 16 + k]) : twx_at((g0 + c) * (long long)i);
                    if (INV) wv.im = -wv.im;
                    r = cmul(r, wv);
                }
                __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u2v, r), ry, out_lane, k * out_k, SA & 3);
            }
        }
        if (nxt >= last()) break;
        grp = nxt;
        __syncthreads();  // every read of sbuf / ktab done before the next group is staged
    }
}


template <bool INV, bool TW, bool CFAST, bool OFAST, int LA = 0, int SA = 0>
__global__ void __launch_bounds__(1024)
fft1024_pipe_kernel(const cf* __restrict__ x, cf* __restrict__ y, const cf* __restrict__ tw,
                    const cf* __restrict__ twx, long long count, long long G, long long S0, long long S1,
                    long long Si, long long T1, long long So) {
    fft1024_pipe_body<INV, TW, CFAST, OFAST, 16, 8, LA, SA>(x, y, tw, twx, count, G, S0, S1, Si, T1, So);
}


}  // namespace

// M = 1024, complex f32, K <= 8 taps per branch; false = not applicable.  LAB: chan1024_kernel
// (0 = the product kernels)
template <int LAB>
bool try_launch_chan1024_t(const ChanArgs& a, hipStream_t s, hipError_t* err) {
    if (a.M != 1024 || a.K < 1 || a.K > 8 || a.fast <= 0) return false;
    // the 512-thread form loads 16 bytes per lane: 1024-thread form for an input
    // that is only 8-byte aligned
    const int var = (a.fast == 2 || a.fast == 4) && ((uintptr_t)a.x & 15) ? 1 : a.fast;
    // chunk of F frames (a whole number of rounds); each chunk re-reads K-1 warm-up
    // frames (L2 hits when the neighbouring chunk is in flight on the same XCD)
    const int R = var == 2 || var == 4 || var == 5 || var == 6 ? 8 : 16;  // frames per step (chunks: whole steps)
    long long Fd = (long long)(a.frames * a.streams) / 512;
    Fd = Fd < 64 ? 64 : (Fd > 256 ? 256 : Fd);
    const int F = (int)(((a.frames_per_block > 0 ? a.frames_per_block : Fd) + R - 1) / R * R);
    const long long cps = ((long long)a.frames + F - 1) / F, C = cps * (long long)a.streams;
    if (C > (1LL << 30)) return false;
    // resident workgroups: 256 CUs x (2 of 512 threads | 1 of 1024)
    const long long resident = var == 2 || var == 4 ? 512 : 256;
    int xcd = a.xcd_order ? 1 : 0;
    long long G = C < resident ? C : resident;
    if (xcd) {
        G = G / 8 * 8;  // whole workgroups per XCD
        if (G == 0) xcd = 0, G = C;
    }
    dim3 grid((unsigned)G);
#define SDSP_CHAN_T(KV, T, PF, R)                                                                          \
    hipLaunchKernelGGL((chan1024_kernel<KV, T, PF, R, LAB>), grid, dim3(T), 0, s, (const f2*)a.x, (const f2*)a.hist, \
                       (const float*)a.cb, (f2*)a.y, (const f2*)a.tw, (long long)a.n, (long long)a.frames, F, (int)cps, \
                       (int)C, xcd)
#define SDSP_CHAN(KV)                                                   \
    case KV:                                                            \
        if (var == 2) SDSP_CHAN_T(KV, 512, false, 8);                   \
        else if (var == 3) SDSP_CHAN_T(KV, 1024, true, 16);             \
        else if (var == 4) SDSP_CHAN_T(KV, 512, true, 8);               \
        else if (var == 5) SDSP_CHAN_T(KV, 1024, true, 8);              \
        else if (var == 6) SDSP_CHAN_T(KV, 1024, true, 4);              \
        else SDSP_CHAN_T(KV, 1024, false, 16);                          \
        break;
    switch (a.K) {
        SDSP_CHAN(1) SDSP_CHAN(2) SDSP_CHAN(3) SDSP_CHAN(4) SDSP_CHAN(5) SDSP_CHAN(6) SDSP_CHAN(7) SDSP_CHAN(8)
    }
#undef SDSP_CHAN
#undef SDSP_CHAN_T
    *err = hipGetLastError();
    return true;
}

bool try_launch_chan1024(const ChanArgs& a, hipStream_t s, hipError_t* err) {
    return try_launch_chan1024_t<0>(a, s, err);
}

// four-step pass of L = 1024 on the wave FFT; false = not applicable.  LA / SA: the pipelined
// kernel's load / store policy (0 = the product)
template <int LA, int SA>
bool try_launch_fft1024_pass_t(const FftPass& p, hipStream_t s, hipError_t* err) {
    // p.wave1024 (SDSP_TUNE_FFT_WAVE1024): 16 (default) the pipelined persistent kernel, 1 the
    // one-shot kernel with 16 transforms per workgroup, 8 one-shot with 8, 0 the generic
    // Stockham pass
    const int tpb = p.wave1024 == 0 || p.wave1024 == 8 || p.wave1024 == 1 ? p.wave1024 : 16;
    if (tpb == 0 || p.L != 1024 || p.count % 16 != 0 || p.G % 16 != 0) return false;
    if (!(p.S1 == 1 || p.Si == 1) || !(p.T1 == 1 || p.So == 1)) return false;
    if (p.Ntw && (p.Ntw != (1LL << 20) || !p.twx)) return false;
    if (tpb == 16) {
        int dev = 0, cus = 256;  // (the current device's CU count)
        if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
        const long long groups = p.count / 16;
        const dim3 g2((unsigned)(groups < cus ? groups : cus));
        const bool cf_ = p.S1 == 1, of_ = p.T1 == 1;
        // 16-byte strided-side loads: every group's base and row offset 16-byte aligned
        const bool wide = cf_ && ((uintptr_t)p.x & 15) == 0 && (p.S0 & 1) == 0 && (p.Si & 1) == 0;
#define SDSP_PIPE5(INV, TW, C, O, LAV)                                                                              \
    hipLaunchKernelGGL((fft1024_pipe_kernel<INV, TW, C, O, LAV, SA>), g2, dim3(1024), 0, s, (const cf*)p.x, (cf*)p.y, \
                       (const cf*)p.tw, (const cf*)p.twx, p.count, p.G, p.S0, p.S1, p.Si, p.T1, p.So)
#define SDSP_PIPE4(INV, TW, C, O)                                            \
    do {                                                                      \
        if constexpr (C) {                                                    \
            if (wide) SDSP_PIPE5(INV, TW, C, O, (LA | 16));                   \
            else SDSP_PIPE5(INV, TW, C, O, LA);                               \
        } else {                                                              \
            SDSP_PIPE5(INV, TW, C, O, LA);                                    \
        }                                                                     \
    } while (0)
#define SDSP_PIPE(INV, TW)                                                                         \
    do {                                                                                           \
        if (cf_) { if (of_) SDSP_PIPE4(INV, TW, true, true); else SDSP_PIPE4(INV, TW, true, false); }   \
        else { if (of_) SDSP_PIPE4(INV, TW, false, true); else SDSP_PIPE4(INV, TW, false, false); } \
    } while (0)
        if (p.inverse) {
            if (p.Ntw) SDSP_PIPE(true, true); else SDSP_PIPE(true, false);
        } else {
            if (p.Ntw) SDSP_PIPE(false, true); else SDSP_PIPE(false, false);
        }
#undef SDSP_PIPE
#undef SDSP_PIPE4
#undef SDSP_PIPE5
        *err = hipGetLastError();
        return true;
    }
    dim3 grid((unsigned)(p.count / (tpb == 1 ? 16 : tpb)));
#define SDSP_P1024(INV, TW, TPB)                                                                                  \
    hipLaunchKernelGGL((fft1024_pass_kernel<INV, TW, TPB>), grid, dim3(64 * TPB), 0, s, (const cf*)p.x, (cf*)p.y, \
                       (const cf*)p.tw, (const cf*)p.twx, p.count, p.G, p.S0, p.S1, p.Si, p.T1, p.So)
#define SDSP_P1024_T(TPB)                                                                 \
    if (p.inverse) {                                                                      \
        if (p.Ntw) SDSP_P1024(true, true, TPB); else SDSP_P1024(true, false, TPB);        \
    } else {                                                                              \
        if (p.Ntw) SDSP_P1024(false, true, TPB); else SDSP_P1024(false, false, TPB);      \
    }
    if (tpb == 1) {
        SDSP_P1024_T(16)
    } else {
        SDSP_P1024_T(8)
    }
#undef SDSP_P1024_T
#undef SDSP_P1024
    *err = hipGetLastError();
    return true;
}

bool try_launch_fft1024_pass(const FftPass& p, hipStream_t s, hipError_t* err) {
    return try_launch_fft1024_pass_t<0, 0>(p, s, err);
}

}  // namespace sdsp
