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
//       P2 lane (n0, k2):      DFT16 over n1, * W1024^(16 n0 k1)
//       P3 lane l, c = l + 64 j: DFT4 over n0 -> X[c + 256 k0] (coalesced stores)
//     with two wave-local LDS transposes, so the four FFTs need no workgroup
//     barrier.  Outputs: natural channel order, as kern_fft.hip.
// Arithmetic: fused multiply-add, f32; parity is the §8d tolerance against the
// f64 restatement (tests/test_gpu_fft.py).
#include "sdsp_device.hpp"
#include <cstdlib>

#include "sdsp_kernels.hpp"

namespace sdsp {

namespace {

struct cf { float re, im; };
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

typedef float f2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void st_nt(cf* p, cf v) {  // one 8-byte streaming store
    __builtin_nontemporal_store(f2v{v.re, v.im}, reinterpret_cast<f2v*>(p));
}

constexpr int kM = 1024;
constexpr int kThreads = 1024;           // one branch per thread, 16 waves
constexpr int kNB = kM / kThreads;       // branches per thread
constexpr int kFrames = kThreads / 64;   // frames per round: one FFT per wave

// Wave buffer: 64 rows of 18 complex (16 + 2 pad): every LDS address below is
// a lane base plus a compile-time offset, and 16 lanes reading the same slot
// of 16 consecutive rows hit distinct banks.
constexpr int kRow = 18;
constexpr int kBuf = 64 * kRow;

// P1 and P2 of one wave's 1024-point FFT: buffer holds v[p] at index p on
// entry; on exit the P3 inputs of column c = (k2 + 16 k1) sit at buf[4 c + n0]
__device__ __forceinline__ void fft1024_p12(cf* __restrict__ buf, const cf* __restrict__ stw, int L) {
    cf v[16];
#pragma unroll
    for (int n2 = 0; n2 < 16; ++n2) v[n2] = buf[L + 64 * n2];
    dft16(v);
#pragma unroll
    for (int k2 = 1; k2 < 16; ++k2) v[k2] = cmul(v[k2], stw[(L * k2) & (kM - 1)]);
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
    for (int k1 = 1; k1 < 16; ++k1) v[k1] = cmul(v[k1], stw[(16 * n0 * k1) & (kM - 1)]);
    wave_sync();
    const int k2 = L >> 2;
#pragma unroll
    for (int k1 = 0; k1 < 16; ++k1) buf[(k2 + 16 * k1) * 4 + n0] = v[k1];
    wave_sync();
}

// one frame's FFT by one wave: buffer holds v[p] at index p on entry,
// natural-order X written to yf
__device__ __forceinline__ void fft1024_wave(cf* __restrict__ buf, const cf* __restrict__ stw, int L,
                                             cf* __restrict__ yf, bool store) {
    fft1024_p12(buf, stw, L);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int c = L + 64 * j;
        cf a0 = buf[c * 4 + 0], a1 = buf[c * 4 + 1], a2 = buf[c * 4 + 2], a3 = buf[c * 4 + 3];
        dft4(a0, a1, a2, a3);
        if (store) {
            st_nt(yf + c, a0);
            st_nt(yf + c + 256, a1);
            st_nt(yf + c + 512, a2);
            st_nt(yf + c + 768, a3);
        }
    }
    wave_sync();
}

// the same FFT leaving natural-order X in buf[0, 1024)
__device__ __forceinline__ void fft1024_wave_lds(cf* __restrict__ buf, const cf* __restrict__ stw, int L) {
    fft1024_p12(buf, stw, L);
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

template <int K>
__global__ void __launch_bounds__(kThreads)
chan1024_kernel(const cf* __restrict__ x, const cf* __restrict__ hist, const float* __restrict__ cb,
                cf* __restrict__ y, const cf* __restrict__ tw, long long n, long long frames, int F) {
    __shared__ cf stw[kM];
    __shared__ cf sbuf[kFrames * kBuf];
    const int t = threadIdx.x, L = t & 63, w = t >> 6;
    const int s = blockIdx.y;
    const long long H = (long long)(K - 1) * kM;
    static_assert(kFrames % 8 == 0, "ring slots are frame mod 8");
    x += (long long)s * n;
    y += (long long)s * n;
    hist += (long long)s * H;
    const long long m0 = (long long)blockIdx.x * F;
    const long long m_end = m0 + F < frames ? m0 + F : frames;
    for (int i = t; i < kM; i += kThreads) stw[i] = tw[i];

    // branches p_j = t + kThreads j
    float c[kNB][K];
#pragma unroll
    for (int j = 0; j < kNB; ++j)
#pragma unroll
        for (int i = 0; i < K; ++i) c[j][i] = cb[(t + kThreads * j) * K + i];

    // input sample of branch p_j at frame f: x[f*M + M-1-p_j]; before the call: history
    auto ext = [&](long long f, int j) -> cf {
        const long long q = f * kM + (kM - 1 - t - kThreads * j);
        if (q >= 0) return q < n ? x[q] : cf{0.0f, 0.0f};
        return H + q >= 0 ? hist[H + q] : cf{0.0f, 0.0f};
    };

    cf ring[kNB][8];
#pragma unroll
    for (int j = 0; j < kNB; ++j)
#pragma unroll
        for (int r = 0; r < 8; ++r) ring[j][r] = cf{0.0f, 0.0f};
    // warm-up: frames m0-1 .. m0-K+1 into slots 7 .. 8-K+1 (slot = frame - m0 mod 8)
#pragma unroll
    for (int q = 1; q < K; ++q)
#pragma unroll
        for (int j = 0; j < kNB; ++j) ring[j][8 - q] = ext(m0 - q, j);

    // a round's new samples: plain loads when those frames exist (uniform test; a
    // per-load branch would serialise the HBM round trips), else guarded
    // a round's new samples: plain loads when those frames exist (uniform test; a
    // per-load branch would serialise the HBM round trips), else guarded
    cf nx[kFrames][kNB];
    auto load_round = [&](long long f0) {
        if (f0 + kFrames <= frames) {
            const int off = kM - 1 - t;  // uniform frame base (SGPRs) + 32-bit lane offset
#pragma unroll
            for (int f = 0; f < kFrames; ++f) {
                const cf* xf = x + (f0 + f) * kM;
#pragma unroll
                for (int j = 0; j < kNB; ++j) nx[f][j] = xf[off - kThreads * j];
            }
        } else {
#pragma unroll
            for (int f = 0; f < kFrames; ++f)
#pragma unroll
                for (int j = 0; j < kNB; ++j) nx[f][j] = ext(f0 + f, j);
        }
    };
    __syncthreads();

    for (long long mb = m0; mb < m_end; mb += kFrames) {
        load_round(mb);
        // PFB: frame mb + g into buffer g (ring slot g mod 8)
#pragma unroll
        for (int g = 0; g < kFrames; ++g) {
#pragma unroll
            for (int j = 0; j < kNB; ++j) {
                ring[j][g & 7] = nx[g][j];
                cf acc = {0.0f, 0.0f};
#pragma unroll
                for (int i = 0; i < K; ++i) {
                    const cf h = ring[j][(g - i) & 7];
                    acc.re = __builtin_fmaf(c[j][i], h.re, acc.re);
                    acc.im = __builtin_fmaf(c[j][i], h.im, acc.im);
                }
                sbuf[g * kBuf + t + kThreads * j] = acc;
            }
        }
        __syncthreads();
        const long long f = mb + w;
        fft1024_wave(sbuf + w * kBuf, stw, L, y + f * kM, f < m_end);
        __syncthreads();
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

}  // namespace

// M = 1024, complex f32, K <= 8 taps per branch; false = not applicable
bool try_launch_chan1024(const ChanArgs& a, hipStream_t s, hipError_t* err) {
    if (a.M != 1024 || a.K < 1 || a.K > 8) return false;
    // frames per workgroup (multiple of kFrames): each workgroup re-reads K-1 warm-up frames
    // default: as long as the grid keeps >= ~2 workgroups per CU (measured on cfg5: 64 -> 256
    // frames per workgroup 0.525 -> 0.499 ms, warm-up traffic 11% -> 3%)
    long long Fd = (long long)(a.frames * a.streams) / 512;
    Fd = Fd < 64 ? 64 : (Fd > 256 ? 256 : Fd);
    const int F = (int)(((a.frames_per_block > 0 ? a.frames_per_block : Fd) + kFrames - 1) / kFrames * kFrames);
    static_assert(64 % kFrames == 0, "F");
    dim3 grid((unsigned)((a.frames + F - 1) / F), (unsigned)a.streams);
#define SDSP_CHAN(KV)                                                                                          \
    case KV:                                                                                                   \
        hipLaunchKernelGGL((chan1024_kernel<KV>), grid, dim3(kThreads), 0, s, (const cf*)a.x, (const cf*)a.hist,    \
                           (const float*)a.cb, (cf*)a.y, (const cf*)a.tw, (long long)a.n, (long long)a.frames, F); \
        break;
    switch (a.K) {
        SDSP_CHAN(1) SDSP_CHAN(2) SDSP_CHAN(3) SDSP_CHAN(4) SDSP_CHAN(5) SDSP_CHAN(6) SDSP_CHAN(7) SDSP_CHAN(8)
    }
#undef SDSP_CHAN
    *err = hipGetLastError();
    return true;
}

// four-step pass of L = 1024 on the wave FFT; false = not applicable
bool try_launch_fft1024_pass(const FftPass& p, hipStream_t s, hipError_t* err) {
    static const int tpb = [] {
        const char* e = std::getenv("SDSP_FFT_WAVE1024");
        const int v = e ? std::atoi(e) : 16;
        return v == 0 || v == 8 ? v : 16;
    }();
    if (tpb == 0 || p.L != 1024 || p.count % tpb != 0 || p.G % tpb != 0) return false;
    if (!(p.S1 == 1 || p.Si == 1) || !(p.T1 == 1 || p.So == 1)) return false;
    if (p.Ntw && (p.Ntw != (1LL << 20) || !p.twx)) return false;
    dim3 grid((unsigned)(p.count / tpb));
#define SDSP_P1024(INV, TW, TPB)                                                                                  \
    hipLaunchKernelGGL((fft1024_pass_kernel<INV, TW, TPB>), grid, dim3(64 * TPB), 0, s, (const cf*)p.x, (cf*)p.y, \
                       (const cf*)p.tw, (const cf*)p.twx, p.count, p.G, p.S0, p.S1, p.Si, p.T1, p.So)
#define SDSP_P1024_T(TPB)                                                                 \
    if (p.inverse) {                                                                      \
        if (p.Ntw) SDSP_P1024(true, true, TPB); else SDSP_P1024(true, false, TPB);        \
    } else {                                                                              \
        if (p.Ntw) SDSP_P1024(false, true, TPB); else SDSP_P1024(false, false, TPB);      \
    }
    if (tpb == 16) {
        SDSP_P1024_T(16)
    } else {
        SDSP_P1024_T(8)
    }
#undef SDSP_P1024_T
#undef SDSP_P1024
    *err = hipGetLastError();
    return true;
}

}  // namespace sdsp
