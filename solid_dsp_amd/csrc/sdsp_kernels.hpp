// Internal launcher interface between the C-ABI runtime (runtime.cpp) and the
// kernel translation units.  Not installed; no torch types anywhere.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

namespace sdsp {

struct FirArgs {
    const void* x;         // device input, channel-major [channels][n]
    const void* hist;      // device history [channels][L-1], oldest first
    const void* taps_rev;  // device reversed taps cr[i] = h[L-1-i]
    const void* scale;     // host pointer to one Coef
    void* y;               // device output [channels][nout]
    size_t n, nout, channels;
    int L, M;
    size_t j0;             // block-relative index of the first emitting input (decimator)
    bool exact;
    int seg = 0;           // polyphase decimator: outputs per lane group (0 = auto)
};

hipError_t launch_fir_direct(int dtype, const FirArgs& a, hipStream_t s);
hipError_t launch_decim_direct(int dtype, const FirArgs& a, hipStream_t s);
// column-parallel polyphase decimator (kern_decim.hip); false = not applicable
bool try_launch_decim_poly(int dtype, const FirArgs& a, hipStream_t s, hipError_t* err);
hipError_t launch_hist_update(int dtype, const void* x, const void* old_hist, void* new_hist, size_t n, int Lm1,
                              size_t channels, hipStream_t s);

// overlap-save (N = 4096) for 32-bit complex samples
constexpr int kOlsOneShot = 0;     // interior segments: one-shot XCD-ordered kernel (kern_fir_ols_os.hip)
constexpr int kOlsPersistent = 1;  // persistent packed kernel, kOlsSegsPerBlock segments per workgroup
constexpr int kOlsScalar = 2;      // scalar persistent kernel for every segment (kern_fir_ols.hip)
constexpr int kOlsOneShotWide = 3;  // the one-shot kernel with 16-byte lanes (pair exchange by DPP)
constexpr int kOlsSegsPerBlock = 16;
// W4096 column bases [3][256], W256 row bases [3][16], then the first powers alone: {C1, D1}
// per column [256] and {E1, F1} per row [16] (kern_fir_ols_os.hip, runtime.cpp ols_build)
constexpr int kOlsOsTabCD = 768 + 48, kOlsOsTabEF = kOlsOsTabCD + 256;
constexpr int kOlsOsTabF4 = kOlsOsTabEF + 16;

struct OlsPlan {
    void* d_H;    // [256][16] c32: H[k0 + 16 k1 + 256 k2] / N * scale, row t = 16 k0 + k1
    void* d_tw1;  // [256][16] c32: W4096^(t*k)
    void* d_tw2;  // [16][16]  c32: W256^(a*b)
    int halo_rows;  // h2: halo = 256*h2 >= L-1
    int kernel = kOlsOneShot;
    void* d_pkt = nullptr;    // k-pair major tables: [0, 2048) float4 spectrum rows, [2048, 4096) W4096 rows,
                              // [4096, 4224) W256 rows (runtime.cpp ols_build)
    void* d_ostab = nullptr;  // one-shot kernel tables (kOlsOsTabF4 float4, runtime.cpp ols_build)
                              // (C1 C2 | C3 D1 | D2 D3), then [16][8] float4 W256 rows
    // real taps (conjugate-symmetric spectrum): the half-spectrum table of the one-shot kernel,
    // float4 [4][kOlsHalfRow] (runtime.cpp ols_build), else null
    void* d_hhalf = nullptr;
};
constexpr int kOlsHalfRow = 257;  // 256 lanes + the tail entry of lane (0, 0)
constexpr int kOlsN = 4096;
// new_hist: the next call's history buffer.  *hist_done = true when the launch also wrote it
// (the one-shot kernel does, for n >= L - 1); otherwise the caller runs the history update.
hipError_t launch_fir_ols(const OlsPlan& p, const void* x, const void* hist, void* new_hist, void* y, size_t n,
                          int L, size_t channels, int num_cus, hipStream_t s, bool* hist_done);
// interior segments [lo, hi) of a call: whole input window and all outputs inside the stream
void ols_interior_range(long long n, int h2, long long* lo, long long* hi);
// interior-segment kernels (16-byte rows)
hipError_t launch_fir_ols_os(const OlsPlan& p, const void* x, const void* hist, void* new_hist, void* y, size_t n,
                             int Lm1, size_t channels, hipStream_t s, bool wide);
hipError_t launch_fir_ols_pk(const OlsPlan& p, const void* x, void* y, size_t n, size_t channels, hipStream_t s,
                             long long lo, long long hi);

// polyphase filterbank / interpolator: out[j*M + p] = sum_{i<K} cb[p*K + i] * ext(j - i)
struct PfbArgs {
    const void* x;
    const void* hist;  // [channels][H] oldest first; ext(j<0) = hist[H + j]
    const void* cb;    // device branch coefs [M][K] (stored order, pfb.rs:33-40)
    void* y;           // [channels][n*M]
    size_t n, channels;
    int K, M, H;
    bool exact;
};
hipError_t launch_pfb(int dtype, const PfbArgs& a, hipStream_t s);

// one-sample FIR step (kern_fir_step.hip): shifts the delay line (last Lm1 of
// hist_in + sample -> hist_out), if emit writes one output to `out`, then
// releases *flag = seq (both host-mapped); the sample is passed by value
struct FirStepArgs {
    const void* sample;  // host pointer, copied into the launch
    const void* hist_in;
    void* hist_out;
    const void* taps_rev;
    const void* scale;  // host pointer to one Coef
    void* out;
    unsigned* flag;
    unsigned seq;
    int Lm1, L;
    bool emit, exact;
};
hipError_t launch_fir_step(int dtype, const FirStepArgs& a, hipStream_t s);

// IIR: SOS cascade (sections > 0) or Normal DF-II (sections == 0)
struct IirArgs {
    const void* x;
    void* y;
    const void* coefs;   // SOS: [S][5] (b0,b1,b2,a1,a2)/a0 ; Normal: num[nb] then den[na-1]
    const void* P;       // scan: [8][2S][2S] A^(B 2^k) (Coef type)
    const void* st_in;   // [channels][state]
    void* st_out;
    size_t n, nout, channels;
    int sections, nb, na, cap;
    int Mi, Md;          // interpolation (zero stuffing) / decimation factors
    size_t phase;        // DecimatingIIRFilter index before this block
    bool algo_scan;
    int wc;              // warm-up chunks (scan)
    const void* Cr = nullptr;  // wave scan: [B][2S] output response to the state, c A^i (Coef type)
    int ws_variant = 0;        // wave scan chunk: 0 = 256 bytes, 1 = 128 bytes
    // exact inter-wave carries (wc == 0: cascades whose state response does not decay):
    // Phi[t-1] = A^(64 B t) (t = tiles per wave, 1..8), scratch G / Cin [channels][waves][2S]
    const void* Phi = nullptr;
    void* G = nullptr;
    void* Cin = nullptr;
    size_t scratch_waves = 0;  // capacity of G / Cin per channel
};
// waves the exact-carry wave scan launches for this call (sizes G / Cin)
size_t iir_wscan_waves(int dtype, const IirArgs& a, int* tpw = nullptr);  // waves (and tiles per wave) of one call
hipError_t launch_iir(int dtype, const IirArgs& a, hipStream_t s);
int iir_scan_chunk(int dtype);  // samples per lane chunk of the scan kernel
// wave-level scan (kern_iir_wscan.hip): SOS cascades, with rate changes; wc <= 32
// warm-up chunks, or wc == 0 with Phi/G/Cin: aggregate pass, carry scan, output pass
hipError_t launch_iir_wscan(int dtype, const IirArgs& a, hipStream_t s);
int iir_wscan_chunk(int dtype, int variant);  // samples per lane chunk of the wave scan

// batched FFT (power of two: Stockham in LDS; otherwise direct DFT)
struct FftArgs {
    const void* x;
    void* y;
    const void* tw;  // [N] e^{-j 2 pi m / N}
    int N, logN;
    bool pow2, inverse;
    size_t batch;
};
hipError_t launch_fft(bool f64, const FftArgs& a, hipStream_t s);
// strided pass of the four-step FFT (kern_fft.hip fft_pass_kernel); Ntw = 0: no inter-pass twiddle
struct FftPass {
    const void* x;
    void* y;
    const void* tw;  // [L] e^{-j 2 pi m / L}
    int L, logL;
    long long count, G, S0, S1, Si, T1, So, Ntw;
    bool inverse;
    const void* twx = nullptr;  // c32 [Tl | Th] inter-pass twiddle tables when Ntw = 2^20 (L = 1024 path)
    int group = 4;      // generic pass: at most this many transforms per workgroup (SDSP_TUNE_FFT_GROUP)
    int wave1024 = 16;  // L = 1024 c32 passes (SDSP_TUNE_FFT_WAVE1024): 16 pipelined persistent kernel,
                        // 1 / 8 one-shot with 16 / 8 transforms per workgroup, 0 the generic pass
};
// L = 1024, complex f32 pass on the wave FFT (kern_chan1024.hip); false = not applicable
bool try_launch_fft1024_pass(const FftPass& p, hipStream_t s, hipError_t* err);
hipError_t launch_fft_pass(bool f64, const FftPass& p, hipStream_t s);
// Bluestein steps: 0 chirp in (x[N] -> a[M], zero padded), 1 a *= B, 2 chirp out (a -> y[N])
hipError_t launch_bluestein(bool f64, int step, const void* in, void* out, const void* w_or_B, long long N, long long M,
                            long long batch, hipStream_t s);

// PFB + FFT channeliser (M power of two)
struct ChanArgs {
    const void* x;     // [streams][n]
    const void* hist;  // [streams][(K-1) M]
    const void* cb;    // [M][K] real branch coefficients (stored order)
    void* y;           // [streams][frames][M]
    const void* tw;
    int M, logM, K;
    size_t n, frames, streams;
    int fast = 3;  // streaming kernel where it applies: 0 off, 1/3 = 1024-thread, 2/4 = 512-thread, 3/4 prefetching (sdsp_chan_set_tuning)
    int frames_per_block = 0;  // streaming kernel: frames per workgroup (0 = default)
    bool xcd_order = true;     // streaming kernel: XCD-contiguous chunk order
};
hipError_t launch_chan(bool f64, const ChanArgs& a, hipStream_t s);
// streaming M = 1024 kernel (kern_chan1024.hip); false = not applicable
bool try_launch_chan1024(const ChanArgs& a, hipStream_t s, hipError_t* err);

// batched DotProduct::execute
struct DotArgs {
    const void* coefs;
    int it;  // min(samples, len)
    const void* s;
    size_t stride, batch;
    void* out;
};
hipError_t launch_dot(int dtype, const DotArgs& a, hipStream_t s);

// AutoCorrelator (kern_rx.hip); prec 0 = complex f32, 1 = complex f64.  hist: [channels][H]
// oldest first (H = window size), K = max(W - delay, 0) product terms per output
// kernel (SDSP_TUNE_ACORR_KERNEL): 0 the pipelined kernel on interior tiles where it applies, else the
// one-shot kernel staging the delayed input in LDS; 1 the one-shot kernel everywhere (staged); 2 the
// one-shot kernel with two loads per product (no staging)
hipError_t launch_acorr(int prec, const void* x, const void* hist, void* y, size_t n, int H, int d, int K,
                        size_t channels, hipStream_t s, int kernel = 0);
hipError_t launch_acorr_current(int prec, const void* hist, void* out, int H, int d, int K, size_t channels,
                                hipStream_t s);
hipError_t launch_acorr_energy(int prec, const void* x, const void* hist, size_t n, int H, int W, size_t channels,
                               double* energy, hipStream_t s);
// NCO mix_up / mix_down over a block (kern_rx.hip): theta_i = theta0 + i dtheta (u32)
hipError_t launch_nco_mix(int prec, bool down, const void* x, void* y, size_t n, const double* table, uint32_t theta0,
                          uint32_t dtheta, int num_cus, hipStream_t s);
// AGC bank (src/auto_gain_control/mod.rs): state is sdsp_agc_state[channels] in
// device memory; cplx = Complex<f64> samples, else f64
// pipe: agc_pipe_kernel for calls it admits (SDSP_TUNE_AGC_KERNEL 0), else agc_kernel
hipError_t launch_agc(bool cplx, const void* x, void* y, size_t n, void* state, size_t channels, hipStream_t s,
                      bool pipe = true);
hipError_t launch_agc_init(bool cplx, const void* x, size_t n, void* state, double* levels, size_t channels,
                           hipStream_t s);

hipError_t launch_bw_copy(const void* a, void* b, size_t bytes, int num_cus, hipStream_t s);
hipError_t launch_synth_f32(float* out, uint64_t seed, uint64_t channel, uint64_t start, size_t count,
                            hipStream_t s);

}  // namespace sdsp
