// C-ABI runtime for FFT (src/fft/mod.rs:175-215), the PFB + FFT channeliser
// (build-defined) and batched DotProduct::execute
// (src/dot_product/mod.rs:153-171).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <string>
#include <vector>

#include "sdsp.h"
#include "sdsp_host.hpp"
#include "sdsp_kernels.hpp"

using namespace sdsp;

namespace {

#define F_TRY(expr, what)                                      \
    do {                                                       \
        hipError_t _e = (expr);                                \
        if (_e != hipSuccess) return device_status(_e, what);  \
    } while (0)

struct Guard {
    int prev = -1;
    explicit Guard(int d) {
        (void)hipGetDevice(&prev);
        if (prev != d) (void)hipSetDevice(d);
    }
    ~Guard() {
        int cur = -1;
        (void)hipGetDevice(&cur);
        if (prev >= 0 && cur != prev) (void)hipSetDevice(prev);
    }
};

int check_gfx950(int device) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0 || device < 0 || device >= n) {
        set_error("no HIP device visible (libsdsp has no CPU execution path)");
        return SDSP_E_NO_DEVICE;
    }
    hipDeviceProp_t p;
    if (hipGetDeviceProperties(&p, device) != hipSuccess || std::strncmp(p.gcnArchName, "gfx950", 6) != 0) {
        set_error("libsdsp is built for gfx950");
        return SDSP_E_NO_DEVICE;
    }
    return SDSP_OK;
}

bool is_pow2(size_t n) { return n && !(n & (n - 1)); }
int ilog2(size_t n) {
    int l = 0;
    while ((size_t)1 << l < n) ++l;
    return l;
}

// e^{-j 2 pi m / N}, computed in f64, stored as c32 or c64
int make_twiddles(DevBuf& buf, size_t N, bool f64) {
    std::vector<double> w(2 * N);
    for (size_t m = 0; m < N; ++m) {
        const double a = -2.0 * M_PI * (double)m / (double)N;
        w[2 * m] = std::cos(a);
        w[2 * m + 1] = std::sin(a);
    }
    if (f64) {
        F_TRY(buf.ensure(w.size() * 8), "alloc twiddles");
        F_TRY(hipMemcpy(buf.p, w.data(), w.size() * 8, hipMemcpyHostToDevice), "copy twiddles");
    } else {
        std::vector<float> f(w.begin(), w.end());
        F_TRY(buf.ensure(f.size() * 4), "alloc twiddles");
        F_TRY(hipMemcpy(buf.p, f.data(), f.size() * 4, hipMemcpyHostToDevice), "copy twiddles");
    }
    return SDSP_OK;
}

}  // namespace

namespace {

// power-of-two transform: Stockham in LDS (N <= 4096) or the four-step
// decomposition N = N1 N2 (two strided passes, inter-pass twiddle) above
struct Pow2Plan {
    size_t N = 0;
    int group = 4, wave1024 = 16;  // pass kernel knobs (SDSP_TUNE_FFT_GROUP / SDSP_TUNE_FFT_WAVE1024)
    int logN = 0, l1 = 0, l2 = 0;
    DevBuf tw, tw1, tw2, twx;
    bool four_step() const { return N > 4096; }
    int build(size_t n, bool f64) {
        N = n;
        logN = ilog2(n);
        if (!four_step()) return make_twiddles(tw, N, f64);
        l1 = logN / 2;
        l2 = logN - l1;
        int st = make_twiddles(tw1, (size_t)1 << l1, f64);
        if (st) return st;
        st = make_twiddles(tw2, (size_t)1 << l2, f64);
        if (st || f64 || l1 != 10 || l2 != 10) return st;
        // 2^20 = 1024 x 1024, complex f32: the wave-FFT passes take the inter-pass
        // twiddle W_N^m as Th[m >> 10] * Tl[m & 1023] (each from f64)
        std::vector<float> t(4 * 1024);
        for (int j = 0; j < 1024; ++j) {
            const double a = -2.0 * M_PI * (double)j / (double)N, b = -2.0 * M_PI * (double)j * 1024.0 / (double)N;
            t[2 * j] = (float)std::cos(a);
            t[2 * j + 1] = (float)std::sin(a);
            t[2048 + 2 * j] = (float)std::cos(b);
            t[2048 + 2 * j + 1] = (float)std::sin(b);
        }
        F_TRY(twx.ensure(t.size() * 4), "alloc twiddles");
        F_TRY(hipMemcpy(twx.p, t.data(), t.size() * 4, hipMemcpyHostToDevice), "copy twiddles");
        return SDSP_OK;
    }
    // in -> out (may alias); tmp: batch * N samples when four_step()
    hipError_t run(bool f64, const void* in, void* out, void* tmp, size_t batch, bool inverse, hipStream_t s) const {
        if (!four_step()) {
            FftArgs a{in, out, tw.p, (int)N, logN, true, inverse, batch};
            return launch_fft(f64, a, s);
        }
        const long long n = (long long)N, N1 = 1LL << l1, N2 = 1LL << l2;
        // pass 1: columns n2 (length N1, stride N2) -> tmp[k1][n2] * W_N^(n2 k1)
        FftPass p1{in, tmp, tw1.p, (int)N1, l1, (long long)batch * N2, N2, n, 1, N2, 1, N2, n, inverse, twx.p,
                   group, wave1024};
        hipError_t e = launch_fft_pass(f64, p1, s);
        if (e != hipSuccess) return e;
        // pass 2: rows k1 (length N2) -> out[k1 + N1 k2]
        FftPass p2{tmp, out, tw2.p, (int)N2, l2, (long long)batch * N1, N1, n, N2, 1, 1, N1, 0, inverse, nullptr,
                   group, wave1024};
        return launch_fft_pass(f64, p2, s);
    }
};

// iterative radix-2 FFT in f64 on the host (Bluestein filter spectrum, plan time only)
void host_fft_pow2(std::vector<double>& a, size_t M) {
    for (size_t i = 1, j = 0; i < M; ++i) {
        size_t bit = M >> 1;
        for (; j & bit; bit >>= 1) j ^= bit;
        j ^= bit;
        if (i < j) {
            std::swap(a[2 * i], a[2 * j]);
            std::swap(a[2 * i + 1], a[2 * j + 1]);
        }
    }
    for (size_t len = 2; len <= M; len <<= 1) {
        for (size_t k = 0; k < len / 2; ++k) {
            const double ang = -2.0 * M_PI * (double)k / (double)len;
            const double wr = std::cos(ang), wi = std::sin(ang);
            for (size_t i = 0; i < M; i += len) {
                double* u = &a[2 * (i + k)];
                double* v = &a[2 * (i + k + len / 2)];
                const double tr = v[0] * wr - v[1] * wi, ti = v[0] * wi + v[1] * wr;
                v[0] = u[0] - tr;
                v[1] = u[1] - ti;
                u[0] += tr;
                u[1] += ti;
            }
        }
    }
}

int upload(DevBuf& buf, const std::vector<double>& v, bool f64) {
    if (f64) {
        F_TRY(buf.ensure(v.size() * 8), "alloc");
        F_TRY(hipMemcpy(buf.p, v.data(), v.size() * 8, hipMemcpyHostToDevice), "upload");
    } else {
        std::vector<float> f(v.begin(), v.end());
        F_TRY(buf.ensure(f.size() * 4), "alloc");
        F_TRY(hipMemcpy(buf.p, f.data(), f.size() * 4, hipMemcpyHostToDevice), "upload");
    }
    return SDSP_OK;
}

constexpr size_t kDirectMax = 512;  // non-power-of-two sizes up to this run the direct DFT

}  // namespace

struct sdsp_fft {
    size_t N = 0;
    int direction = 0;  // 0 FORWARD, 1 REVERSE
    bool f64 = true;
    int device = 0;
    int kind = 0;       // 0 direct DFT, 1 power of two, 2 Bluestein
    DevBuf tw, stage_in, stage_out;
    Pow2Plan p2;        // kind 1: the transform; kind 2: the length-M convolution transform
    size_t M = 0;       // Bluestein convolution length (power of two >= 2N - 1)
    DevBuf chirp, spec; // Bluestein: w[N] of the direction, B[M] = FFT_M(conj chirp) / M
    DevBuf work, tmp;   // device scratch, grown with the batch
    hipStream_t stream = nullptr;
};

struct sdsp_chan {
    int dtype = SDSP_RC32, device = 0;
    size_t M = 0, K = 0, streams = 1;
    std::vector<unsigned char> taps;
    DevBuf cb, tw, hist[2], stage_in, stage_out;
    int cur = 0;
    int fast = 5;  // streaming M = 1024 kernel variant (SDSP_TUNE_CHAN_STREAMING): 8-frame rounds
    int fpb = 0;       // its frames per workgroup (SDSP_TUNE_CHAN_FRAMES_PER_BLOCK, 0 = default)
    bool xcd = true;   // XCD-contiguous chunk order (SDSP_TUNE_CHAN_XCD_ORDER)
    hipStream_t stream = nullptr;
    StreamFence fence;  // last caller stream an execute call was queued on
};

extern "C" {

// FFT::new(nfft, direction, flags)   src/fft/mod.rs:175-186
int sdsp_fft_create(sdsp_fft** out, size_t nfft, int direction, int precision, int device) {
    if (!out) return SDSP_E_INVALID_ARGUMENT;
    *out = nullptr;
    if (nfft == 0 || nfft > (1u << 24)) {  // the reference panics on a zero-length plan
        set_error("FFT size must be in [1, 2^24]");
        return SDSP_E_INVALID_ARGUMENT;
    }
    if (direction != 0 && direction != 1) return SDSP_E_INVALID_ARGUMENT;
    int st = check_gfx950(device);
    if (st) return st;
    Guard g(device);
    sdsp_fft* h = new sdsp_fft();
    h->N = nfft;
    h->direction = direction;
    h->f64 = precision != 0;
    h->device = device;
    hipError_t e = hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking);
    if (e != hipSuccess) { delete h; return device_status(e, "stream"); }
    if (is_pow2(nfft)) {
        h->kind = 1;
        st = h->p2.build(nfft, h->f64);
    } else if (nfft <= kDirectMax) {
        h->kind = 0;
        st = make_twiddles(h->tw, nfft, h->f64);
    } else {
        // Bluestein: X[k] = w[k] sum_n (x[n] w[n]) conj(w[k - n]),  w[n] = e^{-/+ j pi n^2 / N}
        h->kind = 2;
        size_t M = 1;
        while (M < 2 * nfft - 1) M <<= 1;
        h->M = M;
        const double sgn = direction == 1 ? 1.0 : -1.0;
        std::vector<double> w(2 * nfft), bb(2 * M, 0.0);
        for (size_t n = 0; n < nfft; ++n) {
            const unsigned long long q = (unsigned long long)((unsigned __int128)n * n % (2 * (unsigned __int128)nfft));
            const double ang = sgn * M_PI * (double)q / (double)nfft;
            w[2 * n] = std::cos(ang);
            w[2 * n + 1] = std::sin(ang);
            bb[2 * n] = w[2 * n];  // conj(w)
            bb[2 * n + 1] = -w[2 * n + 1];
            if (n) {
                bb[2 * (M - n)] = w[2 * n];
                bb[2 * (M - n) + 1] = -w[2 * n + 1];
            }
        }
        host_fft_pow2(bb, M);
        for (auto& v : bb) v /= (double)M;
        st = upload(h->chirp, w, h->f64);
        if (!st) st = upload(h->spec, bb, h->f64);
        if (!st) st = h->p2.build(M, h->f64);
    }
    if (st) { sdsp_fft_destroy(h); return st; }
    *out = h;
    return SDSP_OK;
}

void sdsp_fft_destroy(sdsp_fft* h) {
    if (!h) return;
    {
        Guard g(h->device);
        if (h->stream) { (void)hipStreamSynchronize(h->stream); (void)hipStreamDestroy(h->stream); }
        h->tw.release();
        h->stage_in.release();
        h->stage_out.release();
        h->p2.tw.release();
        h->p2.tw1.release();
        h->p2.tw2.release();
        h->p2.twx.release();
        h->chirp.release();
        h->spec.release();
        h->work.release();
        h->tmp.release();
    }
    delete h;
}

size_t sdsp_fft_len(const sdsp_fft* h) { return h ? h->N : 0; }

int sdsp_fft_set_tuning(sdsp_fft* h, int key, int value) {
    if (!h) return SDSP_E_INVALID_ARGUMENT;
    if (key == SDSP_TUNE_FFT_GROUP && value >= 1 && value <= 64) h->p2.group = value;
    else if (key == SDSP_TUNE_FFT_WAVE1024 && (value == 0 || value == 1 || value == 8 || value == 16))
        h->p2.wave1024 = value;
    else return SDSP_E_INVALID_ARGUMENT;
    return SDSP_OK;
}

int sdsp_fft_execute_device(sdsp_fft* h, const void* d_in, void* d_out, size_t batch, void* stream) {
    if (!h) return SDSP_E_INVALID_ARGUMENT;
    if (batch == 0) return SDSP_OK;
    Guard g(h->device);
    hipStream_t s = stream ? (hipStream_t)stream : h->stream;
    const size_t cb = h->f64 ? 16 : 8;
    const bool inv = h->direction == 1;
    if (h->kind == 0) {
        if (d_in == d_out) {  // the direct DFT reads every input per output: work from a copy
            F_TRY(h->work.ensure(batch * h->N * cb), "dft scratch");
            F_TRY(hipMemcpyAsync(h->work.p, d_in, batch * h->N * cb, hipMemcpyDeviceToDevice, s), "dft copy");
            d_in = h->work.p;
        }
        FftArgs a{d_in, d_out, h->tw.p, (int)h->N, ilog2(h->N), false, inv, batch};
        F_TRY(launch_fft(h->f64, a, s), "fft");
    } else if (h->kind == 1) {
        if (h->p2.four_step()) F_TRY(h->tmp.ensure(batch * h->N * cb), "fft scratch");
        F_TRY(h->p2.run(h->f64, d_in, d_out, h->tmp.p, batch, inv, s), "fft");
    } else {
        const long long N = (long long)h->N, M = (long long)h->M;
        F_TRY(h->work.ensure(batch * h->M * cb), "bluestein scratch");
        if (h->p2.four_step()) F_TRY(h->tmp.ensure(batch * h->M * cb), "bluestein scratch");
        F_TRY(launch_bluestein(h->f64, 0, d_in, h->work.p, h->chirp.p, N, M, (long long)batch, s), "bluestein in");
        F_TRY(h->p2.run(h->f64, h->work.p, h->work.p, h->tmp.p, batch, false, s), "bluestein fft");
        F_TRY(launch_bluestein(h->f64, 1, nullptr, h->work.p, h->spec.p, N, M, (long long)batch, s), "bluestein mul");
        F_TRY(h->p2.run(h->f64, h->work.p, h->work.p, h->tmp.p, batch, true, s), "bluestein ifft");
        F_TRY(launch_bluestein(h->f64, 2, h->work.p, d_out, h->chirp.p, N, M, (long long)batch, s), "bluestein out");
    }
    return SDSP_OK;
}

// plan kind (0 direct DFT, 1 power of two in LDS, 2 Bluestein, 3 four-step power of two)
int sdsp_fft_method(const sdsp_fft* h) {
    if (!h) return -1;
    if (h->kind == 1 && h->p2.four_step()) return 3;
    return h->kind;
}

// FFT::execute(&[Complex]) -> Vec<Complex> over `batch` contiguous transforms   src/fft/mod.rs:188-215
int sdsp_fft_execute(sdsp_fft* h, const void* in, void* out, size_t batch) {
    if (!h) return SDSP_E_INVALID_ARGUMENT;
    if (batch == 0) return SDSP_OK;
    Guard g(h->device);
    const size_t bytes = h->N * batch * (h->f64 ? 16 : 8);
    F_TRY(h->stage_in.ensure(bytes), "stage");
    F_TRY(h->stage_out.ensure(bytes), "stage");
    F_TRY(hipMemcpyAsync(h->stage_in.p, in, bytes, hipMemcpyHostToDevice, h->stream), "H2D");
    int st = sdsp_fft_execute_device(h, h->stage_in.p, h->stage_out.p, batch, h->stream);
    if (st) return st;
    F_TRY(hipMemcpyAsync(out, h->stage_out.p, bytes, hipMemcpyDeviceToHost, h->stream), "D2H");
    F_TRY(hipStreamSynchronize(h->stream), "sync");
    return SDSP_OK;
}

// ---- channeliser -----------------------------------------------------------
int sdsp_chan_create(sdsp_chan** out, int dtype, const void* taps, size_t len, size_t M, int device) {
    if (!out) return SDSP_E_INVALID_ARGUMENT;
    *out = nullptr;
    if (dtype != SDSP_RC32 && dtype != SDSP_RC64) {
        set_error("channeliser takes real taps and complex samples (SDSP_RC32 / SDSP_RC64)");
        return SDSP_E_UNSUPPORTED;
    }
    if (M == 0) { set_error("FIR Filter Error NotEnoughFilters"); return SDSP_E_NOT_ENOUGH_FILTERS; }
    if (len == 0) { set_error("FIR Filter Error CoefficientsLengthZero"); return SDSP_E_COEFFICIENTS_LENGTH_ZERO; }
    if (!is_pow2(M) || M < 4 || M > 4096) {
        set_error("channel count must be a power of two in [4, 4096]");
        return SDSP_E_UNSUPPORTED;
    }
    const size_t K = len / M;
    if (K == 0) { set_error("fewer taps than channels"); return SDSP_E_INVALID_ARGUMENT; }
    int st = check_gfx950(device);
    if (st) return st;
    Guard g(device);
    sdsp_chan* h = new sdsp_chan();
    h->dtype = dtype;
    h->device = device;
    h->M = M;
    h->K = K;
    const size_t cbytes = coef_bytes(dtype);
    h->taps.assign((const unsigned char*)taps, (const unsigned char*)taps + len * cbytes);
    // branch coefficients, stored order: cb[p][K-1-idx] = h[p + idx M]   (pfb.rs:33-40)
    std::vector<unsigned char> cb(M * K * cbytes);
    for (size_t p = 0; p < M; ++p)
        for (size_t idx = 0; idx < K; ++idx)
            std::memcpy(&cb[(p * K + (K - 1 - idx)) * cbytes], &h->taps[(p + idx * M) * cbytes], cbytes);
    hipError_t e = hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking);
    if (e == hipSuccess) e = h->cb.ensure(cb.size());
    if (e == hipSuccess) e = hipMemcpy(h->cb.p, cb.data(), cb.size(), hipMemcpyHostToDevice);
    if (e != hipSuccess) { st = device_status(e, "chan create"); sdsp_chan_destroy(h); return st; }
    st = make_twiddles(h->tw, M, dtype == SDSP_RC64);
    if (!st) st = sdsp_chan_set_streams(h, 1);
    if (st) { sdsp_chan_destroy(h); return st; }
    *out = h;
    return SDSP_OK;
}

void sdsp_chan_destroy(sdsp_chan* h) {
    if (!h) return;
    {
        Guard g(h->device);
        (void)h->fence.wait();
        if (h->stream) { (void)hipStreamSynchronize(h->stream); (void)hipStreamDestroy(h->stream); }
        h->cb.release(); h->tw.release(); h->hist[0].release(); h->hist[1].release();
        h->stage_in.release(); h->stage_out.release();
    }
    delete h;
}

int sdsp_chan_set_streams(sdsp_chan* h, size_t streams) {
    if (!h || streams == 0) return SDSP_E_INVALID_ARGUMENT;
    Guard g(h->device);
    F_TRY(h->fence.wait(), "wait for queued work");  // a queued block may still read the history
    h->streams = streams;
    const size_t hb = streams * (h->K - 1) * h->M * sample_bytes(h->dtype);
    for (int i = 0; i < 2; ++i) {
        F_TRY(h->hist[i].ensure(hb), "alloc history");
        if (hb) F_TRY(hipMemsetAsync(h->hist[i].p, 0, hb, h->stream), "zero history");
    }
    h->cur = 0;
    F_TRY(hipStreamSynchronize(h->stream), "sync");
    return SDSP_OK;
}

int sdsp_chan_set_tuning(sdsp_chan* h, int key, int value) {
    if (!h) return SDSP_E_INVALID_ARGUMENT;
    if (key == SDSP_TUNE_CHAN_STREAMING && value >= 0 && value <= 6) h->fast = value;
    else if (key == SDSP_TUNE_CHAN_FRAMES_PER_BLOCK && value >= 0) h->fpb = value;
    else if (key == SDSP_TUNE_CHAN_XCD_ORDER) h->xcd = value != 0;
    else return SDSP_E_INVALID_ARGUMENT;
    return SDSP_OK;
}

int sdsp_chan_reset(sdsp_chan* h) { return h ? sdsp_chan_set_streams(h, h->streams) : SDSP_E_INVALID_ARGUMENT; }

int sdsp_chan_execute_block_device(sdsp_chan* h, const void* d_in, size_t n, void* d_out, size_t* frames,
                                   void* stream) {
    if (!h) return SDSP_E_INVALID_ARGUMENT;
    if (n % h->M) {
        set_error("channeliser blocks must be a whole number of M-sample frames");
        return SDSP_E_INVALID_ARGUMENT;
    }
    const size_t fr = n / h->M;
    if (frames) *frames = fr;
    if (fr == 0) return SDSP_OK;
    const size_t bytes = h->streams * n * sample_bytes(h->dtype);
    if (ranges_overlap(d_in, bytes, d_out, bytes)) {
        set_error("input and output blocks overlap (in-place channelising is not supported)");
        return SDSP_E_INVALID_ARGUMENT;
    }
    Guard g(h->device);
    hipStream_t s = stream ? (hipStream_t)stream : h->stream;
    F_TRY(h->fence.order_before(s), "order after queued work");  // the history this launch reads
    ChanArgs a{d_in, h->hist[h->cur].p, h->cb.p, d_out, h->tw.p, (int)h->M, ilog2(h->M), (int)h->K, n, fr, h->streams};
    a.fast = h->fast;
    a.frames_per_block = h->fpb;
    a.xcd_order = h->xcd;
    F_TRY(launch_chan(h->dtype == SDSP_RC64, a, s), "channeliser");
    const int H = (int)((h->K - 1) * h->M);
    F_TRY(launch_hist_update(h->dtype, d_in, h->hist[h->cur].p, h->hist[h->cur ^ 1].p, n, H, h->streams, s),
          "history update");
    h->cur ^= 1;
    F_TRY(h->fence.record(s), "record fence");
    return SDSP_OK;
}

int sdsp_chan_execute_block(sdsp_chan* h, const void* in, size_t n, void* out, size_t* frames) {
    if (!h) return SDSP_E_INVALID_ARGUMENT;
    Guard g(h->device);
    const size_t bytes = h->streams * n * sample_bytes(h->dtype);
    if (n % h->M) {
        set_error("channeliser blocks must be a whole number of M-sample frames");
        return SDSP_E_INVALID_ARGUMENT;
    }
    if (frames) *frames = n / h->M;
    if (n == 0) return SDSP_OK;
    F_TRY(h->stage_in.ensure(bytes), "stage");
    F_TRY(h->stage_out.ensure(bytes), "stage");
    F_TRY(hipMemcpyAsync(h->stage_in.p, in, bytes, hipMemcpyHostToDevice, h->stream), "H2D");
    int st = sdsp_chan_execute_block_device(h, h->stage_in.p, n, h->stage_out.p, nullptr, h->stream);
    if (st) return st;
    F_TRY(hipMemcpyAsync(out, h->stage_out.p, bytes, hipMemcpyDeviceToHost, h->stream), "D2H");
    F_TRY(hipStreamSynchronize(h->stream), "sync");
    return SDSP_OK;
}

int sdsp_chan_synchronize(sdsp_chan* h) {
    if (!h) return SDSP_E_INVALID_ARGUMENT;
    Guard g(h->device);
    F_TRY(h->fence.wait(), "wait for queued work");
    F_TRY(hipStreamSynchronize(h->stream), "sync");
    return SDSP_OK;
}

// ---- DotProduct ---------------------------------------------------------------
// batch vectors of n samples (stride samples apart), coefficients as given to
// DotProduct::new(&coefs, direction) (0 FORWARD, 1 REVERSE), device buffers.
int sdsp_dot_execute_batched_device(int dtype, const void* coefs, size_t len, int direction, const void* d_samples,
                                    size_t n, size_t stride, size_t batch, void* d_out, void* stream) {
    if (dtype < 0 || dtype > 5 || direction < 0 || direction > 1) return SDSP_E_INVALID_ARGUMENT;
    if (batch == 0) return SDSP_OK;
    int dev = 0;
    F_TRY(hipGetDevice(&dev), "device");
    int st = check_gfx950(dev);
    if (st) return st;
    const size_t cb = coef_bytes(dtype);
    std::vector<unsigned char> c((const unsigned char*)coefs, (const unsigned char*)coefs + len * cb);
    if (direction == 1)
        for (size_t i = 0; i < len / 2; ++i)
            std::swap_ranges(&c[i * cb], &c[i * cb] + cb, &c[(len - 1 - i) * cb]);
    DevBuf d_c;
    F_TRY(d_c.ensure(c.size()), "alloc coefs");
    hipStream_t s = (hipStream_t)stream;
    F_TRY(hipMemcpyAsync(d_c.p, c.data(), c.size(), hipMemcpyHostToDevice, s), "copy coefs");
    DotArgs a{d_c.p, (int)std::min(n, len), d_samples, stride, batch, d_out};
    F_TRY(launch_dot(dtype, a, s), "dot");
    F_TRY(hipStreamSynchronize(s), "sync");  // d_c is released on return
    return SDSP_OK;
}

// single DotProduct::execute over host buffers (out = one sample)
int sdsp_dot_execute(int dtype, const void* coefs, size_t len, int direction, const void* samples, size_t n,
                     void* out) {
    if (dtype < 0 || dtype > 5) return SDSP_E_INVALID_ARGUMENT;
    int dev = 0;
    F_TRY(hipGetDevice(&dev), "device");
    int st = check_gfx950(dev);
    if (st) return st;
    const size_t sb = sample_bytes(dtype);
    DevBuf s, o;
    F_TRY(s.ensure(std::max<size_t>(n, 1) * sb), "alloc");
    F_TRY(o.ensure(sb), "alloc");
    if (n) F_TRY(hipMemcpy(s.p, samples, n * sb, hipMemcpyHostToDevice), "H2D");
    st = sdsp_dot_execute_batched_device(dtype, coefs, len, direction, s.p, n, n, 1, o.p, nullptr);
    if (st) return st;
    F_TRY(hipMemcpy(out, o.p, sb, hipMemcpyDeviceToHost), "D2H");
    return SDSP_OK;
}

}  // extern "C"
