// C-ABI runtime of libsdsp.so: handles, HBM-resident delay lines, streams,
// kernel selection.  Every exported function cites the reference method it
// replaces in include/sdsp.h.
//
// There is deliberately no CPU execution path: if no gfx950 device is usable
// the create calls fail with SDSP_E_NO_DEVICE and nothing runs.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cctype>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "sdsp.h"
#include "sdsp_host.hpp"
#include "sdsp_kernels.hpp"

namespace sdsp {

static thread_local std::string g_last_error;
void set_error(const std::string& msg) { g_last_error = msg; }

// Process-wide starting algorithm of new FIR-type and IIR handles: SDSP_ALGO_EXACT unless
// sdsp_set_default_algo or the SDSP_DEFAULT_ALGO environment variable ("auto" / "exact" / "fma",
// or 0 / 1 / 2; read once, at the first handle or query) says otherwise -- so a deployment can move
// an unchanged reference-API caller onto the fast paths without a per-handle set_algo call.
static std::atomic<int> g_default_algo{-1};  // -1: not yet read from the environment
static int parse_algo_env(const char* e) {
    if (!e) return SDSP_ALGO_EXACT;
    std::string v(e);
    for (auto& ch : v) ch = (char)std::tolower((unsigned char)ch);
    if (v == "auto" || v == "0") return SDSP_ALGO_AUTO;
    if (v == "fma" || v == "2") return SDSP_ALGO_FMA;
    return SDSP_ALGO_EXACT;  // "exact", "1", anything else
}
int default_algo() {
    int v = g_default_algo.load();
    if (v >= 0) return v;
    int expect = -1;
    g_default_algo.compare_exchange_strong(expect, parse_algo_env(std::getenv("SDSP_DEFAULT_ALGO")));
    return g_default_algo.load();
}
int device_status(hipError_t e, const char* what) {
    if (e == hipSuccess) return SDSP_OK;
    set_error(std::string(what) + ": " + hipGetErrorString(e));
    return e == hipErrorOutOfMemory ? SDSP_E_OUT_OF_MEMORY : SDSP_E_DEVICE;
}
#define SDSP_TRY(expr, what)                              \
    do {                                                  \
        hipError_t _e = (expr);                           \
        if (_e != hipSuccess) return device_status(_e, what); \
    } while (0)

struct DeviceInfo {
    bool ok = false;
    int cus = 256;
};

static int check_device(int device, DeviceInfo* info) {
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count <= 0) {
        set_error("no HIP device visible (libsdsp has no CPU execution path)");
        return SDSP_E_NO_DEVICE;
    }
    if (device < 0 || device >= count) {
        set_error("device index out of range");
        return SDSP_E_NO_DEVICE;
    }
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) != hipSuccess) {
        set_error("hipGetDeviceProperties failed");
        return SDSP_E_NO_DEVICE;
    }
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) {
        set_error(std::string("libsdsp is built for gfx950; device is ") + prop.gcnArchName);
        return SDSP_E_NO_DEVICE;
    }
    info->ok = true;
    info->cus = prop.multiProcessorCount;
    return SDSP_OK;
}

struct DeviceGuard {
    int prev = -1;
    explicit DeviceGuard(int d) {
        (void)hipGetDevice(&prev);
        if (prev != d) (void)hipSetDevice(d);
    }
    ~DeviceGuard() {
        int cur = -1;
        (void)hipGetDevice(&cur);
        if (prev >= 0 && cur != prev) (void)hipSetDevice(prev);
    }
};

static hipStream_t pick(void* user, hipStream_t own) { return user ? (hipStream_t)user : own; }

}  // namespace sdsp

using namespace sdsp;

// ===========================================================================
// FIR / decimating FIR
// ===========================================================================
struct sdsp_fir {
    int dtype = 0, device = 0, cus = 256;
    mutable unsigned long long device_ops = 0;  // sdsp_fir_device_ops
    size_t L = 0, M = 1, channels = 1;
    std::vector<unsigned char> taps;   // original order (host copy for coefficients / design queries)
    std::vector<unsigned char> scale;  // one Coef
    DevBuf d_taps_rev;                 // cr[i] = h[L-1-i]  (DotProduct REVERSE, dot_product/mod.rs:73-81)
    DevBuf d_hist[2];                  // [channels][L-1] oldest first
    int cur = 0;
    size_t ci = 0;                     // DecimatingFIRFilter::current_item (decim.rs:7)
    int algo = SDSP_ALGO_EXACT;        // reference-order kernel unless the caller opts in (sdsp.h)
    hipStream_t stream = nullptr;
    mutable StreamFence fence;         // last stream an execute call was queued on
    DevBuf stage_in, stage_out;
    HostMapped step_out;  // per-sample execute on the device: output at [0, 16), completion flag at [16, 20)
    unsigned step_seq = 0;
    // host delay line for per-sample calls and small host blocks (runtime_host_step below):
    // hbuf holds 2(L-1) samples, the window (oldest first) is hbuf[hpos, hpos + L-1)
    std::vector<unsigned char> hbuf;
    size_t hpos = 0;
    bool host_valid = false;  // hbuf holds the current window (single-channel handles only)
    bool dev_stale = false;   // the host consumed samples after d_hist[cur] was last written
    int host_step = 1;        // SDSP_TUNE_HOST_STEP
    size_t host_macs = 1u << 16;  // host blocks: n * L up to this many multiply-adds
    // overlap-save plan
    bool ols_ok = false;
    int ols_kernel = kOlsOneShot;  // SDSP_TUNE_OLS_KERNEL
    int decim_seg = 0;  // outputs per lane group of the polyphase decimator (0 = auto)
    OlsPlan ols{};
    DevBuf d_H, d_tw1, d_tw2, d_pkt, d_ostab, d_hhalf;
};

namespace {

int fir_alloc_state(sdsp_fir* h) {
    SDSP_TRY(h->fence.wait(), "wait for queued work");
    const size_t hb = h->channels * (h->L - 1) * sample_bytes(h->dtype);
    for (int i = 0; i < 2; ++i) {
        SDSP_TRY(h->d_hist[i].ensure(hb), "alloc history");
        if (hb) SDSP_TRY(hipMemsetAsync(h->d_hist[i].p, 0, hb, h->stream), "zero history");
    }
    h->cur = 0;
    h->ci = 0;
    SDSP_TRY(hipStreamSynchronize(h->stream), "sync");
    const size_t lm1 = h->L - 1, sb = sample_bytes(h->dtype);
    h->hbuf.assign(2 * lm1 * sb, 0);  // the zeroed window, both copies
    h->hpos = 0;
    h->host_valid = h->channels == 1;
    h->dev_stale = false;
    return SDSP_OK;
}

bool ols_applicable(const sdsp_fir* h) {
    return (h->dtype == SDSP_RC32 || h->dtype == SDSP_CC32) && h->M == 1 && h->L >= 2 && h->L - 1 <= 256 * 15;
}

// spectrum of g[i] = scale * h[L-1-i] in the lane layout of kern_fir_ols.hip
int ols_build(sdsp_fir* h) {
    SDSP_TRY(h->fence.wait(), "wait for queued work");
    const int N = kOlsN;
    const size_t L = h->L;
    const int h2 = (int)((L - 1 + 255) / 256);
    std::vector<cd> g(N, cd{0.0, 0.0});
    const cd s = coef_at(h->scale.data(), h->dtype, 0);
    for (size_t i = 0; i < L; ++i) {
        cd c = coef_at(h->taps.data(), h->dtype, L - 1 - i);
        g[i] = coef_is_complex(h->dtype) ? cmul(c, s) : cd{c.re * s.re, c.re * s.im};
    }
    // direct DFT in f64 (one-time, O(N L))
    std::vector<cd> G(N);
    const double w = -2.0 * M_PI / N;
    for (int k = 0; k < N; ++k) {
        double re = 0.0, im = 0.0;
        for (size_t i = 0; i < L; ++i) {
            const long long ph = ((long long)i * k) % N;
            const double c = std::cos(w * (double)ph), sn = std::sin(w * (double)ph);
            re += g[i].re * c - g[i].im * sn;
            im += g[i].re * sn + g[i].im * c;
        }
        G[k] = {re / N, im / N};
    }
    std::vector<float> Hs(2 * 4096), tw1(2 * 4096), tw2(2 * 256);
    for (int t = 0; t < 256; ++t) {
        const int k0 = t >> 4, k1 = t & 15;
        for (int k2 = 0; k2 < 16; ++k2) {
            const cd v = G[k0 + 16 * k1 + 256 * k2];
            Hs[2 * (t * 16 + k2)] = (float)v.re;
            Hs[2 * (t * 16 + k2) + 1] = (float)v.im;
        }
        for (int k = 0; k < 16; ++k) {
            const long long ph = ((long long)t * k) % 4096;
            tw1[2 * (t * 16 + k)] = (float)std::cos(-2.0 * M_PI * ph / 4096.0);
            tw1[2 * (t * 16 + k) + 1] = (float)std::sin(-2.0 * M_PI * ph / 4096.0);
        }
    }
    for (int a = 0; a < 16; ++a)
        for (int b = 0; b < 16; ++b) {
            const int ph = (a * b) % 256;
            tw2[2 * (a * 16 + b)] = (float)std::cos(-2.0 * M_PI * ph / 256.0);
            tw2[2 * (a * 16 + b) + 1] = (float)std::sin(-2.0 * M_PI * ph / 256.0);
        }
    SDSP_TRY(h->d_H.ensure(Hs.size() * 4), "alloc H");
    SDSP_TRY(h->d_tw1.ensure(tw1.size() * 4), "alloc tw1");
    SDSP_TRY(h->d_tw2.ensure(tw2.size() * 4), "alloc tw2");
    SDSP_TRY(hipMemcpyAsync(h->d_H.p, Hs.data(), Hs.size() * 4, hipMemcpyHostToDevice, h->stream), "copy H");
    SDSP_TRY(hipMemcpyAsync(h->d_tw1.p, tw1.data(), tw1.size() * 4, hipMemcpyHostToDevice, h->stream), "copy tw1");
    SDSP_TRY(hipMemcpyAsync(h->d_tw2.p, tw2.data(), tw2.size() * 4, hipMemcpyHostToDevice, h->stream), "copy tw2");
    // the same tables for the packed kernel, k-pair major so that a table load is one
    // coalesced 16-byte access per lane: float4 (p, i) = entries 2p, 2p + 1 of row i;
    // [0, 2048): H rows t, [2048, 4096): tw1 rows, [4096, 4224): tw2 rows
    std::vector<float> pkt(4 * 4224);
    for (int q = 0; q < 8; ++q) {
        for (int i = 0; i < 256; ++i)
            for (int e = 0; e < 4; ++e) {
                pkt[4 * (q * 256 + i) + e] = Hs[2 * (i * 16 + 2 * q) + e];
                pkt[4 * (2048 + q * 256 + i) + e] = tw1[2 * (i * 16 + 2 * q) + e];
            }
        for (int i = 0; i < 16; ++i)
            for (int e = 0; e < 4; ++e) pkt[4 * (4096 + q * 16 + i) + e] = tw2[2 * (i * 16 + 2 * q) + e];
    }
    SDSP_TRY(h->d_pkt.ensure(pkt.size() * 4), "alloc packed tables");
    SDSP_TRY(hipMemcpyAsync(h->d_pkt.p, pkt.data(), pkt.size() * 4, hipMemcpyHostToDevice, h->stream),
             "copy packed tables");
    // one-shot kernel (kern_fir_ols_os.hip): per column c the twiddle bases C_b = W4096^(b c),
    // D_a = W4096^(4 a c) (b, a = 1..3) as float4 [q][c] = (C1 C2 | C3 D1 | D2 D3), then per
    // row l the W256 bases E_b = W256^(b l), F_a = W256^(4 a l) as float4 [768 + 16 q + l], then
    // the first powers alone (kOlsOsTabCD, kOlsOsTabEF: the default kernel's two loads)
    std::vector<float> os(4 * kOlsOsTabF4);
    auto put = [&](size_t f4, int half, long long m, int nn) {
        const double ang = -2.0 * M_PI * (double)(m % nn) / nn;
        os[4 * f4 + 2 * half] = (float)std::cos(ang);
        os[4 * f4 + 2 * half + 1] = (float)std::sin(ang);
    };
    for (int c = 0; c < 256; ++c) {
        put(c, 0, c, 4096);
        put(c, 1, 2LL * c, 4096);
        put(256 + c, 0, 3LL * c, 4096);
        put(256 + c, 1, 4LL * c, 4096);
        put(512 + c, 0, 8LL * c, 4096);
        put(512 + c, 1, 12LL * c, 4096);
    }
    for (int c = 0; c < 256; ++c) {  // {C1, D1} per column
        put(kOlsOsTabCD + c, 0, c, 4096);
        put(kOlsOsTabCD + c, 1, 4LL * c, 4096);
    }
    for (int l = 0; l < 16; ++l) {  // {E1, F1} per row
        put(kOlsOsTabEF + l, 0, l, 256);
        put(kOlsOsTabEF + l, 1, 4LL * l, 256);
    }
    for (int l = 0; l < 16; ++l) {
        put(768 + l, 0, l, 256);
        put(768 + l, 1, 2LL * l, 256);
        put(784 + l, 0, 3LL * l, 256);
        put(784 + l, 1, 4LL * l, 256);
        put(800 + l, 0, 8LL * l, 256);
        put(800 + l, 1, 12LL * l, 256);
    }
    SDSP_TRY(h->d_ostab.ensure(os.size() * 4), "alloc one-shot tables");
    SDSP_TRY(hipMemcpyAsync(h->d_ostab.p, os.data(), os.size() * 4, hipMemcpyHostToDevice, h->stream),
             "copy one-shot tables");
    // real taps: H[N - k] = conj(H[k]), so the one-shot kernel reads bins k2 < 8 of every lane from
    // a half table and the others as the conjugates of its mirror lane's (kern_fir_ols_os.hip):
    // float4 [p][i] = {H(i, 2p), H(i, 2p + 1)} for p < 4, H(i, k2) = G[k0 + 16 k1 + 256 k2] of
    // lane i = 16 k0 + k1; entry i = 256 is the mirror of lane (0, 0), whose bins k2 >= 8 mirror
    // k2' = 16 - k2 (k2' = 8 included): stored so that the kernel's conj-and-swap yields them
    const bool real_taps = !coef_is_complex(h->dtype);
    if (real_taps) {
        std::vector<float> hh(4 * 4 * kOlsHalfRow);
        auto set = [&](int q, int i, int half, cd v) {
            hh[4 * (q * kOlsHalfRow + i) + 2 * half] = (float)v.re;
            hh[4 * (q * kOlsHalfRow + i) + 2 * half + 1] = (float)v.im;
        };
        for (int q = 0; q < 4; ++q) {
            for (int i = 0; i < 256; ++i) {
                const int k0 = i >> 4, k1 = i & 15;
                set(q, i, 0, G[k0 + 16 * k1 + 256 * (2 * q)]);
                set(q, i, 1, G[k0 + 16 * k1 + 256 * (2 * q + 1)]);
            }
            // lane (0, 0), pair p = 7 - q of its bins k2 = 2p, 2p + 1: stored as
            // {conj H(256 (2p + 1)), conj H(256 (2p))} at the mirror slot
            const int pp = 7 - q;
            const cd a = G[256 * (2 * pp + 1)], b = G[256 * (2 * pp)];
            set(q, 256, 0, cd{a.re, -a.im});
            set(q, 256, 1, cd{b.re, -b.im});
        }
        SDSP_TRY(h->d_hhalf.ensure(hh.size() * 4), "alloc half spectrum");
        SDSP_TRY(hipMemcpyAsync(h->d_hhalf.p, hh.data(), hh.size() * 4, hipMemcpyHostToDevice, h->stream),
                 "copy half spectrum");
    }
    SDSP_TRY(hipStreamSynchronize(h->stream), "sync");
    h->ols = OlsPlan{};
    h->ols.d_hhalf = real_taps ? h->d_hhalf.p : nullptr;
    h->ols.d_H = h->d_H.p;
    h->ols.d_tw1 = h->d_tw1.p;
    h->ols.d_tw2 = h->d_tw2.p;
    h->ols.halo_rows = h2;
    h->ols.kernel = h->ols_kernel;
    h->ols.d_pkt = h->d_pkt.p;
    h->ols.d_ostab = h->d_ostab.p;
    h->ols_ok = true;
    return SDSP_OK;
}

int fir_resolve_algo(const sdsp_fir* h, size_t n) {
    if (h->algo == SDSP_ALGO_FFT) return ols_applicable(h) ? SDSP_ALGO_FFT : SDSP_ALGO_EXACT;
    if (h->algo != SDSP_ALGO_AUTO) return h->algo;
    // AUTO: overlap-save for long 32-bit complex blocks, reference-order direct form otherwise
    if (ols_applicable(h) && n >= (size_t)(1 << 16)) return SDSP_ALGO_FFT;
    return SDSP_ALGO_EXACT;
}
// AUTO on a decimating handle: the fused multiply-add kernels for long 32-bit blocks (n inputs)
static int decim_resolve_algo(const sdsp_fir* h, size_t n) {
    if (h->algo != SDSP_ALGO_AUTO) return h->algo;
    return h->dtype <= SDSP_CC32 && n >= (size_t)(1 << 16) ? SDSP_ALGO_FMA : SDSP_ALGO_EXACT;
}

int fir_create_common(sdsp_fir** out, int dtype, const void* taps, size_t len, const void* scale, size_t M,
                      int device) {
    *out = nullptr;
    if (dtype < 0 || dtype > 5) {
        set_error("bad dtype");
        return SDSP_E_INVALID_ARGUMENT;
    }
    if (len == 0) {
        set_error("FIR Filter Error CoefficientsLengthZero");
        return SDSP_E_COEFFICIENTS_LENGTH_ZERO;
    }
    if (M < 1) {
        set_error("FIR Filter Error DecimationLessThanOne");
        return SDSP_E_DECIMATION_LESS_THAN_ONE;
    }
    if (len > (1u << 30)) {
        set_error("tap count too large");
        return SDSP_E_INVALID_ARGUMENT;
    }
    DeviceInfo info;
    int st = check_device(device, &info);
    if (st) return st;
    DeviceGuard g(device);
    sdsp_fir* h = new sdsp_fir();
    h->dtype = dtype;
    h->device = device;
    h->algo = default_algo();
    h->cus = info.cus;
    h->L = len;
    h->M = M;
    const size_t cb = coef_bytes(dtype);
    h->taps.assign((const unsigned char*)taps, (const unsigned char*)taps + len * cb);
    h->scale.assign((const unsigned char*)scale, (const unsigned char*)scale + cb);
    std::vector<unsigned char> rev(len * cb);
    for (size_t i = 0; i < len; ++i) std::memcpy(&rev[i * cb], &h->taps[(len - 1 - i) * cb], cb);
    hipError_t e = hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking);
    if (e == hipSuccess) e = h->d_taps_rev.ensure(rev.size());
    if (e == hipSuccess) e = hipMemcpy(h->d_taps_rev.p, rev.data(), rev.size(), hipMemcpyHostToDevice);
    if (e != hipSuccess) {
        st = device_status(e, "fir create");
        sdsp_fir_destroy(h);
        return st;
    }
    st = fir_alloc_state(h);
    if (st) {
        sdsp_fir_destroy(h);
        return st;
    }
    *out = h;
    return SDSP_OK;
}

}  // namespace

namespace {
// ---------------------------------------------------------------------------
// Host step: Filter::execute(sample), DecimatingFIRFilter::push and small host
// blocks run on the host against the handle's own delay line, in
// the reference's arithmetic (fir/mod.rs:209-212, decim.rs:115-118, 221-228:
// acc = 0; acc += cr[i] x[n-i] for i = 0..L-1; y = acc * scale; num-complex
// products, no contraction -- this TU is built with -ffp-contract=off).  It is
// the product's own small-work path, not a fallback: creating a handle still
// requires the gfx950 device, and every block above the threshold runs on it.
// Coherence: the state is the last L-1 inputs, so it moves between host and
// device only when the side that runs next does not hold it -- one D2H of L-1
// samples before the first host step after device work (host_pull), one H2D
// before the first device call after host steps (host_flush).
template <typename T> struct hcx {
    T re, im;
};
template <typename T> inline T hmul(T a, T b) { return a * b; }
template <typename T> inline hcx<T> hmul(T a, hcx<T> b) { return {a * b.re, a * b.im}; }
template <typename T> inline hcx<T> hmul(hcx<T> a, T b) { return {a.re * b, a.im * b}; }
template <typename T> inline hcx<T> hmul(hcx<T> a, hcx<T> b) {
    return {a.re * b.re - a.im * b.im, a.re * b.im + a.im * b.re};
}
template <typename T> inline T hadd(T a, T b) { return a + b; }
template <typename T> inline hcx<T> hadd(hcx<T> a, hcx<T> b) { return {a.re + b.re, a.im + b.im}; }
// fused forms: fmac_ of sdsp_device.hpp (the device FMA kernels), one rounding per fma
inline float hfma(float acc, float c, float x) { return std::fma(c, x, acc); }
inline double hfma(double acc, double c, double x) { return std::fma(c, x, acc); }
template <typename T> inline hcx<T> hfma(hcx<T> acc, T c, hcx<T> x) { return {hfma(acc.re, c, x.re), hfma(acc.im, c, x.im)}; }
template <typename T> inline hcx<T> hfma(hcx<T> acc, hcx<T> c, hcx<T> x) {
    return {hfma(hfma(acc.re, c.re, x.re), -c.im, x.im), hfma(hfma(acc.im, c.re, x.im), c.im, x.re)};
}
template <typename T> inline T hzero() { return T{}; }

template <typename C, typename I>
void host_step_t(sdsp_fir* h, const unsigned char* sample, unsigned char* out, bool emit, bool fused) {
    const size_t L = h->L, lm1 = L - 1;
    I x;
    std::memcpy(&x, sample, sizeof(I));
    I* b = reinterpret_cast<I*>(h->hbuf.data());
    if (emit) {
        const I* w = b + h->hpos;  // window oldest first: x[n - i] = w[lm1 - i]
        const C* taps = reinterpret_cast<const C*>(h->taps.data());  // cr[i] = h[L-1-i]
        I acc = hzero<I>();
        if (fused) {
            acc = hfma(acc, taps[L - 1], x);
            for (size_t i = 1; i < L; ++i) acc = hfma(acc, taps[L - 1 - i], w[lm1 - i]);
        } else {
            acc = hadd(acc, hmul(taps[L - 1], x));
            for (size_t i = 1; i < L; ++i) acc = hadd(acc, hmul(taps[L - 1 - i], w[lm1 - i]));
        }
        C sc;
        std::memcpy(&sc, h->scale.data(), sizeof(C));
        const I y = hmul(acc, sc);
        std::memcpy(out, &y, sizeof(I));
    }
    if (lm1) {  // Window::push (src/window/mod.rs:36-41) on the doubled buffer
        b[h->hpos] = x;
        b[h->hpos + lm1] = x;
        h->hpos = h->hpos + 1 == lm1 ? 0 : h->hpos + 1;
    }
}

void host_step(sdsp_fir* h, const unsigned char* sample, unsigned char* out, bool emit) {
    const bool fused = h->algo == SDSP_ALGO_FMA;
    switch (h->dtype) {
        case SDSP_RR32: return host_step_t<float, float>(h, sample, out, emit, fused);
        case SDSP_RC32: return host_step_t<float, hcx<float>>(h, sample, out, emit, fused);
        case SDSP_CC32: return host_step_t<hcx<float>, hcx<float>>(h, sample, out, emit, fused);
        case SDSP_RR64: return host_step_t<double, double>(h, sample, out, emit, fused);
        case SDSP_RC64: return host_step_t<double, hcx<double>>(h, sample, out, emit, fused);
        case SDSP_CC64: return host_step_t<hcx<double>, hcx<double>>(h, sample, out, emit, fused);
    }
}

// the host window := the device history (after device work)
int host_pull(sdsp_fir* h) {
    if (h->host_valid) return SDSP_OK;
    SDSP_TRY(h->fence.wait(), "wait for queued work");
    SDSP_TRY(hipStreamSynchronize(h->stream), "sync");
    const size_t lm1 = h->L - 1, sb = sample_bytes(h->dtype);
    h->hbuf.resize(2 * lm1 * sb);
    ++h->device_ops;
    if (lm1) {
        SDSP_TRY(hipMemcpy(h->hbuf.data(), h->d_hist[h->cur].p, lm1 * sb, hipMemcpyDeviceToHost), "pull history");
        std::memcpy(h->hbuf.data() + lm1 * sb, h->hbuf.data(), lm1 * sb);
    }
    h->hpos = 0;
    h->host_valid = true;
    return SDSP_OK;
}

// the device history := the host window (before device work after host steps).  No
// kernel can be reading d_hist here: host steps start only after host_pull's
// synchronisation, a synchronising host call, or a state reset.
int host_flush(const sdsp_fir* hc) {
    sdsp_fir* h = const_cast<sdsp_fir*>(hc);
    if (!h->dev_stale) return SDSP_OK;
    ++h->device_ops;
    const size_t lm1 = h->L - 1, sb = sample_bytes(h->dtype);
    if (lm1)
        SDSP_TRY(hipMemcpy(h->d_hist[h->cur].p, h->hbuf.data() + h->hpos * sb, lm1 * sb, hipMemcpyHostToDevice),
                 "flush history");
    h->dev_stale = false;
    return SDSP_OK;
}

// keep a valid host window current across a device block whose input the host holds
void host_feed(sdsp_fir* h, const unsigned char* in, size_t n) {
    const size_t lm1 = h->L - 1, sb = sample_bytes(h->dtype);
    if (!h->host_valid || !lm1 || !n) return;
    if (n >= lm1) {
        std::memcpy(h->hbuf.data(), in + (n - lm1) * sb, lm1 * sb);
        std::memcpy(h->hbuf.data() + lm1 * sb, in + (n - lm1) * sb, lm1 * sb);
        h->hpos = 0;
        return;
    }
    for (size_t i = 0; i < n; ++i) {
        std::memcpy(h->hbuf.data() + h->hpos * sb, in + i * sb, sb);
        std::memcpy(h->hbuf.data() + (h->hpos + lm1) * sb, in + i * sb, sb);
        h->hpos = h->hpos + 1 == lm1 ? 0 : h->hpos + 1;
    }
}

bool host_eligible(const sdsp_fir* h, size_t n) {
    return h->host_step && h->channels == 1 && h->algo != SDSP_ALGO_FFT && n * h->L <= h->host_macs;
}

// n inputs through the host step; outputs (when `out`) where the phase emits (decim.rs:221-228)
int host_run(sdsp_fir* h, const unsigned char* in, size_t n, unsigned char* out, size_t* n_out) {
    int st = host_pull(h);
    if (st) return st;
    const size_t sb = sample_bytes(h->dtype);
    size_t k = 0;
    for (size_t i = 0; i < n; ++i) {
        const bool emit = out && (h->M == 1 || (h->M - 1 - h->ci) % h->M == 0);
        host_step(h, in + i * sb, emit ? out + k * sb : nullptr, emit);
        h->ci = (h->ci + 1) % h->M;
        k += emit;
    }
    if (n) h->dev_stale = true;
    if (n_out) *n_out = k;
    return SDSP_OK;
}

// one input through the single-launch device step kernel (kern_fir_step.hip,
// SDSP_TUNE_HOST_STEP = 0): the delay line shifts on the device, the output (when
// the phase emits and `want` is set) lands in host-mapped memory
int fir_step_device(sdsp_fir* h, const void* sample, void* out, size_t* n_out, bool want) {
    SDSP_TRY(h->fence.wait(), "wait for queued work");
    ++h->device_ops;
    int st = host_flush(h);
    if (st) return st;
    if (!h->step_out.host) {
        SDSP_TRY(h->step_out.ensure(32), "alloc mapped output");
        std::memset(h->step_out.host, 0, 32);  // pinned memory is not zeroed: no stale flag value
    }
    const bool emit = want && (h->M == 1 || (h->M - 1 - h->ci) % h->M == 0);  // decim.rs:221-231
    unsigned* flag_h = reinterpret_cast<unsigned*>((char*)h->step_out.host + 16);
    unsigned seq = ++h->step_seq;
    if (seq == 0) seq = h->step_seq = 1;  // the flag's initial 0 never matches
    FirStepArgs a{sample, h->d_hist[h->cur].p, h->d_hist[h->cur ^ 1].p, h->d_taps_rev.p, h->scale.data(),
                  h->step_out.dev, reinterpret_cast<unsigned*>((char*)h->step_out.dev + 16), seq, (int)h->L - 1,
                  (int)h->L, emit, h->algo != SDSP_ALGO_FMA};
    SDSP_TRY(launch_fir_step(h->dtype, a, h->stream), "fir step");
    h->cur ^= 1;
    h->ci = (h->ci + 1) % h->M;
    h->host_valid = false;
    // the flag is released after the whole workgroup's delay-line stores; the fence orders any
    // later launch on a caller stream after the kernel itself
    SDSP_TRY(h->fence.record(h->stream), "record fence");
    SDSP_TRY(wait_host_flag(flag_h, seq, h->stream), "fir step wait");
    if (emit && out) std::memcpy(out, h->step_out.host, sample_bytes(h->dtype));
    if (n_out) *n_out = emit ? 1 : 0;
    return SDSP_OK;
}

int fir_step(sdsp_fir* h, const void* sample, void* out, size_t* n_out, bool want) {
    if (!h || !sample || h->channels != 1) return SDSP_E_INVALID_ARGUMENT;
    DeviceGuard g(h->device);
    if (!h->host_step) return fir_step_device(h, sample, out, n_out, want);
    size_t k = 0;
    int st = host_run(h, (const unsigned char*)sample, 1, want ? (unsigned char*)out : nullptr, &k);
    if (n_out) *n_out = k;
    return st;
}
}  // namespace

extern "C" {

const char* sdsp_last_error(void) { return g_last_error.c_str(); }
const char* sdsp_version(void) { return "sdsp 0.1.0 (gfx950)"; }
size_t sdsp_sample_size(int dtype) { return sample_bytes(dtype); }
size_t sdsp_coef_size(int dtype) { return coef_bytes(dtype); }

int sdsp_device_count(void) {
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess) return 0;
    int n = 0;
    for (int d = 0; d < count; ++d) {
        hipDeviceProp_t p;
        if (hipGetDeviceProperties(&p, d) == hipSuccess && std::strncmp(p.gcnArchName, "gfx950", 6) == 0) ++n;
    }
    return n;
}

int sdsp_fir_create(sdsp_fir** out, int dtype, const void* taps, size_t len, const void* scale, int device) {
    return fir_create_common(out, dtype, taps, len, scale, 1, device);
}

int sdsp_decim_create(sdsp_fir** out, int dtype, const void* taps, size_t len, const void* scale,
                      size_t decimation, int device) {
    return fir_create_common(out, dtype, taps, len, scale, decimation, device);
}

void sdsp_fir_destroy(sdsp_fir* h) {
    if (!h) return;
    {
        DeviceGuard g(h->device);
        (void)h->fence.wait();  // work queued on a caller stream may still read the tables / history
        if (h->stream) {
            (void)hipStreamSynchronize(h->stream);
            (void)hipStreamDestroy(h->stream);
        }
        h->d_taps_rev.release();
        h->d_hist[0].release();
        h->d_hist[1].release();
        h->stage_in.release();
        h->stage_out.release();
        h->d_H.release();
        h->d_tw1.release();
        h->d_tw2.release();
        h->d_pkt.release();
        h->d_ostab.release();
        h->d_hhalf.release();
    }
    delete h;
}

int sdsp_fir_set_channels(sdsp_fir* h, size_t channels) {
    if (!h || channels == 0) return SDSP_E_INVALID_ARGUMENT;
    DeviceGuard g(h->device);
    h->channels = channels;
    return fir_alloc_state(h);
}

int sdsp_fir_set_algo(sdsp_fir* h, int algo) {
    if (!h || algo < 0 || algo > 3) return SDSP_E_INVALID_ARGUMENT;
    if (algo == SDSP_ALGO_FFT && !ols_applicable(h)) {
        set_error("overlap-save needs 32-bit complex samples, no decimation and L-1 <= 3840");
        return SDSP_E_UNSUPPORTED;
    }
    h->algo = algo;
    return SDSP_OK;
}

int sdsp_fir_get_algo(const sdsp_fir* h) { return h ? h->algo : -1; }

int sdsp_set_default_algo(int algo) {
    if (algo != SDSP_ALGO_AUTO && algo != SDSP_ALGO_EXACT && algo != SDSP_ALGO_FMA) {
        set_error("default algorithm: SDSP_ALGO_AUTO, SDSP_ALGO_EXACT or SDSP_ALGO_FMA");
        return SDSP_E_INVALID_ARGUMENT;
    }
    sdsp::g_default_algo.store(algo);
    return SDSP_OK;
}

int sdsp_get_default_algo(void) { return sdsp::default_algo(); }

int sdsp_fir_set_tuning(sdsp_fir* h, int key, int value) {
    if (!h) return SDSP_E_INVALID_ARGUMENT;
    switch (key) {
        case SDSP_TUNE_OLS_KERNEL:  // every value computes the full output (performance only)
            if (value < kOlsOneShot || value > kOlsOneShotWide) return SDSP_E_INVALID_ARGUMENT;
            h->ols_kernel = value;
            h->ols.kernel = value;
            return SDSP_OK;
        case SDSP_TUNE_DECIM_SEG:
            if (value < 0) return SDSP_E_INVALID_ARGUMENT;
            h->decim_seg = value;
            return SDSP_OK;
        case SDSP_TUNE_HOST_STEP:
            if (value < 0 || value > 1) return SDSP_E_INVALID_ARGUMENT;
            if (!value) {  // the device kernels take over: they need the newest window
                DeviceGuard g(h->device);
                int st = host_flush(h);
                if (st) return st;
            }
            h->host_step = value;
            return SDSP_OK;
        case SDSP_TUNE_HOST_BLOCK_MACS:
            if (value < 0) return SDSP_E_INVALID_ARGUMENT;
            h->host_macs = (size_t)value;
            return SDSP_OK;
        default:
            set_error("unknown or retired tuning key");
            return SDSP_E_INVALID_ARGUMENT;
    }
}

int sdsp_fir_clone(const sdsp_fir* h, sdsp_fir** out) {
    if (!h || !out) return SDSP_E_INVALID_ARGUMENT;
    int st = fir_create_common(out, h->dtype, h->taps.data(), h->L, h->scale.data(), h->M, h->device);
    if (st) return st;
    sdsp_fir* c = *out;
    DeviceGuard g(h->device);
    c->algo = h->algo;
    if (h->channels != 1) {
        st = sdsp_fir_set_channels(c, h->channels);
        if (st) return st;
    }
    c->ols_kernel = h->ols_kernel;
    c->decim_seg = h->decim_seg;
    const size_t hb = h->channels * (h->L - 1) * sample_bytes(h->dtype);
    SDSP_TRY(h->fence.wait(), "wait for queued work");
    SDSP_TRY(hipStreamSynchronize(h->stream), "sync");
    st = host_flush(h);
    if (st) return st;
    if (hb) SDSP_TRY(hipMemcpy(c->d_hist[0].p, h->d_hist[h->cur].p, hb, hipMemcpyDeviceToDevice), "clone state");
    c->cur = 0;
    c->ci = h->ci;
    c->host_step = h->host_step;
    c->host_macs = h->host_macs;
    c->host_valid = false;
    return SDSP_OK;
}

int sdsp_fir_set_scale(sdsp_fir* h, const void* scale) {
    if (!h || !scale) return SDSP_E_INVALID_ARGUMENT;
    DeviceGuard g(h->device);
    SDSP_TRY(h->fence.wait(), "wait for queued work");  // the next run rebuilds tables a queued kernel may read
    std::memcpy(h->scale.data(), scale, h->scale.size());
    h->ols_ok = false;
    return SDSP_OK;
}
int sdsp_fir_get_scale(const sdsp_fir* h, void* scale) {
    if (!h || !scale) return SDSP_E_INVALID_ARGUMENT;
    std::memcpy(scale, h->scale.data(), h->scale.size());
    return SDSP_OK;
}
size_t sdsp_fir_len(const sdsp_fir* h) { return h ? h->L : 0; }
size_t sdsp_fir_decimation(const sdsp_fir* h) { return h ? h->M : 0; }

int sdsp_fir_coefficients(const sdsp_fir* h, void* out) {
    if (!h || !out) return SDSP_E_INVALID_ARGUMENT;
    const size_t cb = coef_bytes(h->dtype);
    unsigned char* o = (unsigned char*)out;
    for (size_t i = 0; i < h->L; ++i) std::memcpy(o + i * cb, &h->taps[(h->L - 1 - i) * cb], cb);
    return SDSP_OK;
}

size_t sdsp_fir_output_count(const sdsp_fir* h, size_t n) {
    if (!h) return 0;
    if (h->M == 1) return n;
    const size_t j0 = (h->M - 1 - h->ci) % h->M;  // first input index whose push wraps the phase to 0
    return j0 < n ? (n - 1 - j0) / h->M + 1 : 0;
}

int sdsp_fir_execute_block_device(sdsp_fir* h, const void* d_in, size_t n, void* d_out, size_t* n_out,
                                  void* stream) {
    if (!h) return SDSP_E_INVALID_ARGUMENT;
    DeviceGuard g(h->device);
    hipStream_t s = pick(stream, h->stream);
    const size_t nout = sdsp_fir_output_count(h, n);
    if (n_out) *n_out = nout;
    if (n == 0) return SDSP_OK;
    const size_t sb = sample_bytes(h->dtype);
    if (ranges_overlap(d_in, h->channels * n * sb, d_out, h->channels * nout * sb)) {
        set_error("input and output blocks overlap (in-place filtering is not supported)");
        return SDSP_E_INVALID_ARGUMENT;
    }
    int hst = host_flush(h);
    if (hst) return hst;
    ++h->device_ops;
    h->host_valid = false;  // the input is device-resident: the host window is re-read when needed
    // work queued on another stream (the fence) reads or writes the history this launch uses
    SDSP_TRY(h->fence.order_before(s), "order after queued work");
    const void* hist = h->d_hist[h->cur].p;
    bool hist_done = false;  // the overlap-save launch wrote the next history itself
    if (h->M == 1) {
        const int algo = fir_resolve_algo(h, n);
        if (algo == SDSP_ALGO_FFT) {
            if (!h->ols_ok) {
                int st = ols_build(h);
                if (st) return st;
            }
            SDSP_TRY(launch_fir_ols(h->ols, d_in, hist, h->d_hist[h->cur ^ 1].p, d_out, n, (int)h->L, h->channels,
                                    h->cus, s, &hist_done),
                     "fir ols");
        } else {
            FirArgs a{d_in, hist, h->d_taps_rev.p, h->scale.data(), d_out, n, n, h->channels, (int)h->L, 1, 0,
                      algo != SDSP_ALGO_FMA};
            SDSP_TRY(launch_fir_direct(h->dtype, a, s), "fir direct");
        }
    } else {
        const size_t j0 = (h->M - 1 - h->ci) % h->M;
        const int algo = decim_resolve_algo(h, n) == SDSP_ALGO_FMA ? SDSP_ALGO_FMA : SDSP_ALGO_EXACT;
        FirArgs a{d_in, hist, h->d_taps_rev.p, h->scale.data(), d_out, n, nout, h->channels, (int)h->L, (int)h->M,
                  j0, algo != SDSP_ALGO_FMA};
        a.seg = h->decim_seg;
        SDSP_TRY(launch_decim_direct(h->dtype, a, s), "decim direct");
        h->ci = (h->ci + n) % h->M;
    }
    if (!hist_done)
        SDSP_TRY(launch_hist_update(h->dtype, d_in, hist, h->d_hist[h->cur ^ 1].p, n, (int)h->L - 1, h->channels, s),
                 "history update");
    h->cur ^= 1;
    SDSP_TRY(h->fence.record(s), "record fence");
    return SDSP_OK;
}

int sdsp_fir_execute_block(sdsp_fir* h, const void* in, size_t n, void* out, size_t* n_out) {
    if (!h) return SDSP_E_INVALID_ARGUMENT;
    DeviceGuard g(h->device);
    SDSP_TRY(h->fence.wait(), "wait for queued work");
    const size_t sb = sample_bytes(h->dtype);
    const size_t nout = sdsp_fir_output_count(h, n);
    if (n_out) *n_out = nout;
    if (n == 0) return SDSP_OK;
    if (host_eligible(h, n)) return host_run(h, (const unsigned char*)in, n, (unsigned char*)out, nullptr);
    const bool keep = h->host_valid;
    SDSP_TRY(h->stage_in.ensure(h->channels * n * sb), "stage in");
    SDSP_TRY(h->stage_out.ensure(h->channels * std::max<size_t>(nout, 1) * sb), "stage out");
    SDSP_TRY(hipMemcpyAsync(h->stage_in.p, in, h->channels * n * sb, hipMemcpyHostToDevice, h->stream), "H2D");
    int st = sdsp_fir_execute_block_device(h, h->stage_in.p, n, h->stage_out.p, nullptr, h->stream);
    if (st) return st;
    if (nout)
        SDSP_TRY(hipMemcpyAsync(out, h->stage_out.p, h->channels * nout * sb, hipMemcpyDeviceToHost, h->stream),
                 "D2H");
    SDSP_TRY(hipStreamSynchronize(h->stream), "sync");
    h->host_valid = keep;  // the host holds the input: move its window on without a read-back
    host_feed(h, (const unsigned char*)in, n);
    return SDSP_OK;
}

int sdsp_fir_execute(sdsp_fir* h, const void* sample, void* out, size_t* n_out) {
    if (!out) return SDSP_E_INVALID_ARGUMENT;
    return fir_step(h, sample, out, n_out, true);
}

int sdsp_decim_write(sdsp_fir* h, const void* samples, size_t n) {
    if (!h) return SDSP_E_INVALID_ARGUMENT;
    if (n == 0) return SDSP_OK;
    DeviceGuard g(h->device);
    SDSP_TRY(h->fence.wait(), "wait for queued work");
    if (host_eligible(h, n)) return host_run(h, (const unsigned char*)samples, n, nullptr, nullptr);
    int hst = host_flush(h);
    if (hst) return hst;
    const size_t sb = sample_bytes(h->dtype);
    ++h->device_ops;
    SDSP_TRY(h->stage_in.ensure(h->channels * n * sb), "stage in");
    SDSP_TRY(hipMemcpyAsync(h->stage_in.p, samples, h->channels * n * sb, hipMemcpyHostToDevice, h->stream), "H2D");
    SDSP_TRY(launch_hist_update(h->dtype, h->stage_in.p, h->d_hist[h->cur].p, h->d_hist[h->cur ^ 1].p, n,
                                (int)h->L - 1, h->channels, h->stream),
             "history update");
    h->cur ^= 1;
    h->ci = (h->ci + n) % h->M;
    SDSP_TRY(hipStreamSynchronize(h->stream), "sync");
    host_feed(h, (const unsigned char*)samples, n);
    return SDSP_OK;
}

int sdsp_decim_push(sdsp_fir* h, const void* sample) {
    if (h && h->channels != 1) return sdsp_decim_write(h, sample, 1);  // one sample per channel
    return fir_step(h, sample, nullptr, nullptr, false);
}

int sdsp_fir_reset(sdsp_fir* h) {
    if (!h) return SDSP_E_INVALID_ARGUMENT;
    DeviceGuard g(h->device);
    return fir_alloc_state(h);
}

size_t sdsp_fir_state_len(const sdsp_fir* h) { return h ? h->channels * (h->L - 1) : 0; }

int sdsp_fir_get_state(const sdsp_fir* h, void* hist, size_t* phase) {
    if (!h) return SDSP_E_INVALID_ARGUMENT;
    DeviceGuard g(h->device);
    const size_t hb = h->channels * (h->L - 1) * sample_bytes(h->dtype);
    SDSP_TRY(h->fence.wait(), "wait for queued work");
    SDSP_TRY(hipStreamSynchronize(h->stream), "sync");
    if (h->dev_stale) {  // the host window is the newer one
        if (hb && hist) std::memcpy(hist, h->hbuf.data() + h->hpos * sample_bytes(h->dtype), hb);
    } else if (hb && hist) {
        SDSP_TRY(hipMemcpy(hist, h->d_hist[h->cur].p, hb, hipMemcpyDeviceToHost), "get state");
    }
    if (phase) *phase = h->ci;
    return SDSP_OK;
}

int sdsp_fir_set_state(sdsp_fir* h, const void* hist, size_t phase) {
    if (!h || phase >= h->M) return SDSP_E_INVALID_ARGUMENT;
    DeviceGuard g(h->device);
    const size_t hb = h->channels * (h->L - 1) * sample_bytes(h->dtype);
    SDSP_TRY(h->fence.wait(), "wait for queued work");
    SDSP_TRY(hipStreamSynchronize(h->stream), "sync");
    if (hb && hist) SDSP_TRY(hipMemcpy(h->d_hist[h->cur].p, hist, hb, hipMemcpyHostToDevice), "set state");
    h->ci = phase;
    h->dev_stale = false;
    h->host_valid = false;  // re-read on the next host step
    return SDSP_OK;
}

int sdsp_fir_frequency_response(const sdsp_fir* h, double f, double* re_im) {
    if (!h || !re_im) return SDSP_E_INVALID_ARGUMENT;
    // coefficients() returns the REVERSED stored taps (fir/mod.rs:173-176, used at :263-273)
    std::vector<cd> c(h->L);
    for (size_t i = 0; i < h->L; ++i) c[i] = coef_at(h->taps.data(), h->dtype, h->L - 1 - i);
    const bool real = !coef_is_complex(h->dtype);
    cd o = poly_response(c, real, f);
    cd s = coef_at(h->scale.data(), h->dtype, 0);
    cd r = real ? cmul(s.re, o) : cmul(s, o);
    re_im[0] = r.re;
    re_im[1] = r.im;
    return SDSP_OK;
}

int sdsp_fir_group_delay(const sdsp_fir* h, double f, double* delay) {
    if (!h || !delay) return SDSP_E_INVALID_ARGUMENT;
    std::vector<cd> c(h->L);
    for (size_t i = 0; i < h->L; ++i) c[i] = coef_at(h->taps.data(), h->dtype, h->L - 1 - i);
    double d = 0.0;
    if (fir_group_delay(c, !coef_is_complex(h->dtype), f, &d)) d = 0.0;  // errors map to 0.0 (:293-303)
    *delay = d;
    return SDSP_OK;
}

unsigned long long sdsp_fir_device_ops(const sdsp_fir* h) { return h ? h->device_ops : 0; }

int sdsp_fir_synchronize(sdsp_fir* h) {
    if (!h) return SDSP_E_INVALID_ARGUMENT;
    DeviceGuard g(h->device);
    SDSP_TRY(h->fence.wait(), "wait for queued work");
    SDSP_TRY(hipStreamSynchronize(h->stream), "sync");
    return SDSP_OK;
}

}  // extern "C"

// ===========================================================================
// Polyphase filterbank / interpolating FIR
// ===========================================================================
struct sdsp_pfb {
    int dtype = 0, device = 0;
    size_t M = 0, K = 0, channels = 1;
    bool interp = false;
    std::vector<unsigned char> cb;     // [M][K] branch coefficients, stored order
    std::vector<unsigned char> scale;  // kept, never applied (pfb.rs:85-90)
    DevBuf d_cb;
    DevBuf d_hist[2];  // [channels][K] : the Window(K), oldest first
    int cur = 0;
    int algo = SDSP_ALGO_EXACT;
    hipStream_t stream = nullptr;
    mutable StreamFence fence;  // last caller stream an execute call was queued on
    DevBuf stage_in, stage_out;
};

namespace {

int pfb_alloc_state(sdsp_pfb* h) {
    SDSP_TRY(h->fence.wait(), "wait for queued work");
    const size_t hb = h->channels * h->K * sample_bytes(h->dtype);
    for (int i = 0; i < 2; ++i) {
        SDSP_TRY(h->d_hist[i].ensure(hb), "alloc window");
        SDSP_TRY(hipMemsetAsync(h->d_hist[i].p, 0, hb, h->stream), "zero window");
    }
    h->cur = 0;
    SDSP_TRY(hipStreamSynchronize(h->stream), "sync");
    return SDSP_OK;
}

int pfb_create_common(sdsp_pfb** out, int dtype, const unsigned char* taps, size_t len, size_t M,
                      const unsigned char* scale, bool interp, int device) {
    *out = nullptr;
    const size_t cbytes = coef_bytes(dtype);
    const size_t K = len / M;
    if (K == 0) {  // the reference panics in Window::new(0) (src/window/mod.rs:18)
        set_error("fewer taps than filters: sub-filter length 0");
        return SDSP_E_INVALID_ARGUMENT;
    }
    DeviceInfo info;
    int st = check_device(device, &info);
    if (st) return st;
    DeviceGuard g(device);
    sdsp_pfb* h = new sdsp_pfb();
    h->dtype = dtype;
    h->device = device;
    h->algo = default_algo() == SDSP_ALGO_FMA ? SDSP_ALGO_FMA : SDSP_ALGO_EXACT;  // (EXACT / FMA only)
    h->M = M;
    h->K = K;
    h->interp = interp;
    h->scale.assign(scale, scale + cbytes);
    h->cb.resize(M * K * cbytes);
    // rev_sub_coefs[K - index - 1] = coefficients[filter + index * filters]  (pfb.rs:33-40)
    for (size_t p = 0; p < M; ++p)
        for (size_t idx = 0; idx < K; ++idx)
            std::memcpy(&h->cb[(p * K + (K - idx - 1)) * cbytes], taps + (p + idx * M) * cbytes, cbytes);
    hipError_t e = hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking);
    if (e == hipSuccess) e = h->d_cb.ensure(h->cb.size());
    if (e == hipSuccess) e = hipMemcpy(h->d_cb.p, h->cb.data(), h->cb.size(), hipMemcpyHostToDevice);
    if (e != hipSuccess) {
        st = device_status(e, "pfb create");
        sdsp_pfb_destroy(h);
        return st;
    }
    st = pfb_alloc_state(h);
    if (st) {
        sdsp_pfb_destroy(h);
        return st;
    }
    *out = h;
    return SDSP_OK;
}

}  // namespace

extern "C" {

int sdsp_pfb_create(sdsp_pfb** out, int dtype, const void* taps, size_t len, size_t filters, const void* scale,
                    int device) {
    if (!out) return SDSP_E_INVALID_ARGUMENT;
    *out = nullptr;
    if (dtype < 0 || dtype > 5) return SDSP_E_INVALID_ARGUMENT;
    if (filters == 0) {  // pfb.rs:25-26
        set_error("FIR Filter Error NotEnoughFilters");
        return SDSP_E_NOT_ENOUGH_FILTERS;
    }
    if (len == 0) {  // pfb.rs:27-28
        set_error("FIR Filter Error CoefficientsLengthZero");
        return SDSP_E_COEFFICIENTS_LENGTH_ZERO;
    }
    return pfb_create_common(out, dtype, (const unsigned char*)taps, len, filters, (const unsigned char*)scale,
                             false, device);
}

int sdsp_interp_create(sdsp_pfb** out, int dtype, const void* taps, size_t len, size_t M, int device) {
    if (!out) return SDSP_E_INVALID_ARGUMENT;
    *out = nullptr;
    if (dtype < 0 || dtype > 5) return SDSP_E_INVALID_ARGUMENT;
    if (len == 0) {  // interp.rs:28-29
        set_error("FIR Filter Error CoefficientsLengthZero");
        return SDSP_E_COEFFICIENTS_LENGTH_ZERO;
    }
    if (M < 1) {  // interp.rs:30-31
        set_error("FIR Filter Error InterpolationLessThanOne");
        return SDSP_E_INTERPOLATION_LESS_THAN_ONE;
    }
    // sub-filter length computed in f32 (interp.rs:35-40), taps zero-padded to K*M (:43-46)
    const float q = (float)len / (float)M;
    const size_t K = (q == std::floor(q)) ? (size_t)q : (size_t)std::ceil(q);
    const size_t cbytes = coef_bytes(dtype);
    std::vector<unsigned char> eff(K * M * cbytes, 0);
    std::memcpy(eff.data(), taps, std::min(len, K * M) * cbytes);
    std::vector<unsigned char> one(cbytes, 0);
    if (coef_is_f32(dtype)) { float v = 1.0f; std::memcpy(one.data(), &v, 4); }
    else { double v = 1.0; std::memcpy(one.data(), &v, 8); }
    return pfb_create_common(out, dtype, eff.data(), K * M, M, one.data(), true, device);
}

void sdsp_pfb_destroy(sdsp_pfb* h) {
    if (!h) return;
    {
        DeviceGuard g(h->device);
        if (h->stream) {
            (void)hipStreamSynchronize(h->stream);
            (void)hipStreamDestroy(h->stream);
        }
        h->d_cb.release();
        h->d_hist[0].release();
        h->d_hist[1].release();
        h->stage_in.release();
        h->stage_out.release();
    }
    delete h;
}

int sdsp_pfb_clone(const sdsp_pfb* h, sdsp_pfb** out) {
    if (!h || !out) return SDSP_E_INVALID_ARGUMENT;
    DeviceInfo info;
    int st = check_device(h->device, &info);
    if (st) return st;
    DeviceGuard g(h->device);
    sdsp_pfb* c = new sdsp_pfb();
    c->dtype = h->dtype; c->device = h->device; c->M = h->M; c->K = h->K; c->channels = h->channels;
    c->interp = h->interp; c->cb = h->cb; c->scale = h->scale; c->algo = h->algo;
    hipError_t e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
    if (e == hipSuccess) e = c->d_cb.ensure(c->cb.size());
    if (e == hipSuccess) e = hipMemcpy(c->d_cb.p, c->cb.data(), c->cb.size(), hipMemcpyHostToDevice);
    if (e != hipSuccess) { st = device_status(e, "pfb clone"); sdsp_pfb_destroy(c); return st; }
    st = pfb_alloc_state(c);
    if (st) { sdsp_pfb_destroy(c); return st; }
    const size_t hb = h->channels * h->K * sample_bytes(h->dtype);
    e = h->fence.wait();
    if (e == hipSuccess) e = hipStreamSynchronize(h->stream);
    if (e == hipSuccess) e = hipMemcpy(c->d_hist[0].p, h->d_hist[h->cur].p, hb, hipMemcpyDeviceToDevice);
    if (e != hipSuccess) { st = device_status(e, "pfb clone state"); sdsp_pfb_destroy(c); return st; }
    *out = c;
    return SDSP_OK;
}

size_t sdsp_pfb_len(const sdsp_pfb* h) { return h ? h->M : 0; }
size_t sdsp_pfb_subfilter_len(const sdsp_pfb* h) { return h ? h->K : 0; }
int sdsp_pfb_set_scale(sdsp_pfb* h, const void* scale) {
    if (!h || !scale) return SDSP_E_INVALID_ARGUMENT;
    std::memcpy(h->scale.data(), scale, h->scale.size());
    return SDSP_OK;
}
int sdsp_pfb_get_scale(const sdsp_pfb* h, void* scale) {
    if (!h || !scale) return SDSP_E_INVALID_ARGUMENT;
    std::memcpy(scale, h->scale.data(), h->scale.size());
    return SDSP_OK;
}
int sdsp_pfb_coefficients(const sdsp_pfb* h, void* out) {
    if (!h || !out) return SDSP_E_INVALID_ARGUMENT;
    std::memcpy(out, h->cb.data(), h->cb.size());
    return SDSP_OK;
}

int sdsp_pfb_set_algo(sdsp_pfb* h, int algo) {
    if (!h || (algo != SDSP_ALGO_EXACT && algo != SDSP_ALGO_FMA)) return SDSP_E_INVALID_ARGUMENT;
    h->algo = algo;
    return SDSP_OK;
}

int sdsp_pfb_set_channels(sdsp_pfb* h, size_t channels) {
    if (!h || channels == 0) return SDSP_E_INVALID_ARGUMENT;
    DeviceGuard g(h->device);
    h->channels = channels;
    return pfb_alloc_state(h);
}

int sdsp_pfb_execute_block_device(sdsp_pfb* h, const void* d_in, size_t n, void* d_out, void* stream) {
    if (!h) return SDSP_E_INVALID_ARGUMENT;
    if (n == 0) return SDSP_OK;
    DeviceGuard g(h->device);
    hipStream_t s = pick(stream, h->stream);
    const size_t sb = sample_bytes(h->dtype);
    if (ranges_overlap(d_in, h->channels * n * sb, d_out, h->channels * n * h->M * sb)) {
        set_error("input and output blocks overlap (in-place filtering is not supported)");
        return SDSP_E_INVALID_ARGUMENT;
    }
    // work queued on another stream (the fence) reads or writes the window this launch uses
    SDSP_TRY(h->fence.order_before(s), "order after queued work");
    PfbArgs a{d_in, h->d_hist[h->cur].p, h->d_cb.p, d_out, n, h->channels, (int)h->K, (int)h->M, (int)h->K,
              h->algo != SDSP_ALGO_FMA};
    SDSP_TRY(launch_pfb(h->dtype, a, s), "pfb");
    SDSP_TRY(launch_hist_update(h->dtype, d_in, h->d_hist[h->cur].p, h->d_hist[h->cur ^ 1].p, n, (int)h->K,
                                h->channels, s),
             "window update");
    h->cur ^= 1;
    SDSP_TRY(h->fence.record(s), "record fence");
    return SDSP_OK;
}

int sdsp_pfb_execute_block(sdsp_pfb* h, const void* in, size_t n, void* out) {
    if (!h) return SDSP_E_INVALID_ARGUMENT;
    if (n == 0) return SDSP_OK;
    DeviceGuard g(h->device);
    SDSP_TRY(h->fence.wait(), "wait for queued work");
    const size_t sb = sample_bytes(h->dtype);
    SDSP_TRY(h->stage_in.ensure(h->channels * n * sb), "stage in");
    SDSP_TRY(h->stage_out.ensure(h->channels * n * h->M * sb), "stage out");
    SDSP_TRY(hipMemcpyAsync(h->stage_in.p, in, h->channels * n * sb, hipMemcpyHostToDevice, h->stream), "H2D");
    int st = sdsp_pfb_execute_block_device(h, h->stage_in.p, n, h->stage_out.p, h->stream);
    if (st) return st;
    SDSP_TRY(hipMemcpyAsync(out, h->stage_out.p, h->channels * n * h->M * sb, hipMemcpyDeviceToHost, h->stream),
             "D2H");
    SDSP_TRY(hipStreamSynchronize(h->stream), "sync");
    return SDSP_OK;
}

int sdsp_pfb_push(sdsp_pfb* h, const void* sample) {
    if (!h || h->channels != 1) return SDSP_E_INVALID_ARGUMENT;
    DeviceGuard g(h->device);
    SDSP_TRY(h->fence.wait(), "wait for queued work");
    const size_t sb = sample_bytes(h->dtype);
    SDSP_TRY(h->stage_in.ensure(sb), "stage in");
    SDSP_TRY(hipMemcpyAsync(h->stage_in.p, sample, sb, hipMemcpyHostToDevice, h->stream), "H2D");
    SDSP_TRY(launch_hist_update(h->dtype, h->stage_in.p, h->d_hist[h->cur].p, h->d_hist[h->cur ^ 1].p, 1,
                                (int)h->K, 1, h->stream),
             "window push");
    h->cur ^= 1;
    SDSP_TRY(hipStreamSynchronize(h->stream), "sync");
    return SDSP_OK;
}

int sdsp_pfb_execute(sdsp_pfb* h, size_t index, void* out) {
    if (!h || h->channels != 1 || index >= h->M) return SDSP_E_INVALID_ARGUMENT;
    DeviceGuard g(h->device);
    SDSP_TRY(h->fence.wait(), "wait for queued work");
    const size_t sb = sample_bytes(h->dtype);
    SDSP_TRY(h->stage_out.ensure(h->M * sb), "stage out");
    // all branches on the current window: x = newest sample, history = the K-1 before it
    const unsigned char* win = (const unsigned char*)h->d_hist[h->cur].p;
    PfbArgs a{win + (h->K - 1) * sb, win, h->d_cb.p, h->stage_out.p, 1, 1, (int)h->K, (int)h->M,
              (int)h->K - 1, h->algo != SDSP_ALGO_FMA};
    SDSP_TRY(launch_pfb(h->dtype, a, h->stream), "pfb execute");
    SDSP_TRY(hipMemcpyAsync(out, (unsigned char*)h->stage_out.p + index * sb, sb, hipMemcpyDeviceToHost, h->stream),
             "D2H");
    SDSP_TRY(hipStreamSynchronize(h->stream), "sync");
    return SDSP_OK;
}

int sdsp_pfb_reset(sdsp_pfb* h) {
    if (!h) return SDSP_E_INVALID_ARGUMENT;
    DeviceGuard g(h->device);
    return pfb_alloc_state(h);
}

// InterpolatingFIRFilter::frequency_response / group_delay over the flattened
// branch coefficients (interp.rs:113-137); PolyPhaseFilterBank has no Filter impl.
int sdsp_pfb_frequency_response(const sdsp_pfb* h, double f, double* re_im) {
    if (!h || !re_im) return SDSP_E_INVALID_ARGUMENT;
    std::vector<cd> c(h->M * h->K);
    for (size_t i = 0; i < c.size(); ++i) c[i] = coef_at(h->cb.data(), h->dtype, i);
    const bool real = !coef_is_complex(h->dtype);
    cd o = poly_response(c, real, f);
    cd s = coef_at(h->scale.data(), h->dtype, 0);
    cd r = real ? cmul(s.re, o) : cmul(s, o);
    re_im[0] = r.re;
    re_im[1] = r.im;
    return SDSP_OK;
}

int sdsp_pfb_group_delay(const sdsp_pfb* h, double f, double* delay) {
    if (!h || !delay) return SDSP_E_INVALID_ARGUMENT;
    std::vector<cd> c(h->M * h->K);
    for (size_t i = 0; i < c.size(); ++i) c[i] = coef_at(h->cb.data(), h->dtype, i);
    double d = 0.0;
    if (fir_group_delay(c, !coef_is_complex(h->dtype), f, &d)) d = 0.0;
    *delay = d;
    return SDSP_OK;
}

int sdsp_pfb_synchronize(sdsp_pfb* h) {
    if (!h) return SDSP_E_INVALID_ARGUMENT;
    DeviceGuard g(h->device);
    SDSP_TRY(hipStreamSynchronize(h->stream), "sync");
    return SDSP_OK;
}

// ===========================================================================
// utilities
// ===========================================================================
int sdsp_bandwidth_copy_device(const void* d_src, void* d_dst, size_t bytes, void* stream) {
    int dev = 0;
    SDSP_TRY(hipGetDevice(&dev), "get device");
    hipDeviceProp_t p;
    SDSP_TRY(hipGetDeviceProperties(&p, dev), "props");
    SDSP_TRY(launch_bw_copy(d_src, d_dst, bytes, p.multiProcessorCount, (hipStream_t)stream), "bw copy");
    return SDSP_OK;
}

int sdsp_synth_f32_device(void* d_out, uint64_t seed, uint64_t channel, uint64_t start, size_t count,
                          void* stream) {
    SDSP_TRY(launch_synth_f32((float*)d_out, seed, channel, start, count, (hipStream_t)stream), "synth");
    return SDSP_OK;
}

}  // extern "C"
