// C-ABI runtime for the IIR family: IIRFilter (Normal / SecondOrder),
// SecondOrderFilter, DecimatingIIRFilter, InterpolatingIIRFilter
// (src/filter/iir/{mod,sos,decim,interp}.rs).  Coefficient normalisation by
// a0 happens here, once, in the handle's Coef precision exactly as the
// reference does it (sos.rs:61-68, mod.rs:111-118); the streaming recurrence
// runs in kern_iir.hip.
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

#define IIR_TRY(expr, what)                                    \
    do {                                                       \
        hipError_t _e = (expr);                                \
        if (_e != hipSuccess) return device_status(_e, what);  \
    } while (0)

constexpr int kMaxGroupSections = 8;  // sections per kernel launch (longer cascades chain launches)
constexpr int kScanLanes = 256;
constexpr int kMaxNormalCap = 32;

struct Group {
    int first = 0, count = 0;  // sections [first, first+count)
    int wc = 0;                // warm-up chunks for the scan path (0: scan not applicable)
    DevBuf d_P;                // [8][2c][2c]
    struct WaveScan {          // wave-scan tables per chunk-size variant (256 B, 128 B)
        int wc = 0;
        bool exact = false;    // wc == 0 but bounded: exact inter-wave carries (Phi)
        DevBuf d_P, d_Cr;      // [6][2c][2c], [B][2c] output response to the state
        DevBuf d_Phi;          // exact carries: [8][2c][2c] A^(64 B t), t = 1..8
        long long phi_wmax[9] = {-1, -1, -1, -1, -1, -1, -1, -1, -1};  // per tpw: waves the carry chain admits
    } ws[6];
    // SOS wave scan in b0-factored coordinates (kern_iir_wscan.hip sys_step): the group's
    // coefficients (1, b1/b0, b2/b0, a1, a2) per section, (G b0, G b1, G b2, a1, a2) for the last
    // (G = prod of the b0 before it), and on the device the state scales G_q and their inverses
    std::vector<double> wc64;
    std::vector<double> wscale;  // [2 count]: reference state = kernel state * wscale
    DevBuf d_wcoefs;
};

struct DeviceGuardI {
    int prev = -1;
    explicit DeviceGuardI(int d) {
        (void)hipGetDevice(&prev);
        if (prev != d) (void)hipSetDevice(d);
    }
    ~DeviceGuardI() {
        int cur = -1;
        (void)hipGetDevice(&cur);
        if (prev >= 0 && cur != prev) (void)hipSetDevice(prev);
    }
};

using Mat = std::vector<double>;  // row-major D x D
Mat matmul(const Mat& a, const Mat& b, int D) {
    Mat c(D * D, 0.0);
    for (int i = 0; i < D; ++i)
        for (int k = 0; k < D; ++k) {
            const double v = a[i * D + k];
            if (v == 0.0) continue;
            for (int j = 0; j < D; ++j) c[i * D + j] += v * b[k * D + j];
        }
    return c;
}
Mat matpow(Mat a, long long e, int D) {
    Mat r(D * D, 0.0);
    for (int i = 0; i < D; ++i) r[i * D + i] = 1.0;
    while (e > 0) {
        if (e & 1) r = matmul(r, a, D);
        a = matmul(a, a, D);
        e >>= 1;
    }
    return r;
}
double norm_inf(const Mat& a, int D) {
    double m = 0.0;
    for (int i = 0; i < D; ++i) {
        double s = 0.0;
        for (int j = 0; j < D; ++j) s += std::fabs(a[i * D + j]);
        m = std::max(m, s);
    }
    return m;
}

}  // namespace

struct sdsp_iir {
    int dtype = 0, device = 0, cus = 256;
    int type = 1;       // 0 Normal, 1 SecondOrder
    int mode = 0;       // 0 IIRFilter, 1 DecimatingIIRFilter, 2 InterpolatingIIRFilter
    size_t M = 1;
    size_t channels = 1;
    size_t phase = 0;   // DecimatingIIRFilter::index (decim.rs:9)
    std::vector<unsigned char> ff, fb;   // as given (Coef type)
    std::vector<double> c64;             // normalised coefficients widened (host queries)
    std::vector<unsigned char> cdev;     // normalised coefficients in the Coef type (device layout)
    int S = 0, nb = 0, na = 0, cap = 0;
    std::vector<Group> groups;
    DevBuf d_coefs, d_coefs_nrm, d_state[2], d_tmp[2], d_carry[2];
    int cur = 0;
    int algo = SDSP_ALGO_EXACT;  // reference-order recurrence unless the caller opts in (sdsp.h)
    int wscan = 1;  // 0: block scan; 1-6: wave-scan variant 0-5 (kern_iir_wscan.hip; sdsp_iir_set_tuning)
    hipStream_t stream = nullptr;
    mutable StreamFence fence;  // last caller stream an execute call was queued on
    DevBuf stage_in, stage_out;
    size_t state_per_ch() const { return type == 1 ? (size_t)(2 * S) : (size_t)(cap - 1); }
};

namespace {

bool is_f32(int dt) { return dt == SDSP_RR32 || dt == SDSP_RC32; }

// one Coef value from raw bytes
double cval(const std::vector<unsigned char>& v, int dt, size_t i) {
    if (is_f32(dt)) { float f; std::memcpy(&f, v.data() + 4 * i, 4); return f; }
    double d; std::memcpy(&d, v.data() + 8 * i, 8); return d;
}
// normalised value computed in the Coef type: num / den
double cdiv_t(double num, double den, int dt) {
    if (is_f32(dt)) return (double)((float)num / (float)den);
    return num / den;
}
void push_coef(std::vector<unsigned char>& out, double v, int dt) {
    if (is_f32(dt)) { float f = (float)v; const unsigned char* p = (const unsigned char*)&f; out.insert(out.end(), p, p + 4); }
    else { const unsigned char* p = (const unsigned char*)&v; out.insert(out.end(), p, p + 8); }
}

int iir_alloc_state(sdsp_iir* h) {
    IIR_TRY(h->fence.wait(), "wait for queued work");
    const size_t sb = sample_bytes(h->dtype) * h->channels * h->state_per_ch();
    for (int i = 0; i < 2; ++i) {
        IIR_TRY(h->d_state[i].ensure(sb), "alloc state");
        if (sb) IIR_TRY(hipMemsetAsync(h->d_state[i].p, 0, sb, h->stream), "zero state");
    }
    h->cur = 0;
    h->phase = 0;
    IIR_TRY(hipStreamSynchronize(h->stream), "sync");
    return SDSP_OK;
}


// state dimension of a scanned group: the SOS sections' (w1, w2) pairs, or the
// Normal DF-II delay line (cap - 1 values)
int group_dim(const sdsp_iir* h, const Group& g) { return h->type == 1 ? 2 * g.count : h->cap - 1; }

// run the group's system over x from state s (in place) in precision T: sections
// [first, first+count) of the SOS cascade (sos.rs:92-114), or the Normal DF-II
// recurrence (mod.rs:272-279).  The coefficients are the handle's (already rounded
// to the Coef type), so T = float reproduces an f32 handle's arithmetic.
// cf: the group's SOS coefficients, 5 per section (the handle's normalised ones, or the wave
// scan's b0-factored set, group_coefs)
template <typename T>
void sys_run(const sdsp_iir* h, const Group& g, const double* cf, const T* x, T* y, size_t n, std::vector<T>& s) {
    if (h->type == 0) {
        const int D = h->cap - 1, nb = h->nb, na1 = h->na - 1;
        const double* num = h->c64.data();
        const double* den = h->c64.data() + nb;
        for (size_t k = 0; k < n; ++k) {
            T d = 0;
            for (int i = 0; i < na1; ++i) d += (T)den[i] * s[i];
            const T v = x[k] - d;
            T out = (T)num[0] * v;
            for (int i = 1; i < nb; ++i) out += (T)num[i] * s[i - 1];
            for (int i = D - 1; i > 0; --i) s[i] = s[i - 1];
            if (D > 0) s[0] = v;
            if (y) y[k] = out;
        }
        return;
    }
    for (size_t i = 0; i < n; ++i) {
        T v = x[i];
        for (int q = 0; q < g.count; ++q) {
            const double* c = cf + 5 * q;
            const T w = v - ((T)c[3] * s[2 * q] + (T)c[4] * s[2 * q + 1]);
            v = (T)c[0] * w + (T)c[1] * s[2 * q] + (T)c[2] * s[2 * q + 1];
            s[2 * q + 1] = s[2 * q];
            s[2 * q] = w;
        }
        if (y) y[i] = v;
    }
}

// the coefficients a group's system runs on: the wave scan's b0-factored set (scaled, SOS only)
// or the handle's normalised coefficients
const double* group_coefs(const sdsp_iir* h, const Group& g, bool scaled) {
    if (h->type != 1) return nullptr;
    return scaled ? g.wc64.data() : &h->c64[5 * (size_t)g.first];
}

// state-transition matrix of the group's system (zero input), row-major
Mat sys_A(const sdsp_iir* h, const Group& g, const double* cf) {
    const int D = group_dim(h, g);
    Mat A(D * D, 0.0);
    const double zero = 0.0;
    for (int j = 0; j < D; ++j) {
        std::vector<double> s(D, 0.0);
        s[j] = 1.0;
        sys_run<double>(h, g, cf, &zero, nullptr, 1, s);
        for (int i = 0; i < D; ++i) A[i * D + j] = s[i];
    }
    return A;
}

// Is carrying chunk states through A^B as accurate as the recurrence itself?  A
// cascade that integrates its input (e.g. active_lag: poles at 1 and 1 - 1.6e-6)
// grows states ~1e6 x its output, and re-associating the recurrence through powers
// of A then loses 3-6 digits against the reference-order loop (measured: 8e-6
// relative at 2^18 samples, against 2e-9 for the serial f64 loop); a high-order
// direct-form polynomial does the same through its companion matrix.  Host probe
// over 2^14 pseudo-random samples in the handle's precision T: zero-state chunks
// corrected by carried states against the serial loop, both measured against the
// serial loop in f64; admitted when the carried form is within 10x the serial
// form's own error (plus 1e-13 / 1e-7 of slack).
template <typename T>
double probe_rel(const std::vector<T>& a, const std::vector<double>& ref) {
    double num = 0.0, den = 0.0;
    for (size_t i = 0; i < ref.size(); ++i) {
        num += ((double)a[i] - ref[i]) * ((double)a[i] - ref[i]);
        den += ref[i] * ref[i];
    }
    return (std::isfinite(num) && den > 0.0) ? std::sqrt(num / den) : INFINITY;
}

template <typename T>
bool carry_well_conditioned_t(const sdsp_iir* h, const Group& g, const double* cf, int B, const Mat& AB) {
    const int D = group_dim(h, g);
    const size_t n = 1 << 14;
    std::vector<double> x64(n), ref(n);
    uint64_t r = 0x9E3779B97F4A7C15ULL;
    for (auto& v : x64) {
        r = r * 6364136223846793005ULL + 1442695040888963407ULL;
        v = (double)(float)((double)(r >> 11) * (1.0 / 9007199254740992.0) * 2.0 - 1.0);
    }
    std::vector<double> s64(D, 0.0);
    sys_run<double>(h, g, cf, x64.data(), ref.data(), n, s64);
    std::vector<T> x(x64.begin(), x64.end()), ys(n), yc(n);
    std::vector<T> st(D, 0);
    sys_run<T>(h, g, cf, x.data(), ys.data(), n, st);
    std::vector<T> cr(D * (size_t)B), ABt(AB.begin(), AB.end());
    for (int d = 0; d < D; ++d) {  // Cr[i][d]: output response to basis state e_d
        std::vector<T> zs(D, 0), zero(B, 0), out(B);
        zs[d] = 1;
        sys_run<T>(h, g, cf, zero.data(), out.data(), B, zs);
        for (int i = 0; i < B; ++i) cr[(size_t)i * D + d] = out[i];
    }
    std::vector<T> I(D, 0), e(D), nI(D);
    for (size_t k = 0; k < n; k += B) {
        std::fill(e.begin(), e.end(), T(0));
        sys_run<T>(h, g, cf, &x[k], &yc[k], B, e);
        for (int i = 0; i < B; ++i)
            for (int d = 0; d < D; ++d) yc[k + i] += cr[(size_t)i * D + d] * I[d];
        for (int a = 0; a < D; ++a) {
            T v = 0;
            for (int b = 0; b < D; ++b) v += ABt[a * D + b] * I[b];
            nI[a] = v + e[a];
        }
        I = nI;
    }
    const double e_ser = probe_rel(ys, ref), e_car = probe_rel(yc, ref);
    return e_car <= 10.0 * e_ser + (sizeof(T) == 8 ? 1e-13 : 1e-7);
}

bool carry_well_conditioned(const sdsp_iir* h, const Group& g, const double* cf, int B, const Mat& AB) {
    return is_f32(h->dtype) ? carry_well_conditioned_t<float>(h, g, cf, B, AB)
                            : carry_well_conditioned_t<double>(h, g, cf, B, AB);
}

// Scan tables for chunks of B samples: warm-up chunks wc (smallest m with
// ||A^(mB)||_inf < tol, m <= max_wc; 0 = the scan is not admissible), P_k =
// A^(B 2^k) for k < nP, and optionally Cr[i][d] (i < B): the cascade output i
// steps after starting from basis state e_d with zero input.
int scan_tables(const sdsp_iir* h, const Group& g, bool scaled, int B, int max_wc, int nP, int* wc, DevBuf* dP,
                DevBuf* dCr, DevBuf* dPhi = nullptr, bool* exact = nullptr) {
    const double tol = is_f32(h->dtype) ? 1e-9 : 1e-17;
    const int D = group_dim(h, g);
    const double* cf = group_coefs(h, g, scaled);
    const Mat A = sys_A(h, g, cf);
    const Mat AB = matpow(A, B, D);
    Mat Am = AB;
    *wc = 0;
    for (int m = 1; m <= max_wc; ++m) {
        const double nrm = norm_inf(Am, D);
        if (!std::isfinite(nrm)) break;
        if (nrm < tol) { *wc = m; break; }
        Am = matmul(Am, AB, D);
    }
    if (exact) *exact = false;
    if (*wc > 0 && h->type == 0 && !carry_well_conditioned(h, g, cf, B, AB)) {
        *wc = 0;  // a direct-form polynomial whose companion powers lose digits: serial only
        return SDSP_OK;
    }
    if (*wc == 0) {
        // a state response that does not die out (e.g. a pole at z = 1, the active_lag PLL
        // filter): exact carries between waves instead of warm-up, provided the powers of A
        // over the longest wave segment stay bounded
        if (!exact || !dPhi) return SDSP_OK;
        const Mat A64 = matpow(AB, 64, D);
        Mat At = A64;
        std::vector<unsigned char> Phi;
        for (int t = 1; t <= 8; ++t) {
            const double nrm = norm_inf(At, D);
            if (!std::isfinite(nrm) || nrm > 1e6) return SDSP_OK;
            for (double v : At) push_coef(Phi, v, h->dtype);
            At = matmul(At, A64, D);
        }
        if (!carry_well_conditioned(h, g, cf, B, AB)) return SDSP_OK;
        IIR_TRY(dPhi->ensure(Phi.size()), "alloc Phi");
        IIR_TRY(hipMemcpy(dPhi->p, Phi.data(), Phi.size(), hipMemcpyHostToDevice), "copy Phi");
        *exact = true;
    }
    std::vector<unsigned char> P;
    Mat Pk = AB;
    for (int k = 0; k < nP; ++k) {
        for (double v : Pk) push_coef(P, v, h->dtype);
        Pk = matmul(Pk, Pk, D);
    }
    IIR_TRY(dP->ensure(P.size()), "alloc P");
    IIR_TRY(hipMemcpy(dP->p, P.data(), P.size(), hipMemcpyHostToDevice), "copy P");
    if (!dCr) return SDSP_OK;
    std::vector<double> resp((size_t)B * D);
    for (int d = 0; d < D; ++d) {  // output response to basis state e_d, zero input
        std::vector<double> st(D, 0.0), zero(B, 0.0), out(B);
        st[d] = 1.0;
        sys_run<double>(h, g, cf, zero.data(), out.data(), B, st);
        for (int i = 0; i < B; ++i) resp[(size_t)i * D + d] = out[i];
    }
    std::vector<unsigned char> Cr;
    if (h->dtype == 0 && B % 2 == 0) {  // real f32: sample pairs, [B/2][D][2] (packed correction)
        for (int q = 0; q < B / 2; ++q)
            for (int d = 0; d < D; ++d)
                for (int i = 2 * q; i < 2 * q + 2; ++i) push_coef(Cr, resp[(size_t)i * D + d], h->dtype);
    } else {
        for (double v : resp) push_coef(Cr, v, h->dtype);
    }
    IIR_TRY(dCr->ensure(Cr.size()), "alloc Cr");
    IIR_TRY(hipMemcpy(dCr->p, Cr.data(), Cr.size(), hipMemcpyHostToDevice), "copy Cr");
    return SDSP_OK;
}

// Exact inter-wave carries (wc == 0) run through Phi = A^(64 B tpw) and, in the
// one-block carry kernel, Phi^R (R = ceil(W / 256), by repeated squaring in the Coef
// type) and 256 chained applications of it: the carried state is multiplied by
// powers of Phi up to Phi^W.  The plan-time probe covers chunk carries over 2^14
// samples only, so each call also bounds the powers it will use: every
// power Phi^m with m < 2^(j+1) is a product of a subset of the repeated squares
// Phi^(2^0) .. Phi^(2^j), so ||Phi^m||_inf <= prod_{i<=j} max(1, ||Phi^(2^i)||_inf); a call
// of W waves is admitted while that product stays <= 1e6 for 2^(j+1) > W (computed in
// f64, once per tpw, cached as the largest W admitted).  This is a bound, not a
// heuristic, on the growth of the carried state; a marginally stable system whose
// powers grow (a double pole at z = 1: ||A^m|| ~ m) is admitted for short calls and
// runs the reference-order recurrence for long ones, and systems with bounded powers
// (a single pole at z = 1, poles on the unit circle) admit long calls.
bool exact_carry_bounded(const sdsp_iir* h, Group& g, int wv, size_t waves, int tpw) {
    if (tpw < 1 || tpw > 8) return false;
    long long& wmax = g.ws[wv].phi_wmax[tpw];
    if (wmax < 0) {
        const int D = group_dim(h, g), B = iir_wscan_chunk(h->dtype, wv);
        Mat P = matpow(matpow(sys_A(h, g, group_coefs(h, g, true)), B, D), 64LL * tpw, D);
        wmax = 0;
        double bound = 1.0;  // >= ||Phi^m||_inf for every m < 2^(j+1)
        for (int j = 0; j < 48; ++j) {
            const double nrm = norm_inf(P, D);
            if (!std::isfinite(nrm)) break;
            bound *= nrm > 1.0 ? nrm : 1.0;
            if (bound > 1e6) break;
            wmax = (2LL << j) - 1;  // powers up to 2^(j+1) - 1: products of Phi^(2^0) .. Phi^(2^j)
            P = matmul(P, P, D);
        }
    }
    return (long long)waves <= wmax;
}

// The wave scan's b0-factored coefficient set of an SOS group (kern_iir_wscan.hip sys_step):
// section q < count - 1 runs w = v - a1 w1 - a2 w2, out = w + (b1/b0) w1 + (b2/b0) w2 on states
// divided by G_q = prod_{j<q} b0_j, and the last section (G b0, G b1, G b2) gives the reference's
// output.  Saves one multiply per section but the last per sample (cfg3: 20 -> 17 operations in
// the zero-state run).  The values are formed in f64 from the handle's normalised coefficients and
// rounded to the Coef type once.  False when a section but the last has b0 = 0 or a scale leaves
// [1e-30, 1e30].
bool wscan_coefs(const sdsp_iir* h, Group& g) {
    g.wc64.assign(5 * (size_t)g.count, 0.0);
    g.wscale.assign(2 * (size_t)g.count, 1.0);
    double G = 1.0;
    for (int q = 0; q < g.count; ++q) {
        const double* c = &h->c64[5 * (size_t)(g.first + q)];
        double* o = &g.wc64[5 * (size_t)q];
        g.wscale[2 * q] = g.wscale[2 * q + 1] = G;
        if (!(std::fabs(G) >= 1e-30 && std::fabs(G) <= 1e30)) return false;
        o[3] = c[3];
        o[4] = c[4];
        if (q + 1 < g.count) {
            if (c[0] == 0.0 || !std::isfinite(c[1] / c[0]) || !std::isfinite(c[2] / c[0])) return false;
            o[0] = 1.0;
            o[1] = c[1] / c[0];
            o[2] = c[2] / c[0];
            G *= c[0];
        } else {
            o[0] = G * c[0];
            o[1] = G * c[1];
            o[2] = G * c[2];
        }
    }
    if (!is_f32(h->dtype)) return true;
    for (double& v : g.wc64) v = (double)(float)v;  // the values the f32 kernel multiplies by
    return true;
}

int plan_groups(sdsp_iir* h) {
    h->groups.clear();
    if (h->type == 0) {  // Normal DF-II: one dense system of cap - 1 states on the wave scan (D <= 8)
        const int D = h->cap - 1;
        if (D < 1 || D > 8) return SDSP_OK;
        h->groups.emplace_back();
        Group& g = h->groups.back();
        // 256-byte chunks (variant 0), and for real f32 also 128-byte chunks (variant 1, the
        // default there as for the SOS cascades: h->wscan = 2)
        for (int v = 0; v < (h->dtype == SDSP_RR32 ? 2 : 1); ++v) {
            const int Bw = iir_wscan_chunk(h->dtype, v);
            int st = scan_tables(h, g, false, Bw, 32, 7, &g.ws[v].wc, &g.ws[v].d_P, &g.ws[v].d_Cr, &g.ws[v].d_Phi,
                                 &g.ws[v].exact);
            if (st) return st;
        }
        // the kernel's coefficient layout: num[0..D] then den[0..D), zero padded
        std::vector<unsigned char> c;
        for (int i = 0; i <= D; ++i) push_coef(c, i < h->nb ? h->c64[i] : 0.0, h->dtype);
        for (int i = 0; i < D; ++i) push_coef(c, i < h->na - 1 ? h->c64[h->nb + i] : 0.0, h->dtype);
        IIR_TRY(h->d_coefs_nrm.ensure(c.size()), "alloc normal coefs");
        IIR_TRY(hipMemcpy(h->d_coefs_nrm.p, c.data(), c.size(), hipMemcpyHostToDevice), "copy normal coefs");
        return SDSP_OK;
    }
    if (h->type != 1) return SDSP_OK;
    for (int f = 0; f < h->S; f += kMaxGroupSections) {
        h->groups.emplace_back();
        Group& g = h->groups.back();
        g.first = f;
        g.count = std::min(kMaxGroupSections, h->S - f);
        // block scan (kern_iir.hip): 8 powers, warm-up up to half the block's lanes
        int st = scan_tables(h, g, false, iir_scan_chunk(h->dtype), kScanLanes / 2, 8, &g.wc, &g.d_P, nullptr);
        if (st) return st;
        // wave scan (kern_iir_wscan.hip) in b0-factored coordinates; a section other than the last
        // with b0 = 0 (or scales out of range) has no such form: its group stays off the wave scan
        if (!wscan_coefs(h, g)) continue;
        // one table set per chunk size: 6 powers, warm-up <= 32 chunks; without a decaying state
        // response the single-chunk variants carry exactly
        for (int v = 0; v < 6; ++v) {
            const int Bw = iir_wscan_chunk(h->dtype, v);
            if (Bw == 0) continue;
            if (g.wc == 0 && v != 0 && v != 1) continue;
            st = scan_tables(h, g, true, Bw, 32, 7, &g.ws[v].wc, &g.ws[v].d_P, &g.ws[v].d_Cr, &g.ws[v].d_Phi,
                             &g.ws[v].exact);
            if (st) return st;
        }
        std::vector<unsigned char> c;  // device layout: 5 count coefficients, count * 2 scales, inverses
        for (double v : g.wc64) push_coef(c, v, h->dtype);
        for (double v : g.wscale) push_coef(c, v, h->dtype);
        for (double v : g.wscale) push_coef(c, 1.0 / v, h->dtype);
        IIR_TRY(g.d_wcoefs.ensure(c.size()), "alloc wave-scan coefs");
        IIR_TRY(hipMemcpy(g.d_wcoefs.p, c.data(), c.size(), hipMemcpyHostToDevice), "copy wave-scan coefs");
    }
    return SDSP_OK;
}

int iir_check(size_t nff, size_t nfb, int type) {
    if (type == 0) {  // IIRFilter::new Normal (mod.rs:99-104)
        if (nff == 0) { set_error("IIR Filter Error NumeratorLengthZero"); return SDSP_E_NUMERATOR_LENGTH_ZERO; }
        if (nfb == 0) { set_error("IIR Filter Error DenominatorLengthZero"); return SDSP_E_DENOMINATOR_LENGTH_ZERO; }
        return SDSP_OK;
    }
    if (type != 1) { set_error("bad IIR type"); return SDSP_E_INVALID_ARGUMENT; }
    // SecondOrder (mod.rs:131-142)
    if (nff != nfb) { set_error("IIR Filter Error SecondOrderSectionSizeMismatch"); return SDSP_E_SOS_SIZE_MISMATCH; }
    if (nff == 0) { set_error("IIR Filter Error SecondOrderSectionSizeZero"); return SDSP_E_SOS_SIZE_ZERO; }
    if (nff % 3 != 0) {
        set_error("IIR Filter Error SecondOrderSectionSizeNotMultpleOf3");
        return SDSP_E_SOS_SIZE_NOT_MULTIPLE_OF_3;
    }
    return SDSP_OK;
}

int iir_create(sdsp_iir** out, int dtype, const void* ff, size_t nff, const void* fb, size_t nfb, int type, int mode,
               size_t M, int device) {
    *out = nullptr;
    if (!(dtype == SDSP_RR32 || dtype == SDSP_RC32 || dtype == SDSP_RR64 || dtype == SDSP_RC64)) {
        set_error("IIR filters take real coefficients (the reference implements Conj/Real for f64 only)");
        return SDSP_E_UNSUPPORTED;
    }
    if (mode != 0) {  // decim.rs:191-200, interp.rs:185-194: empty checks, then the factor
        if (nff == 0) { set_error("IIR Filter Error NumeratorLengthZero"); return SDSP_E_NUMERATOR_LENGTH_ZERO; }
        if (nfb == 0) { set_error("IIR Filter Error DenominatorLengthZero"); return SDSP_E_DENOMINATOR_LENGTH_ZERO; }
        if (M < 1) {
            set_error(mode == 1 ? "IIR Filter Error DecimationLessThanOne" : "IIR Filter Error InterpolationLessThanOne");
            return mode == 1 ? SDSP_E_IIR_DECIMATION_LESS_THAN_ONE : SDSP_E_IIR_INTERPOLATION_LESS_THAN_ONE;
        }
    }
    int st = iir_check(nff, nfb, type);
    if (st) return st;
    const size_t cb = coef_bytes(dtype);
    sdsp_iir* h = new sdsp_iir();
    h->dtype = dtype;
    h->device = device;
    h->algo = default_algo();
    h->type = type;
    // real f32: 128-byte chunks (B = 32; cfg3 1.75 -> 1.72 ms, its compute-only ablation 1.63 ->
    // 1.40 ms); wider samples keep 256-byte chunks so a chunk holds >= 16 samples per scan
    h->wscan = dtype == SDSP_RR32 ? 2 : 1;
    h->mode = mode;
    h->M = mode ? M : 1;
    h->ff.assign((const unsigned char*)ff, (const unsigned char*)ff + nff * cb);
    h->fb.assign((const unsigned char*)fb, (const unsigned char*)fb + nfb * cb);
    if (type == 1) {
        h->S = (int)(nff / 3);
        for (int s = 0; s < h->S; ++s) {  // sos.rs:61-68: b = ff/a0, a = fb/a0 in the Coef type
            const double a0 = cval(h->fb, dtype, 3 * s);
            const double v[5] = {cdiv_t(cval(h->ff, dtype, 3 * s), a0, dtype), cdiv_t(cval(h->ff, dtype, 3 * s + 1), a0, dtype),
                                 cdiv_t(cval(h->ff, dtype, 3 * s + 2), a0, dtype), cdiv_t(cval(h->fb, dtype, 3 * s + 1), a0, dtype),
                                 cdiv_t(cval(h->fb, dtype, 3 * s + 2), a0, dtype)};
            for (double x : v) { h->c64.push_back(x); push_coef(h->cdev, x, dtype); }
        }
    } else {
        h->nb = (int)nff;
        h->na = (int)nfb;
        h->cap = (int)std::max(nff, nfb);  // mod.rs:105-109
        if (h->cap > kMaxNormalCap) {
            delete h;
            set_error("Normal IIR order above 31 is not supported on the device");
            return SDSP_E_UNSUPPORTED;
        }
        const double a0 = cval(h->fb, dtype, 0);
        for (size_t i = 0; i < nff; ++i) { const double v = cdiv_t(cval(h->ff, dtype, i), a0, dtype); h->c64.push_back(v); push_coef(h->cdev, v, dtype); }
        for (size_t i = 1; i < nfb; ++i) { const double v = cdiv_t(cval(h->fb, dtype, i), a0, dtype); h->c64.push_back(v); push_coef(h->cdev, v, dtype); }
    }
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0 || device < 0 || device >= ndev) {
        delete h;
        set_error("no HIP device visible (libsdsp has no CPU execution path)");
        return SDSP_E_NO_DEVICE;
    }
    DeviceGuardI g(device);
    hipDeviceProp_t p;
    if (hipGetDeviceProperties(&p, device) != hipSuccess || std::strncmp(p.gcnArchName, "gfx950", 6) != 0) {
        delete h;
        set_error("libsdsp is built for gfx950");
        return SDSP_E_NO_DEVICE;
    }
    h->cus = p.multiProcessorCount;
    hipError_t e = hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking);
    if (e == hipSuccess) e = h->d_coefs.ensure(h->cdev.size());
    if (e == hipSuccess) e = hipMemcpy(h->d_coefs.p, h->cdev.data(), h->cdev.size(), hipMemcpyHostToDevice);
    if (e != hipSuccess) {
        st = device_status(e, "iir create");
        sdsp_iir_destroy(h);
        return st;
    }
    st = plan_groups(h);
    if (!st) st = iir_alloc_state(h);
    if (st) {
        sdsp_iir_destroy(h);
        return st;
    }
    *out = h;
    return SDSP_OK;
}

// wave-scan variant index for this group (-1: none applies)
int group_wscan(const sdsp_iir* h, const Group& g, bool rate_change) {
    if (h->type == 0) {
        if (h->wscan < 1) return -1;
        const int wv = h->wscan == 2 && h->dtype == SDSP_RR32 && (g.ws[1].wc > 0 || g.ws[1].exact) ? 1 : 0;
        return (g.ws[wv].wc > 0 || g.ws[wv].exact) ? wv : -1;
    }
    int wv = h->wscan - 1;
    if ((rate_change || g.wc == 0) && (wv == 2 || wv == 3)) wv = 0;  // paired kernels: decaying, no rate change
    if (wv < 0) return -1;
    return (g.ws[wv].wc > 0 || g.ws[wv].exact) ? wv : -1;
}

bool group_scan(const sdsp_iir* h, const Group& g, size_t nd, bool rate_change) {
    if (h->type == 0 && group_wscan(h, g, rate_change) < 0) return false;
    if (g.wc == 0 && group_wscan(h, g, rate_change) < 0) return false;
    if (h->algo == SDSP_ALGO_EXACT) return false;
    if (h->algo == SDSP_ALGO_AUTO && nd < 8192) return false;
    return true;
}

}  // namespace

extern "C" {

int sdsp_iir_create(sdsp_iir** out, int dtype, const void* ff, size_t nff, const void* fb, size_t nfb, int type,
                    int device) {
    if (!out) return SDSP_E_INVALID_ARGUMENT;
    return iir_create(out, dtype, ff, nff, fb, nfb, type, 0, 1, device);
}
int sdsp_iir_decim_create(sdsp_iir** out, int dtype, const void* ff, size_t nff, const void* fb, size_t nfb, int type,
                          size_t M, int device) {
    if (!out) return SDSP_E_INVALID_ARGUMENT;
    return iir_create(out, dtype, ff, nff, fb, nfb, type, 1, M, device);
}
int sdsp_iir_interp_create(sdsp_iir** out, int dtype, const void* ff, size_t nff, const void* fb, size_t nfb,
                           int type, size_t M, int device) {
    if (!out) return SDSP_E_INVALID_ARGUMENT;
    return iir_create(out, dtype, ff, nff, fb, nfb, type, 2, M, device);
}
int sdsp_sos_create(sdsp_iir** out, const double* ff, size_t nff, const double* fb, size_t nfb, int device) {
    if (!out) return SDSP_E_INVALID_ARGUMENT;
    *out = nullptr;
    if (nff < 3 || nfb < 3) {  // sos.rs:56-60
        set_error("Second Order Error CoefficientsNotInRange");
        return SDSP_E_SOS_COEFFICIENTS_NOT_IN_RANGE;
    }
    return iir_create(out, SDSP_RR64, ff, 3, fb, 3, 1, 0, 1, device);
}

void sdsp_iir_destroy(sdsp_iir* h) {
    if (!h) return;
    {
        DeviceGuardI g(h->device);
        (void)h->fence.wait();
        if (h->stream) {
            (void)hipStreamSynchronize(h->stream);
            (void)hipStreamDestroy(h->stream);
        }
        h->d_coefs.release();
        h->d_coefs_nrm.release();
        for (int i = 0; i < 2; ++i) { h->d_state[i].release(); h->d_tmp[i].release(); h->d_carry[i].release(); }
        for (auto& g : h->groups) {
            g.d_P.release();
            g.d_wcoefs.release();
            for (auto& w : g.ws) { w.d_P.release(); w.d_Cr.release(); w.d_Phi.release(); }
        }
        h->stage_in.release();
        h->stage_out.release();
    }
    delete h;
}

int sdsp_iir_clone(const sdsp_iir* h, sdsp_iir** out) {
    if (!h || !out) return SDSP_E_INVALID_ARGUMENT;
    const size_t cb = coef_bytes(h->dtype);
    int st = iir_create(out, h->dtype, h->ff.data(), h->ff.size() / cb, h->fb.data(), h->fb.size() / cb, h->type,
                        h->mode, h->M, h->device);
    if (st) return st;
    sdsp_iir* c = *out;
    DeviceGuardI g(h->device);
    c->algo = h->algo;
    c->wscan = h->wscan;
    if (h->channels != 1) {
        st = sdsp_iir_set_channels(c, h->channels);
        if (st) return st;
    }
    IIR_TRY(h->fence.wait(), "wait for queued work");
    IIR_TRY(hipStreamSynchronize(h->stream), "sync");
    const size_t sb = sample_bytes(h->dtype) * h->channels * h->state_per_ch();
    if (sb) IIR_TRY(hipMemcpy(c->d_state[0].p, h->d_state[h->cur].p, sb, hipMemcpyDeviceToDevice), "clone state");
    c->cur = 0;
    c->phase = h->phase;
    return SDSP_OK;
}

int sdsp_iir_set_channels(sdsp_iir* h, size_t channels) {
    if (!h || channels == 0) return SDSP_E_INVALID_ARGUMENT;
    DeviceGuardI g(h->device);
    h->channels = channels;
    return iir_alloc_state(h);
}

int sdsp_iir_set_algo(sdsp_iir* h, int algo) {
    if (!h || !(algo == SDSP_ALGO_AUTO || algo == SDSP_ALGO_EXACT || algo == SDSP_ALGO_FMA)) return SDSP_E_INVALID_ARGUMENT;
    h->algo = algo;  // FMA = always the block-parallel scan where the cascade admits it
    return SDSP_OK;
}

int sdsp_iir_set_tuning(sdsp_iir* h, int key, int value) {
    if (!h) return SDSP_E_INVALID_ARGUMENT;
    if (key != SDSP_TUNE_IIR_WAVE_SCAN) return SDSP_E_INVALID_ARGUMENT;
    if (value < 0 || value > 6) return SDSP_E_INVALID_ARGUMENT;
    h->wscan = value;
    return SDSP_OK;
}

int sdsp_iir_scan_info(const sdsp_iir* h, int group, int* warmup_chunks, int* chunk) {
    if (!h || group < 0 || group >= (int)h->groups.size()) return SDSP_E_INVALID_ARGUMENT;
    if (warmup_chunks) *warmup_chunks = h->groups[group].wc;
    if (chunk) *chunk = iir_scan_chunk(h->dtype);
    return SDSP_OK;
}

int sdsp_iir_wscan_mode(const sdsp_iir* h, int group) {
    if (!h || group < 0 || group >= (int)h->groups.size()) return -1;
    const int wv = group_wscan(h, h->groups[group], false);
    if (wv < 0) return 0;
    return h->groups[group].ws[wv].wc > 0 ? 1 : 2;
}

size_t sdsp_iir_output_count(const sdsp_iir* h, size_t n) {
    if (!h) return 0;
    if (h->mode == 2) return n * h->M;
    if (h->mode == 1) {
        const size_t j0 = (h->M - 1 - h->phase) % h->M;
        return j0 < n ? (n - 1 - j0) / h->M + 1 : 0;
    }
    return n;
}

int sdsp_iir_execute_block_device(sdsp_iir* h, const void* d_in, size_t n, void* d_out, size_t* n_out, void* stream) {
    if (!h) return SDSP_E_INVALID_ARGUMENT;
    DeviceGuardI g(h->device);
    hipStream_t s = stream ? (hipStream_t)stream : h->stream;
    const size_t nout = sdsp_iir_output_count(h, n);
    if (n_out) *n_out = nout;
    if (n == 0) return SDSP_OK;
    if (ranges_overlap(d_in, h->channels * n * sample_bytes(h->dtype), d_out,
                       h->channels * nout * sample_bytes(h->dtype))) {
        set_error("input and output blocks overlap (in-place filtering is not supported)");
        return SDSP_E_INVALID_ARGUMENT;
    }
    // work queued on another stream (the fence) reads or writes the state this launch uses
    IIR_TRY(h->fence.order_before(s), "order after queued work");
    const int Mi = h->mode == 2 ? (int)h->M : 1;
    const int Md = h->mode == 1 ? (int)h->M : 1;
    const size_t nd = n * Mi;
    const size_t sbytes = sample_bytes(h->dtype);
    unsigned char* st_in = (unsigned char*)h->d_state[h->cur].p;
    unsigned char* st_out = (unsigned char*)h->d_state[h->cur ^ 1].p;
    const size_t cb = coef_bytes(h->dtype);
    if (h->type == 0) {
        IirArgs a{d_in, d_out, h->d_coefs.p, nullptr, st_in, st_out, n, nout, h->channels, 0, h->nb, h->na, h->cap,
                  Mi, Md, h->phase, false, 0};
        const bool rc = Mi != 1 || Md != 1;
        bool scanned = false;
        if (!h->groups.empty() && group_scan(h, h->groups[0], nd, rc)) {  // dense-system wave scan
            Group& gr = h->groups[0];
            const int wv = group_wscan(h, gr, rc);
            IirArgs b = a;
            b.coefs = h->d_coefs_nrm.p;
            b.algo_scan = true;
            b.P = gr.ws[wv].d_P.p;
            b.Cr = gr.ws[wv].d_Cr.p;
            b.wc = gr.ws[wv].wc;
            b.ws_variant = wv;
            int tpw = 0;
            const size_t W = iir_wscan_waves(h->dtype, b, &tpw);
            if (b.wc > 0 || exact_carry_bounded(h, gr, wv, W, tpw)) {  // else the reference-order recurrence
                if (b.wc == 0) {
                    b.Phi = gr.ws[wv].d_Phi.p;
                    const size_t bytes = h->channels * W * (size_t)(h->cap - 1) * sbytes;
                    IIR_TRY(h->d_carry[0].ensure(bytes), "iir carry scratch");
                    IIR_TRY(h->d_carry[1].ensure(bytes), "iir carry scratch");
                    b.G = h->d_carry[0].p;
                    b.Cin = h->d_carry[1].p;
                    b.scratch_waves = W;
                }
                IIR_TRY(launch_iir_wscan(h->dtype, b, s), "iir normal wave scan");
                scanned = true;
            }
        }
        if (!scanned) IIR_TRY(launch_iir(h->dtype, a, s), "iir normal");
    } else {
        const size_t ng = h->groups.size();
        if (ng > 1) {
            IIR_TRY(h->d_tmp[0].ensure(nd * h->channels * sbytes), "iir tmp");
            IIR_TRY(h->d_tmp[1].ensure(nd * h->channels * sbytes), "iir tmp");
        }
        size_t soff = 0;
        const void* src = d_in;
        for (size_t gi = 0; gi < ng; ++gi) {
            Group& gr = h->groups[gi];
            const bool first = gi == 0, last = gi + 1 == ng;
            void* dst = last ? d_out : h->d_tmp[gi & 1].p;
            const size_t n_g = first ? n : nd;
            const bool rc = (first && Mi != 1) || (last && Md != 1);
            IirArgs a{src, dst, (const unsigned char*)h->d_coefs.p + 5 * gr.first * cb, gr.d_P.p,
                      st_in + soff, st_out + soff, n_g, last ? nout : nd, h->channels, gr.count, 0, 0, 0,
                      first ? Mi : 1, last ? Md : 1, last ? h->phase : 0, group_scan(h, gr, nd, rc), gr.wc};
            const int wv = group_wscan(h, gr, rc);
            bool wave_scan = a.algo_scan && wv >= 0;
            if (wave_scan && gr.ws[wv].wc == 0) {  // exact carries: the powers of Phi this call uses stay bounded
                IirArgs b = a;
                b.wc = 0;
                b.ws_variant = wv;
                int tpw = 0;
                const size_t W = iir_wscan_waves(h->dtype, b, &tpw);
                wave_scan = exact_carry_bounded(h, gr, wv, W, tpw);
            }
            if (wave_scan) {
                a.coefs = gr.d_wcoefs.p;  // the b0-factored set (sys_step)
                a.P = gr.ws[wv].d_P.p;
                a.Cr = gr.ws[wv].d_Cr.p;
                a.wc = gr.ws[wv].wc;
                a.ws_variant = wv;
                if (a.wc == 0) {  // exact inter-wave carries: scratch for the aggregate pass
                    a.Phi = gr.ws[wv].d_Phi.p;
                    const size_t W = iir_wscan_waves(h->dtype, a);
                    const size_t bytes = h->channels * W * 2 * gr.count * sbytes;
                    IIR_TRY(h->d_carry[0].ensure(bytes), "iir carry scratch");
                    IIR_TRY(h->d_carry[1].ensure(bytes), "iir carry scratch");
                    a.G = h->d_carry[0].p;
                    a.Cin = h->d_carry[1].p;
                    a.scratch_waves = W;
                }
                IIR_TRY(launch_iir_wscan(h->dtype, a, s), "iir sos wave scan");
            } else if (a.algo_scan && (gr.wc == 0 || wv >= 0)) {  // block scan needs the decaying response;
                a.algo_scan = false;                             // an unbounded carry chain runs serial
                IIR_TRY(launch_iir(h->dtype, a, s), "iir sos");
            } else {
                IIR_TRY(launch_iir(h->dtype, a, s), "iir sos");
            }
            soff += h->channels * 2 * gr.count * sbytes;
            src = dst;
        }
    }
    h->cur ^= 1;
    if (h->mode == 1) h->phase = (h->phase + nd) % h->M;
    IIR_TRY(h->fence.record(s), "record fence");
    return SDSP_OK;
}

int sdsp_iir_execute_block(sdsp_iir* h, const void* in, size_t n, void* out, size_t* n_out) {
    if (!h) return SDSP_E_INVALID_ARGUMENT;
    DeviceGuardI g(h->device);
    const size_t sb = sample_bytes(h->dtype);
    const size_t nout = sdsp_iir_output_count(h, n);
    if (n_out) *n_out = nout;
    if (n == 0) return SDSP_OK;
    IIR_TRY(h->stage_in.ensure(h->channels * n * sb), "stage in");
    IIR_TRY(h->stage_out.ensure(h->channels * std::max<size_t>(nout, 1) * sb), "stage out");
    IIR_TRY(hipMemcpyAsync(h->stage_in.p, in, h->channels * n * sb, hipMemcpyHostToDevice, h->stream), "H2D");
    int st = sdsp_iir_execute_block_device(h, h->stage_in.p, n, h->stage_out.p, nullptr, h->stream);
    if (st) return st;
    if (nout) IIR_TRY(hipMemcpyAsync(out, h->stage_out.p, h->channels * nout * sb, hipMemcpyDeviceToHost, h->stream), "D2H");
    IIR_TRY(hipStreamSynchronize(h->stream), "sync");
    return SDSP_OK;
}

int sdsp_iir_execute(sdsp_iir* h, const void* sample, void* out, size_t* n_out) {
    if (!h || h->channels != 1) return SDSP_E_INVALID_ARGUMENT;
    return sdsp_iir_execute_block(h, sample, 1, out, n_out);
}

int sdsp_iir_reset(sdsp_iir* h) {
    if (!h) return SDSP_E_INVALID_ARGUMENT;
    DeviceGuardI g(h->device);
    return iir_alloc_state(h);
}

size_t sdsp_iir_state_len(const sdsp_iir* h) { return h ? h->channels * h->state_per_ch() : 0; }

int sdsp_iir_get_state(const sdsp_iir* h, void* state, size_t* phase) {
    if (!h) return SDSP_E_INVALID_ARGUMENT;
    DeviceGuardI g(h->device);
    IIR_TRY(h->fence.wait(), "wait for queued work");
    IIR_TRY(hipStreamSynchronize(h->stream), "sync");
    const size_t sb = sample_bytes(h->dtype) * h->channels * h->state_per_ch();
    if (state && sb) IIR_TRY(hipMemcpy(state, h->d_state[h->cur].p, sb, hipMemcpyDeviceToHost), "get state");
    if (phase) *phase = h->phase;
    return SDSP_OK;
}

int sdsp_iir_set_state(sdsp_iir* h, const void* state, size_t phase) {
    if (!h || phase >= h->M) return SDSP_E_INVALID_ARGUMENT;
    DeviceGuardI g(h->device);
    IIR_TRY(h->fence.wait(), "wait for queued work");
    IIR_TRY(hipStreamSynchronize(h->stream), "sync");
    const size_t sb = sample_bytes(h->dtype) * h->channels * h->state_per_ch();
    if (state && sb) IIR_TRY(hipMemcpy(h->d_state[h->cur].p, state, sb, hipMemcpyHostToDevice), "set state");
    h->phase = phase;
    return SDSP_OK;
}

// numerator_coefs() / denominator_coefs() exactly as the reference stores them
// (mod.rs:123-127 Normal: b/a0 and a[1..]/a0; :156-157 SecondOrder: raw ff and fb)
size_t sdsp_iir_num_coefs(const sdsp_iir* h, int which) {
    if (!h) return 0;
    const size_t cb = coef_bytes(h->dtype);
    if (h->type == 1) return (which == 0 ? h->ff.size() : h->fb.size()) / cb;
    return which == 0 ? (size_t)h->nb : (size_t)(h->na - 1);
}
int sdsp_iir_coefficients(const sdsp_iir* h, double* num, double* den) {
    if (!h) return SDSP_E_INVALID_ARGUMENT;
    const size_t nn = sdsp_iir_num_coefs(h, 0), nd = sdsp_iir_num_coefs(h, 1);
    if (h->type == 1) {
        for (size_t i = 0; i < nn; ++i) if (num) num[i] = cval(h->ff, h->dtype, i);
        for (size_t i = 0; i < nd; ++i) if (den) den[i] = cval(h->fb, h->dtype, i);
    } else {
        for (size_t i = 0; i < nn; ++i) if (num) num[i] = h->c64[i];
        for (size_t i = 0; i < nd; ++i) if (den) den[i] = h->c64[nn + i];
    }
    return SDSP_OK;
}

// Filter::frequency_response (mod.rs:336-372): Normal = B/A over the stored
// coefficient vectors; SecondOrder starts from h = 0 and multiplies, so it is 0.
int sdsp_iir_frequency_response(const sdsp_iir* h, double f, double* re_im) {
    if (!h || !re_im) return SDSP_E_INVALID_ARGUMENT;
    if (h->type == 0) {
        std::vector<cd> b(h->nb), a(h->na - 1);
        for (int i = 0; i < h->nb; ++i) b[i] = {h->c64[i], 0.0};
        for (int i = 0; i < h->na - 1; ++i) a[i] = {h->c64[h->nb + i], 0.0};
        cd r = cdiv(poly_response(b, true, f), poly_response(a, true, f));
        re_im[0] = r.re;
        re_im[1] = r.im;
        return SDSP_OK;
    }
    cd acc = {0.0, 0.0};
    for (int s = 0; s < h->S; ++s) {
        const double* c = &h->c64[5 * s];
        // section response (sos.rs:171-190): numerator_coefs = a[1..], denominator_coefs = b
        std::vector<cd> num = {{c[3], 0.0}, {c[4], 0.0}}, den = {{c[0], 0.0}, {c[1], 0.0}, {c[2], 0.0}};
        acc = cmul(acc, cdiv(poly_response(num, true, f), poly_response(den, true, f)));
    }
    re_im[0] = acc.re;
    re_im[1] = acc.im;
    return SDSP_OK;
}

// Filter::group_delay (mod.rs:392-413; SecondOrderFilter::group_delay sos.rs:208-230)
int sdsp_iir_group_delay(const sdsp_iir* h, double f, double* delay) {
    if (!h || !delay) return SDSP_E_INVALID_ARGUMENT;
    if (h->type == 0) {
        std::vector<double> b(h->c64.begin(), h->c64.begin() + h->nb), a(h->c64.begin() + h->nb, h->c64.end());
        double d = 0.0;
        if (iir_group_delay(b, a, f, &d)) d = 0.0;
        *delay = d;
        return SDSP_OK;
    }
    double total = 0.0;
    for (int s = 0; s < h->S; ++s) {
        const double* c = &h->c64[5 * s];
        std::vector<double> num = {c[3], c[4]}, den = {c[0], c[1], c[2]};  // swapped names (sos.rs:72-73)
        double d = 0.0;
        const double sec = iir_group_delay(num, den, f, &d) ? 0.0 : d + 2.0;
        total = total + sec + 2.0;
    }
    *delay = total;
    return SDSP_OK;
}

// SecondOrderFilter accessors (sos.rs:116-150): numerator_coefs = a[1..]/a0, denominator_coefs = b/a0
int sdsp_sos_section_coefs(const sdsp_iir* h, int section, double* num2, double* den3) {
    if (!h || h->type != 1 || section < 0 || section >= h->S) return SDSP_E_INVALID_ARGUMENT;
    const double* c = &h->c64[5 * section];
    if (num2) { num2[0] = c[3]; num2[1] = c[4]; }
    if (den3) { den3[0] = c[0]; den3[1] = c[1]; den3[2] = c[2]; }
    return SDSP_OK;
}

int sdsp_iir_synchronize(sdsp_iir* h) {
    if (!h) return SDSP_E_INVALID_ARGUMENT;
    DeviceGuardI g(h->device);
    IIR_TRY(h->fence.wait(), "wait for queued work");
    IIR_TRY(hipStreamSynchronize(h->stream), "sync");
    return SDSP_OK;
}

}  // extern "C"
