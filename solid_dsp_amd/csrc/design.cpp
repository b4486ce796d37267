// Host-side f64 design and analysis functions of the C ABI.
//
// These stay on the host in the reference too (SURVEY §2 "host-only" rows):
// they produce taps for the streaming objects and back Filter::frequency_response
// / Filter::group_delay.  Restated from:
//   sinc, besseli/lnbesseli, gamma/lngamma   src/math/mod.rs:17-183
//   kaiser window                            src/windows/kaiser.rs:33-46
//   kaiser_beta, firdes_kaiser, firdes_notch src/filter/firdes/mod.rs:243-368
//   besselj                                  src/math/mod.rs:102-146
//   length / attenuation / transition estimates, firdes_doppler, filter_autocorrelation,
//   filter_crosscorrelation, filter_isi, filter_energy   src/filter/firdes/mod.rs:46-640
//   active_lag, active_proportional_integral src/filter/iirdes/pll/mod.rs:24-99
//   fir_group_delay, iir_group_delay         src/group_delay/mod.rs:51-129
// num-complex 0.4 arithmetic (Mul, Div, from_polar) is reproduced operation
// by operation; this TU is compiled with -ffp-contract=off.
#include <cmath>
#include <complex>
#include <vector>

#include "sdsp.h"
#include "sdsp_host.hpp"

namespace sdsp {
namespace {
const double PI = 3.14159265358979323846;

double sinc(double x) {
    if (std::fabs(x) < 0.01) return std::cos(PI * x / 2.0) * std::cos(PI * x / 4.0) * std::cos(PI * x / 8.0);
    return std::sin(PI * x) / (PI * x);
}
double lngamma(double z) {
    if (z < 0.0) return 0.0;
    if (z < 10.0) return lngamma(z + 1.0) - std::log(z);
    double g = 0.5 * (std::log(2.0 * PI) - std::log(z));
    return g + z * (std::log(z + (1.0 / (12.0 * z - 0.1 / z))) - 1.0);
}
double gamma_fn(double z) {
    if (z < 0.0) return PI / (gamma_fn(1.0 - z) * std::sin(PI * z));
    return std::exp(lngamma(z));
}
double lnbesseli(double z, double nu) {
    if (z == 0.0) return nu == 0.0 ? 0.0 : -1.7976931348623157e308;
    if (nu == 0.5) return 0.5 * std::log(2.0 / (PI * z)) + std::log(std::sinh(z));
    if (z < 0.001 * std::sqrt(nu + 1.0)) return -gamma_fn(nu + 1.0) + nu * std::log(0.5 * z);
    double t0 = nu * std::log(0.5 * z);
    double y = 0.0;
    for (int k = 0; k < 64; ++k) {
        double t1 = 2.0 * (double)k * std::log(0.5 * z);
        double t2 = lngamma((double)k + 1.0);
        double t3 = lngamma(nu + (double)k + 1.0);
        y += std::exp(t1 - t2 - t3);
    }
    return t0 + std::log(y);
}
double besseli(double z, double nu) {
    if (z == 0.0) return nu == 0.0 ? 1.0 : 0.0;
    if (nu == 0.5) return std::sqrt(2.0 / (PI * z)) * std::sinh(z);
    if (z < 0.001 * std::sqrt(nu + 1.0)) return std::pow(0.5 * z, nu) / gamma_fn(nu + 1.0);
    return std::exp(lnbesseli(z, nu));
}
double kaiser_w(size_t i, size_t n, double beta) {
    double t = (double)i - (double)(n - 1) / 2.0;
    double r = 2.0 * t / (double)(n - 1);
    return besseli(beta * std::sqrt(1.0 - r * r), 0.0) / besseli(beta, 0.0);
}
// Bessel function of the first kind: the 128-term series of math/mod.rs:102-146
double besselj(double z, double nu) {
    if (z == 0.0) return nu == 0.0 ? 1.0 : 0.0;
    if (z < 0.001 * std::sqrt(nu + 1.0)) return std::pow(0.5 * z, nu) / gamma_fn(nu + 1.0);
    double J = 0.0;
    const double abs_nu = std::fabs(nu);
    for (int i = 0; i < 128; ++i) {
        const double t0 = 2.0 * (double)i + abs_nu;
        const double t1 = t0 * std::log(z);
        const double t2 = t0 * std::log(2.0);
        const double t3 = lngamma((double)i + 1.0);
        const double t4 = lngamma(abs_nu + (double)i + 1.0);
        if (i % 2 == 0) J += std::exp(t1 - t2 - t3 - t4);
        else J -= std::exp(t1 - t2 - t3 - t4);
    }
    return J;
}
// the length estimates (firdes/mod.rs:199-240); 0 ok, 1 Bandwidth, 2 StopBandLevel
int est_kaiser(double df, double as, double* out) {
    if (!(df >= 0.0 && df <= 0.5)) return 1;
    if (as <= 0.0) return 2;
    *out = (as - 7.95) / (14.26 * df);
    return 0;
}
int est_herrmann(double df, double as, double* out) {
    if (!(df >= 0.0 && df <= 0.5)) return 1;
    if (as <= 0.0) return 2;
    if (as > 105.0) {
        *out = (as - 7.95) / (14.26 * df);
        return 0;
    }
    const double nas = as + 7.4;
    const double d1 = std::pow(10.0, -nas / 20.0), d2 = std::pow(10.0, -nas / 20.0);
    const double t1 = std::log10(d1), t2 = std::log10(d2);
    const double d_inf = (0.005309 * t1 * t1 + 0.07114 * t1 - 0.4761) * t2 - (0.002660 * t1 * t1 + 0.59410 * t1 + 0.4278);
    const double f = 11.012 + 0.51244 * (t1 - t2);
    *out = (d_inf - f * df * df) / df + 1.0;
    return 0;
}
int est_len(double df, double as, int method, double* out) {
    return method == 0 ? est_kaiser(df, as, out) : est_herrmann(df, as, out);
}
double autocorr(const double* h, size_t n, ptrdiff_t lag) {  // firdes/mod.rs:443-456
    const size_t l = lag < 0 ? (size_t)0 - (size_t)lag : (size_t)lag;
    if (l >= n) return 0.0;
    double r = 0.0;
    for (size_t i = l; i < n; ++i) r += h[i] * h[i - l];
    return r;
}
}  // namespace

// ---- num-complex operations -------------------------------------------------
cd cmul(cd a, cd b) { return {a.re * b.re - a.im * b.im, a.re * b.im + a.im * b.re}; }
cd cmul(double a, cd b) { return {a * b.re, a * b.im}; }
cd cadd(cd a, cd b) { return {a.re + b.re, a.im + b.im}; }
cd cdiv(cd a, cd b) {
    double nrm = b.re * b.re + b.im * b.im;
    return {(a.re * b.re + a.im * b.im) / nrm, (a.im * b.re - a.re * b.im) / nrm};
}
cd from_polar(double r, double t) { return {r * std::cos(t), r * std::sin(t)}; }

// sum_i c[i] e^{+j 2 pi f i}   (the loops of fir/mod.rs:263-273, iir/mod.rs:343-358, sos.rs:171-190)
cd poly_response(const std::vector<cd>& c, bool real, double f) {
    cd out = {0.0, 0.0};
    for (size_t i = 0; i < c.size(); ++i) {
        cd p = from_polar(1.0, f * 2.0 * PI * (double)i);
        out = cadd(out, real ? cmul(c[i].re, p) : cmul(c[i], p));
    }
    return out;
}

// src/group_delay/mod.rs:51-79
int fir_group_delay(const std::vector<cd>& h, bool real, double f, double* out) {
    *out = 0.0;
    if (h.empty()) return 1;
    if (f < -0.5 || f > 0.5) return 2;
    cd t0 = {0.0, 0.0}, t1 = {0.0, 0.0};
    for (size_t i = 0; i < h.size(); ++i) {
        cd rot = from_polar(1.0, f * 2.0 * PI * (double)i);
        cd a = real ? cmul(h[i].re, rot) : cmul(h[i], rot);
        t0 = cadd(t0, cd{a.re * (double)i, a.im * (double)i});
        t1 = cadd(t1, a);
    }
    *out = cdiv(t0, t1).re;
    return 0;
}

// src/group_delay/mod.rs:82-129 (real coefficients: Conj is the identity on f64)
int iir_group_delay(const std::vector<double>& b, const std::vector<double>& a, double f, double* out) {
    *out = 0.0;
    if (b.empty() || a.empty()) return 1;
    if (f < -0.5 || f > 0.5) return 2;
    size_t n = b.size() + a.size() - 1;
    std::vector<double> c(n, 0.0);
    for (size_t i = 0; i < a.size(); ++i)
        for (size_t j = 0; j < b.size(); ++j) c[i + j] = c[i + j] + a[a.size() - i - 1] * b[j];
    cd t0 = {0.0, 0.0}, t1 = {0.0, 0.0};
    for (size_t i = 0; i < n; ++i) {
        cd c0 = cmul(c[i], from_polar(1.0, f * 2.0 * PI * (double)i));
        t0 = cadd(t0, cd{c0.re * (double)i, c0.im * (double)i});
        t1 = cadd(t1, c0);
    }
    if (std::hypot(t1.re, t1.im) <= 0.00000000001) return 3;
    *out = cdiv(t0, t1).re - (double)(a.size() - 1);
    return 0;
}

}  // namespace sdsp

using namespace sdsp;

extern "C" {

double sdsp_kaiser_beta(double as) {
    double a = std::fabs(as);
    if (a > 50.0) return 0.1102 * (a - 8.7);
    if (a > 21.0) return 0.5842 * std::pow(a - 21.0, 0.4) + 0.07886 * (a - 21.0);
    return 0.0;
}

// FirdesErrorCode: 1 Bandwidth, 2 StopBandLevel, 3 Mu, 4 SemiLength
int sdsp_firdes_kaiser(size_t n, double fc, double as, double mu, double* h) {
    if (!(mu >= -0.5 && mu <= 0.5)) return 3;
    if (!(fc >= 0.0 && fc <= 0.5)) return 1;
    if (as <= 0.0) return 2;
    double beta = sdsp_kaiser_beta(as);
    for (size_t i = 0; i < n; ++i) {
        double t = (double)i - ((double)(n - 1)) / 2.0 + mu;
        h[i] = sinc(2.0 * fc * t) * kaiser_w(i, n, beta);
    }
    return 0;
}

int sdsp_firdes_notch(size_t m, double f0, double as, double* h) {
    if (!(m >= 1 && m <= 1000)) return 4;
    if (!(f0 >= 0.0 && f0 <= 0.5)) return 1;
    if (as <= 0.0) return 2;
    double beta = sdsp_kaiser_beta(as);
    size_t n = 2 * m + 1;
    double scale = 0.0;
    for (size_t i = 0; i < n; ++i) {
        double tone = -std::cos(2.0 * PI * f0 * ((double)i - (double)m));
        h[i] = tone * kaiser_w(i, n, beta);
        scale += h[i] * tone;
    }
    for (size_t i = 0; i < n; ++i) h[i] /= scale;
    h[m] += 1.0;
    return 0;
}

int sdsp_active_lag(double bw, double zeta, double k, double* num3, double* den3) {
    if (bw <= 0.0) return 1;
    if (zeta <= 0.0) return 2;
    if (k <= 0.0) return 3;
    double t1 = k / (bw * bw);
    double t2 = 2.0 * zeta / bw - 1.0 / k;
    num3[0] = 2.0 * k * (1.0 + t2 / 2.0);
    num3[1] = 2.0 * k * 2.0;
    num3[2] = 2.0 * k * (1.0 - t2 / 2.0);
    den3[0] = 1.0 + t1 / 2.0;
    den3[1] = -t1;
    den3[2] = -1.0 + t1 / 2.0;
    return 0;
}

int sdsp_active_proportional_integral(double bw, double zeta, double k, double* num3, double* den3) {
    if (bw <= 0.0) return 1;
    if (zeta <= 0.0) return 2;
    if (k <= 0.0) return 3;
    double t1 = k / (bw * bw);
    double t2 = 2.0 * zeta / bw - 1.0 / k;
    num3[0] = 2.0 * k * (1.0 + t2 / 2.0);
    num3[1] = 2.0 * k * 2.0;
    num3[2] = 2.0 * k * (1.0 - t2 / 2.0);
    den3[0] = t1 / 2.0;
    den3[1] = -t1;
    den3[2] = t1 / 2.0;
    return 0;
}

int sdsp_firdes_estimate_length_kaiser(double df, double as, double* len) { return est_kaiser(df, as, len); }
int sdsp_firdes_estimate_length_herrmann(double df, double as, double* len) { return est_herrmann(df, as, len); }

int sdsp_firdes_estimate_length(double df, double as, int method, size_t* len) {
    double v = 0.0;
    const int rc = est_len(df, as, method, &v);
    if (rc) return rc;
    // Rust `f64 as usize`: NaN and negatives to 0, saturating at the top
    *len = !(v > 0.0) ? 0 : v >= 18446744073709551615.0 ? (size_t)-1 : (size_t)v;
    return 0;
}

int sdsp_firdes_estimate_stop_band_attenuation(double df, size_t n, int method, double* as) {
    double as0 = 0.01, as1 = 200.0, as_hat = 0.0;
    for (int i = 0; i < 20; ++i) {
        as_hat = 0.5 * (as1 + as0);
        double n_hat = 0.0;
        const int rc = est_len(df, as_hat, method, &n_hat);
        if (rc) return rc;
        if (n_hat < (double)n) as0 = as_hat;
        else as1 = as_hat;
    }
    *as = as_hat;
    return 0;
}

int sdsp_firdes_estimate_transition(double as, size_t n, int method, double* df) {
    double df0 = 0.001, df1 = 0.499, df_hat = 0.0;
    for (int i = 0; i < 20; ++i) {
        df_hat = 0.5 * (df1 + df0);
        double n_hat = 0.0;
        const int rc = est_len(df_hat, as, method, &n_hat);
        if (rc) return rc;
        if (n_hat < (double)n) df1 = df_hat;
        else df0 = df_hat;
    }
    *df = df_hat;
    return 0;
}

int sdsp_firdes_doppler(size_t n, double fd, double k, double theta, double* h) {
    const double beta = 4.0;
    for (size_t i = 0; i < n; ++i) {
        const double t = (double)i - ((double)n - 1.0) / 2.0;
        const double j = 1.5 * besselj(std::fabs(2.0 * PI * fd * t), 0.0);
        const double r = 1.5 * k / (k + 1.0) * std::cos(2.0 * PI * fd * t * std::cos(theta));
        h[i] = (j + r) * kaiser_w(i, n, beta);
    }
    return 0;
}

double sdsp_filter_autocorrelation(const double* h, size_t n, ptrdiff_t lag) { return autocorr(h, n, lag); }

double sdsp_filter_crosscorrelation(const double* h, size_t nh, const double* g, size_t ng, ptrdiff_t lag) {
    if (nh < ng) return sdsp_filter_crosscorrelation(g, ng, h, nh, lag);  // firdes/mod.rs:487-527
    if (lag <= -(ptrdiff_t)ng) return 0.0;
    if (lag >= (ptrdiff_t)nh) return 0.0;
    const size_t ig = lag < 0 ? (size_t)(-lag) : 0, ih = lag > 0 ? (size_t)lag : 0;
    ptrdiff_t m;
    if (lag < 0) m = (ptrdiff_t)ng + lag;
    else if (lag < (ptrdiff_t)(nh - ng)) m = (ptrdiff_t)ng;
    else m = (ptrdiff_t)nh - lag;
    double r = 0.0;
    for (ptrdiff_t i = 0; i < m; ++i) r += h[ih + i] * g[ig + i];
    return r;
}

int sdsp_filter_isi(const double* h, size_t n, size_t sps, size_t delay, double* rms, double* max) {
    *rms = 0.0;
    *max = 0.0;
    if (2 * sps * delay + 1 != n) return 0;  // firdes/mod.rs:552-577: (0, 0)
    const double rxx0 = autocorr(h, n, 0);
    double isi_rms = 0.0, isi_max = 0.0;
    for (size_t i = 1; i < 2 * delay; ++i) {
        const double e = std::fabs(autocorr(h, n, (ptrdiff_t)(i * sps)) / rxx0);
        isi_rms += e * e;
        if (i == 1 || e > isi_max) isi_max = e;
    }
    *rms = std::sqrt(isi_rms / (2.0 * (double)delay));
    *max = isi_max;
    return 0;
}

int sdsp_filter_energy(const double* h, size_t n, double fc, size_t fft_size, double* energy) {
    if (!(fc >= 0.0 && fc <= 0.5)) return 1;  // firdes/mod.rs:602-640
    if (n == 0) return 5;
    if (fft_size == 0) return 6;
    double e_total = 0.0, e_stop = 0.0;
    for (size_t i = 0; i < fft_size; ++i) {
        const double f = 0.5 * (double)i / (double)fft_size;
        // DotProduct::<f64>::new(filter, FORWARD).execute(&ejwt): 0 + h0 e0 + h1 e1 + ... (f64 * Complex)
        cd v = {0.0, 0.0};
        for (size_t k = 0; k < n; ++k) v = cadd(v, cmul(h[k], from_polar(1.0, 2.0 * PI * f * (double)k)));
        const double e2 = cmul(v, cd{v.re, -v.im}).re;
        e_total += e2;
        if (f > fc) e_stop += e2;
    }
    *energy = e_stop / e_total;
    return 0;
}

int sdsp_fir_group_delay_taps(const double* h, size_t n, double f, double* out) {
    std::vector<cd> c(n);
    for (size_t i = 0; i < n; ++i) c[i] = {h[i], 0.0};
    return fir_group_delay(c, true, f, out);
}

int sdsp_iir_group_delay_taps(const double* b, size_t nb, const double* a, size_t na, double f, double* out) {
    return iir_group_delay(std::vector<double>(b, b + nb), std::vector<double>(a, a + na), f, out);
}

}  // extern "C"
