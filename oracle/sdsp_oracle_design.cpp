// ============================================================================
// sdsp_oracle_design.cpp — CPU RESTATEMENT of the reference's host-side f64
// tap design chain and PLL loop-filter design.  TEST INFRASTRUCTURE ONLY
// (see sdsp_oracle.cpp header).  Also holds the synthetic stream generator
// used to check the device generator bit-for-bit.
//
//   sinc                 src/math/mod.rs:17-27
//   besseli / lnbesseli  src/math/mod.rs:41-100
//   gamma / lngamma      src/math/mod.rs:155-183
//   kaiser window        src/windows/kaiser.rs:33-46
//   kaiser_beta          src/filter/firdes/mod.rs:243-253
//   firdes_kaiser        src/filter/firdes/mod.rs:278-305
//   firdes_notch         src/filter/firdes/mod.rs:329-368
//   estimate_* lengths   src/filter/firdes/mod.rs:71-240
//   besselj              src/math/mod.rs:102-146
//   firdes_doppler       src/filter/firdes/mod.rs:389-419
//   filter_autocorrelation / crosscorrelation / isi / energy   src/filter/firdes/mod.rs:443-640
//   active_lag / active_proportional_integral   src/filter/iirdes/pll/mod.rs:24-99
// ============================================================================
#include <cmath>
#include <cstdint>
#include <cstddef>

namespace {
const double PI = 3.14159265358979323846;  // std::f64::consts::PI

double sinc(double x) {  // src/math/mod.rs:17-27
    if (std::fabs(x) < 0.01) return std::cos(PI * x / 2.0) * std::cos(PI * x / 4.0) * std::cos(PI * x / 8.0);
    return std::sin(PI * x) / (PI * x);
}
double lngamma(double z) {  // src/math/mod.rs:171-183
    if (z < 0.0) return 0.0;
    if (z < 10.0) return lngamma(z + 1.0) - std::log(z);
    double g = 0.5 * (std::log(2.0 * PI) - std::log(z));
    return g + z * (std::log(z + (1.0 / (12.0 * z - 0.1 / z))) - 1.0);
}
double gamma_(double z) {  // src/math/mod.rs:155-169
    if (z < 0.0) {
        double t0 = gamma_(1.0 - z);
        double t1 = std::sin(PI * z);
        return PI / (t0 * t1);
    }
    return std::exp(lngamma(z));
}
double lnbesseli(double z, double nu) {  // src/math/mod.rs:66-100
    if (z == 0.0) return nu == 0.0 ? 0.0 : -1.7976931348623157e308;
    if (nu == 0.5) return 0.5 * std::log(2.0 / (PI * z)) + std::log(std::sinh(z));
    if (z < 0.001 * std::sqrt(nu + 1.0)) return -gamma_(nu + 1.0) + nu * std::log(0.5 * z);
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
double besseli(double z, double nu) {  // src/math/mod.rs:41-64
    if (z == 0.0) return nu == 0.0 ? 1.0 : 0.0;
    if (nu == 0.5) return std::sqrt(2.0 / (PI * z)) * std::sinh(z);
    if (z < 0.001 * std::sqrt(nu + 1.0)) return std::pow(0.5 * z, nu) / gamma_(nu + 1.0);
    return std::exp(lnbesseli(z, nu));
}
double kaiser(size_t i, size_t n, double beta) {  // src/windows/kaiser.rs:33-46
    double t = (double)i - (double)(n - 1) / 2.0;
    double r = 2.0 * t / (double)(n - 1);
    double a = besseli(beta * std::sqrt(1.0 - r * r), 0.0);
    double b = besseli(beta, 0.0);
    return a / b;
}
double herrmann(double df, double as) {  // src/filter/firdes/mod.rs:213-240
    if (as > 105.0) return (as - 7.95) / (14.26 * df);
    double nas = as + 7.4;
    double d1 = std::pow(10.0, -nas / 20.0);
    double d2 = std::pow(10.0, -nas / 20.0);
    double t1 = std::log10(d1);
    double t2 = std::log10(d2);
    double d_inf = (0.005309 * t1 * t1 + 0.07114 * t1 - 0.4761) * t2 - (0.002660 * t1 * t1 + 0.59410 * t1 + 0.4278);
    double f = 11.012 + 0.51244 * (t1 - t2);
    return (d_inf - f * df * df) / df + 1.0;
}
double kaiser_len(double df, double as) { return (as - 7.95) / (14.26 * df); }  // :199-211
double besselj(double z, double nu) {  // src/math/mod.rs:102-146
    if (z == 0.0) return nu == 0.0 ? 1.0 : 0.0;
    if (z < 0.001 * std::sqrt(nu + 1.0)) return std::pow(0.5 * z, nu) / gamma_(nu + 1.0);
    double J = 0.0;
    double abs_nu = std::fabs(nu);
    for (size_t i = 0; i < 128; ++i) {
        double t0 = 2.0 * (double)i + abs_nu;
        double t1 = t0 * std::log(z);
        double t2 = t0 * std::log(2.0);
        double t3 = lngamma((double)i + 1.0);
        double t4 = lngamma(abs_nu + (double)i + 1.0);
        if (i % 2 == 0) J += std::exp(t1 - t2 - t3 - t4);
        else J -= std::exp(t1 - t2 - t3 - t4);
    }
    return J;
}

inline uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}
}  // namespace

extern "C" {

double orc_sinc(double x) { return sinc(x); }
double orc_besseli(double z, double nu) { return besseli(z, nu); }
double orc_lngamma(double z) { return lngamma(z); }
double orc_kaiser(size_t i, size_t n, double beta) { return kaiser(i, n, beta); }

double orc_kaiser_beta(double as) {  // src/filter/firdes/mod.rs:243-253
    double a = std::fabs(as);
    if (a > 50.0) return 0.1102 * (a - 8.7);
    if (a > 21.0) return 0.5842 * std::pow(a - 21.0, 0.4) + 0.07886 * (a - 21.0);
    return 0.0;
}

// returns 0 ok, else FirdesErrorCode+1 (Bandwidth=1, StopBandLevel=2, Mu=3, SemiLength=4)
int orc_firdes_kaiser(size_t n, double fc, double as, double mu, double* h) {  // :278-305
    if (!(mu >= -0.5 && mu <= 0.5)) return 3;
    if (!(fc >= 0.0 && fc <= 0.5)) return 1;
    if (as <= 0.0) return 2;
    double beta = orc_kaiser_beta(as);
    for (size_t i = 0; i < n; ++i) {
        double t = (double)i - ((double)(n - 1)) / 2.0 + mu;
        double h1 = sinc(2.0 * fc * t);
        double h2 = kaiser(i, n, beta);
        h[i] = h1 * h2;
    }
    return 0;
}

int orc_firdes_notch(size_t m, double f0, double as, double* h) {  // :329-368, h has 2m+1
    if (!(m >= 1 && m <= 1000)) return 4;
    if (!(f0 >= 0.0 && f0 <= 0.5)) return 1;
    if (as <= 0.0) return 2;
    double beta = orc_kaiser_beta(as);
    size_t n = 2 * m + 1;
    double scale = 0.0;
    for (size_t i = 0; i < n; ++i) {
        double tone = -std::cos(2.0 * PI * f0 * ((double)i - (double)m));
        double w = kaiser(i, n, beta);
        h[i] = tone * w;
        scale += h[i] * tone;
    }
    for (size_t i = 0; i < n; ++i) h[i] /= scale;
    h[m] += 1.0;
    return 0;
}

// method 0 = Kaiser, 1 = Herrmann   (:71-94; returns (usize) truncation)
int orc_estimate_req_filter_len(double df, double as, int method, size_t* out) {
    if (!(df >= 0.0 && df <= 0.5)) return 1;
    if (as <= 0.0) return 2;
    double v = method == 0 ? kaiser_len(df, as) : herrmann(df, as);
    *out = (size_t)v;  // Rust `as usize` saturates; lengths here are positive
    return 0;
}
double orc_estimate_req_filter_as(double df, size_t n, int method) {  // :117-145
    double as0 = 0.01, as1 = 200.0, as_hat = 0.0;
    for (int i = 0; i < 20; ++i) {
        as_hat = 0.5 * (as1 + as0);
        double n_hat = method == 0 ? kaiser_len(df, as_hat) : herrmann(df, as_hat);
        if (n_hat < (double)n) as0 = as_hat; else as1 = as_hat;
    }
    return as_hat;
}
double orc_estimate_req_filter_df(double as, size_t n, int method) {  // :168-196
    double df0 = 0.001, df1 = 0.499, df_hat = 0.0;
    for (int i = 0; i < 20; ++i) {
        df_hat = 0.5 * (df1 + df0);
        double n_hat = method == 0 ? kaiser_len(df_hat, as) : herrmann(df_hat, as);
        if (n_hat < (double)n) df1 = df_hat; else df0 = df_hat;
    }
    return df_hat;
}

// :389-419 (beta 4; kaiser() cannot fail here: index < length, beta >= 0)
void orc_firdes_doppler(size_t n, double fd, double K, double theta, double* h) {
    double beta = 4.0;
    for (size_t i = 0; i < n; ++i) {
        double t = (double)i - ((double)n - 1.0) / 2.0;
        double j = 1.5 * besselj(std::fabs(2.0 * PI * fd * t), 0.0);
        double r = 1.5 * K / (K + 1.0) * std::cos(2.0 * PI * fd * t * std::cos(theta));
        double w = kaiser(i, n, beta);
        h[i] = (j + r) * w;
    }
}
double orc_filter_autocorrelation(const double* f, size_t n, long lag_s) {  // :443-456
    size_t lag = lag_s < 0 ? (size_t)(-lag_s) : (size_t)lag_s;  // isize::unsigned_abs
    if (lag >= n) return 0.0;
    double rxx = 0.0;
    for (size_t i = lag; i < n; ++i) rxx += f[i] * f[i - lag];
    return rxx;
}
double orc_filter_crosscorrelation(const double* h, size_t nh, const double* g, size_t ng, long lag) {  // :487-527
    if (nh < ng) return orc_filter_crosscorrelation(g, ng, h, nh, lag);
    if (lag <= -(long)ng) return 0.0;
    if (lag >= (long)nh) return 0.0;
    size_t ig = 0, ih = 0;
    if (lag < 0) ig = (size_t)(-lag);
    if (lag > 0) ih = (size_t)lag;
    long n;
    if (lag < 0) n = (long)ng + lag;
    else if (lag < (long)(nh - ng)) n = (long)ng;
    else n = (long)nh - lag;
    double rxy = 0.0;
    for (size_t i = 0; i < (size_t)n; ++i) rxy += h[ih + i] * g[ig + i];
    return rxy;
}
void orc_filter_isi(const double* f, size_t n, size_t sps, size_t delay, double* rms, double* mx) {  // :552-577
    *rms = 0.0;
    *mx = 0.0;
    if (2 * sps * delay + 1 != n) return;
    double rxx0 = orc_filter_autocorrelation(f, n, 0);
    double isi_rms = 0.0, isi_max = 0.0;
    for (size_t i = 1; i < 2 * delay; ++i) {
        double e = std::fabs(orc_filter_autocorrelation(f, n, (long)(i * sps)) / rxx0);
        isi_rms += e * e;
        if (i == 1 || e > isi_max) isi_max = e;
    }
    *rms = std::sqrt(isi_rms / (2.0 * (double)delay));
    *mx = isi_max;
}
// :602-640; 0 ok, 1 Bandwidth, 5 FilterSize, 6 FFTSize.  DotProduct<f64> FORWARD over
// Complex<f64> samples: sum = 0; sum += c[k] * ejwt[k] (f64 * Complex: (c re, c im)).
int orc_filter_energy(const double* f, size_t n, double fc, size_t fft_size, double* out) {
    if (!(fc >= 0.0 && fc <= 0.5)) return 1;
    if (n == 0) return 5;
    if (fft_size == 0) return 6;
    double e_total = 0.0, e_stopband = 0.0;
    for (size_t i = 0; i < fft_size; ++i) {
        double fr = 0.5 * (double)i / (double)fft_size;
        double vr = 0.0, vi = 0.0;
        for (size_t k = 0; k < n; ++k) {
            double th = 2.0 * PI * fr * (double)k;
            double er = 1.0 * std::cos(th), ei = 1.0 * std::sin(th);  // Complex::from_polar(1.0, th)
            vr += f[k] * er;
            vi += f[k] * ei;
        }
        double e2 = vr * vr - vi * (-vi);  // (v * v.conj()).re
        e_total += e2;
        if (fr > fc) e_stopband += e2;
    }
    *out = e_stopband / e_total;
    return 0;
}

// src/filter/iirdes/pll/mod.rs:24-52 ; returns 0 ok, 1 bandwidth, 2 damping, 3 gain
int orc_active_lag(double bw, double zeta, double k, double* num3, double* den3) {
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
// :71-99
int orc_active_pi(double bw, double zeta, double k, double* num3, double* den3) {
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

// Synthetic stream (build-defined; not part of the reference):
//   key = seed ^ (channel * 0x9E3779B97F4A7C15)
//   v(i) = mix64(key + (i + 1) * 0x9E3779B97F4A7C15)    (first SplitMix64 draw at key+i)
//   x(i) = ((v >> 40) * 2^-24) * 2 - 1                 (exact in f32, U[-1,1))
// complex sample n uses i = 2n (re) and 2n+1 (im).  `count` is in scalars.
void orc_synth_f32(uint64_t seed, uint64_t channel, uint64_t start, size_t count, float* out) {
    const uint64_t g = 0x9E3779B97F4A7C15ULL;
    uint64_t key = seed ^ (channel * g);
    for (size_t j = 0; j < count; ++j) {
        uint64_t i = start + j;
        uint64_t v = mix64(key + (i + 1) * g);
        out[j] = (float)(v >> 40) * (1.0f / 16777216.0f) * 2.0f - 1.0f;
    }
}

}  // extern "C"
