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
