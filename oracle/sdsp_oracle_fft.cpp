// ============================================================================
// sdsp_oracle_fft.cpp — CPU RESTATEMENT of the reference FFT subsystem and of
// the build-defined channeliser composition.  TEST INFRASTRUCTURE ONLY (see
// sdsp_oracle.cpp header).
//
//   planner            src/fft/mod.rs:108-143 (fft_is_radix2, fft_estimate_method)
//   FFT::new/execute   src/fft/mod.rs:175-215
//   DFT leaves         src/fft/dft/mod.rs:12-645 (2,3,4,5,6,7,8,16 + generic dot-product DFT)
//   mixed radix        src/fft/mixed_radix/mod.rs:9-130
//   Rader / Rader2     src/fft/rader/mod.rs:9-89, src/fft/rader2/mod.rs:9-103
//   factor / modpow / primitive_root_prime   src/resources/mod.rs:38-119
//   is_prime_miller_rabin: third-party crate slow_primes 0.1.14 (Cargo.toml:13,
//     not vendored); restated as a deterministic Miller-Rabin over the
//     64-bit witness set, which is exact for every u64.
// All arithmetic follows num-complex 0.4 operation by operation (no FMA; the
// Makefile builds with -ffp-contract=off).  Parity of this restatement is
// pinned against numpy.fft in tests (the reference has no FFT tests).
//
// Channeliser (build-defined, no reference equivalent):
//   v_p[m] = sum_{i<K} h[p+(K-1-i)M] * x[(m-i)M + (M-1-p)]   (PFB coefficient
//            layout of src/filter/fir/pfb.rs:33-40, commutator phase M-1-p)
//   X_c[m] = FFT::new(M, FORWARD).execute(v[m])[c]
// ============================================================================
#include <cmath>
#include <cstdint>
#include <cstring>
#include <memory>
#include <vector>

namespace {

struct C {
    double re, im;
};
inline C add(C a, C b) { return {a.re + b.re, a.im + b.im}; }
inline C sub(C a, C b) { return {a.re - b.re, a.im - b.im}; }
inline C mul(C a, C b) { return {a.re * b.re - a.im * b.im, a.re * b.im + a.im * b.re}; }
inline C neg(C a) { return {-a.re, -a.im}; }
inline C conj(C a) { return {a.re, -a.im}; }
inline C divs(C a, double s) { return {a.re / s, a.im / s}; }  // Complex / T
inline C polar(double r, double t) { return {r * std::cos(t), r * std::sin(t)}; }
const C ZERO = {0.0, 0.0};
const C J = {0.0, 1.0};
const double PI = 3.14159265358979323846;

// src/fft/dft/mod.rs:12-45
const double SQRT_3_2 = 0.866025403784439;
const C G = {-0.5, -SQRT_3_2}, GI = {-0.5, SQRT_3_2};
const C G0 = {0.309016994374947, -0.951056516295154}, G1 = {-0.809016994374947, -0.587785252292473};
const C G0I = {0.309016994374947, 0.951056516295154}, G1I = {-0.809016994374947, 0.587785252292473};
const C G2 = {0.623489801858734, -0.781831482468030}, G3 = {-0.222520933956314, -0.974927912181824};
const C G4 = {-0.900968867902419, -0.433883739117558};
const double R2 = 0.70710678118654752440;  // FRAC_1_SQRT_2
const C G5 = {R2, -R2}, G6 = {R2, R2}, G7 = {-R2, -R2}, G8 = {-R2, R2};
const C G9 = {0.92387950, -0.38268346}, G10 = {0.38268343, -0.92387950}, G11 = {-0.38268343, -0.92387950};
const C G12 = {-0.92387950, -0.38268346}, G13 = {0.92387950, 0.38268346}, G14 = {0.38268343, 0.92387950};
const C G15 = {-0.38268343, 0.92387950}, G16 = {-0.92387950, 0.38268346};

enum Method { M_DFT = 0, M_MIXED = 1, M_RADER = 2, M_RADER2 = 3, M_RADIX2 = 4, M_UNKNOWN = 5 };

// ---- src/resources/mod.rs ----------------------------------------------------
std::vector<size_t> factor(size_t n) {  // :38-53
    std::vector<size_t> f;
    while (n > 1 && f.size() < 64) {
        for (size_t i = 2; i <= n; ++i)
            if (n % i == 0) {
                f.push_back(i);
                n /= i;
                break;
            }
    }
    return f;
}
size_t modpow(size_t base, size_t exp, size_t n) {  // :70-77
    size_t c = 1;
    for (size_t i = 0; i < exp; ++i) c = (c * base) % n;
    return c;
}
size_t primitive_root_prime(size_t n) {  // :91-119
    std::vector<size_t> fs;
    size_t m = n - 1;
    while (m > 1 && fs.size() < 64) {
        for (size_t k = 2; k <= m; ++k)
            if (m % k == 0) {
                bool seen = false;
                for (size_t x : fs) seen |= x == k;
                if (!seen) fs.push_back(k);
                m /= k;
                break;
            }
    }
    size_t h = 0;
    for (size_t g = 2; g < n; ++g) {
        h = g;
        bool root = true;
        for (size_t f : fs)
            if (modpow(g, (n - 1) / f, n) == 1) {
                root = false;
                break;
            }
        if (root) break;
    }
    return h;
}

// slow_primes::is_prime_miller_rabin (deterministic for u64)
uint64_t mulmod(uint64_t a, uint64_t b, uint64_t m) { return (unsigned __int128)a * b % m; }
uint64_t powmod(uint64_t a, uint64_t e, uint64_t m) {
    uint64_t r = 1;
    a %= m;
    while (e) {
        if (e & 1) r = mulmod(r, a, m);
        a = mulmod(a, a, m);
        e >>= 1;
    }
    return r;
}
bool is_prime(uint64_t n) {
    if (n < 2) return false;
    for (uint64_t p : {2ull, 3ull, 5ull, 7ull, 11ull, 13ull, 17ull, 19ull, 23ull, 29ull, 31ull, 37ull}) {
        if (n % p == 0) return n == p;
    }
    uint64_t d = n - 1;
    int s = 0;
    while ((d & 1) == 0) { d >>= 1; ++s; }
    for (uint64_t a : {2ull, 3ull, 5ull, 7ull, 11ull, 13ull, 17ull, 19ull, 23ull, 29ull, 31ull, 37ull}) {
        uint64_t x = powmod(a, d, n);
        if (x == 1 || x == n - 1) continue;
        bool comp = true;
        for (int r = 1; r < s; ++r) {
            x = mulmod(x, x, n);
            if (x == n - 1) { comp = false; break; }
        }
        if (comp) return false;
    }
    return true;
}

// ---- src/fft/mod.rs:108-143 ---------------------------------------------------
bool fft_is_radix2(size_t n) {
    size_t d = 0, t = n;
    for (int i = 0; i < 64; ++i) { d += t & 1; t >>= 1; }
    return d == 1;
}
int estimate_method(size_t n) {
    if (n == 0) return M_UNKNOWN;
    if (n <= 8 || n == 11 || n == 13 || n == 16 || n == 17) return M_DFT;
    if (fft_is_radix2(n)) return M_MIXED;
    if (is_prime(n)) return fft_is_radix2(n - 1) ? M_RADER : M_RADER2;
    return M_MIXED;
}
size_t estimate_mixed_radix(size_t n) {  // mixed_radix/mod.rs:9-38
    std::vector<size_t> f = factor(n);
    if (f.size() < 2) return 0;
    size_t num2 = 0;
    for (size_t i = 0; i < f.size(); ++i) {
        num2 = i;
        if (f[i] != 2) break;
    }
    if (num2 > 0) {
        if (n % 16 == 0) return 16;
        if (n % 8 == 0) return 8;
        if (n % 4 == 0) return 4;
        return 2;
    }
    return f[0];
}

struct FFT {
    size_t n = 0;
    bool forward = true;
    int method = M_DFT;
    // DFT generic
    std::vector<std::vector<C>> dps;
    // mixed radix
    size_t p = 0, q = 0;
    std::vector<C> twiddle;
    std::unique_ptr<FFT> p_fft, q_fft;
    // rader / rader2
    std::vector<size_t> seq;
    std::vector<C> dft;
    size_t nprime = 0;
    std::unique_ptr<FFT> fft, ifft;

    static std::unique_ptr<FFT> make(size_t n, bool forward);
    std::vector<C> execute(const std::vector<C>& x) const;
};

std::unique_ptr<FFT> FFT::make(size_t n, bool forward) {
    auto f = std::make_unique<FFT>();
    f->n = n;
    f->forward = forward;
    f->method = estimate_method(n);
    const double d = forward ? -1.0 : 1.0;
    switch (f->method) {
        case M_DFT:
            if (!(n == 2 || n == 3 || n == 4 || n == 5 || n == 6 || n == 7 || n == 8 || n == 16)) {
                // dft/mod.rs:80-98: generic plan; the twiddle vector is reused across i
                std::vector<C> tw(n, ZERO);
                for (size_t i = 0; i < n; ++i) {
                    for (size_t j = 1; j < n; ++j)
                        tw[j - 1] = polar(1.0, d * 2.0 * PI * (double)(i * j) / (double)n);
                    f->dps.emplace_back(tw.begin(), tw.begin() + (n > 0 ? n - 1 : 0));
                }
            }
            break;
        case M_RADER: {  // rader/mod.rs:9-57
            size_t g = primitive_root_prime(n);
            for (size_t i = 0; i < n - 1; ++i) f->seq.push_back(modpow(g, i + 1, n));
            std::vector<C> tdb;
            for (size_t i = 0; i < n - 1; ++i) tdb.push_back(polar(1.0, d * 2.0 * PI * (double)f->seq[i] / (double)n));
            f->fft = make(n - 1, true);
            f->ifft = make(n - 1, false);
            f->dft = f->fft->execute(tdb);
            break;
        }
        case M_RADER2: {  // rader2/mod.rs:9-68
            size_t g = primitive_root_prime(n);
            for (size_t i = 0; i < n - 1; ++i) f->seq.push_back(modpow(g, i + 1, n));
            size_t np = (2 * n - 4) - 1;
            size_t m = 0;
            while (np > 0) { np >>= 1; ++m; }
            np = (size_t)1 << m;
            f->nprime = np;
            std::vector<C> tdb;
            for (size_t i = 0; i < np; ++i)
                tdb.push_back(polar(1.0, d * 2.0 * PI * (double)f->seq[i % (n - 1)] / (double)n));
            f->fft = make(np, true);
            f->ifft = make(np, false);
            f->dft = f->fft->execute(tdb);
            break;
        }
        case M_MIXED:
        default: {  // mixed_radix/mod.rs:40-85
            f->method = M_MIXED;
            f->q = estimate_mixed_radix(n);
            if (f->q == 0 || n % f->q != 0) return nullptr;  // the reference panics
            f->p = n / f->q;
            for (size_t i = 0; i < n; ++i) f->twiddle.push_back(polar(1.0, d * 2.0 * PI * (double)i / (double)n));
            f->p_fft = make(f->p, forward);
            f->q_fft = make(f->q, forward);
            if (!f->p_fft || !f->q_fft) return nullptr;
            break;
        }
    }
    return f;
}

// Complex * Complex::new(0,1) etc. written out as the reference writes them
std::vector<C> dft2(const std::vector<C>& x) { return {add(x[0], x[1]), sub(x[0], x[1])}; }
std::vector<C> dft3(const std::vector<C>& x, bool fwd) {
    std::vector<C> o(3);
    o[0] = add(add(x[0], x[1]), x[2]);
    C ta = add(add(x[0], mul(x[1], G)), mul(x[2], GI));
    C tb = add(add(x[0], mul(x[1], GI)), mul(x[2], G));
    o[1] = fwd ? ta : tb;
    o[2] = fwd ? tb : ta;
    return o;
}
std::vector<C> dft4(const std::vector<C>& x, bool fwd) {  // :177-215
    std::vector<C> o = {x[0], x[2], x[1], x[3]};
    C tmp = o[1]; o[1] = sub(o[0], tmp); o[0] = add(o[0], tmp);
    tmp = o[3]; o[3] = sub(o[2], tmp); o[2] = add(o[2], tmp);
    tmp = o[2]; o[2] = sub(o[0], tmp); o[0] = add(o[0], tmp);
    tmp = C{o[3].im, -o[3].re};
    if (fwd) { o[3] = sub(o[1], tmp); o[1] = add(o[1], tmp); }
    else { o[3] = add(o[1], tmp); o[1] = sub(o[1], tmp); }
    return o;
}
C sum_all(const std::vector<C>& x, size_t n) {  // Iterator::sum: fold from zero
    C s = ZERO;
    for (size_t i = 0; i < n; ++i) s = add(s, x[i]);
    return s;
}
C lin(const std::vector<C>& x, std::initializer_list<C> g) {  // x0 + x1*g1 + x2*g2 + ...
    C s = x[0];
    size_t i = 1;
    for (C w : g) s = add(s, mul(x[i++], w));
    return s;
}
std::vector<C> dft5(const std::vector<C>& x, bool fwd) {  // :217-247
    std::vector<C> o(5);
    o[0] = sum_all(x, 5);
    if (fwd) {
        o[1] = lin(x, {G0, G1, G1I, G0I});
        o[2] = lin(x, {G1, G0I, G0, G1I});
        o[3] = lin(x, {G1I, G0, G0I, G1});
        o[4] = lin(x, {G0I, G1I, G1, G0});
    } else {
        o[1] = lin(x, {G0I, G1I, G1, G0});
        o[2] = lin(x, {G1I, G0, G0I, G1});
        o[3] = lin(x, {G1, G0I, G0, G1I});
        o[4] = lin(x, {G0, G1, G1I, G0I});
    }
    return o;
}
std::vector<C> dft6(const std::vector<C>& x, bool fwd) {  // :249-285
    std::vector<C> o(6);
    o[0] = sum_all(x, 6);
    C g1, g2, g3, g4;
    if (fwd) { g1 = neg(GI); g2 = G; g3 = GI; g4 = neg(G); }
    else { g1 = neg(G); g2 = GI; g3 = G; g4 = neg(GI); }
    // o[1] = x0 + x1*g1 + x2*g2 - x3 + x4*g3 + x5*g4  (left to right)
    o[1] = add(add(sub(add(add(x[0], mul(x[1], g1)), mul(x[2], g2)), x[3]), mul(x[4], g3)), mul(x[5], g4));
    o[2] = add(add(add(add(add(x[0], mul(x[1], g2)), mul(x[2], g3)), x[3]), mul(x[4], g2)), mul(x[5], g3));
    o[3] = sub(add(sub(add(sub(x[0], x[1]), x[2]), x[3]), x[4]), x[5]);
    o[4] = add(add(add(add(add(x[0], mul(x[1], g3)), mul(x[2], g2)), x[3]), mul(x[4], g3)), mul(x[5], g2));
    o[5] = add(add(sub(add(add(x[0], mul(x[1], g4)), mul(x[2], g3)), x[3]), mul(x[4], g2)), mul(x[5], g1));
    return o;
}
std::vector<C> dft7(const std::vector<C>& x, bool fwd) {  // :287-361
    std::vector<C> o(7);
    o[0] = sum_all(x, 7);
    C g1 = fwd ? G2 : conj(G2), g2 = fwd ? G3 : conj(G3), g3 = fwd ? G4 : conj(G4);
    C g4 = conj(g3), g5 = conj(g2), g6 = conj(g1);
    o[1] = lin(x, {g1, g2, g3, g4, g5, g6});
    o[2] = lin(x, {g2, g4, g6, g1, g3, g5});
    o[3] = lin(x, {g3, g6, g2, g5, g1, g4});
    o[4] = lin(x, {g4, g1, g5, g2, g6, g3});
    o[5] = lin(x, {g5, g3, g1, g6, g4, g2});
    o[6] = lin(x, {g6, g5, g4, g3, g2, g1});
    return o;
}
// butterfly helpers: (a, b) <- (a + y, a - y)
inline void bf(std::vector<C>& o, int a, int b, C y) { o[b] = sub(o[a], y); o[a] = add(o[a], y); }
std::vector<C> dft8(const std::vector<C>& x, bool fwd) {  // :363-443
    std::vector<C> o = {x[0], x[4], x[2], x[6], x[1], x[5], x[3], x[7]};
    bf(o, 0, 1, o[1]); bf(o, 2, 3, o[3]); bf(o, 4, 5, o[5]); bf(o, 6, 7, o[7]);
    bf(o, 0, 2, o[2]); bf(o, 4, 6, o[6]);
    C yp, yp1;
    if (fwd) { yp = C{o[3].im, -o[3].re}; yp1 = C{o[7].im, -o[7].re}; }
    else { yp = C{-o[3].im, o[3].re}; yp1 = C{-o[7].im, o[7].re}; }
    bf(o, 1, 3, yp);
    bf(o, 5, 7, yp1);
    bf(o, 0, 4, o[4]);
    C yp2;
    if (fwd) { yp = mul(o[5], G5); yp1 = C{o[6].im, -o[6].re}; yp2 = mul(o[7], G7); }
    else { yp = mul(o[5], G6); yp1 = C{-o[6].im, o[6].re}; yp2 = mul(o[7], G8); }
    bf(o, 1, 5, yp);
    bf(o, 2, 6, yp1);
    bf(o, 3, 7, yp2);
    return o;
}
std::vector<C> dft16(const std::vector<C>& x, bool fwd) {  // :445-645
    static const int ord[16] = {0, 8, 4, 12, 2, 10, 6, 14, 1, 9, 5, 13, 3, 11, 7, 15};
    std::vector<C> o(16);
    for (int i = 0; i < 16; ++i) o[i] = x[ord[i]];
    for (int i = 0; i < 16; i += 2) bf(o, i, i + 1, o[i + 1]);
    for (int i : {0, 4, 8, 12}) bf(o, i, i + 2, o[i + 2]);
    // multiply by -j (forward: -o * j) or +j (reverse: o * j) as full complex products
    auto rot = [&](C v) { return fwd ? mul(neg(v), J) : mul(v, J); };
    for (int i : {1, 5, 9, 13}) bf(o, i, i + 2, rot(o[i + 2]));
    bf(o, 0, 4, o[4]);
    bf(o, 8, 12, o[12]);
    bf(o, 1, 5, mul(o[5], fwd ? G5 : G6));
    bf(o, 9, 13, mul(o[13], fwd ? G5 : G6));
    bf(o, 2, 6, rot(o[6]));
    bf(o, 10, 14, rot(o[14]));
    bf(o, 3, 7, mul(o[7], fwd ? G7 : G8));
    bf(o, 11, 15, mul(o[15], fwd ? G7 : G8));
    bf(o, 0, 8, o[8]);
    bf(o, 1, 9, mul(o[9], fwd ? G9 : G13));
    bf(o, 2, 10, mul(o[10], fwd ? G5 : G6));
    bf(o, 3, 11, mul(o[11], fwd ? G10 : G14));
    bf(o, 4, 12, rot(o[12]));
    bf(o, 5, 13, mul(o[13], fwd ? G11 : G15));
    bf(o, 6, 14, mul(o[14], fwd ? G7 : G8));
    bf(o, 7, 15, mul(o[15], fwd ? G12 : G16));
    return o;
}

std::vector<C> FFT::execute(const std::vector<C>& x) const {
    switch (method) {
        case M_DFT:
            switch (n) {
                case 2: return dft2(x);
                case 3: return dft3(x, forward);
                case 4: return dft4(x, forward);
                case 5: return dft5(x, forward);
                case 6: return dft6(x, forward);
                case 7: return dft7(x, forward);
                case 8: return dft8(x, forward);
                case 16: return dft16(x, forward);
                default: {  // dft_execute (:100-112): dot(twiddle_i, x[1..]) + x[0]
                    std::vector<C> out;
                    for (size_t i = 0; i < n; ++i) {
                        C s = ZERO;
                        const std::vector<C>& tw = dps[i];
                        size_t it = std::min(tw.size(), x.size() > 0 ? x.size() - 1 : 0);
                        for (size_t j = 0; j < it; ++j) s = add(s, mul(tw[j], x[j + 1]));
                        out.push_back(add(s, x[0]));
                    }
                    return out;
                }
            }
        case M_MIXED: {  // mixed_radix/mod.rs:87-130
            std::vector<C> out(n, ZERO), pv(p, ZERO), qv(q, ZERO);
            std::vector<C> inter(x.begin(), x.begin() + n);
            for (size_t i = 0; i < q; ++i) {
                for (size_t j = 0; j < p; ++j) pv[j] = x[q * j + i];
                std::vector<C> t = p_fft->execute(pv);
                for (size_t j = 0; j < p; ++j) inter[q * j + i] = mul(t[j], twiddle[i * j]);
            }
            for (size_t i = 0; i < p; ++i) {
                for (size_t j = 0; j < q; ++j) qv[j] = inter[q * i + j];
                std::vector<C> t = q_fft->execute(qv);
                for (size_t j = 0; j < q; ++j) out[p * j + i] = t[j];
            }
            return out;
        }
        case M_RADER: {  // rader/mod.rs:59-89
            std::vector<C> out(n, ZERO), tdb;
            for (size_t i = 0; i < n - 1; ++i) tdb.push_back(x[seq[n - i - 2]]);
            std::vector<C> fdb = fft->execute(tdb);
            for (size_t i = 0; i < fdb.size(); ++i) fdb[i] = mul(fdb[i], dft[i]);
            tdb = ifft->execute(fdb);
            out[0] = sum_all(x, n);
            for (size_t i = 0; i < n - 1; ++i) out[seq[i]] = add(divs(tdb[i], (double)(n - 1)), x[0]);
            return out;
        }
        case M_RADER2: {  // rader2/mod.rs:70-103
            std::vector<C> out(n, ZERO), xp(nprime, ZERO);
            xp[0] = x[seq[n - 2]];
            for (size_t i = 1; i < n - 1; ++i) xp[i + nprime - n + 1] = x[seq[n - i - 2]];
            std::vector<C> xi = fft->execute(xp);
            for (size_t i = 0; i < xi.size(); ++i) xi[i] = mul(xi[i], dft[i]);
            xp = ifft->execute(xi);
            out[0] = sum_all(x, n);
            for (size_t i = 0; i < n - 1; ++i) out[seq[i]] = add(divs(xp[i], (double)nprime), x[0]);
            return out;
        }
    }
    return {};
}

}  // namespace

extern "C" {

// direction: 0 FORWARD, 1 REVERSE
void* orc_fft_new(size_t n, int direction) { return FFT::make(n, direction == 0).release(); }
int orc_fft_method(void* h) { return ((FFT*)h)->method; }
// in/out: n complex<f64>
int orc_fft_execute(void* h, const void* in, void* out) {
    const FFT* f = (const FFT*)h;
    std::vector<C> x((const C*)in, (const C*)in + f->n);
    std::vector<C> y = f->execute(x);
    if (y.size() != f->n) return 1;
    std::memcpy(out, y.data(), f->n * sizeof(C));
    return 0;
}
void orc_fft_free(void* h) { delete (FFT*)h; }

// channeliser over one stream: h (L taps, f64), M channels, x (n complex f64,
// n a multiple of M), out (n/M frames x M).  Branch windows start at zero.
size_t orc_channelize(const void* taps, size_t L, size_t M, const void* in, size_t n, void* out) {
    const double* h = (const double*)taps;
    const C* x = (const C*)in;
    C* y = (C*)out;
    const size_t K = L / M;
    auto fft = FFT::make(M, true);
    if (!fft || K == 0) return 0;
    // branch p coefficients, stored order (pfb.rs:33-40): c_p[K-1-idx] = h[p + idx M]
    std::vector<std::vector<double>> cb(M, std::vector<double>(K));
    for (size_t p = 0; p < M; ++p)
        for (size_t idx = 0; idx < K; ++idx) cb[p][K - idx - 1] = h[p + idx * M];
    // branch windows (newest first), Window(K) semantics
    std::vector<std::vector<C>> win(M, std::vector<C>(K, ZERO));
    const size_t frames = n / M;
    std::vector<C> v(M);
    for (size_t m = 0; m < frames; ++m) {
        for (size_t p = 0; p < M; ++p) {
            std::vector<C>& w = win[p];
            std::memmove(w.data() + 1, w.data(), (K - 1) * sizeof(C));
            w[0] = x[m * M + (M - 1 - p)];
            C s = ZERO;  // DotProduct::execute, real taps x complex
            for (size_t i = 0; i < K; ++i) s = add(s, C{cb[p][i] * w[i].re, cb[p][i] * w[i].im});
            v[p] = s;
        }
        std::vector<C> X = fft->execute(v);
        std::memcpy(y + m * M, X.data(), M * sizeof(C));
    }
    return frames;
}

}  // extern "C"
