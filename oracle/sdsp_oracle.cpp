// ============================================================================
// sdsp_oracle.cpp — CPU RESTATEMENT OF juliantos/solid-dsp's STREAMING FILTER
// PATH.  TEST INFRASTRUCTURE ONLY.
//
// This file is the parity oracle and the "port" CPU baseline.  It is never
// linked into, loaded by, or called from the product library
// (solid_dsp_amd/csrc).  Only tests/, __graft_entry__.smoke() and bench.py's
// cpu_baseline leg may load oracle/_build/libsdsp_oracle.so, and only as the
// checker / the timed CPU reference.
//
// It follows the reference Rust sources literally (paths relative to the
// reference checkout):
//   * newest-first shift-register delay line that memmoves cap-1 elements per
//     push and copies `cap` elements on every to_vec()   src/window/mod.rs:17-77
//   * DotProduct: FORWARD / REVERSE coefficient copy, strictly left-to-right
//     accumulation from zero, separate multiply and add (Rust never contracts
//     to FMA; this file is compiled with -ffp-contract=off)
//                                                   src/dot_product/mod.rs:57-171
//   * num-complex 0.4 arithmetic (third-party, not vendored; semver range
//     `num = "0.4"` in Cargo.toml:8-14):  real*complex = (s*re, s*im);
//     complex*complex = (ar*br - ai*bi, ar*bi + ai*br); componentwise add/sub;
//     div = ((a c + b d)/|z|^2, (b c - a d)/|z|^2); from_polar(r,t) =
//     (r cos t, r sin t).
//   * every filter object's per-sample execute loop (file:line at each class).
//
// Parity pinning: tests/test_oracle_kats.py checks this restatement against
// every known-answer doctest the reference holds for the path.
// ============================================================================
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <vector>
#include <new>
#include <algorithm>

#if defined(__FP_FAST_FMA) && !defined(SDSP_ORACLE_ALLOW_FMA)
// -ffp-contract=off is enforced by the Makefile; explicit fma is never used.
#endif

namespace orc {

// --------------------------------------------------------------------------
// Scalar / complex arithmetic with num-complex 0.4 semantics
// --------------------------------------------------------------------------
template <typename T> struct cpx { T re, im; };

template <typename T> inline T zero() { return T(0); }
template <> inline cpx<float> zero<cpx<float>>() { return {0.0f, 0.0f}; }
template <> inline cpx<double> zero<cpx<double>>() { return {0.0, 0.0}; }

template <typename T> inline T mul(T a, T b) { return a * b; }
template <typename T> inline cpx<T> mul(T a, cpx<T> b) { return {a * b.re, a * b.im}; }
template <typename T> inline cpx<T> mul(cpx<T> a, T b) { return {a.re * b, a.im * b}; }
template <typename T> inline cpx<T> mul(cpx<T> a, cpx<T> b) {
    T re = a.re * b.re - a.im * b.im;
    T im = a.re * b.im + a.im * b.re;
    return {re, im};
}
template <typename T> inline T add(T a, T b) { return a + b; }
template <typename T> inline cpx<T> add(cpx<T> a, cpx<T> b) { return {a.re + b.re, a.im + b.im}; }
template <typename T> inline T sub(T a, T b) { return a - b; }
template <typename T> inline cpx<T> sub(cpx<T> a, cpx<T> b) { return {a.re - b.re, a.im - b.im}; }
template <typename T> inline cpx<T> cdiv(cpx<T> a, cpx<T> b) {
    T norm = b.re * b.re + b.im * b.im;
    return {(a.re * b.re + a.im * b.im) / norm, (a.im * b.re - a.re * b.im) / norm};
}
inline cpx<double> from_polar(double r, double t) { return {r * std::cos(t), r * std::sin(t)}; }

// Out type of Coef * In (num-complex Mul impls)
template <typename C, typename I> struct out_of { using type = decltype(mul(C(), I())); };

// --------------------------------------------------------------------------
// msb_index  src/resources/mod.rs:21-23
// --------------------------------------------------------------------------
inline size_t msb_index(size_t x) { return x == 0 ? 0 : (size_t)(64 - __builtin_clzll((unsigned long long)x)); }

// --------------------------------------------------------------------------
// Window<T>  src/window/mod.rs:9-77   (delay is always 0 on the filter path)
// --------------------------------------------------------------------------
template <typename T> struct Window {
    size_t capacity, delay;
    std::vector<T> buf;  // capacity + delay, zero initialised (alloc_zeroed, :21-25)
    Window(size_t cap, size_t d) : capacity(cap), delay(d), buf(cap + d, zero<T>()) {
        if (cap == 0) std::abort();  // assert!(capacity > 0)  :18
    }
    // to_vec: fresh heap copy of `capacity` elements from `delay`  :44-51
    std::vector<T> to_vec() const { return std::vector<T>(buf.begin() + delay, buf.begin() + delay + capacity); }
    // reset: fresh zeroed buffer  :54-56
    void reset() { std::fill(buf.begin(), buf.end(), zero<T>()); }
    // push: memmove(buf+1, buf, cap-1); buf[0] = x   :63-71
    void push(T x) {
        std::memmove(buf.data() + 1, buf.data(), (capacity - 1) * sizeof(T));
        buf[0] = x;
    }
    void write(const T* xs, size_t n) { for (size_t i = 0; i < n; ++i) push(xs[i]); }  // :73-77
};

// --------------------------------------------------------------------------
// DotProduct<T>  src/dot_product/mod.rs:37-171
// --------------------------------------------------------------------------
enum Direction { FORWARD = 0, REVERSE = 1 };
template <typename T> struct DotProduct {
    std::vector<T> c;
    DotProduct() {}
    DotProduct(const T* coefs, size_t len, Direction d) : c(coefs, coefs + len) {   // :57-87
        if (d == REVERSE) std::reverse(c.begin(), c.end());
    }
    size_t len() const { return c.size(); }
    // Execute::execute  :153-171  — sum = O::zero(); sum += value * sample (in order)
    template <typename I> typename out_of<T, I>::type execute(const I* s, size_t n) const {
        using O = typename out_of<T, I>::type;
        size_t it = n < c.size() ? n : c.size();
        O sum = zero<O>();
        for (size_t i = 0; i < it; ++i) sum = add(sum, mul(c[i], s[i]));
        return sum;
    }
};

// --------------------------------------------------------------------------
// Host-side f64 group delay  src/group_delay/mod.rs:51-129
// --------------------------------------------------------------------------
inline cpx<double> as_c(double x) { return {x, 0.0}; }
inline cpx<double> as_c(cpx<double> x) { return x; }
inline cpx<double> as_c(float x) { return {(double)x, 0.0}; }
inline cpx<double> as_c(cpx<float> x) { return {(double)x.re, (double)x.im}; }
inline cpx<double> coef_mul_polar(double c, cpx<double> p) { return mul(c, p); }
inline cpx<double> coef_mul_polar(cpx<double> c, cpx<double> p) { return mul(c, p); }
inline double conj_(double c) { return c; }

// fir_group_delay  :51-79   (returns 0 on error like the Filter impls do)
template <typename C> double fir_group_delay(const std::vector<C>& h, double f, int* err) {
    *err = 0;
    if (h.empty()) { *err = 1; return 0.0; }
    if (f < -0.5 || f > 0.5) { *err = 2; return 0.0; }
    cpx<double> t0 = {0.0, 0.0}, t1 = {0.0, 0.0};
    for (size_t i = 0; i < h.size(); ++i) {
        cpx<double> rot = from_polar(1.0, f * 2.0 * M_PI * (double)i);
        cpx<double> a = coef_mul_polar(h[i], rot);
        t0 = add(t0, mul(a, (double)i));
        t1 = add(t1, a);
    }
    return cdiv(t0, t1).re;
}

// iir_group_delay  :82-129  (f64 coefficients only: Conj is implemented for f64)
inline double iir_group_delay(const std::vector<double>& b, const std::vector<double>& a, double f, int* err) {
    *err = 0;
    if (b.empty() || a.empty()) { *err = 1; return 0.0; }
    if (f < -0.5 || f > 0.5) { *err = 2; return 0.0; }
    size_t n = b.size() + a.size() - 1;
    std::vector<double> c(n, 0.0);
    for (size_t i = 0; i < a.size(); ++i)
        for (size_t j = 0; j < b.size(); ++j) {
            double s = conj_(a[a.size() - i - 1]) * b[j];
            c[i + j] = c[i + j] + s;
        }
    cpx<double> t0 = {0.0, 0.0}, t1 = {0.0, 0.0};
    for (size_t i = 0; i < n; ++i) {
        cpx<double> c0 = mul(c[i], from_polar(1.0, f * 2.0 * M_PI * (double)i));
        t0 = add(t0, mul(c0, (double)i));
        t1 = add(t1, c0);
    }
    if (std::hypot(t1.re, t1.im) <= 0.00000000001) { *err = 3; return 0.0; }
    return cdiv(t0, t1).re - (double)(a.size() - 1);
}

// frequency response helper: scale * sum_i c[i] * e^{+j 2 pi f i}
template <typename C> cpx<double> poly_response(const std::vector<C>& c, double f) {
    cpx<double> out = {0.0, 0.0};
    for (size_t i = 0; i < c.size(); ++i)
        out = add(out, coef_mul_polar(c[i], from_polar(1.0, f * 2.0 * M_PI * (double)i)));
    return out;
}
inline double widen(float x) { return x; }
inline double widen(double x) { return x; }
inline cpx<double> widen(cpx<float> x) { return {x.re, x.im}; }
inline cpx<double> widen(cpx<double> x) { return x; }
template <typename C> std::vector<decltype(widen(C()))> widen_vec(const std::vector<C>& v) {
    std::vector<decltype(widen(C()))> o; o.reserve(v.size());
    for (auto& x : v) o.push_back(widen(x));
    return o;
}

// --------------------------------------------------------------------------
// Object model for the C API below
// --------------------------------------------------------------------------
struct Obj {
    virtual ~Obj() {}
    // returns number of outputs written
    virtual size_t execute_block(const void* in, size_t n, void* out) = 0;
    virtual size_t execute(const void* in, void* out) { return execute_block(in, 1, out); }
    virtual void push(const void*) {}
    virtual void write(const void*, size_t) {}
    virtual void reset() {}
    virtual double group_delay(double) { return 0.0; }
    virtual cpx<double> frequency_response(double) { return {0.0, 0.0}; }
    virtual Obj* clone() const = 0;
    // SecondOrder IIR state (w1, w2) per section, the device handle's layout (sdsp_iir_get_state):
    // copied to st (set = 0) or from st (set = 1) as the sample type; 1 = not an SOS cascade
    virtual int sos_state(void*, int) { return 1; }
};

// FIRFilter<Coef,In>  src/filter/fir/mod.rs:58-304
template <typename C, typename I> struct FIR : Obj {
    using O = typename out_of<C, I>::type;
    C scale;
    Window<I> window;
    DotProduct<C> coefs;
    FIR(const C* h, size_t L, C s) : scale(s), window((size_t)1 << msb_index(L), 0), coefs(h, L, REVERSE) {}  // :79-88
    O step(I x) {  // execute  :209-212
        window.push(x);
        std::vector<I> w = window.to_vec();
        return mul(coefs.execute(w.data(), w.size()), scale);
    }
    size_t execute_block(const void* in, size_t n, void* out) override {  // :235-241
        const I* x = (const I*)in; O* y = (O*)out;
        for (size_t i = 0; i < n; ++i) y[i] = step(x[i]);
        return n;
    }
    // frequency_response uses coefficients(), i.e. the REVERSED stored taps  :263-273
    cpx<double> frequency_response(double f) override {
        cpx<double> o = poly_response(widen_vec(coefs.c), f);
        return mul(widen(scale), o);
    }
    double group_delay(double f) override { int e; return fir_group_delay(widen_vec(coefs.c), f, &e); }  // :293-303
    Obj* clone() const override { return new FIR(*this); }
};

// DecimatingFIRFilter  src/filter/fir/decim.rs:5-281
template <typename C, typename I> struct Decim : Obj {
    using O = typename out_of<C, I>::type;
    FIR<C, I> f;
    size_t ci = 0, M;
    Decim(const C* h, size_t L, C s, size_t m) : f(h, L, s), M(m) {}
    void push(const void* p) override {  // :115-118
        ci = (ci + 1) % M;
        f.window.push(*(const I*)p);
    }
    void write(const void* p, size_t n) override {  // :136-139
        ci = (ci + n) % M;
        f.window.write((const I*)p, n);
    }
    size_t execute_block(const void* in, size_t n, void* out) override {  // :221-228, :250-256
        const I* x = (const I*)in; O* y = (O*)out; size_t k = 0;
        for (size_t i = 0; i < n; ++i) {
            push(&x[i]);
            if (ci == 0) {
                std::vector<I> w = f.window.to_vec();
                y[k++] = mul(f.coefs.execute(w.data(), w.size()), f.scale);
            }
        }
        return k;
    }
    cpx<double> frequency_response(double fr) override { return f.frequency_response(fr); }
    double group_delay(double fr) override { return f.group_delay(fr); }
    Obj* clone() const override { return new Decim(*this); }
};

// PolyPhaseFilterBank  src/filter/fir/pfb.rs:3-91
template <typename C, typename I> struct PFB : Obj {
    using O = typename out_of<C, I>::type;
    C scale;
    size_t K, M;
    Window<I> window;
    std::vector<DotProduct<C>> coefs;
    PFB(const C* h, size_t L, size_t m, C s) : scale(s), K(L / m), M(m), window(L / m, 0) {  // :24-49
        for (size_t p = 0; p < M; ++p) {
            std::vector<C> rev(K, zero<C>());
            for (size_t idx = 0; idx < K; ++idx) rev[K - idx - 1] = h[p + idx * M];
            coefs.emplace_back(rev.data(), K, FORWARD);
        }
    }
    void push(const void* p) override { window.push(*(const I*)p); }  // :81-83
    void reset() override { window.reset(); }                           // :77-79
    O branch(size_t p) {                                                // execute(index) :85-90 (no scale)
        std::vector<I> w = window.to_vec();
        return coefs[p].execute(w.data(), w.size());
    }
    // all-branches block: push, then emit branch 0..M-1 (the interpolator's loop)
    size_t execute_block(const void* in, size_t n, void* out) override {
        const I* x = (const I*)in; O* y = (O*)out; size_t k = 0;
        for (size_t i = 0; i < n; ++i) {
            push(&x[i]);
            for (size_t p = 0; p < M; ++p) y[k++] = branch(p);
        }
        return k;
    }
    std::vector<C> flat() const {
        std::vector<C> o;
        for (auto& d : coefs) o.insert(o.end(), d.c.begin(), d.c.end());
        return o;
    }
    cpx<double> frequency_response(double f) override {   // interp.rs:113-124 form (flat branches)
        return mul(widen(scale), poly_response(widen_vec(flat()), f));
    }
    double group_delay(double f) override { int e; return fir_group_delay(widen_vec(flat()), f, &e); }
    Obj* clone() const override { return new PFB(*this); }
};

// InterpolatingFIRFilter  src/filter/fir/interp.rs:6-138
template <typename C, typename I> struct Interp : Obj {
    PFB<C, I>* bank;
    size_t M;
    static std::vector<C> pad(const C* h, size_t L, size_t m) {  // :27-54, K computed in f32
        float q = (float)L / (float)m;
        size_t K = (q == std::floor(q)) ? (size_t)q : (size_t)std::ceil(q);
        std::vector<C> e(h, h + L);
        e.resize(K * m, zero<C>());
        return e;
    }
    Interp(const C* h, size_t L, size_t m) : M(m) {
        std::vector<C> e = pad(h, L, m);
        C one; set_one(one);
        bank = new PFB<C, I>(e.data(), e.size(), m, one);
    }
    Interp(const Interp& o) : bank(new PFB<C, I>(*o.bank)), M(o.M) {}
    ~Interp() { delete bank; }
    static void set_one(float& x) { x = 1.0f; }
    static void set_one(double& x) { x = 1.0; }
    static void set_one(cpx<float>& x) { x = {1.0f, 0.0f}; }
    static void set_one(cpx<double>& x) { x = {1.0, 0.0}; }
    size_t execute_block(const void* in, size_t n, void* out) override { return bank->execute_block(in, n, out); }  // :102-111
    cpx<double> frequency_response(double f) override { return bank->frequency_response(f); }
    double group_delay(double f) override { return bank->group_delay(f); }
    Obj* clone() const override { return new Interp(*this); }
};

// SecondOrderFilter<C,T>  src/filter/iir/sos.rs:34-231  (C = f64 or f32 restatement)
template <typename C, typename T> struct SOS {
    Window<T> wbuf;
    DotProduct<C> num;  // holds a[1..]/a0  (field names swapped, :72-73)
    DotProduct<C> den;  // holds b/a0
    SOS(const C* ff, const C* fb) : wbuf(3, 0) {  // :55-75
        C a0 = fb[0];
        C b[3] = {ff[0] / a0, ff[1] / a0, ff[2] / a0};
        C a[3] = {fb[0] / a0, fb[1] / a0, fb[2] / a0};
        num = DotProduct<C>(a + 1, 2, FORWARD);
        den = DotProduct<C>(b, 3, FORWARD);
    }
    T step(T x) {  // execute  :92-114
        std::vector<T> buffer = wbuf.to_vec();
        buffer[2] = buffer[1];
        buffer[1] = buffer[0];
        T d = num.execute(buffer.data() + 1, 2);
        T mixed = sub(x, d);
        wbuf.push(mixed);
        std::vector<T> b2 = wbuf.to_vec();
        return den.execute(b2.data(), 3);
    }
    // group_delay  :208-230 — iir_group_delay(numerator_coefs()=a[1..], denominator_coefs()=b) + 2
    double group_delay(double f) {
        int e;
        double d = iir_group_delay(widen_vec(num.c), widen_vec(den.c), f, &e);
        return e ? 0.0 : d + 2.0;
    }
};

enum IIRType { NORMAL = 0, SECOND_ORDER = 1 };

// IIRFilter<Coef,In>  src/filter/iir/mod.rs:62-414  (Coef real: f64, or f32 for the f32 restatement)
template <typename C, typename I> struct IIR : Obj {
    int type;
    Window<I> buffer;
    DotProduct<C> num, den;
    std::vector<SOS<C, I>> sections;
    IIR(const C* ff, size_t nff, const C* fb, size_t nfb, int t)
        : type(t), buffer(t == NORMAL ? (nfb > nff ? nfb : nff) : (nff / 3) * 2, 0) {
        if (t == NORMAL) {  // :101-129
            C a0 = fb[0];
            std::vector<C> n_, d_;
            for (size_t i = 0; i < nff; ++i) n_.push_back(ff[i] / a0);
            for (size_t i = 0; i < nfb; ++i) d_.push_back(fb[i] / a0);
            num = DotProduct<C>(n_.data(), n_.size(), FORWARD);
            den = DotProduct<C>(d_.data() + 1, d_.size() - 1, FORWARD);
        } else {  // :131-162
            for (size_t i = 0; i < nff / 3; ++i) sections.emplace_back(ff + 3 * i, fb + 3 * i);
            num = DotProduct<C>(ff, nff, FORWARD);
            den = DotProduct<C>(fb, nfb, FORWARD);
        }
    }
    I step(I x) {  // execute :270-289
        if (type == NORMAL) {
            std::vector<I> b = buffer.to_vec();
            I d = den.execute(b.data(), b.size() - 1);
            I mixed = sub(x, d);
            buffer.push(mixed);
            std::vector<I> b2 = buffer.to_vec();
            return num.execute(b2.data(), b2.size());
        }
        I v = sections[0].step(x);
        for (size_t s = 1; s < sections.size(); ++s) v = sections[s].step(v);
        return v;
    }
    size_t execute_block(const void* in, size_t n, void* out) override {  // :310-316
        const I* x = (const I*)in; I* y = (I*)out;
        for (size_t i = 0; i < n; ++i) y[i] = step(x[i]);
        return n;
    }
    cpx<double> frequency_response(double f) override {  // :336-372
        if (type == NORMAL) {
            cpx<double> b = poly_response(widen_vec(num.c), f);
            cpx<double> a = poly_response(widen_vec(den.c), f);
            return cdiv(b, a);
        }
        cpx<double> h = {0.0, 0.0};  // starts at zero: SecondOrder response is identically 0
        for (auto& s : sections) {
            cpx<double> r = cdiv(poly_response(widen_vec(s.num.c), f), poly_response(widen_vec(s.den.c), f));
            h = mul(h, r);
        }
        return h;
    }
    double group_delay(double f) override {  // :392-413
        if (type == NORMAL) {
            int e; double d = iir_group_delay(widen_vec(num.c), widen_vec(den.c), f, &e);
            return e ? 0.0 : d;
        }
        double d = 0.0;
        for (auto& s : sections) d = d + s.group_delay(f) + 2.0;
        return d;
    }
    Obj* clone() const override { return new IIR(*this); }
    // the delay line of section q after a step is [w, w1_old, w2_old] newest first: the state the
    // next step reads is (buf[0], buf[1]) (sos.rs:92-114; buf[2] is overwritten before use)
    int sos_state(void* st, int set) override {
        if (type != SECOND_ORDER) return 1;
        I* p = (I*)st;
        for (size_t q = 0; q < sections.size(); ++q) {
            auto& b = sections[q].wbuf.buf;
            if (set) {
                b[0] = p[2 * q];
                b[1] = p[2 * q + 1];
            } else {
                p[2 * q] = b[0];
                p[2 * q + 1] = b[1];
            }
        }
        return 0;
    }
};

// DecimatingIIRFilter  src/filter/iir/decim.rs:190-233
template <typename C, typename I> struct IIRDecim : Obj {
    IIR<C, I> f; size_t M, index = 0;
    IIRDecim(const C* ff, size_t nff, const C* fb, size_t nfb, int t, size_t m) : f(ff, nff, fb, nfb, t), M(m) {}
    size_t execute_block(const void* in, size_t n, void* out) override {
        const I* x = (const I*)in; I* y = (I*)out; size_t k = 0;
        for (size_t i = 0; i < n; ++i) {
            index = (index + 1) % M;
            I v = f.step(x[i]);
            if (index == 0) y[k++] = v;
        }
        return k;
    }
    cpx<double> frequency_response(double fr) override { return f.frequency_response(fr); }
    double group_delay(double fr) override { return f.group_delay(fr); }
    Obj* clone() const override { return new IIRDecim(*this); }
};

// InterpolatingIIRFilter  src/filter/iir/interp.rs:184-221
template <typename C, typename I> struct IIRInterp : Obj {
    IIR<C, I> f; size_t M;
    IIRInterp(const C* ff, size_t nff, const C* fb, size_t nfb, int t, size_t m) : f(ff, nff, fb, nfb, t), M(m) {}
    size_t execute_block(const void* in, size_t n, void* out) override {
        const I* x = (const I*)in; I* y = (I*)out; size_t k = 0;
        for (size_t i = 0; i < n; ++i) {
            y[k++] = f.step(x[i]);
            for (size_t j = 1; j < M; ++j) y[k++] = f.step(zero<I>());
        }
        return k;
    }
    cpx<double> frequency_response(double fr) override { return f.frequency_response(fr); }
    double group_delay(double fr) override { return f.group_delay(fr); }
    Obj* clone() const override { return new IIRInterp(*this); }
};

}  // namespace orc

using namespace orc;

// dtype codes shared with include/sdsp.h: (Coef, In)
enum { RR32 = 0, RC32 = 1, CC32 = 2, RR64 = 3, RC64 = 4, CC64 = 5 };

extern "C" {

size_t orc_msb_index(size_t x) { return msb_index(x); }

// ---- FIR family ----------------------------------------------------------
#define ORC_DISPATCH_FIR(T, ...)                                                          \
    switch (dtype) {                                                                      \
        case RR32: return new T<float, float>(__VA_ARGS__(float));                        \
        case RC32: return new T<float, cpx<float>>(__VA_ARGS__(float));                   \
        case CC32: return new T<cpx<float>, cpx<float>>(__VA_ARGS__(cpx<float>));         \
        case RR64: return new T<double, double>(__VA_ARGS__(double));                     \
        case RC64: return new T<double, cpx<double>>(__VA_ARGS__(double));                \
        case CC64: return new T<cpx<double>, cpx<double>>(__VA_ARGS__(cpx<double>));      \
    }                                                                                     \
    return nullptr;

// error codes mirror FIRErrorCode (src/filter/fir/mod.rs:40-45) + 1
void* orc_fir_new(int dtype, const void* taps, size_t L, const void* scale, int* err) {
    *err = 0;
    if (L == 0) { *err = 1; return nullptr; }
#define A(C) (const C*)taps, L, *(const C*)scale
    ORC_DISPATCH_FIR(FIR, A)
#undef A
}
void* orc_decim_new(int dtype, const void* taps, size_t L, const void* scale, size_t M, int* err) {
    *err = 0;
    if (L == 0) { *err = 1; return nullptr; }
    if (M < 1) { *err = 2; return nullptr; }
#define A(C) (const C*)taps, L, *(const C*)scale, M
    ORC_DISPATCH_FIR(Decim, A)
#undef A
}
void* orc_pfb_new(int dtype, const void* taps, size_t L, size_t M, const void* scale, int* err) {
    *err = 0;
    if (M == 0) { *err = 4; return nullptr; }
    if (L == 0) { *err = 1; return nullptr; }
    if (L / M == 0) { *err = 90; return nullptr; }  // reference panics (Window::new(0) assert)
#define A(C) (const C*)taps, L, M, *(const C*)scale
    ORC_DISPATCH_FIR(PFB, A)
#undef A
}
void* orc_interp_new(int dtype, const void* taps, size_t L, size_t M, int* err) {
    *err = 0;
    if (L == 0) { *err = 1; return nullptr; }
    if (M < 1) { *err = 3; return nullptr; }
#define A(C) (const C*)taps, L, M
    ORC_DISPATCH_FIR(Interp, A)
#undef A
}

size_t orc_execute_block(void* h, const void* in, size_t n, void* out) { return ((Obj*)h)->execute_block(in, n, out); }
void orc_push(void* h, const void* x) { ((Obj*)h)->push(x); }
void orc_write(void* h, const void* x, size_t n) { ((Obj*)h)->write(x, n); }
void orc_reset(void* h) { ((Obj*)h)->reset(); }
void* orc_clone(void* h) { return ((Obj*)h)->clone(); }
void orc_free(void* h) { delete (Obj*)h; }
int orc_sos_state(void* h, void* st, int set) { return ((Obj*)h)->sos_state(st, set); }
double orc_group_delay(void* h, double f) { return ((Obj*)h)->group_delay(f); }
void orc_frequency_response(void* h, double f, double* out2) {
    cpx<double> r = ((Obj*)h)->frequency_response(f);
    out2[0] = r.re; out2[1] = r.im;
}

// PFB execute(index) on the current window (no push)
int orc_pfb_execute(void* h, int dtype, size_t index, void* out) {
    switch (dtype) {
#define C_(K, C, I) case K: { auto* p = (PFB<C, I>*)h; if (index >= p->M) return 1; *(typename PFB<C, I>::O*)out = p->branch(index); return 0; }
        C_(RR32, float, float) C_(RC32, float, cpx<float>) C_(CC32, cpx<float>, cpx<float>)
        C_(RR64, double, double) C_(RC64, double, cpx<double>) C_(CC64, cpx<double>, cpx<double>)
#undef C_
    }
    return 2;
}

// ---- IIR family (Coef real) ------------------------------------------------
// err mirrors IIRErrorCode order (src/filter/iir/mod.rs:41-49) + 10
static int iir_check(const void*, size_t nff, const void*, size_t nfb, int type) {
    if (type == NORMAL) {
        if (nff == 0) return 10;
        if (nfb == 0) return 11;
    } else {
        if (nff != nfb) return 13;
        if (nff == 0) return 12;
        if (nff % 3 != 0) return 14;
    }
    return 0;
}
#define ORC_DISPATCH_IIR(T, ...)                                                   \
    switch (dtype) {                                                               \
        case RR32: return new T<float, float>(__VA_ARGS__(float));                 \
        case RC32: return new T<float, cpx<float>>(__VA_ARGS__(float));            \
        case RR64: return new T<double, double>(__VA_ARGS__(double));              \
        case RC64: return new T<double, cpx<double>>(__VA_ARGS__(double));         \
    }                                                                              \
    *err = 90; return nullptr;

void* orc_iir_new(int dtype, const void* ff, size_t nff, const void* fb, size_t nfb, int type, int* err) {
    *err = iir_check(ff, nff, fb, nfb, type);
    if (*err) return nullptr;
#define A(C) (const C*)ff, nff, (const C*)fb, nfb, type
    ORC_DISPATCH_IIR(IIR, A)
#undef A
}
void* orc_iir_decim_new(int dtype, const void* ff, size_t nff, const void* fb, size_t nfb, int type, size_t M, int* err) {
    *err = 0;
    if (nff == 0) { *err = 10; return nullptr; }
    if (nfb == 0) { *err = 11; return nullptr; }
    if (M < 1) { *err = 15; return nullptr; }
    *err = iir_check(ff, nff, fb, nfb, type);
    if (*err) return nullptr;
#define A(C) (const C*)ff, nff, (const C*)fb, nfb, type, M
    ORC_DISPATCH_IIR(IIRDecim, A)
#undef A
}
void* orc_iir_interp_new(int dtype, const void* ff, size_t nff, const void* fb, size_t nfb, int type, size_t M, int* err) {
    *err = 0;
    if (nff == 0) { *err = 10; return nullptr; }
    if (nfb == 0) { *err = 11; return nullptr; }
    if (M < 1) { *err = 16; return nullptr; }
    *err = iir_check(ff, nff, fb, nfb, type);
    if (*err) return nullptr;
#define A(C) (const C*)ff, nff, (const C*)fb, nfb, type, M
    ORC_DISPATCH_IIR(IIRInterp, A)
#undef A
}

// SecondOrderFilter alone (f64 coefs, f64 samples)  src/filter/iir/sos.rs
struct SOSObj { SOS<double, double> s; };
void* orc_sos_new(const double* ff, size_t nff, const double* fb, size_t nfb, int* err) {
    *err = 0;
    if (nff < 3 || nfb < 3) { *err = 20; return nullptr; }
    return new SOSObj{SOS<double, double>(ff, fb)};
}
double orc_sos_execute(void* h, double x) { return ((SOSObj*)h)->s.step(x); }
double orc_sos_group_delay(void* h, double f) { return ((SOSObj*)h)->s.group_delay(f); }
void orc_sos_coefs(void* h, double* num2, double* den3) {
    auto* p = (SOSObj*)h;
    for (int i = 0; i < 2; ++i) num2[i] = p->s.num.c[i];
    for (int i = 0; i < 3; ++i) den3[i] = p->s.den.c[i];
}
void orc_sos_free(void* h) { delete (SOSObj*)h; }

// ---- DotProduct (f64 / c64) -----------------------------------------------
// kind: 0 = f64 coef x f64 samples, 1 = f64 x c64, 2 = c64 x c64
void orc_dot_execute(int kind, const void* coefs, size_t len, int direction, const void* s, size_t n, double* out) {
    if (kind == 0) {
        DotProduct<double> d((const double*)coefs, len, (Direction)direction);
        out[0] = d.execute((const double*)s, n); out[1] = 0.0;
    } else if (kind == 1) {
        DotProduct<double> d((const double*)coefs, len, (Direction)direction);
        cpx<double> r = d.execute((const cpx<double>*)s, n); out[0] = r.re; out[1] = r.im;
    } else {
        DotProduct<cpx<double>> d((const cpx<double>*)coefs, len, (Direction)direction);
        cpx<double> r = d.execute((const cpx<double>*)s, n); out[0] = r.re; out[1] = r.im;
    }
}

// ---- Group delay entry points (src/group_delay/mod.rs) ----------------------
double orc_fir_group_delay(const double* h, size_t n, double f, int* err) {
    return fir_group_delay(std::vector<double>(h, h + n), f, err);
}
double orc_iir_group_delay(const double* b, size_t nb, const double* a, size_t na, double f, int* err) {
    return iir_group_delay(std::vector<double>(b, b + nb), std::vector<double>(a, a + na), f, err);
}

}  // extern "C"
