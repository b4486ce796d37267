// ============================================================================
// sdsp_oracle_rx.cpp — CPU RESTATEMENT of the receive-chain objects next to the
// filter path: AutoCorrelator, NCO and AGC.
// TEST INFRASTRUCTURE ONLY (see sdsp_oracle.cpp's header): loaded by tests/ and
// bench.py's cpu_baseline leg, never by the product library.
//
// Follows the reference literally (paths relative to the reference checkout):
//   * AutoCorrelator  src/filter/auto_correlator/mod.rs:26-214, on two
//     Window<Complex<C>> (src/window/mod.rs:17-77) — the delayed window has
//     capacity + delay zeroed slots but push() only shifts the first
//     capacity - 1, so slots [capacity, capacity + delay) stay zero and
//     to_vec() (which starts at `delay`) reads them: the unfilled-delay tail.
//     push() needs Complex<C>: Real<Output = f64> (:99-102), i.e. C = f64 in the
//     reference; the C = f32 instance here is the same sequence of operations
//     at f32 (energy still accumulated in f64), the checker of the c32 kernel.
//   * NCO  src/nco/mod.rs:27-187: 1024-entry f64 sine table, u32 phase,
//     index = ((theta + 2^21) >> 22) & 0x3ff, cos = table[(index + 256) & 0x3ff],
//     constrain(), step(), pll_step(), mix_up / mix_down (num-complex Mul).
//     mix_up_block / mix_down_block (:153-172) index a Vec of length 0 and panic
//     for any non-empty input; the block restatement here is the per-sample
//     composition `mix_up(x); step()` those functions spell out.
//   * AGC  src/auto_gain_control/mod.rs:97-677 for f64 and Complex<f64> samples:
//     execute (:214-246), update_squelch_mode (:631-677; the usize timer wraps as
//     in a release build), init (:568-586) and the setters, with libm's exp/ln/log10.
// Compiled with -ffp-contract=off (no FMA, as rustc).
// ============================================================================
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>

namespace orx {

template <typename T> struct cpx { T re, im; };
template <typename T> inline cpx<T> cmul(cpx<T> a, cpx<T> b) { return {a.re * b.re - a.im * b.im, a.re * b.im + a.im * b.re}; }
template <typename T> inline cpx<T> cadd(cpx<T> a, cpx<T> b) { return {a.re + b.re, a.im + b.im}; }
template <typename T> inline cpx<T> conj(cpx<T> a) { return {a.re, -a.im}; }

// Window<T> with a delay  src/window/mod.rs:17-77
template <typename T> struct Window {
    size_t capacity, delay;
    std::vector<T> buf;  // capacity + delay zeroed slots (alloc_zeroed :21-26)
    Window(size_t cap, size_t d) : capacity(cap), delay(d), buf(cap + d, T{}) {}
    void push(T x) {  // memmove(buf + 1, buf, capacity - 1); buf[0] = x   :63-71
        std::memmove(buf.data() + 1, buf.data(), (capacity - 1) * sizeof(T));
        buf[0] = x;
    }
    std::vector<T> to_vec() const { return std::vector<T>(buf.begin() + delay, buf.begin() + delay + capacity); }
    void reset() { std::fill(buf.begin(), buf.end(), T{}); }
};

// AutoCorrelator<C>  src/filter/auto_correlator/mod.rs:26-214
template <typename C> struct AutoCorrelator {
    using X = cpx<C>;
    size_t window_size, delay;
    Window<X> window, window_with_delay;
    std::vector<double> energy_buffer;
    double energy_sum = 0.0;
    size_t energy_index = 0;
    AutoCorrelator(size_t w, size_t d)  // :51-62
        : window_size(w), delay(d), window(w, 0), window_with_delay(w, d), energy_buffer(w, 0.0) {}
    void reset() {  // :76-85
        window.reset();
        window_with_delay.reset();
        energy_sum = 0.0;
        std::fill(energy_buffer.begin(), energy_buffer.end(), 0.0);
        energy_index = 0;
    }
    void push(X x) {  // :99-111
        window.push(x);
        window_with_delay.push(conj(x));
        const double e2 = (double)cmul(x, conj(x)).re;  // (sample * sample.conj()).real()
        energy_sum -= energy_buffer[energy_index];
        energy_sum += e2;
        energy_buffer[energy_index] = e2;
        energy_index = (energy_index + 1) % window_size;
    }
    X execute() const {  // :156-163  zip(to_vec, to_vec).map(x * y).sum(), from Complex::zero
        const std::vector<X> a = window.to_vec(), b = window_with_delay.to_vec();
        X s{C(0), C(0)};
        for (size_t i = 0; i < a.size(); ++i) s = cadd(s, cmul(a[i], b[i]));
        return s;
    }
};

// NCO  src/nco/mod.rs:27-187
inline uint32_t constrain(double theta) {  // :175-187
    const double d = theta / (2.0 * M_PI);
    double f = d - std::trunc(d);  // f64::fract
    if (f < 0.0) f += 1.0;
    return (uint32_t)(f * (double)0xffffffffu);  // `as u32` saturates; f * (2^32 - 1) < 2^32
}
struct NCO {
    double table[1024];
    uint32_t theta = 0, delta_theta = 0;
    double alpha, beta;
    NCO() {  // :36-50
        for (int i = 0; i < 1024; ++i) table[i] = std::sin(2.0 * M_PI * (double)i / 1024.0);
        alpha = 0.1;
        beta = std::sqrt(alpha);
    }
    size_t index() const { return (size_t)(((uint32_t)(theta + (1u << 21)) >> 22) & 0x3ff); }  // :99-101
    double sin_() const { return table[index()]; }
    double cos_() const { return table[(index() + 256) & 0x3ff]; }
    void step() { theta += delta_theta; }  // wrapping_add  :94-96
    cpx<double> mix_up(cpx<double> x) const { return cmul(cpx<double>{cos_(), sin_()}, x); }  // :141-144
    cpx<double> mix_down(cpx<double> x) const { return cmul(conj(cpx<double>{cos_(), sin_()}), x); }  // :147-150
};

// AGC  src/auto_gain_control/mod.rs:84-677.  T = f64 or Complex<f64> (the trait
// bounds Real<Output = f64> + Mul<f64> admit only these two).
enum Squelch { UNKNOWN, ENABLED, RISE, SIGNALHI, FALL, SINGALLO, TIMEOUT, DISABLED };  // :85-94
struct AGC {
    double gain = 1.0, scale = 1.0, bandwidth = 0.1, alpha = 0.1, energy_estimate = 1.0;  // new  :136-149
    bool lock = false;
    int squelch_mode = DISABLED;
    double squelch_threshold = 0.0;
    uint64_t squelch_timeout = 100, squelch_timer = 0;

    void reset() {  // :178-188
        gain = 1.0;
        energy_estimate = 1.0;
        lock = false;
        squelch_mode = squelch_mode == DISABLED ? DISABLED : ENABLED;
    }
    double get_rssi() const { return std::log10(gain) * -20.0; }  // :442-444
    void update_squelch_mode() {  // :631-677
        const bool exceeded = get_rssi() > squelch_threshold;
        switch (squelch_mode) {
            case ENABLED: squelch_mode = exceeded ? RISE : ENABLED; break;
            case RISE: squelch_mode = exceeded ? SIGNALHI : FALL; break;
            case SIGNALHI: squelch_mode = exceeded ? SIGNALHI : FALL; break;
            case FALL:
                squelch_timer = squelch_timeout;
                squelch_mode = exceeded ? SIGNALHI : SINGALLO;
                break;
            case SINGALLO:
                squelch_timer -= 1;  // usize; wraps as a release build does (debug panics at 0)
                squelch_mode = squelch_timer == 0 ? TIMEOUT : exceeded ? SIGNALHI : SINGALLO;
                break;
            case TIMEOUT: squelch_mode = ENABLED; break;
            default: squelch_mode = DISABLED;
        }
    }
    // execute  :214-246 for an unlocked AGC, after `out` and its energy: the
    // energy update, the gain update and the squelch; true when the squelch hands
    // back the input (mode ENABLED)
    bool update(double ee) {
        energy_estimate = (1.0 - alpha) * energy_estimate + ee * alpha;
        if (energy_estimate > 0.000001) gain *= std::exp(-0.5 * alpha * std::log(energy_estimate));
        if (gain > 1000000.0) gain = 1000000.0;
        update_squelch_mode();
        return squelch_mode == ENABLED;
    }
    double execute(double x) {
        const double out = x * gain;
        if (lock) {
            energy_estimate = (1.0 - alpha) * energy_estimate + out * out * alpha;
            return out;
        }
        return update(out * out) ? x : out * scale;  // (out.conj() * out).real() for f64
    }
    cpx<double> execute(cpx<double> x) {
        const cpx<double> out{x.re * gain, x.im * gain};
        const double ee = cmul(conj(out), out).re;
        if (lock) {
            energy_estimate = (1.0 - alpha) * energy_estimate + ee * alpha;
            return out;
        }
        return update(ee) ? x : cpx<double>{out.re * scale, out.im * scale};
    }
};

}  // namespace orx

using namespace orx;

extern "C" {

// ---- AutoCorrelator: precision 0 = C f32, 1 = C f64 ------------------------
struct AcObj {
    int prec;
    AutoCorrelator<float>* f;
    AutoCorrelator<double>* d;
};
void* orc_acorr_new(size_t window_size, size_t delay, int prec) {
    if (window_size == 0) return nullptr;  // Window::new asserts capacity > 0
    auto* o = new AcObj{prec, nullptr, nullptr};
    if (prec == 0) o->f = new AutoCorrelator<float>(window_size, delay);
    else o->d = new AutoCorrelator<double>(window_size, delay);
    return o;
}
void orc_acorr_free(void* h) {
    auto* o = (AcObj*)h;
    delete o->f;
    delete o->d;
    delete o;
}
void orc_acorr_reset(void* h) {
    auto* o = (AcObj*)h;
    if (o->f) o->f->reset(); else o->d->reset();
}
// write (push only, :128-137)
void orc_acorr_write(void* h, const void* x, size_t n) {
    auto* o = (AcObj*)h;
    for (size_t i = 0; i < n; ++i) {
        if (o->f) o->f->push(((const cpx<float>*)x)[i]);
        else o->d->push(((const cpx<double>*)x)[i]);
    }
}
// execute_block (:181-191): push, then execute, per sample
void orc_acorr_execute_block(void* h, const void* x, size_t n, void* out) {
    auto* o = (AcObj*)h;
    for (size_t i = 0; i < n; ++i) {
        if (o->f) {
            o->f->push(((const cpx<float>*)x)[i]);
            ((cpx<float>*)out)[i] = o->f->execute();
        } else {
            o->d->push(((const cpx<double>*)x)[i]);
            ((cpx<double>*)out)[i] = o->d->execute();
        }
    }
}
void orc_acorr_execute(void* h, void* out) {
    auto* o = (AcObj*)h;
    if (o->f) *(cpx<float>*)out = o->f->execute();
    else *(cpx<double>*)out = o->d->execute();
}
double orc_acorr_get_energy(void* h) {  // :212-214
    auto* o = (AcObj*)h;
    return o->f ? o->f->energy_sum : o->d->energy_sum;
}

// ---- NCO ---------------------------------------------------------------------
void* orc_nco_new() { return new NCO(); }
void orc_nco_free(void* h) { delete (NCO*)h; }
uint32_t orc_nco_constrain(double t) { return constrain(t); }
void orc_nco_set_frequency(void* h, double dt) { ((NCO*)h)->delta_theta = constrain(dt); }  // :59-61
void orc_nco_adjust_frequency(void* h, double dt) { ((NCO*)h)->delta_theta += constrain(dt); }  // :64-66
void orc_nco_set_phase(void* h, double phi) { ((NCO*)h)->theta = constrain(phi); }  // :79-81
void orc_nco_adjust_phase(void* h, double dphi) { ((NCO*)h)->theta += constrain(dphi); }  // :84-86
void orc_nco_reset(void* h) { ((NCO*)h)->theta = 0; ((NCO*)h)->delta_theta = 0; }  // :53-56
void orc_nco_state(void* h, uint32_t* theta, uint32_t* dtheta) {
    *theta = ((NCO*)h)->theta;
    *dtheta = ((NCO*)h)->delta_theta;
}
void orc_nco_sincos(void* h, double* sc) { sc[0] = ((NCO*)h)->sin_(); sc[1] = ((NCO*)h)->cos_(); }
int orc_nco_set_pll_bandwidth(void* h, double bw) {  // :124-132
    if (bw < 0.0) return 1;
    ((NCO*)h)->alpha = bw;
    ((NCO*)h)->beta = std::sqrt(bw);
    return 0;
}
void orc_nco_pll_step(void* h, double dphi) {  // :135-138
    auto* p = (NCO*)h;
    p->delta_theta += constrain(dphi * p->alpha);
    p->theta += constrain(dphi * p->beta);
}
void orc_nco_step(void* h) { ((NCO*)h)->step(); }
// per sample: out = mix_up(x) (down = 0) or mix_down(x) (down = 1), then step()
void orc_nco_mix_block(void* h, int down, const double* x, size_t n, double* out) {
    auto* p = (NCO*)h;
    for (size_t i = 0; i < n; ++i) {
        const cpx<double> v{x[2 * i], x[2 * i + 1]};
        const cpx<double> r = down ? p->mix_down(v) : p->mix_up(v);
        out[2 * i] = r.re;
        out[2 * i + 1] = r.im;
        p->step();
    }
}

// ---- AGC: sample_type 0 = f64, 1 = Complex<f64> -------------------------------
void* orc_agc_new() { return new AGC(); }
void orc_agc_free(void* h) { delete (AGC*)h; }
void orc_agc_reset(void* h) { ((AGC*)h)->reset(); }
void orc_agc_execute_block(void* h, int sample_type, const double* x, size_t n, double* out) {  // :273-285
    auto* a = (AGC*)h;
    for (size_t i = 0; i < n; ++i) {
        if (sample_type == 1) {
            const cpx<double> r = a->execute(cpx<double>{x[2 * i], x[2 * i + 1]});
            out[2 * i] = r.re;
            out[2 * i + 1] = r.im;
        } else {
            out[i] = a->execute(x[i]);
        }
    }
}
int orc_agc_init(void* h, int sample_type, const double* x, size_t n, double* level) {  // :568-586
    if (n == 0) return 44;
    double x2 = 0.0;
    for (size_t i = 0; i < n; ++i) {
        if (sample_type == 1) {
            const cpx<double> v{x[2 * i], x[2 * i + 1]};
            x2 += cmul(v, conj(v)).re;
        } else {
            x2 += x[i] * x[i];
        }
    }
    x2 = std::sqrt(x2 / (double)n) + 1e-16;
    *level = x2;
    if (x2 <= 0.0) return 41;
    ((AGC*)h)->gain = 1.0 / x2;  // set_signal_level  :416-428
    ((AGC*)h)->energy_estimate = 1.0;
    return 0;
}
int orc_agc_set_bandwidth(void* h, double bw) {  // :374-386
    if (!(bw >= 0.0 && bw <= 1.0)) return 40;
    ((AGC*)h)->bandwidth = bw;
    ((AGC*)h)->alpha = bw;
    return 0;
}
void orc_agc_set_rssi(void* h, double rssi) {  // :458-466
    auto* a = (AGC*)h;
    a->gain = std::pow(10.0, -rssi / 20.0);
    if (a->gain < 1e-16) a->gain = 1e-16;
    a->energy_estimate = 1.0;
}
void orc_agc_set_gain(void* h, double g) { ((AGC*)h)->gain = g; }
void orc_agc_set_scale(void* h, double s) { ((AGC*)h)->scale = s; }
void orc_agc_lock(void* h, int on) { ((AGC*)h)->lock = on != 0; }
void orc_agc_squelch(void* h, int enable) { ((AGC*)h)->squelch_mode = enable ? ENABLED : DISABLED; }
void orc_agc_squelch_set_threshold(void* h, double t) { ((AGC*)h)->squelch_threshold = t; }
void orc_agc_squelch_set_timeout(void* h, uint64_t t) { ((AGC*)h)->squelch_timeout = t; }
double orc_agc_get_gain(void* h) { return ((AGC*)h)->gain; }
double orc_agc_get_energy(void* h) { return ((AGC*)h)->energy_estimate; }
double orc_agc_get_rssi(void* h) { return ((AGC*)h)->get_rssi(); }
int orc_agc_get_mode(void* h) { return ((AGC*)h)->squelch_mode; }
uint64_t orc_agc_get_timer(void* h) { return ((AGC*)h)->squelch_timer; }

}  // extern "C"
