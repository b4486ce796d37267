// C-ABI runtime for the receive-chain objects next to the filter path
// (SURVEY §8f rows 3-4): AutoCorrelator (src/filter/auto_correlator/mod.rs),
// NCO (src/nco/mod.rs) and the AGC bank (src/auto_gain_control/mod.rs).  The
// sample streams run in kern_rx.hip; the NCO's scalar phase/frequency registers
// are host state, as in the reference; the AGC state lives on the device (the
// recurrence updates it every sample) with a host copy for setters and getters.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstring>
#include <vector>

#include "sdsp.h"
#include "sdsp_host.hpp"
#include "sdsp_kernels.hpp"

using namespace sdsp;

namespace {

#define R_TRY(expr, what)                                      \
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

int check_gfx950(int device, int* cus) {
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
    if (cus) *cus = p.multiProcessorCount;
    return SDSP_OK;
}

hipStream_t pick(void* user, hipStream_t own) { return user ? (hipStream_t)user : own; }
size_t cbytes(int prec) { return prec == 0 ? 8 : 16; }
int hist_dtype(int prec) { return prec == 0 ? SDSP_RC32 : SDSP_RC64; }  // sample size 8 / 16 bytes

// constrain()  src/nco/mod.rs:175-187
uint32_t constrain(double theta) {
    const double d = theta / (2.0 * M_PI);
    double f = d - std::trunc(d);  // f64::fract
    if (f < 0.0) f += 1.0;
    return (uint32_t)(f * (double)0xffffffffu);
}

}  // namespace

// ===========================================================================
// AutoCorrelator
// ===========================================================================
struct sdsp_acorr {
    int prec = 1, device = 0;
    size_t W = 0, d = 0, channels = 1;
    DevBuf hist[2];  // [channels][W] oldest first
    int cur = 0;
    DevBuf energy;   // [channels] f64
    DevBuf stage_in, stage_out;
    hipStream_t stream = nullptr;
    int kernel = 0;  // SDSP_TUNE_ACORR_KERNEL
    StreamFence fence;  // the last block queued (on a caller stream or the handle's)
    int K() const { return W > d ? (int)(W - d) : 0; }
};

namespace {
int acorr_alloc(sdsp_acorr* h) {
    const size_t hb = h->channels * h->W * cbytes(h->prec);
    R_TRY(h->fence.wait(), "wait for queued work");  // a queued block may still read the history
    for (int i = 0; i < 2; ++i) {
        R_TRY(h->hist[i].ensure(hb), "alloc history");
        R_TRY(hipMemsetAsync(h->hist[i].p, 0, hb, h->stream), "zero history");
    }
    R_TRY(h->energy.ensure(h->channels * 8), "alloc energy");
    R_TRY(hipMemsetAsync(h->energy.p, 0, h->channels * 8, h->stream), "zero energy");
    h->cur = 0;
    R_TRY(hipStreamSynchronize(h->stream), "sync");
    return SDSP_OK;
}
}  // namespace

extern "C" {

int sdsp_acorr_create(sdsp_acorr** out, size_t window_size, size_t delay, int precision, int device) {
    if (!out) return SDSP_E_INVALID_ARGUMENT;
    *out = nullptr;
    if (window_size == 0 || (precision != 0 && precision != 1)) {
        set_error("window_size must be > 0 (Window::new asserts capacity > 0); precision 0 = c32, 1 = c64");
        return SDSP_E_INVALID_ARGUMENT;
    }
    if (window_size > (1u << 30) || delay > (1u << 30)) {
        set_error("window_size / delay too large");
        return SDSP_E_INVALID_ARGUMENT;
    }
    int st = check_gfx950(device, nullptr);
    if (st) return st;
    Guard g(device);
    auto* h = new sdsp_acorr();
    h->prec = precision;
    h->device = device;
    h->W = window_size;
    h->d = delay;
    if (hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking) != hipSuccess) {
        delete h;
        set_error("hipStreamCreate failed");
        return SDSP_E_DEVICE;
    }
    st = acorr_alloc(h);
    if (st) {
        sdsp_acorr_destroy(h);
        return st;
    }
    *out = h;
    return SDSP_OK;
}

void sdsp_acorr_destroy(sdsp_acorr* h) {
    if (!h) return;
    {
        Guard g(h->device);
        (void)h->fence.wait();
        if (h->stream) {
            (void)hipStreamSynchronize(h->stream);
            (void)hipStreamDestroy(h->stream);
        }
        h->hist[0].release();
        h->hist[1].release();
        h->energy.release();
        h->stage_in.release();
        h->stage_out.release();
    }
    delete h;
}

int sdsp_acorr_set_tuning(sdsp_acorr* h, int key, int value) {
    if (!h || key != SDSP_TUNE_ACORR_KERNEL || value < 0 || value > 2) return SDSP_E_INVALID_ARGUMENT;
    h->kernel = value;
    return SDSP_OK;
}

int sdsp_acorr_set_channels(sdsp_acorr* h, size_t channels) {
    if (!h || channels == 0) return SDSP_E_INVALID_ARGUMENT;
    Guard g(h->device);
    h->channels = channels;
    return acorr_alloc(h);
}

int sdsp_acorr_reset(sdsp_acorr* h) {
    if (!h) return SDSP_E_INVALID_ARGUMENT;
    Guard g(h->device);
    return acorr_alloc(h);
}

size_t sdsp_acorr_window_size(const sdsp_acorr* h) { return h ? h->W : 0; }
size_t sdsp_acorr_delay(const sdsp_acorr* h) { return h ? h->d : 0; }

// push n samples per channel; with d_out, the execute() value after every push
static int acorr_run(sdsp_acorr* h, const void* d_in, size_t n, void* d_out, hipStream_t s) {
    if (n == 0) return SDSP_OK;
    // blocks queued on another stream read and write the history this launch uses
    R_TRY(h->fence.order_before(s), "order after queued work");
    const void* hist = h->hist[h->cur].p;
    if (d_out)
        R_TRY(launch_acorr(h->prec, d_in, hist, d_out, n, (int)h->W, (int)h->d, h->K(), h->channels, s, h->kernel),
              "acorr");
    R_TRY(launch_acorr_energy(h->prec, d_in, hist, n, (int)h->W, (int)h->W, h->channels, (double*)h->energy.p, s),
          "acorr energy");
    R_TRY(launch_hist_update(hist_dtype(h->prec), d_in, hist, h->hist[h->cur ^ 1].p, n, (int)h->W, h->channels, s),
          "history update");
    h->cur ^= 1;
    R_TRY(h->fence.record(s), "record fence");
    return SDSP_OK;
}

int sdsp_acorr_execute_block_device(sdsp_acorr* h, const void* d_in, size_t n, void* d_out, void* stream) {
    if (!h || (n && (!d_in || !d_out))) return SDSP_E_INVALID_ARGUMENT;
    Guard g(h->device);
    return acorr_run(h, d_in, n, d_out, pick(stream, h->stream));
}

int sdsp_acorr_write_device(sdsp_acorr* h, const void* d_in, size_t n, void* stream) {
    if (!h || (n && !d_in)) return SDSP_E_INVALID_ARGUMENT;
    Guard g(h->device);
    return acorr_run(h, d_in, n, nullptr, pick(stream, h->stream));
}

static int acorr_host(sdsp_acorr* h, const void* in, size_t n, void* out) {
    if (!h || (n && !in)) return SDSP_E_INVALID_ARGUMENT;
    if (n == 0) return SDSP_OK;
    Guard g(h->device);
    R_TRY(h->fence.wait(), "wait for queued work");  // host slices: the last block first, on the host
    const size_t bytes = h->channels * n * cbytes(h->prec);
    R_TRY(h->stage_in.ensure(bytes), "stage in");
    R_TRY(hipMemcpyAsync(h->stage_in.p, in, bytes, hipMemcpyHostToDevice, h->stream), "H2D");
    if (out) R_TRY(h->stage_out.ensure(bytes), "stage out");
    int st = acorr_run(h, h->stage_in.p, n, out ? h->stage_out.p : nullptr, h->stream);
    if (st) return st;
    if (out) R_TRY(hipMemcpyAsync(out, h->stage_out.p, bytes, hipMemcpyDeviceToHost, h->stream), "D2H");
    R_TRY(hipStreamSynchronize(h->stream), "sync");
    return SDSP_OK;
}

int sdsp_acorr_execute_block(sdsp_acorr* h, const void* in, size_t n, void* out) {
    if (n && !out) return SDSP_E_INVALID_ARGUMENT;
    return acorr_host(h, in, n, out);
}

int sdsp_acorr_write(sdsp_acorr* h, const void* in, size_t n) { return acorr_host(h, in, n, nullptr); }

int sdsp_acorr_push(sdsp_acorr* h, const void* sample) {
    if (!h || h->channels != 1) return SDSP_E_INVALID_ARGUMENT;
    return acorr_host(h, sample, 1, nullptr);
}

int sdsp_acorr_execute(sdsp_acorr* h, void* out) {
    if (!h || !out) return SDSP_E_INVALID_ARGUMENT;
    Guard g(h->device);
    const size_t bytes = h->channels * cbytes(h->prec);
    R_TRY(h->stage_out.ensure(bytes), "stage out");
    R_TRY(h->fence.wait(), "wait for queued work");  // host-side op: wait for the last block on the host
    R_TRY(launch_acorr_current(h->prec, h->hist[h->cur].p, h->stage_out.p, (int)h->W, (int)h->d, h->K(), h->channels,
                               h->stream),
          "acorr execute");
    R_TRY(hipMemcpyAsync(out, h->stage_out.p, bytes, hipMemcpyDeviceToHost, h->stream), "D2H");
    R_TRY(hipStreamSynchronize(h->stream), "sync");
    return SDSP_OK;
}

int sdsp_acorr_get_energy(sdsp_acorr* h, double* energy) {
    if (!h || !energy) return SDSP_E_INVALID_ARGUMENT;
    Guard g(h->device);
    R_TRY(h->fence.wait(), "wait for queued work");  // host-side op: wait for the last block on the host
    R_TRY(hipMemcpyAsync(energy, h->energy.p, h->channels * 8, hipMemcpyDeviceToHost, h->stream), "D2H");
    R_TRY(hipStreamSynchronize(h->stream), "sync");
    return SDSP_OK;
}

int sdsp_acorr_synchronize(sdsp_acorr* h) {
    if (!h) return SDSP_E_INVALID_ARGUMENT;
    Guard g(h->device);
    R_TRY(h->fence.wait(), "wait for queued work");
    R_TRY(hipStreamSynchronize(h->stream), "sync");
    return SDSP_OK;
}

}  // extern "C"

// ===========================================================================
// NCO
// ===========================================================================
struct sdsp_nco {
    int device = 0, cus = 256;
    uint32_t theta = 0, delta_theta = 0;
    double alpha = 0.1, beta = 0.0;
    double table[1024];
    DevBuf d_table, stage_in, stage_out;
    hipStream_t stream = nullptr;
    size_t index() const { return (size_t)(((uint32_t)(theta + (1u << 21)) >> 22) & 0x3ffu); }  // :99-101
};

extern "C" {

int sdsp_nco_create(sdsp_nco** out, int device) {  // NCO::new  src/nco/mod.rs:36-50
    if (!out) return SDSP_E_INVALID_ARGUMENT;
    *out = nullptr;
    int cus = 256;
    int st = check_gfx950(device, &cus);
    if (st) return st;
    Guard g(device);
    auto* h = new sdsp_nco();
    h->device = device;
    h->cus = cus;
    for (int i = 0; i < 1024; ++i) h->table[i] = std::sin(2.0 * M_PI * (double)i / 1024.0);
    h->alpha = 0.1;
    h->beta = std::sqrt(h->alpha);
    if (hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking) != hipSuccess) {
        delete h;
        set_error("hipStreamCreate failed");
        return SDSP_E_DEVICE;
    }
    if (h->d_table.ensure(sizeof(h->table)) != hipSuccess ||
        hipMemcpy(h->d_table.p, h->table, sizeof(h->table), hipMemcpyHostToDevice) != hipSuccess) {
        sdsp_nco_destroy(h);
        set_error("NCO table upload failed");
        return SDSP_E_DEVICE;
    }
    *out = h;
    return SDSP_OK;
}

void sdsp_nco_destroy(sdsp_nco* h) {
    if (!h) return;
    {
        Guard g(h->device);
        if (h->stream) {
            (void)hipStreamSynchronize(h->stream);
            (void)hipStreamDestroy(h->stream);
        }
        h->d_table.release();
        h->stage_in.release();
        h->stage_out.release();
    }
    delete h;
}

int sdsp_nco_reset(sdsp_nco* h) {  // :53-56
    if (!h) return SDSP_E_INVALID_ARGUMENT;
    h->theta = 0;
    h->delta_theta = 0;
    return SDSP_OK;
}
uint32_t sdsp_nco_constrain(double theta) { return constrain(theta); }  // :175-187
int sdsp_nco_set_frequency(sdsp_nco* h, double dtheta) {  // :59-61
    if (!h) return SDSP_E_INVALID_ARGUMENT;
    h->delta_theta = constrain(dtheta);
    return SDSP_OK;
}
int sdsp_nco_adjust_frequency(sdsp_nco* h, double dt) {  // :64-66 (u32 add wraps in release builds)
    if (!h) return SDSP_E_INVALID_ARGUMENT;
    h->delta_theta += constrain(dt);
    return SDSP_OK;
}
// get_frequency (:69-76): (delta_theta as u64 / 2^32) is integer division, always 0 for a u32
double sdsp_nco_get_frequency(const sdsp_nco* h) {
    if (!h) return 0.0;
    const double dt = (double)((uint64_t)h->delta_theta / (1ULL << 32)) * 2.0 * M_PI;
    return dt > M_PI ? dt - 2.0 * M_PI : dt;
}
int sdsp_nco_set_phase(sdsp_nco* h, double phi) {  // :79-81
    if (!h) return SDSP_E_INVALID_ARGUMENT;
    h->theta = constrain(phi);
    return SDSP_OK;
}
int sdsp_nco_adjust_phase(sdsp_nco* h, double dphi) {  // :84-86
    if (!h) return SDSP_E_INVALID_ARGUMENT;
    h->theta += constrain(dphi);
    return SDSP_OK;
}
double sdsp_nco_get_phase(const sdsp_nco* h) {  // :89-91 (integer division as get_frequency)
    return h ? (double)((uint64_t)h->theta / (1ULL << 32)) * 2.0 * M_PI : 0.0;
}
int sdsp_nco_step(sdsp_nco* h) {  // :94-96
    if (!h) return SDSP_E_INVALID_ARGUMENT;
    h->theta += h->delta_theta;
    return SDSP_OK;
}
int sdsp_nco_sincos(const sdsp_nco* h, double* sin_cos) {  // :104-117
    if (!h || !sin_cos) return SDSP_E_INVALID_ARGUMENT;
    sin_cos[0] = h->table[h->index()];
    sin_cos[1] = h->table[(h->index() + 256) & 0x3ff];
    return SDSP_OK;
}
int sdsp_nco_set_internal_pll_bandwidth(sdsp_nco* h, double bandwidth) {  // :124-132
    if (!h) return SDSP_E_INVALID_ARGUMENT;
    if (bandwidth < 0.0) {
        set_error("NCO Error Bandwidth out Range [0, inf)");
        return SDSP_E_NCO_BANDWIDTH_OUT_OF_RANGE;
    }
    h->alpha = bandwidth;
    h->beta = std::sqrt(bandwidth);
    return SDSP_OK;
}
int sdsp_nco_pll_step(sdsp_nco* h, double delta_phi) {  // :135-138
    if (!h) return SDSP_E_INVALID_ARGUMENT;
    h->delta_theta += constrain(delta_phi * h->alpha);
    h->theta += constrain(delta_phi * h->beta);
    return SDSP_OK;
}
int sdsp_nco_get_state(const sdsp_nco* h, uint32_t* theta, uint32_t* delta_theta) {
    if (!h) return SDSP_E_INVALID_ARGUMENT;
    if (theta) *theta = h->theta;
    if (delta_theta) *delta_theta = h->delta_theta;
    return SDSP_OK;
}
int sdsp_nco_set_state(sdsp_nco* h, uint32_t theta, uint32_t delta_theta) {
    if (!h) return SDSP_E_INVALID_ARGUMENT;
    h->theta = theta;
    h->delta_theta = delta_theta;
    return SDSP_OK;
}

// mix_up_block / mix_down_block (:153-172) as the per-sample loop they spell out:
// out[i] = mix(x[i]) at theta, then step()
int sdsp_nco_mix_block_device(sdsp_nco* h, int down, int precision, const void* d_in, size_t n, void* d_out,
                              void* stream) {
    if (!h || (precision != 0 && precision != 1) || (n && (!d_in || !d_out))) return SDSP_E_INVALID_ARGUMENT;
    Guard g(h->device);
    R_TRY(launch_nco_mix(precision, down != 0, d_in, d_out, n, (const double*)h->d_table.p, h->theta, h->delta_theta,
                         h->cus, pick(stream, h->stream)),
          "nco mix");
    h->theta += (uint32_t)((uint64_t)n * h->delta_theta);  // n steps, wrapping
    return SDSP_OK;
}

int sdsp_nco_mix_block(sdsp_nco* h, int down, int precision, const void* in, size_t n, void* out) {
    if (!h || (precision != 0 && precision != 1) || (n && (!in || !out))) return SDSP_E_INVALID_ARGUMENT;
    if (n == 0) return SDSP_OK;
    Guard g(h->device);
    const size_t bytes = n * cbytes(precision);
    R_TRY(h->stage_in.ensure(bytes), "stage in");
    R_TRY(h->stage_out.ensure(bytes), "stage out");
    R_TRY(hipMemcpyAsync(h->stage_in.p, in, bytes, hipMemcpyHostToDevice, h->stream), "H2D");
    int st = sdsp_nco_mix_block_device(h, down, precision, h->stage_in.p, n, h->stage_out.p, h->stream);
    if (st) return st;
    R_TRY(hipMemcpyAsync(out, h->stage_out.p, bytes, hipMemcpyDeviceToHost, h->stream), "D2H");
    R_TRY(hipStreamSynchronize(h->stream), "sync");
    return SDSP_OK;
}

int sdsp_nco_synchronize(sdsp_nco* h) {
    if (!h) return SDSP_E_INVALID_ARGUMENT;
    Guard g(h->device);
    R_TRY(hipStreamSynchronize(h->stream), "sync");
    return SDSP_OK;
}

}  // extern "C"

// ===========================================================================
// AGC bank (src/auto_gain_control/mod.rs:97-677)
// ===========================================================================
struct sdsp_agc {
    int device = 0;
    size_t channels = 1;
    std::vector<sdsp_agc_state> host;  // valid when host_valid; the device copy is authoritative after a run
    bool host_valid = true;
    DevBuf d_state, d_levels, stage_in, stage_out;
    hipStream_t stream = nullptr, last = nullptr;
    bool pipe = true;  // SDSP_TUNE_AGC_KERNEL 0
};

namespace {
sdsp_agc_state agc_new_state() {  // AGC::new  :136-149
    sdsp_agc_state s{};
    s.gain = 1.0;
    s.scale = 1.0;
    s.bandwidth = 0.1;
    s.alpha = 0.1;
    s.energy_estimate = 1.0;
    s.lock = 0;
    s.squelch_mode = SDSP_SQUELCH_DISABLED;
    s.squelch_threshold = 0.0;
    s.squelch_timeout = 100;
    s.squelch_timer = 0;
    return s;
}
int agc_pull(sdsp_agc* h) {
    if (h->host_valid) return SDSP_OK;
    if (h->last) R_TRY(hipStreamSynchronize(h->last), "sync");
    R_TRY(hipMemcpy(h->host.data(), h->d_state.p, h->channels * sizeof(sdsp_agc_state), hipMemcpyDeviceToHost),
          "state D2H");
    h->host_valid = true;
    return SDSP_OK;
}
int agc_push(sdsp_agc* h) {
    if (h->last) R_TRY(hipStreamSynchronize(h->last), "sync");
    R_TRY(hipMemcpy(h->d_state.p, h->host.data(), h->channels * sizeof(sdsp_agc_state), hipMemcpyHostToDevice),
          "state H2D");
    return SDSP_OK;
}
// read-modify-write every channel's state
template <typename F> int agc_update(sdsp_agc* h, F f) {
    if (!h) return SDSP_E_INVALID_ARGUMENT;
    Guard g(h->device);
    int st = agc_pull(h);
    if (st) return st;
    for (auto& s : h->host) f(s);
    return agc_push(h);
}
size_t agc_bytes(int sample_type) { return sample_type == 1 ? 16 : 8; }
}  // namespace

extern "C" {

int sdsp_agc_create(sdsp_agc** out, size_t channels, int device) {
    if (!out) return SDSP_E_INVALID_ARGUMENT;
    *out = nullptr;
    if (channels == 0) {
        set_error("channels must be > 0");
        return SDSP_E_INVALID_ARGUMENT;
    }
    int st = check_gfx950(device, nullptr);
    if (st) return st;
    Guard g(device);
    auto* h = new sdsp_agc();
    h->device = device;
    h->channels = channels;
    h->host.assign(channels, agc_new_state());
    if (hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking) != hipSuccess) {
        delete h;
        set_error("hipStreamCreate failed");
        return SDSP_E_DEVICE;
    }
    if (h->d_state.ensure(channels * sizeof(sdsp_agc_state)) != hipSuccess || (st = agc_push(h)) != SDSP_OK) {
        sdsp_agc_destroy(h);
        set_error("AGC state upload failed");
        return st ? st : SDSP_E_DEVICE;
    }
    *out = h;
    return SDSP_OK;
}

void sdsp_agc_destroy(sdsp_agc* h) {
    if (!h) return;
    {
        Guard g(h->device);
        if (h->last) (void)hipStreamSynchronize(h->last);
        if (h->stream) {
            (void)hipStreamSynchronize(h->stream);
            (void)hipStreamDestroy(h->stream);
        }
        h->d_state.release();
        h->d_levels.release();
        h->stage_in.release();
        h->stage_out.release();
    }
    delete h;
}

size_t sdsp_agc_channels(const sdsp_agc* h) { return h ? h->channels : 0; }

int sdsp_agc_set_tuning(sdsp_agc* h, int key, int value) {
    if (!h || key != SDSP_TUNE_AGC_KERNEL || value < 0 || value > 1) return SDSP_E_INVALID_ARGUMENT;
    h->pipe = value == 0;
    return SDSP_OK;
}

int sdsp_agc_reset(sdsp_agc* h) {  // :178-188 (squelch stays enabled if it was on)
    return agc_update(h, [](sdsp_agc_state& s) {
        s.gain = 1.0;
        s.energy_estimate = 1.0;
        s.lock = 0;
        s.squelch_mode = s.squelch_mode == SDSP_SQUELCH_DISABLED ? SDSP_SQUELCH_DISABLED : SDSP_SQUELCH_ENABLED;
    });
}

int sdsp_agc_execute_block_device(sdsp_agc* h, int sample_type, const void* d_in, size_t n, void* d_out,
                                  void* stream) {
    if (!h || (sample_type != 0 && sample_type != 1) || (n && (!d_in || !d_out))) return SDSP_E_INVALID_ARGUMENT;
    if (n == 0) return SDSP_OK;
    Guard g(h->device);
    hipStream_t s = pick(stream, h->stream);
    if (h->last && h->last != s) R_TRY(hipStreamSynchronize(h->last), "sync");  // state hand-off between streams
    R_TRY(launch_agc(sample_type == 1, d_in, d_out, n, h->d_state.p, h->channels, s, h->pipe), "agc");
    h->last = s;
    h->host_valid = false;
    return SDSP_OK;
}

int sdsp_agc_execute_block(sdsp_agc* h, int sample_type, const void* in, size_t n, void* out) {
    if (!h || (sample_type != 0 && sample_type != 1) || (n && (!in || !out))) return SDSP_E_INVALID_ARGUMENT;
    if (n == 0) return SDSP_OK;
    Guard g(h->device);
    const size_t bytes = h->channels * n * agc_bytes(sample_type);
    R_TRY(h->stage_in.ensure(bytes), "stage in");
    R_TRY(h->stage_out.ensure(bytes), "stage out");
    R_TRY(hipMemcpyAsync(h->stage_in.p, in, bytes, hipMemcpyHostToDevice, h->stream), "H2D");
    int st = sdsp_agc_execute_block_device(h, sample_type, h->stage_in.p, n, h->stage_out.p, h->stream);
    if (st) return st;
    R_TRY(hipMemcpyAsync(out, h->stage_out.p, bytes, hipMemcpyDeviceToHost, h->stream), "D2H");
    R_TRY(hipStreamSynchronize(h->stream), "sync");
    return SDSP_OK;
}

int sdsp_agc_init(sdsp_agc* h, int sample_type, const void* in, size_t n, double* levels) {
    if (!h || (sample_type != 0 && sample_type != 1) || (n && !in)) return SDSP_E_INVALID_ARGUMENT;
    if (n == 0) {
        set_error("AGC Error Need more than 0 Samples to operate");
        return SDSP_E_AGC_SAMPLES_TOO_LOW;
    }
    Guard g(h->device);
    int st = agc_pull(h);
    if (st) return st;
    const size_t bytes = h->channels * n * agc_bytes(sample_type);
    R_TRY(h->stage_in.ensure(bytes), "stage in");
    R_TRY(h->d_levels.ensure(h->channels * 8), "levels");
    if (h->last && h->last != h->stream) R_TRY(hipStreamSynchronize(h->last), "sync");
    R_TRY(hipMemcpyAsync(h->stage_in.p, in, bytes, hipMemcpyHostToDevice, h->stream), "H2D");
    R_TRY(launch_agc_init(sample_type == 1, h->stage_in.p, n, h->d_state.p, (double*)h->d_levels.p, h->channels,
                          h->stream),
          "agc init");
    std::vector<double> lv(h->channels);
    R_TRY(hipMemcpyAsync(lv.data(), h->d_levels.p, h->channels * 8, hipMemcpyDeviceToHost, h->stream), "D2H");
    R_TRY(hipStreamSynchronize(h->stream), "sync");
    h->last = h->stream;
    h->host_valid = false;
    if (levels) std::memcpy(levels, lv.data(), h->channels * 8);
    for (double l : lv)
        if (!(l > 0.0)) {
            set_error("AGC Error Level is too low (0, inf)");
            return SDSP_E_AGC_SIGNAL_LEVEL_OUT_OF_RANGE;
        }
    return SDSP_OK;
}

int sdsp_agc_lock(sdsp_agc* h) { return agc_update(h, [](sdsp_agc_state& s) { s.lock = 1; }); }
int sdsp_agc_unlock(sdsp_agc* h) { return agc_update(h, [](sdsp_agc_state& s) { s.lock = 0; }); }

int sdsp_agc_set_bandwidth(sdsp_agc* h, double bw) {  // :374-386
    if (!(bw >= 0.0 && bw <= 1.0)) {
        set_error("AGC Error Bandwidth not in range [0, 1]");
        return h ? SDSP_E_AGC_BANDWIDTH_OUT_OF_RANGE : SDSP_E_INVALID_ARGUMENT;
    }
    return agc_update(h, [bw](sdsp_agc_state& s) {
        s.bandwidth = bw;
        s.alpha = bw;
    });
}
int sdsp_agc_set_signal_level(sdsp_agc* h, double level) {  // :416-428
    if (level <= 0.0) {
        set_error("AGC Error Level is too low (0, inf)");
        return h ? SDSP_E_AGC_SIGNAL_LEVEL_OUT_OF_RANGE : SDSP_E_INVALID_ARGUMENT;
    }
    return agc_update(h, [level](sdsp_agc_state& s) {
        s.gain = 1.0 / level;
        s.energy_estimate = 1.0;
    });
}
int sdsp_agc_set_rssi(sdsp_agc* h, double rssi) {  // :458-466
    return agc_update(h, [rssi](sdsp_agc_state& s) {
        s.gain = std::pow(10.0, -rssi / 20.0);
        if (s.gain < 1e-16) s.gain = 1e-16;
        s.energy_estimate = 1.0;
    });
}
int sdsp_agc_set_gain(sdsp_agc* h, double gain) {  // :497-504
    if (gain <= 0.0) {
        set_error("AGC Error Gain is below Threshold (0, inf)");
        return h ? SDSP_E_AGC_GAIN_BELOW_THRESHOLD : SDSP_E_INVALID_ARGUMENT;
    }
    return agc_update(h, [gain](sdsp_agc_state& s) { s.gain = gain; });
}
int sdsp_agc_set_scale(sdsp_agc* h, double scale) {  // :535-542
    if (scale <= 0.0) {
        set_error("AGC Error Scale is below Threshold (0, inf)");
        return h ? SDSP_E_AGC_SCALE_BELOW_THRESHOLD : SDSP_E_INVALID_ARGUMENT;
    }
    return agc_update(h, [scale](sdsp_agc_state& s) { s.scale = scale; });
}
// update_squelch_mode  :631-677 (one step of the state machine per channel, as execute makes it)
int sdsp_agc_update_squelch_mode(sdsp_agc* h) {
    return agc_update(h, [](sdsp_agc_state& s) {
        const bool hi = std::log10(s.gain) * -20.0 > s.squelch_threshold;  // get_rssi() > threshold
        switch (s.squelch_mode) {
            case SDSP_SQUELCH_ENABLED: s.squelch_mode = hi ? SDSP_SQUELCH_RISE : SDSP_SQUELCH_ENABLED; break;
            case SDSP_SQUELCH_RISE: s.squelch_mode = hi ? SDSP_SQUELCH_SIGNALHI : SDSP_SQUELCH_FALL; break;
            case SDSP_SQUELCH_SIGNALHI: s.squelch_mode = hi ? SDSP_SQUELCH_SIGNALHI : SDSP_SQUELCH_FALL; break;
            case SDSP_SQUELCH_FALL:
                s.squelch_timer = s.squelch_timeout;
                s.squelch_mode = hi ? SDSP_SQUELCH_SIGNALHI : SDSP_SQUELCH_SIGNALLO;
                break;
            case SDSP_SQUELCH_SIGNALLO:
                s.squelch_timer -= 1;  // usize: wraps in release builds
                s.squelch_mode = s.squelch_timer == 0 ? SDSP_SQUELCH_TIMEOUT
                                 : hi                 ? SDSP_SQUELCH_SIGNALHI
                                                      : SDSP_SQUELCH_SIGNALLO;
                break;
            case SDSP_SQUELCH_TIMEOUT: s.squelch_mode = SDSP_SQUELCH_ENABLED; break;
            default: s.squelch_mode = SDSP_SQUELCH_DISABLED; break;
        }
    });
}
int sdsp_agc_squelch_enable(sdsp_agc* h) {
    return agc_update(h, [](sdsp_agc_state& s) { s.squelch_mode = SDSP_SQUELCH_ENABLED; });
}
int sdsp_agc_squelch_disable(sdsp_agc* h) {
    return agc_update(h, [](sdsp_agc_state& s) { s.squelch_mode = SDSP_SQUELCH_DISABLED; });
}
int sdsp_agc_squelch_set_threshold(sdsp_agc* h, double threshold) {
    return agc_update(h, [threshold](sdsp_agc_state& s) { s.squelch_threshold = threshold; });
}
int sdsp_agc_squelch_set_timeout(sdsp_agc* h, uint64_t timeout) {
    return agc_update(h, [timeout](sdsp_agc_state& s) { s.squelch_timeout = timeout; });
}

int sdsp_agc_get_state(sdsp_agc* h, size_t channel, sdsp_agc_state* st) {
    if (!h || !st || channel >= h->channels) return SDSP_E_INVALID_ARGUMENT;
    Guard g(h->device);
    int r = agc_pull(h);
    if (r) return r;
    *st = h->host[channel];
    return SDSP_OK;
}
int sdsp_agc_set_state(sdsp_agc* h, size_t channel, const sdsp_agc_state* st) {
    if (!h || !st || channel >= h->channels) return SDSP_E_INVALID_ARGUMENT;
    Guard g(h->device);
    int r = agc_pull(h);
    if (r) return r;
    h->host[channel] = *st;
    return agc_push(h);
}
int sdsp_agc_synchronize(sdsp_agc* h) {
    if (!h) return SDSP_E_INVALID_ARGUMENT;
    Guard g(h->device);
    if (h->last) R_TRY(hipStreamSynchronize(h->last), "sync");
    return SDSP_OK;
}

}  // extern "C"
