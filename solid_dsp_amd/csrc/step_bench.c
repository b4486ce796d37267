/* Per-sample cost of the drop-in boundary as a compiled caller sees it (bench.py
 * `dropin`): FIRFilter<f64, Complex<f64>>::execute(sample) and
 * DecimatingFIRFilter::push through the C ABI, with the host step (default) and
 * with every call a device launch (SDSP_TUNE_HOST_STEP = 0), on cfg2's taps
 * (firdes_kaiser(256, 0.1, 80), scale 0.2).  Prints one JSON object. */
#define _POSIX_C_SOURCE 199309L
#include <stdio.h>
#include <time.h>

#include "sdsp.h"

static double now_us(void) {
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec * 1e6 + t.tv_nsec * 1e-3;
}

static double per_call(sdsp_fir* h, int calls, int push) {
    double x[2] = {0.5, 0.25}, y[2];
    size_t n = 0;
    double t0 = now_us(), acc = 0.0;
    for (int i = 0; i < calls; ++i) {
        x[0] = 1e-3 * (i & 1023);
        if (push) sdsp_decim_push(h, x);
        else sdsp_fir_execute(h, x, y, &n);
        acc += y[0];
    }
    double dt = (now_us() - t0) / calls;
    if (acc == 1.2345e300) printf("#");
    return dt;
}

int main(void) {
    enum { L = 256 };
    double taps[L], scale = 0.2;
    if (sdsp_firdes_kaiser(L, 0.1, 80.0, 0.0, taps)) return 2;
    sdsp_fir *f = NULL, *d = NULL;
    if (sdsp_fir_create(&f, SDSP_RC64, taps, L, &scale, 0)) {
        fprintf(stderr, "%s\n", sdsp_last_error());
        return 1;
    }
    if (sdsp_decim_create(&d, SDSP_RC64, taps, L, &scale, 32, 0)) return 1;
    per_call(f, 20000, 0);
    const double host_exec = per_call(f, 400000, 0);
    const double host_push = per_call(d, 400000, 1);
    sdsp_fir_set_tuning(f, SDSP_TUNE_HOST_STEP, 0);
    sdsp_fir_set_tuning(d, SDSP_TUNE_HOST_STEP, 0);
    per_call(f, 200, 0);
    const double dev_exec = per_call(f, 4000, 0);
    const double dev_push = per_call(d, 4000, 1);
    printf("{\"execute_us\": %.4f, \"push_us\": %.4f, \"execute_device_step_us\": %.3f, "
           "\"push_device_step_us\": %.3f, \"taps\": %d, \"type\": \"FIRFilter<f64, Complex<f64>>\"}\n",
           host_exec, host_push, dev_exec, dev_push, L);
    sdsp_fir_destroy(f);
    sdsp_fir_destroy(d);
    return 0;
}
