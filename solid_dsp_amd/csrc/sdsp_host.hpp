// Internal host-side helpers shared by runtime.cpp and design.cpp.
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstring>
#include <string>
#include <vector>

namespace sdsp {

struct cd { double re, im; };

cd cmul(cd a, cd b);
cd cmul(double a, cd b);
cd cadd(cd a, cd b);
cd cdiv(cd a, cd b);
cd from_polar(double r, double t);
cd poly_response(const std::vector<cd>& c, bool real, double f);
int fir_group_delay(const std::vector<cd>& h, bool real, double f, double* out);
int iir_group_delay(const std::vector<double>& b, const std::vector<double>& a, double f, double* out);

void set_error(const std::string& msg);
// the algorithm new FIR-type and IIR handles start on (sdsp_set_default_algo; SDSP_DEFAULT_ALGO)
int default_algo();
int device_status(hipError_t e, const char* what);

// dtype traits (sdsp_dtype)
inline size_t sample_bytes(int dt) {
    static const size_t b[6] = {4, 8, 8, 8, 16, 16};
    return (dt >= 0 && dt < 6) ? b[dt] : 0;
}
inline size_t coef_bytes(int dt) {
    static const size_t b[6] = {4, 4, 8, 8, 8, 16};
    return (dt >= 0 && dt < 6) ? b[dt] : 0;
}
inline bool coef_is_complex(int dt) { return dt == 2 || dt == 5; }
inline bool coef_is_f32(int dt) { return dt <= 2; }

// widen one stored coefficient to complex<f64>
inline cd coef_at(const unsigned char* p, int dt, size_t i) {
    switch (dt) {
        case 0: case 1: { float v; std::memcpy(&v, p + 4 * i, 4); return {(double)v, 0.0}; }
        case 2: { float v[2]; std::memcpy(v, p + 8 * i, 8); return {(double)v[0], (double)v[1]}; }
        case 3: case 4: { double v; std::memcpy(&v, p + 8 * i, 8); return {v, 0.0}; }
        case 5: { double v[2]; std::memcpy(v, p + 16 * i, 16); return {v[0], v[1]}; }
    }
    return {0.0, 0.0};
}

// owned device allocation
// pinned host memory mapped into the device address space (coherent): a kernel
// writes it directly, the host reads it after the stream synchronises
struct HostMapped {
    void* host = nullptr;
    void* dev = nullptr;
    HostMapped() = default;
    HostMapped(const HostMapped&) = delete;
    HostMapped& operator=(const HostMapped&) = delete;
    ~HostMapped() {
        if (host) (void)hipHostFree(host);
    }
    hipError_t ensure(size_t bytes) {
        if (host) return hipSuccess;
        hipError_t e = hipHostMalloc(&host, bytes, hipHostMallocMapped | hipHostMallocCoherent);
        if (e != hipSuccess) {
            host = nullptr;
            return e;
        }
        return hipHostGetDevicePointer(&dev, host, 0);
    }
};

// Wait until a kernel has released *flag == seq into host-mapped memory: a short
// spin (the step kernels finish within microseconds of the launch), then the
// stream's own synchronisation, which also surfaces launch errors.
inline hipError_t wait_host_flag(const unsigned* flag, unsigned seq, hipStream_t s) {
    for (int i = 0; i < (1 << 22); ++i) {
        if (__atomic_load_n(flag, __ATOMIC_ACQUIRE) == seq) return hipSuccess;
        __builtin_ia32_pause();
    }
    hipError_t e = hipStreamSynchronize(s);
    if (e != hipSuccess) return e;
    return __atomic_load_n(flag, __ATOMIC_ACQUIRE) == seq ? hipSuccess : hipErrorUnknown;
}

struct DevBuf {
    void* p = nullptr;
    size_t bytes = 0;
    DevBuf() = default;
    DevBuf(const DevBuf&) = delete;
    DevBuf& operator=(const DevBuf&) = delete;
    DevBuf(DevBuf&& o) noexcept : p(o.p), bytes(o.bytes) { o.p = nullptr; o.bytes = 0; }
    DevBuf& operator=(DevBuf&& o) noexcept {
        if (this != &o) { release(); p = o.p; bytes = o.bytes; o.p = nullptr; o.bytes = 0; }
        return *this;
    }
    ~DevBuf() { release(); }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        bytes = 0;
    }
    hipError_t ensure(size_t b) {
        if (b <= bytes && p) return hipSuccess;
        release();
        if (b == 0) b = 16;
        hipError_t e = hipMalloc(&p, b);
        if (e == hipSuccess) bytes = b;
        else p = nullptr;
        return e;
    }
};

// Completion marker of the last work a handle queued, on whichever stream it went
// (a caller's stream or the handle's own).  *_execute_block_device may run on any
// stream: each launch is first ordered after the marker (order_before) and then
// records a new one (record), so a call on a caller stream s1, a call on the handle
// stream and another call on s1 run in that order.  Host-side state operations
// (reset, set_state / get_state, clone, table rebuilds after set_scale) first wait
// for the marker, so a kernel still reading the delay line or the tables is never
// raced by a host copy on the handle's own stream.
//
// The markers rotate through kRing events: a stream never re-records the event it
// has just waited on (a stream waiting on an event that it then re-records every
// call crashed the host side in round 3), and an event is only
// recorded again kRing records later.
struct StreamFence {
    static constexpr int kRing = 4;
    hipEvent_t ev[kRing] = {};
    int cur = 0;                   // ev[cur] is the pending marker
    hipStream_t stream = nullptr;  // where the pending marker was recorded
    bool pending = false;
    StreamFence() = default;
    StreamFence(const StreamFence&) = delete;
    StreamFence& operator=(const StreamFence&) = delete;
    ~StreamFence() {
        for (hipEvent_t e : ev)
            if (e) (void)hipEventDestroy(e);
    }
    // A marker on the legacy default stream is recorded through its null handle: an event
    // recorded on the special handle hipStreamLegacy makes every later hipStreamWaitEvent on
    // it crash inside the runtime (SIGSEGV, any waiting stream), while one recorded on the null
    // stream is waited for normally (tools/fence_probe.hip, profiles/r05/fence_probe.log: the
    // round-4 AutoCorrelator crash, a block on torch's default stream followed by get_energy)
    hipError_t record(hipStream_t s) {
        const int nxt = (cur + 1) % kRing;
        if (!ev[nxt]) {
            hipError_t e = hipEventCreateWithFlags(&ev[nxt], hipEventDisableTiming);
            if (e != hipSuccess) return e;
        }
        hipError_t e = hipEventRecord(ev[nxt], legacy(s) ? nullptr : s);
        if (e != hipSuccess) return e;
        cur = nxt;
        pending = true;
        stream = s;
        return hipSuccess;
    }
    // order work about to be queued on `s` after the pending marker (nothing to do on the
    // marker's own stream: stream order; the null handle and hipStreamLegacy are the same
    // stream).  Device-side waits from any stream, the legacy one included (record() keeps the
    // marker off the hipStreamLegacy handle)
    hipError_t order_before(hipStream_t s) {
        if (!pending || s == stream || (legacy(s) && legacy(stream))) return hipSuccess;
        return hipStreamWaitEvent(s, ev[cur], 0);
    }
    static bool legacy(hipStream_t s) { return s == nullptr || s == hipStreamLegacy; }
    // the marker stays pending until a synchronize has succeeded (a failed wait must
    // not let later host operations skip it)
    hipError_t wait() {
        if (!pending) return hipSuccess;
        const hipError_t e = hipEventSynchronize(ev[cur]);
        if (e == hipSuccess) pending = false;
        return e;
    }
};

// [a, a + na) and [b, b + nb) overlap (byte ranges)
inline bool ranges_overlap(const void* a, size_t na, const void* b, size_t nb) {
    if (!na || !nb) return false;
    const auto pa = reinterpret_cast<uintptr_t>(a), pb = reinterpret_cast<uintptr_t>(b);
    return pa < pb + nb && pb < pa + na;
}

}  // namespace sdsp
