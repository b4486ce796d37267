// Standalone HBM bandwidth probe for the GPU box (calibration, not product).
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/_build/bw_probe tools/bw_probe.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

#define CK(x)                                                                   \
    do {                                                                        \
        hipError_t e = (x);                                                     \
        if (e != hipSuccess) {                                                  \
            std::printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); \
            return 1;                                                           \
        }                                                                       \
    } while (0)

typedef float f4v __attribute__((ext_vector_type(4)));
template <int U, bool NT>
__global__ void __launch_bounds__(256) copy_k(const float4* __restrict__ a_, float4* __restrict__ b_, long long n16) {
    const f4v* a = reinterpret_cast<const f4v*>(a_);
    f4v* b = reinterpret_cast<f4v*>(b_);
    const long long per = 256LL * U;
    for (long long base = (long long)blockIdx.x * per; base < n16; base += (long long)gridDim.x * per) {
        f4v r[U];
#pragma unroll
        for (int k = 0; k < U; ++k) {
            const long long i = base + threadIdx.x + 256 * k;
            if constexpr (NT) r[k] = __builtin_nontemporal_load(a + i);
            else r[k] = a[i];
        }
#pragma unroll
        for (int k = 0; k < U; ++k) {
            const long long i = base + threadIdx.x + 256 * k;
            if constexpr (NT) __builtin_nontemporal_store(r[k], b + i);
            else b[i] = r[k];
        }
    }
}

template <int U>
__global__ void __launch_bounds__(256) read_k(const float4* __restrict__ a, float* __restrict__ out, long long n16) {
    const long long per = 256LL * U;
    float s = 0.f;
    for (long long base = (long long)blockIdx.x * per; base < n16; base += (long long)gridDim.x * per) {
#pragma unroll
        for (int k = 0; k < U; ++k) {
            const float4 v = a[base + threadIdx.x + 256 * k];
            s += v.x + v.y + v.z + v.w;
        }
    }
    if (s == 12345.f) out[blockIdx.x] = s;
}

template <int U>
__global__ void __launch_bounds__(256) write_k(float4* __restrict__ b, long long n16) {
    const long long per = 256LL * U;
    for (long long base = (long long)blockIdx.x * per; base < n16; base += (long long)gridDim.x * per) {
#pragma unroll
        for (int k = 0; k < U; ++k) b[base + threadIdx.x + 256 * k] = make_float4(1.f, 2.f, 3.f, 4.f);
    }
}

// one-shot read: every thread U float4s, grid covers the buffer
template <int U, bool NT>
__global__ void __launch_bounds__(256) read_once_k(const float4* __restrict__ a_, float* __restrict__ out, long long n16) {
    const f4v* a = reinterpret_cast<const f4v*>(a_);
    const long long base = (long long)blockIdx.x * 256 * U + threadIdx.x;
    f4v s = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int k = 0; k < U; ++k) {
        const long long i = base + 256 * k;
        if (i < n16) {
            if constexpr (NT) s += __builtin_nontemporal_load(a + i);
            else s += a[i];
        }
    }
    if (s.x + s.y + s.z + s.w == 12345.f) out[blockIdx.x] = s.x;
}

// decimator-like: 16-lane groups each stream 256-byte rows through their own
// segment of SEG bytes, 8 rows per step
template <bool NT>
__global__ void __launch_bounds__(256) read_seg_k(const float4* __restrict__ a_, float* __restrict__ out, long long n16,
                                                  long long seg16) {
    const f4v* a = reinterpret_cast<const f4v*>(a_);
    const long long grp = ((long long)blockIdx.x * 256 + threadIdx.x) / 16;
    const int q = threadIdx.x % 16;
    const long long b0 = grp * seg16;
    f4v s = {0.f, 0.f, 0.f, 0.f};
    if (b0 < n16) {
        for (long long r = 0; r < seg16; r += 16 * 8) {
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const long long i = b0 + r + u * 16 + q;
                if constexpr (NT) s += __builtin_nontemporal_load(a + i);
                else s += a[i];
            }
        }
    }
    if (s.x + s.y + s.z + s.w == 12345.f) out[blockIdx.x] = s.x;
}

template <typename F>
float time_ms(F f, int reps = 10) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    f();
    f();
    std::vector<float> ts;
    for (int r = 0; r < reps; ++r) {
        hipEventRecord(e0);
        f();
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        ts.push_back(ms);
    }
    std::sort(ts.begin(), ts.end());
    return ts[ts.size() / 2];
}

int main() {
    const size_t bytes = 8ull << 30;
    const long long n16 = bytes / 16;
    float4 *a, *b;
    float* out;
    CK(hipMalloc(&a, bytes));
    CK(hipMalloc(&b, bytes));
    CK(hipMalloc(&out, 1 << 20));
    CK(hipMemset(a, 0, bytes));
    hipDeviceProp_t p;
    CK(hipGetDeviceProperties(&p, 0));
    const int cus = p.multiProcessorCount;
    std::printf("device %s CUs %d\n", p.gcnArchName, cus);
    auto rep = [&](const char* name, float ms, double moved) {
        std::printf("%-36s %8.3f ms  %8.1f GB/s\n", name, ms, moved / ms / 1e6);
    };
    for (int g : {2, 4, 8, 16}) {
        char nm[64];
        std::snprintf(nm, 64, "copy U4 grid=%dxCU", g);
        rep(nm, time_ms([&] { copy_k<4, false><<<cus * g, 256>>>(a, b, n16); }), 2.0 * bytes);
        std::snprintf(nm, 64, "copy U4 nt grid=%dxCU", g);
        rep(nm, time_ms([&] { copy_k<4, true><<<cus * g, 256>>>(a, b, n16); }), 2.0 * bytes);
        std::snprintf(nm, 64, "copy U8 grid=%dxCU", g);
        rep(nm, time_ms([&] { copy_k<8, false><<<cus * g, 256>>>(a, b, n16); }), 2.0 * bytes);
        std::snprintf(nm, 64, "read U8 grid=%dxCU", g);
        rep(nm, time_ms([&] { read_k<8><<<cus * g, 256>>>(a, out, n16); }), 1.0 * bytes);
        std::snprintf(nm, 64, "write U8 grid=%dxCU", g);
        rep(nm, time_ms([&] { write_k<8><<<cus * g, 256>>>(b, n16); }), 1.0 * bytes);
    }
    for (int u : {1, 4}) {
        char nm[64];
        const long long per = 256LL * u;
        const unsigned gb = (unsigned)((n16 + per - 1) / per);
        std::snprintf(nm, 64, "read one-shot U%d", u);
        rep(nm, time_ms([&] { if (u == 1) read_once_k<1, false><<<gb, 256>>>(a, out, n16); else read_once_k<4, false><<<gb, 256>>>(a, out, n16); }), 1.0 * bytes);
        std::snprintf(nm, 64, "read one-shot U%d nt", u);
        rep(nm, time_ms([&] { if (u == 1) read_once_k<1, true><<<gb, 256>>>(a, out, n16); else read_once_k<4, true><<<gb, 256>>>(a, out, n16); }), 1.0 * bytes);
    }
    for (long long segb : {4096LL, 16384LL, 65536LL, 262144LL}) {
        char nm[64];
        const long long seg16 = segb / 16;
        const long long groups = n16 / seg16;
        const unsigned gb = (unsigned)((groups * 16 + 255) / 256);
        std::snprintf(nm, 64, "read segmented %lldB", segb);
        rep(nm, time_ms([&] { read_seg_k<false><<<gb, 256>>>(a, out, n16, seg16); }), 1.0 * bytes);
        std::snprintf(nm, 64, "read segmented %lldB nt", segb);
        rep(nm, time_ms([&] { read_seg_k<true><<<gb, 256>>>(a, out, n16, seg16); }), 1.0 * bytes);
    }
    rep("copy U1 one-shot grid", time_ms([&] { copy_k<1, false><<<(unsigned)(n16 / 256), 256>>>(a, b, n16); }),
        2.0 * bytes);
    rep("hipMemcpyDtoD", time_ms([&] { hipMemcpyAsync(b, a, bytes, hipMemcpyDeviceToDevice, 0); }), 2.0 * bytes);
    CK(hipDeviceSynchronize());
    return 0;
}
