// Copy ceilings at the configs' sizes (calibration, not product): one-shot copies of
// in -> out with 8- or 16-byte lanes and each load / store cache policy, for
// 1 GiB (cfg5: 8 x 2^24 c32), 4 GiB (cfg3: 2^30 f32) and 8 GiB (cfg2: 2^30 c32) each way.
// Policies: 0 default, 2 nontemporal, 16 write-through (sc1).
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/_build/copy_shape_probe tools/copy_shape_probe.hip
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

typedef unsigned u4 __attribute__((ext_vector_type(4)));
typedef unsigned u2 __attribute__((ext_vector_type(2)));

// one-shot: workgroup b copies U consecutive 256-lane rows of W-byte vectors starting at
// b * 256 * U; the buffer descriptors bound every access (num_records = bytes), so a
// partial last workgroup reads zeros and drops its stores
template <int W, int U, int LA, int SA>
__global__ void __launch_bounds__(256) copy_k(const char* __restrict__ a, char* __restrict__ b, unsigned long long bytes) {
    const unsigned long long base = (unsigned long long)blockIdx.x * 256ull * U * W;
    const unsigned long long rem = bytes > base ? bytes - base : 0;
    const unsigned nrec = (unsigned)(rem < 0x80000000ull ? rem : 0x80000000ull);
    const auto ra = __builtin_amdgcn_make_buffer_rsrc((void*)(a + base), (short)0, nrec, 0x00020000);
    const auto rb = __builtin_amdgcn_make_buffer_rsrc((void*)(b + base), (short)0, nrec, 0x00020000);
    if constexpr (W == 16) {
        u4 r[U];
#pragma unroll
        for (int k = 0; k < U; ++k)
            r[k] = __builtin_bit_cast(u4, __builtin_amdgcn_raw_buffer_load_b128(ra, (threadIdx.x + 256 * k) * 16, 0, LA));
#pragma unroll
        for (int k = 0; k < U; ++k) __builtin_amdgcn_raw_buffer_store_b128(r[k], rb, (threadIdx.x + 256 * k) * 16, 0, SA);
    } else {
        u2 r[U];
#pragma unroll
        for (int k = 0; k < U; ++k)
            r[k] = __builtin_bit_cast(u2, __builtin_amdgcn_raw_buffer_load_b64(ra, (threadIdx.x + 256 * k) * 8, 0, LA));
#pragma unroll
        for (int k = 0; k < U; ++k) __builtin_amdgcn_raw_buffer_store_b64(r[k], rb, (threadIdx.x + 256 * k) * 8, 0, SA);
    }
}

// 8-byte lanes in reversed order within each wave's 512 bytes (the channeliser's load shape:
// lane t reads x[M - 1 - t] of a frame)
template <int U, int LA, int SA, bool REVL, bool REVS>
__global__ void __launch_bounds__(256) copy_rev_k(const char* __restrict__ a, char* __restrict__ b, unsigned long long bytes) {
    const unsigned long long base = (unsigned long long)blockIdx.x * 256ull * U * 8;
    const unsigned long long rem = bytes > base ? bytes - base : 0;
    const unsigned nrec = (unsigned)(rem < 0x80000000ull ? rem : 0x80000000ull);
    const auto ra = __builtin_amdgcn_make_buffer_rsrc((void*)(a + base), (short)0, nrec, 0x00020000);
    const auto rb = __builtin_amdgcn_make_buffer_rsrc((void*)(b + base), (short)0, nrec, 0x00020000);
    const unsigned lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const unsigned lo = (wv * 64 + (REVL ? 63 - lane : lane)) * 8, so = (wv * 64 + (REVS ? 63 - lane : lane)) * 8;
    u2 r[U];
#pragma unroll
    for (int k = 0; k < U; ++k) r[k] = __builtin_bit_cast(u2, __builtin_amdgcn_raw_buffer_load_b64(ra, lo + 2048 * k, 0, LA));
#pragma unroll
    for (int k = 0; k < U; ++k) __builtin_amdgcn_raw_buffer_store_b64(r[k], rb, so + 2048 * k, 0, SA);
}

template <typename F>
float time_ms(F f, int reps = 15) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (int i = 0; i < 5; ++i) f();
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

template <int W, int U, int LA, int SA>
void run(const char* a, char* b, unsigned long long bytes, const char* tag) {
    const unsigned long long per = 256ull * U * W;
    const unsigned g = (unsigned)((bytes + per - 1) / per);
    const float ms = time_ms([&] { copy_k<W, U, LA, SA><<<g, 256>>>(a, b, bytes); });
    std::printf("%-6s W=%2d U=%d load=%2d store=%2d  %8.4f ms  %7.1f GB/s\n", tag, W, U, LA, SA, ms,
                2.0 * bytes / ms / 1e6);
}

template <int U, int LA, int SA, bool REVL, bool REVS>
void run_rev(const char* a, char* b, unsigned long long bytes, const char* tag) {
    const unsigned long long per = 256ull * U * 8;
    const unsigned g = (unsigned)((bytes + per - 1) / per);
    const float ms = time_ms([&] { copy_rev_k<U, LA, SA, REVL, REVS><<<g, 256>>>(a, b, bytes); });
    std::printf("%-6s W= 8 U=%d load=%2d store=%2d rev_load=%d rev_store=%d  %8.4f ms  %7.1f GB/s\n", tag, U, LA, SA,
                (int)REVL, (int)REVS, ms, 2.0 * bytes / ms / 1e6);
}

int main() {
    const unsigned long long maxb = 8ull << 30;
    char *a, *b;
    CK(hipMalloc(&a, maxb));
    CK(hipMalloc(&b, maxb));
    CK(hipMemset(a, 1, maxb));
    CK(hipMemset(b, 0, maxb));
    struct Sz { unsigned long long bytes; const char* tag; } sizes[] = {{1ull << 30, "cfg5"}, {4ull << 30, "cfg3"}, {8ull << 30, "cfg2"}};
    for (const auto& s : sizes) {
        run<16, 1, 0, 0>(a, b, s.bytes, s.tag);
        run<16, 1, 2, 2>(a, b, s.bytes, s.tag);
        run<16, 1, 0, 2>(a, b, s.bytes, s.tag);
        run<16, 1, 0, 16>(a, b, s.bytes, s.tag);
        run<16, 1, 2, 16>(a, b, s.bytes, s.tag);
        run<16, 4, 0, 2>(a, b, s.bytes, s.tag);
        run<16, 4, 0, 16>(a, b, s.bytes, s.tag);
        run<8, 2, 0, 0>(a, b, s.bytes, s.tag);
        run<8, 2, 0, 2>(a, b, s.bytes, s.tag);
        run<8, 2, 0, 16>(a, b, s.bytes, s.tag);
        run<8, 8, 0, 2>(a, b, s.bytes, s.tag);
        run_rev<2, 0, 2, false, false>(a, b, s.bytes, s.tag);
        run_rev<2, 0, 2, true, false>(a, b, s.bytes, s.tag);
        run_rev<2, 0, 2, true, true>(a, b, s.bytes, s.tag);
        run_rev<8, 0, 2, false, false>(a, b, s.bytes, s.tag);
        run_rev<8, 0, 2, true, false>(a, b, s.bytes, s.tag);
        CK(hipDeviceSynchronize());
        std::fflush(stdout);
    }
    return 0;
}
