// Strided-run bandwidth probe (calibration, not product): how fast does HBM
// stream runs of G complex-f32 samples (8 G bytes) taken from rows 8 KB apart --
// the column pass of the four-step 2^20-point FFT (cfg8) reads and writes runs of
// 16 samples (128 B) from 1024 rows -- at a fixed 32 KB footprint per 256-lane
// workgroup and 4 workgroups per CU (36 KB LDS pinned), against contiguous 32 KB.
// Each workgroup copies a G x R block (R = 4096 / G rows) of a batch of 1024 x 1024
// matrices from x to the same place in y; blocks are dealt in XCD-contiguous order
// (workgroup b on XCD b % 8 takes the (b / 8)-th block of that XCD's eighth) or
// in launch order.  Lane mapping: the G/2 lanes of a row move one 16-byte vector
// each, 512 / G rows per wave instruction, 8 instructions per lane.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/_build/stride_probe tools/stride_probe.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                   \
    do {                                                                        \
        hipError_t e = (x);                                                     \
        if (e != hipSuccess) {                                                  \
            std::printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); \
            std::exit(1);                                                       \
        }                                                                       \
    } while (0)

typedef float f4v __attribute__((ext_vector_type(4)));

// G samples per run (G/2 float4), rows 1024 samples (512 float4) apart
template <int G, bool XCD, bool NT>
__global__ void __launch_bounds__(256) block_copy(const f4v* __restrict__ x, f4v* __restrict__ y, long long nblk, long long q) {
    extern __shared__ float pin[];
    constexpr int VPR = G / 2;           // float4 per run
    constexpr int R = 4096 / G;          // rows per block (32 KB)
    constexpr int BPM = (1024 / G) * (1024 / R);  // blocks per 1024 x 1024 matrix
    long long b;
    if constexpr (XCD) {
        const int xc = blockIdx.x & 7;
        b = (long long)xc * q + (blockIdx.x >> 3);
        const long long e = (long long)(xc + 1) * q;
        if (b >= (e < nblk ? e : nblk)) return;
    } else {
        b = blockIdx.x;
        if (b >= nblk) return;
    }
    const long long mat = b / BPM;
    const int inm = (int)(b % BPM);
    // column group major inside a matrix: consecutive blocks are the next rows of the same columns
    const int cg = inm / (1024 / R), rg = inm % (1024 / R);
    const long long base = mat * (1024LL * 512) + (long long)rg * R * 512 + (long long)cg * VPR;
    const int t = threadIdx.x;
    // float4 e = 256 i + t of the block: row e / VPR, column e % VPR
    auto off = [&](int i) { const int e = 256 * i + t; return base + (long long)(e / VPR) * 512 + e % VPR; };
    f4v v[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const long long o = off(i);
        v[i] = NT ? __builtin_nontemporal_load(x + o) : x[o];
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const long long o = off(i);
        if (NT) __builtin_nontemporal_store(v[i], y + o);
        else y[o] = v[i];
    }
    if (nblk < 0) pin[t] = v[0].x;
}

int main() {
    const long long nsamp = 256LL << 20;  // 256 matrices of 1024 x 1024 complex f32 = 2 GiB
    f4v *x, *y;
    CK(hipMalloc(&x, nsamp * 8));
    CK(hipMalloc(&y, nsamp * 8));
    CK(hipMemset(x, 0, nsamp * 8));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto time_it = [&](auto launch) {
        for (int r = 0; r < 3; ++r) launch();
        std::vector<float> ts;
        for (int r = 0; r < 15; ++r) {
            CK(hipEventRecord(e0));
            launch();
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            ts.push_back(ms);
        }
        std::sort(ts.begin(), ts.end());
        return ts[ts.size() / 2];
    };
    const long long nblk = nsamp / 4096, q = (nblk + 7) / 8;
    for (int r = 0; r < 200; ++r)  // clocks settle
        hipLaunchKernelGGL((block_copy<1024, true, false>), dim3(8 * q), dim3(256), 36864, 0, x, y, nblk, q);
    CK(hipDeviceSynchronize());
    auto run = [&](auto kern, const char* name, int G, bool xcd, bool nt) {
        const unsigned grid = xcd ? (unsigned)(8 * q) : (unsigned)nblk;
        const float ms = time_it([&] { hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 36864, 0, x, y, nblk, q); });
        std::printf("%-8s run %5d B  %s %s  %.3f ms  %.0f GB/s\n", name, 8 * G, xcd ? "xcd   " : "launch", nt ? "nt   " : "plain",
                    ms, 2.0 * nsamp * 8 / (ms * 1e6));
        std::fflush(stdout);
    };
    for (int rep = 0; rep < 2; ++rep) {
        run(block_copy<16, true, false>, "block", 16, true, false);
        run(block_copy<32, true, false>, "block", 32, true, false);
        run(block_copy<64, true, false>, "block", 64, true, false);
        run(block_copy<128, true, false>, "block", 128, true, false);
        run(block_copy<256, true, false>, "block", 256, true, false);
        run(block_copy<1024, true, false>, "block", 1024, true, false);
        run(block_copy<16, false, false>, "block", 16, false, false);
        run(block_copy<32, false, false>, "block", 32, false, false);
        run(block_copy<64, false, false>, "block", 64, false, false);
        run(block_copy<1024, false, false>, "block", 1024, false, false);
        run(block_copy<16, true, true>, "block", 16, true, true);
        run(block_copy<32, true, true>, "block", 32, true, true);
        run(block_copy<1024, true, true>, "block", 1024, true, true);
    }
    return 0;
}
