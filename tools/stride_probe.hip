// Strided-run bandwidth probe (calibration, not product): how fast does HBM
// stream runs of G complex-f32 samples (8 G bytes) taken from rows 8 KB apart --
// the column pass of the four-step 2^20-point FFT (cfg8) reads and writes runs of
// 16 samples (128 B) from 1024 rows.  A workgroup of T threads copies a G x R block
// (R = 16 T / G rows, 128 T bytes) of a batch of 1024 x 1024 matrices from x to the same
// place in y, with LW-byte lane accesses (16: G/2 lanes per row; 8: G lanes per row, the pass
// kernel's lane shape); T = 256 pins 4 workgroups per CU (36 KB LDS), T = 1024 one (96 KB),
// the pass kernel's 128 KB group per CU.  Blocks are dealt in XCD-contiguous order (workgroup
// b on XCD b % 8 takes the (b / 8)-th block of that XCD's eighth) or in launch order.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/_build/stride_probe tools/stride_probe.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <type_traits>
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

// G samples per run, rows 1024 samples apart; T threads per workgroup (16 T samples =
// 128 T bytes per block: 32 KB at 256, the pass kernel's 128 KB group at 1024), LW bytes per
// lane access (16: G/2 lanes per row, the original probe; 8: G lanes per row, the pass kernel's
// lane shape)
template <int G, int T, int LW, bool XCD, bool NT>
__global__ void __launch_bounds__(T) block_copy(const f4v* __restrict__ x, f4v* __restrict__ y, long long nblk, long long q) {
    extern __shared__ float pin[];
    typedef float f2v __attribute__((ext_vector_type(2)));
    typedef typename std::conditional<LW == 16, f4v, f2v>::type V;
    constexpr int E = LW / 8;            // complex samples per lane access
    constexpr int LPR = G / E;           // lanes per row
    constexpr int R = 16 * T / G;        // rows per block
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
    const long long base = mat * (1024LL * 1024) + (long long)rg * R * 1024 + (long long)cg * G;  // complex units
    const int t = threadIdx.x;
    // access e = T i + t of the block: row e / LPR, samples E (e % LPR) .. + E - 1
    auto off = [&](int i) { const int e = T * i + t; return base + (long long)(e / LPR) * 1024 + (e % LPR) * E; };
    const V* xv = (const V*)x;
    V* yv = (V*)y;
    V v[16 / E];
#pragma unroll
    for (int i = 0; i < 16 / E; ++i) {
        const long long o = off(i) / E;
        v[i] = NT ? __builtin_nontemporal_load(xv + o) : xv[o];
    }
#pragma unroll
    for (int i = 0; i < 16 / E; ++i) {
        const long long o = off(i) / E;
        if (NT) __builtin_nontemporal_store(v[i], yv + o);
        else yv[o] = v[i];
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
    for (int r = 0; r < 200; ++r)  // clocks settle
        hipLaunchKernelGGL((block_copy<1024, 256, 16, true, false>), dim3(8 * ((nsamp / 4096 + 7) / 8)), dim3(256), 36864, 0,
                           x, y, nsamp / 4096, (nsamp / 4096 + 7) / 8);
    CK(hipDeviceSynchronize());
    // T = 256: 36 KB of LDS pins 4 workgroups per CU; T = 1024: 96 KB pins one (the pass kernel's)
    auto run = [&](auto kern, int G, int T, int LW, bool xcd, bool nt) {
        const long long nblk = nsamp / (16 * T), q = (nblk + 7) / 8;
        const unsigned grid = xcd ? (unsigned)(8 * q) : (unsigned)nblk;
        const size_t lds = T == 256 ? 36864 : 98304;
        const float ms = time_it([&] { hipLaunchKernelGGL(kern, dim3(grid), dim3(T), lds, 0, x, y, nblk, q); });
        std::printf("block    run %5d B  T %4d  lane %2d B  %s %s  %.3f ms  %.0f GB/s\n", 8 * G, T, LW,
                    xcd ? "xcd   " : "launch", nt ? "nt   " : "plain", ms, 2.0 * nsamp * 8 / (ms * 1e6));
        std::fflush(stdout);
    };
    for (int rep = 0; rep < 2; ++rep) {
        run(block_copy<16, 256, 16, false, false>, 16, 256, 16, false, false);
        run(block_copy<16, 256, 8, false, false>, 16, 256, 8, false, false);
        run(block_copy<16, 1024, 16, false, false>, 16, 1024, 16, false, false);
        run(block_copy<16, 1024, 8, false, false>, 16, 1024, 8, false, false);
        run(block_copy<16, 256, 16, true, false>, 16, 256, 16, true, false);
        run(block_copy<16, 1024, 8, true, false>, 16, 1024, 8, true, false);
        run(block_copy<32, 256, 16, false, false>, 32, 256, 16, false, false);
        run(block_copy<32, 1024, 8, false, false>, 32, 1024, 8, false, false);
        run(block_copy<1024, 256, 16, false, false>, 1024, 256, 16, false, false);
        run(block_copy<1024, 1024, 8, false, false>, 1024, 1024, 8, false, false);
    }
    return 0;
}
