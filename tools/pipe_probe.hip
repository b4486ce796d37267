// Streaming-structure probe for the overlap-save FIR (calibration, not product).
// Every kernel moves the cfg2 stream shape: segments of 4096 complex-f32
// samples (32 KB) read with a 256-sample halo (segment stride 3840), the 3840
// non-halo samples written back, with a synthetic per-segment compute load of
// `iters` x 16 packed FMAs per lane between the read and the write.
//   A  one-shot: one segment per 256-lane workgroup, XCD-ordered (workgroup b
//      -> XCD b % 8 streams its contiguous eighth), 8 x 16-byte loads per lane
//      into VGPRs, 36 KB LDS pinned so 4 workgroups share a CU (the current
//      product kernel's shape).
//   B  persistent, LDS-DMA double buffer: `wpc` workgroups per CU, each walks
//      an XCD-contiguous segment order (iteration k of the XCD's j-th
//      workgroup takes segment x q + k (G/8) + j), global_load_lds_dwordx4
//      straight into one of two 32 KB LDS buffers, two segments in flight
//      ahead of the one being computed, raw s_barrier + counted vmcnt.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/_build/pipe_probe tools/pipe_probe.hip
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

typedef float f2 __attribute__((ext_vector_type(2)));
typedef float f4v __attribute__((ext_vector_type(4)));

constexpr int kSeg = 4096, kV = 3840;

__device__ __forceinline__ void fake_compute(f4v (&q)[8], int iters, float c) {
    f2 acc[16];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        acc[2 * i] = f2{q[i].x, q[i].y};
        acc[2 * i + 1] = f2{q[i].z, q[i].w};
    }
    const f2 cc = {c, c}, dd = {c * 0.5f, c * 0.25f};
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int j = 0; j < 16; ++j) acc[j] = __builtin_elementwise_fma(acc[j], cc, dd);
    }
    const f2 z = {c - c, c - c};  // runtime zero: the result depends on the compute, the data pass through
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const f2 a = __builtin_elementwise_fma(acc[2 * i], z, f2{q[i].x, q[i].y});
        const f2 b = __builtin_elementwise_fma(acc[2 * i + 1], z, f2{q[i].z, q[i].w});
        q[i] = f4v{a.x, a.y, b.x, b.y};
    }
}

__global__ void __launch_bounds__(256, 4) oneshot_k(const f4v* __restrict__ x, f4v* __restrict__ y, long long nseg,
                                                    long long q, int iters, float c) {
    __shared__ float pin[9216];  // 36 KB: 4 workgroups per CU
    const int t = threadIdx.x;
    const int xc = blockIdx.x & 7;
    const long long seg = (long long)xc * q + (blockIdx.x >> 3);
    const long long xe = (long long)(xc + 1) * q;
    if (seg >= (xe < nseg ? xe : nseg)) return;
    const long long base = seg * (kV / 2);  // float4 units (2 samples each)
    f4v v[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = x[base + t + 256 * i];
    fake_compute(v, iters, c);
#pragma unroll
    for (int i = 0; i < 8; ++i)
        if (i > 0 || t >= 128) y[base + t + 256 * i] = v[i];
    if (iters < 0) pin[t] = v[0].x;
}

// one-shot pattern kernel: U 16-byte vectors per lane (U * 4 KB per workgroup),
// segment stride `stride` samples, the first `skip` samples of a segment not
// written (halo).  LAYOUT 0: lane t, vector i at t + 256 i; 1: wave-contiguous
// (wave w covers U KB); 2: the overlap-save row-pair layout (rows 2i + up).
// MODE 1: the second half of the loads waits for the first (vmcnt); MODE 2: s_sleep
// between stores (spread the write burst); MODE 3: nontemporal loads; MODE 4:
// nontemporal stores; MODE 5: stores in reverse order
template <int U, int LAYOUT, int MODE = 0>
__global__ void __launch_bounds__(256) pat_k(const f4v* __restrict__ x, f4v* __restrict__ y, long long nseg,
                                             long long q, long long stride, int skip) {
    extern __shared__ float pin_dyn[];
    const int t = threadIdx.x;
    const int xc = blockIdx.x & 7;
    const long long seg = (long long)xc * q + (blockIdx.x >> 3);
    const long long xe = (long long)(xc + 1) * q;
    if (seg >= (xe < nseg ? xe : nseg)) return;
    const long long base = seg * (stride / 2);
    auto ix = [&](int i) -> int {
        if constexpr (LAYOUT == 0) return t + 256 * i;
        else if constexpr (LAYOUT == 1) return (t >> 6) * 64 * U + 64 * i + (t & 63);
        else return 256 * i + 128 * ((t >> 4) & 1) + 16 * (t >> 5) + (t & 15);
    };
    f4v v[U];
#pragma unroll
    for (int i = 0; i < U; ++i) {
        if (MODE == 1 && i == U / 2) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if constexpr (MODE == 3) v[i] = __builtin_nontemporal_load(x + base + ix(i));
        else v[i] = x[base + ix(i)];
    }
#pragma unroll
    for (int k = 0; k < U; ++k) {
        const int i = MODE == 5 ? U - 1 - k : k;
        if (MODE == 2 && k) __builtin_amdgcn_s_sleep(8);
        if (ix(i) >= skip / 2) {
            if constexpr (MODE == 4) __builtin_nontemporal_store(v[i], y + base + ix(i));
            else y[base + ix(i)] = v[i];
        }
    }
    if (nseg < 0) pin_dyn[t] = 0.f;
}

// one-shot, NT threads per workgroup = NT/256 consecutive overlap-save segments
// (row-pair layout, halo), each 256-lane group moving its own 32 KB segment
template <int NT>
__global__ void __launch_bounds__(NT) grp_k(const f4v* __restrict__ x, f4v* __restrict__ y, long long nseg,
                                            long long q, long long stride, int skip) {
    extern __shared__ float pin_dyn[];
    const int t = threadIdx.x & 255, g = threadIdx.x >> 8;
    const int xc = blockIdx.x & 7;
    const long long seg = ((long long)xc * q + (blockIdx.x >> 3)) * (NT / 256) + g;
    const long long xe = ((long long)xc + 1) * q * (NT / 256);
    if (seg >= (xe < nseg ? xe : nseg)) return;
    const long long base = seg * (stride / 2);
    auto ix = [&](int i) -> int { return 256 * i + 128 * ((t >> 4) & 1) + 16 * (t >> 5) + (t & 15); };
    f4v v[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = x[base + ix(i)];
#pragma unroll
    for (int i = 0; i < 8; ++i)
        if (ix(i) >= skip / 2) y[base + ix(i)] = v[i];
    if (nseg < 0) pin_dyn[t] = 0.f;
}

template <int N> __device__ __forceinline__ void wait_vm() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }
__device__ __forceinline__ void raw_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
}

__device__ __forceinline__ void lds_read8(f4v (&v)[8], unsigned a) {
#pragma unroll
    for (int i = 0; i < 8; ++i) asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(v[i]) : "v"(a), "n"(4096 * i));
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
}

template <int WPC>
__global__ void __launch_bounds__(256, WPC) pipe_k(const f4v* __restrict__ x, f4v* __restrict__ y, long long nseg,
                                                   long long q, int iters, float c) {
    __shared__ f4v buf[2][2048];  // 2 x 32 KB
    __shared__ float pin[WPC == 2 ? 1024 : 1];
    const int t = threadIdx.x, w = t >> 6, l = t & 63;
    const int xc = blockIdx.x & 7;
    const long long per = gridDim.x >> 3, j = blockIdx.x >> 3;
    const long long s0 = (long long)xc * q, s1 = std::min<long long>(s0 + q, nseg);
    // segments of this workgroup: s0 + j + k per, k = 0 .. nk-1
    const long long nk = s0 + j < s1 ? (s1 - s0 - j + per - 1) / per : 0;
    auto issue = [&](long long k, int b) {
        const f4v* src = x + (s0 + j + k * per) * (kV / 2);
#pragma unroll
        for (int i = 0; i < 8; ++i)
            __builtin_amdgcn_global_load_lds((const void*)(src + 256 * i + 64 * w + l),
                                             (__attribute__((address_space(3))) void*)&buf[b][256 * i + 64 * w], 16, 0, 0);
    };
    if (nk > 0) issue(0, 0);
    if (nk > 1) issue(1, 1);
    for (long long k = 0; k < nk; ++k) {
        const bool more = k + 1 < nk;
        if (more) {
            if (k == 0) wait_vm<8>();
            else if (k == 1) wait_vm<16>();
            else wait_vm<24>();
        } else {
            if (k == 0) wait_vm<0>();
            else if (k == 1) wait_vm<8>();
            else wait_vm<16>();
        }
        raw_barrier();
        const int b = (int)(k & 1);
        // LDS reads as inline asm: the compiler would otherwise put vmcnt(0) in
        // front of them (it cannot tell which DMA wrote the buffer) and drain the
        // loads of the segments in flight
        f4v v[8];
        const unsigned a = (unsigned)(size_t)(__attribute__((address_space(3))) void*)&buf[b][t];
        lds_read8(v, a);
        raw_barrier();
        if (k + 2 < nk) issue(k + 2, b);
        fake_compute(v, iters, c);
        f4v* dst = y + (s0 + j + k * per) * (kV / 2);
#pragma unroll
        for (int i = 0; i < 8; ++i)
            if (i > 0 || t >= 128) dst[t + 256 * i] = v[i];
    }
    if (iters < 0) pin[t & (WPC == 2 ? 1023 : 0)] = 0.f;
}

int main(int argc, char** argv) {
    const long long nsamp = 1LL << 30;
    f4v *x, *y;
    CK(hipMalloc(&x, nsamp * 8 + (1 << 20)));
    CK(hipMalloc(&y, nsamp * 8 + (1 << 20)));
    CK(hipMemset(x, 0, nsamp * 8));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto time_it = [&](auto launch) {
        for (int r = 0; r < 3; ++r) launch();
        std::vector<float> ts;
        for (int r = 0; r < 9; ++r) {
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
    // clock settle
    {
        const long long nseg = nsamp / 4096, q = (nseg + 7) / 8;
        for (int r = 0; r < 100; ++r)
            hipLaunchKernelGGL((pat_k<8, 0>), dim3(8 * q), dim3(256), 0, 0, x, y, nseg, q, 4096LL, 0);
        CK(hipDeviceSynchronize());
    }
    auto pat = [&](auto kern, int U, const char* name, long long stride, int skip, int lds) {
        const long long win = 512LL * U;  // samples read per workgroup
        const long long nseg = (nsamp - win) / stride, q = (nseg + 7) / 8;
        const double bytes = (double)nseg * (win - skip) * 16.0;
        float ms = time_it([&] { hipLaunchKernelGGL(kern, dim3(8 * q), dim3(256), lds, 0, x, y, nseg, q, stride, skip); });
        std::printf("%-22s U %d stride %5lld skip %3d lds %6d  %.3f ms  %.0f GB/s (out-sample bytes)\n", name, U, stride,
                    skip, lds, ms, bytes / ms / 1e6);
        std::fflush(stdout);
    };
    auto grp = [&](auto kern, int nt, long long stride, int skip, int lds) {
        const long long nseg = (nsamp - 4096) / stride, per = nt / 256;
        const long long q = (nseg / per + 7) / 8 + 1;
        const double bytes = (double)nseg * (4096 - skip) * 16.0;
        float ms = time_it([&] { hipLaunchKernelGGL(kern, dim3(8 * q), dim3(nt), lds, 0, x, y, nseg, q, stride, skip); });
        std::printf("grp %4d threads lds %6d  %.3f ms  %.0f GB/s\n", nt, lds, ms, bytes / ms / 1e6);
        std::fflush(stdout);
    };
    for (int rep = 0; rep < 2; ++rep) {
        grp(grp_k<256>, 256, 3840, 256, 36864);
        grp(grp_k<256>, 256, 3840, 256, 90112);
        grp(grp_k<512>, 512, 3840, 256, 73728);
        grp(grp_k<512>, 512, 3840, 256, 90112);
        grp(grp_k<1024>, 1024, 3840, 256, 90112);
        grp(grp_k<1024>, 1024, 3840, 256, 147456);
    }
    for (int rep = 0; rep < 1; ++rep) {
        pat(pat_k<1, 0>, 1, "lin", 512, 0, 0);
        pat(pat_k<2, 0>, 2, "lin", 1024, 0, 36864);
        for (int lds : {36864, 49152, 65536, 90112}) pat(pat_k<8, 2>, 8, "rowpair halo", 3840, 256, lds);
        pat(pat_k<8, 2, 1>, 8, "rowpair halo split", 3840, 256, 36864);
        pat(pat_k<8, 2, 2>, 8, "rowpair halo sleepst", 3840, 256, 36864);
        pat(pat_k<8, 2, 3>, 8, "rowpair halo ntload", 3840, 256, 36864);
        pat(pat_k<8, 2, 4>, 8, "rowpair halo ntstore", 3840, 256, 36864);
        pat(pat_k<8, 2, 5>, 8, "rowpair halo revst", 3840, 256, 36864);
    }
    if (argc > 1) {
        const long long nseg = (nsamp - kSeg) / kV;
        const long long q = (nseg + 7) / 8;
        const double bytes = (double)nseg * kV * 16.0;
        for (int i = 1; i < argc; ++i) {
            const int it = std::atoi(argv[i]);
            float a = time_it([&] { hipLaunchKernelGGL(oneshot_k, dim3(8 * q), dim3(256), 0, 0, x, y, nseg, q, it, 1.0f); });
            float b2 = time_it([&] { hipLaunchKernelGGL(pipe_k<2>, dim3(256 * 2), dim3(256), 0, 0, x, y, nseg, q, it, 1.0f); });
            std::printf("iters %3d  oneshot %.3f ms (%.0f GB/s)  pipe2 %.3f ms (%.0f GB/s)\n", it, a, bytes / a / 1e6, b2,
                        bytes / b2 / 1e6);
        }
    }
    CK(hipGetLastError());
    return 0;
}
