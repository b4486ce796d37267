// HBM access-pattern probe for the overlap-save kernel (calibration, not product).
// Each workgroup (256 lanes) moves `per` segments of 4096 complex-f32 samples
// (32 KB) through registers: 8 x 16-byte loads per lane, then 8 stores.
//   PAT 0: linear (lane t, load i -> float4 index t + 256 i: 4 KB contiguous per WG instruction)
//   PAT 1: the packed OLS row-pair pattern (rows 2i / 2i+1 of a 16 x 256 image, 512 B per half wave)
//   HALO 1: segments advance 3840 samples and row 0 is not stored (the OLS stream shape)
//   lds: dynamic LDS per workgroup, to pin occupancy at the kernel's 2 workgroups per CU
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/_build/pattern_probe tools/pattern_probe.hip
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
            return 1;                                                           \
        }                                                                       \
    } while (0)

typedef float f4v __attribute__((ext_vector_type(4)));

template <int PAT, int HALO, int NT>
__global__ void __launch_bounds__(256) seg_k(const float2* __restrict__ x, float2* __restrict__ y, long long nseg,
                                             int per) {
    extern __shared__ float lds_dyn[];
    const int t = threadIdx.x;
    const int up = (t >> 4) & 1;
    const int colX = 32 * (t >> 5) + 2 * (t & 15);
    const long long stride = HALO ? 3840 : 4096;
    long long s0 = (long long)blockIdx.x * per;
    long long s1 = s0 + per < nseg ? s0 + per : nseg;
    for (long long s = s0; s < s1; ++s) {
        f4v q[8];
        const long long base = s * stride;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const long long off = PAT == 0 ? base + 2 * (t + 256 * i) : base + 512 * i + 256 * up + colX;
            const f4v* p = reinterpret_cast<const f4v*>(x + off);
            q[i] = (NT & 1) ? __builtin_nontemporal_load(p) : *p;
        }
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const long long off = PAT == 0 ? base + 2 * (t + 256 * i) : base + 512 * i + 256 * up + colX;
            const bool halo_row = HALO && (PAT == 0 ? (i == 0 && t < 128) : (i == 0 && !up));
            if (halo_row) continue;
            f4v* p = reinterpret_cast<f4v*>(y + off);
            if (NT & 2) __builtin_nontemporal_store(q[i], p);
            else *p = q[i];
        }
    }
    if (per < 0) lds_dyn[t] = 0.f;  // keep the allocation
}

template <int PAT, int HALO, int NT>
float run(const float2* x, float2* y, long long nsamp, int per, int lds, int reps) {
    const long long stride = HALO ? 3840 : 4096;
    const long long nseg = (nsamp - 4096) / stride;
    const long long blocks = (nseg + per - 1) / per;
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    std::vector<float> ts;
    for (int r = 0; r < reps + 1; ++r) {
        hipEventRecord(e0);
        hipLaunchKernelGGL((seg_k<PAT, HALO, NT>), dim3((unsigned)blocks), dim3(256), lds, 0, x, y, nseg, per);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        if (r) ts.push_back(ms);
    }
    std::sort(ts.begin(), ts.end());
    hipEventDestroy(e0);
    hipEventDestroy(e1);
    const float ms = ts[ts.size() / 2];
    const double bytes = 16.0 * (double)(nseg * stride);  // algorithmic: 8 B in + 8 B out per output sample
    std::printf("PAT %d HALO %d NT %d per %4d lds %6d  %.3f ms  %.1f GB/s\n", PAT, HALO, NT, per, lds, ms,
                bytes / (ms * 1e-3) / 1e9);
    return ms;
}


// ORD 0: load i of lane t at t + 256 i (1 KB per wave instruction, 4 KB apart);
// ORD 1: wave-contiguous, wave w covers [w 64 U, (w + 1) 64 U) (U KB per wave)
// ORD 2: as 0 with workgroups remapped so that each XCD (blockIdx % 8) streams its own
// contiguous eighth of the buffer; ORD 3: as 0, chunk = blockIdx with the low 3 bits
// moved up (chunks 8 apart share an XCD's consecutive workgroups' ... i.e. XCD x gets
// chunks x*?); see remap below
template <int U, int NT, int ORD = 0>
__global__ void __launch_bounds__(256) lin_k(const f4v* __restrict__ x, f4v* __restrict__ y, long long nblk) {
    extern __shared__ float lds_dyn[];
    const int t = threadIdx.x;
    long long blk = blockIdx.x;
    if constexpr (ORD == 2) blk = (blk % 8) * (nblk / 8) + blk / 8;
    const long long base = blk * 256 * U;
    auto ix = [&](int i) -> long long { return ORD != 1 ? t + 256 * i : (t >> 6) * 64 * U + 64 * i + (t & 63); };
    f4v q[U];
#pragma unroll
    for (int i = 0; i < U; ++i) q[i] = (NT & 1) ? __builtin_nontemporal_load(x + base + ix(i)) : x[base + ix(i)];
#pragma unroll
    for (int i = 0; i < U; ++i) {
        if (NT & 2) __builtin_nontemporal_store(q[i], y + base + ix(i));
        else y[base + ix(i)] = q[i];
    }
    if (nblk < 0) lds_dyn[t] = 0.f;
}

template <int U, int NT, int ORD = 0>
void run_lin(const float2* x, float2* y, long long nsamp, int lds, int reps) {
    const long long nblk = nsamp / 2 / (256 * U);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    std::vector<float> ts;
    for (int r = 0; r < reps + 1; ++r) {
        (void)hipEventRecord(e0);
        hipLaunchKernelGGL((lin_k<U, NT, ORD>), dim3((unsigned)nblk), dim3(256), lds, 0, (const f4v*)x, (f4v*)y, nblk);
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms;
        (void)hipEventElapsedTime(&ms, e0, e1);
        if (r) ts.push_back(ms);
    }
    std::sort(ts.begin(), ts.end());
    const float ms = ts[ts.size() / 2];
    std::printf("LIN ORD %d U %d NT %d lds %6d  %.3f ms  %.1f GB/s\n", ORD, U, NT, lds, ms, 16.0 * nsamp / (ms * 1e-3) / 1e9);
}


// Model of the persistent overlap-save loop: `per` segments per workgroup, compute
// emulated by 4 phases of s_sleep (SL x 64 cycles each); loads for segment s + 1 and
// stores of segment s - 1 are issued during segment s, either as one burst of 8
// (after phase 1) or 2 per phase (SPL bit 0: loads, bit 1: stores).
template <int SPL, int SL>
__global__ void __launch_bounds__(256) model_k(const f4v* __restrict__ x, f4v* __restrict__ y, long long nseg, int per) {
    extern __shared__ float lds_dyn[];
    const int t = threadIdx.x;
    const long long s0 = (long long)blockIdx.x * per;
    const long long s1 = s0 + per < nseg ? s0 + per : nseg;
    f4v nq[8], ov[8];
    auto ld = [&](long long sg, int i0, int i1) {
#pragma unroll
        for (int i = 0; i < 8; ++i)
            if (i >= i0 && i < i1) nq[i] = x[sg * 2048 + t + 256 * i];
    };
    auto st = [&](long long sg, int i0, int i1) {
#pragma unroll
        for (int i = 0; i < 8; ++i)
            if (i >= i0 && i < i1) y[sg * 2048 + t + 256 * i] = ov[i];
    };
    auto phase = [] {
        if constexpr (SL > 0) __builtin_amdgcn_s_sleep(SL);
    };
    if (s0 < s1) ld(s0, 0, 8);
    long long os = -1;
    for (long long s = s0; s < s1; ++s) {
        f4v v[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) v[i] = nq[i];
#pragma unroll
        for (int i = 0; i < 8; ++i) asm volatile("" : "+v"(v[i]));
        const long long nx = s + 1 < s1 ? s + 1 : s;
        phase();
        if (SPL & 1) ld(nx, 0, 2); else ld(nx, 0, 8);
        if (os >= 0) { if (SPL & 2) st(os, 0, 2); else st(os, 0, 8); }
        phase();
        if (SPL & 1) ld(nx, 2, 4);
        if ((SPL & 2) && os >= 0) st(os, 2, 4);
        phase();
        if (SPL & 1) ld(nx, 4, 6);
        if ((SPL & 2) && os >= 0) st(os, 4, 6);
        phase();
        if (SPL & 1) ld(nx, 6, 8);
        if ((SPL & 2) && os >= 0) st(os, 6, 8);
#pragma unroll
        for (int i = 0; i < 8; ++i) ov[i] = v[i];
        os = s;
    }
    if (os >= 0) st(os, 0, 8);
    if (per < 0) lds_dyn[t] = 0.f;
}

template <int SPL, int SL>
void run_model(const float2* x, float2* y, long long nsamp, int per, int lds, int reps) {
    const long long nseg = nsamp / 4096;
    const long long blocks = (nseg + per - 1) / per;
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    std::vector<float> ts;
    for (int r = 0; r < reps + 1; ++r) {
        (void)hipEventRecord(e0);
        hipLaunchKernelGGL((model_k<SPL, SL>), dim3((unsigned)blocks), dim3(256), lds, 0, (const f4v*)x, (f4v*)y, nseg, per);
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms;
        (void)hipEventElapsedTime(&ms, e0, e1);
        if (r) ts.push_back(ms);
    }
    std::sort(ts.begin(), ts.end());
    const float ms = ts[ts.size() / 2];
    std::printf("MODEL spread %d sleep %2d per %3d lds %6d  %.3f ms  %.1f GB/s\n", SPL, SL, per, lds, ms,
                16.0 * nsamp / (ms * 1e-3) / 1e9);
}

// Persistent chunked copy: per segment (32 KB per workgroup) U loads then U stores per
// lane, 8/U times; WG b takes `per` consecutive segments (per > 0) or segments
// b, b + G, ... (per == 0, G = grid).
template <int U>
__global__ void __launch_bounds__(256) pchunk_k(const f4v* __restrict__ x, f4v* __restrict__ y, long long nseg, int per) {
    extern __shared__ float lds_dyn[];
    const int t = threadIdx.x;
    long long s0, s1, st;
    if (per > 0) { s0 = (long long)blockIdx.x * per; s1 = s0 + per < nseg ? s0 + per : nseg; st = 1; }
    else { s0 = blockIdx.x; s1 = nseg; st = gridDim.x; }
    for (long long s = s0; s < s1; s += st) {
#pragma unroll
        for (int c = 0; c < 8 / U; ++c) {
            f4v q[U];
#pragma unroll
            for (int i = 0; i < U; ++i) q[i] = x[s * 2048 + t + 256 * (c * U + i)];
#pragma unroll
            for (int i = 0; i < U; ++i) y[s * 2048 + t + 256 * (c * U + i)] = q[i];
        }
    }
    if (per < 0) lds_dyn[t] = 0.f;
}

template <int U>
void run_pchunk(const float2* x, float2* y, long long nsamp, int per, int lds, int grid, int reps) {
    const long long nseg = nsamp / 4096;
    const long long blocks = per > 0 ? (nseg + per - 1) / per : grid;
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    std::vector<float> ts;
    for (int r = 0; r < reps + 1; ++r) {
        (void)hipEventRecord(e0);
        hipLaunchKernelGGL((pchunk_k<U>), dim3((unsigned)blocks), dim3(256), lds, 0, (const f4v*)x, (f4v*)y, nseg, per);
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms;
        (void)hipEventElapsedTime(&ms, e0, e1);
        if (r) ts.push_back(ms);
    }
    std::sort(ts.begin(), ts.end());
    const float ms = ts[ts.size() / 2];
    std::printf("PCHUNK U %d per %3d grid %5lld lds %6d  %.3f ms  %.1f GB/s\n", U, per, blocks, lds, ms,
                16.0 * nsamp / (ms * 1e-3) / 1e9);
}

// Persistent grid with a dynamic work queue per XCD: XCD b % 8 owns one contiguous
// eighth of the segments; its workgroups take the next segment from an atomic counter
// (the index for segment s + 1 is fetched while segment s moves), so the resident
// workgroups of an XCD stay on one compact window, as a one-shot dispatch keeps them.
__global__ void __launch_bounds__(256) dyn_k(const f4v* __restrict__ x, f4v* __restrict__ y, long long nseg,
                                             unsigned long long* ctr) {
    extern __shared__ float lds_dyn[];
    __shared__ long long nxt_s[2];
    const int t = threadIdx.x;
    const int xc = blockIdx.x % 8;
    const long long s8 = (nseg + 7) / 8;
    const long long a = xc * s8;
    const long long e = a + s8 < nseg ? a + s8 : nseg;
    if (t == 0) nxt_s[0] = a + (long long)atomicAdd(ctr + xc, 1ULL);
    __syncthreads();
    long long s = nxt_s[0];
    int par = 1;
    while (s < e) {
        if (t == 0) nxt_s[par] = a + (long long)atomicAdd(ctr + xc, 1ULL);
        f4v q[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) q[i] = x[s * 2048 + t + 256 * i];
#pragma unroll
        for (int i = 0; i < 8; ++i) y[s * 2048 + t + 256 * i] = q[i];
        __syncthreads();
        s = nxt_s[par];
        par ^= 1;
    }
    if (nseg < 0) lds_dyn[t] = 0.f;
}

void run_dyn(const float2* x, float2* y, long long nsamp, int grid, int lds, int reps) {
    const long long nseg = nsamp / 4096;
    unsigned long long* ctr;
    (void)hipMalloc(&ctr, 64);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    std::vector<float> ts;
    for (int r = 0; r < reps + 1; ++r) {
        (void)hipMemset(ctr, 0, 64);
        (void)hipEventRecord(e0);
        hipLaunchKernelGGL(dyn_k, dim3((unsigned)grid), dim3(256), lds, 0, (const f4v*)x, (f4v*)y, nseg, ctr);
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms;
        (void)hipEventElapsedTime(&ms, e0, e1);
        if (r) ts.push_back(ms);
    }
    std::sort(ts.begin(), ts.end());
    const float ms = ts[ts.size() / 2];
    std::printf("DYN grid %5d lds %6d  %.3f ms  %.1f GB/s\n", grid, lds, ms, 16.0 * nsamp / (ms * 1e-3) / 1e9);
    (void)hipFree(ctr);
}

int main() {
    const long long n = 1LL << 30;
    float2 *x, *y;
    CK(hipMalloc(&x, n * sizeof(float2)));
    CK(hipMalloc(&y, n * sizeof(float2)));
    CK(hipMemset(x, 0, n * sizeof(float2)));
    CK(hipMemset(y, 0, n * sizeof(float2)));

    const int L = 70 * 1024;
    const int reps = 5;
    if (getenv("PROBE_DYN")) {
        run_dyn(x, y, n, 512, L, reps);
        run_dyn(x, y, n, 1024, L, reps);
        run_dyn(x, y, n, 512, 0, reps);
        run_dyn(x, y, n, 2048, 0, reps);
        run_lin<8, 0, 2>(x, y, n, L, reps);
        run_pchunk<8>(x, y, n, 16, L, 0, reps);
        return 0;
    }
    if (getenv("PROBE_XCD")) {
        run_lin<2, 0, 0>(x, y, n, L, reps);
        run_lin<2, 0, 2>(x, y, n, L, reps);
        run_lin<8, 0, 0>(x, y, n, L, reps);
        run_lin<8, 0, 2>(x, y, n, L, reps);
        run_lin<1, 0, 0>(x, y, n, 0, reps);
        run_lin<1, 0, 2>(x, y, n, 0, reps);
        run_lin<8, 0, 0>(x, y, n, 0, reps);
        run_lin<8, 0, 2>(x, y, n, 0, reps);
        return 0;
    }
    if (getenv("PROBE_PCHUNK")) {
        for (int U : {1, 2, 8}) {
            for (int per : {1, 16, 0}) {
                if (U == 1) run_pchunk<1>(x, y, n, per, L, 512, reps);
                if (U == 2) run_pchunk<2>(x, y, n, per, L, 512, reps);
                if (U == 8) run_pchunk<8>(x, y, n, per, L, 512, reps);
            }
        }
        run_pchunk<2>(x, y, n, 0, L, 1024, reps);
        run_pchunk<2>(x, y, n, 0, 0, 2048, reps);
        run_pchunk<2>(x, y, n, 4, L, 0, reps);
        run_lin<2, 0>(x, y, n, L, reps);
        return 0;
    }
    if (getenv("PROBE_ORD")) {
        for (int lds : {0, L}) {
            run_lin<8, 0, 0>(x, y, n, lds, reps);
            run_lin<8, 0, 1>(x, y, n, lds, reps);
            run_lin<4, 0, 0>(x, y, n, lds, reps);
            run_lin<4, 0, 1>(x, y, n, lds, reps);
            run_lin<2, 0, 0>(x, y, n, lds, reps);
            run_lin<2, 0, 1>(x, y, n, lds, reps);
            run_lin<8, 3, 1>(x, y, n, lds, reps);
            run_lin<16, 0, 1>(x, y, n, lds, reps);
        }
        return 0;
    }
    if (getenv("PROBE_MODEL")) {
        for (int per : {16}) {
            run_model<0, 0>(x, y, n, per, L, reps);
            run_model<0, 8>(x, y, n, per, L, reps);
            run_model<1, 8>(x, y, n, per, L, reps);
            run_model<2, 8>(x, y, n, per, L, reps);
            run_model<3, 8>(x, y, n, per, L, reps);
            run_model<0, 16>(x, y, n, per, L, reps);
            run_model<1, 16>(x, y, n, per, L, reps);
            run_model<2, 16>(x, y, n, per, L, reps);
            run_model<3, 16>(x, y, n, per, L, reps);
            run_model<0, 24>(x, y, n, per, L, reps);
            run_model<3, 24>(x, y, n, per, L, reps);
            run_model<3, 16>(x, y, n, per, 40000, reps);
            run_model<0, 16>(x, y, n, per, 40000, reps);
        }
        run_lin<1, 0>(x, y, n, 0, reps);
        run_lin<2, 0>(x, y, n, L, reps);
        return 0;
    }
    for (int lds : {0, 40000, L}) {
        run_lin<1, 0>(x, y, n, lds, reps);
        run_lin<2, 0>(x, y, n, lds, reps);
        run_lin<4, 0>(x, y, n, lds, reps);
        run_lin<8, 0>(x, y, n, lds, reps);
        run_lin<1, 3>(x, y, n, lds, reps);
        run_lin<8, 3>(x, y, n, lds, reps);
    }
    for (int per : {1}) {
        for (int lds : {0, L}) {
            run<0, 0, 0>(x, y, n, per, lds, reps);
            run<1, 0, 0>(x, y, n, per, lds, reps);
            run<0, 1, 0>(x, y, n, per, lds, reps);
            run<1, 1, 0>(x, y, n, per, lds, reps);
        }
    }
    run<1, 1, 1>(x, y, n, 1, L, reps);
    run<1, 1, 2>(x, y, n, 1, L, reps);
    run<1, 1, 3>(x, y, n, 1, L, reps);
    run<1, 1, 3>(x, y, n, 1, 0, reps);
    run<0, 0, 3>(x, y, n, 1, 0, reps);
    CK(hipGetLastError());
    CK(hipDeviceSynchronize());
    return 0;
}
