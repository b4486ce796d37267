// Register-FFT issue-rate probe (calibration, not product): a loop of radix-16
// DFTs on 16 complex values per lane, with the workgroups per CU (hence waves per
// SIMD) fixed by a dynamic LDS allocation.  Answers: how much faster does the
// overlap-save kernel's arithmetic issue at 3-4 waves/SIMD than at 2?
// Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -o tools/_build/fft_occ_probe tools/fft_occ_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>

struct cf { float re, im; };
__device__ __forceinline__ cf cadd(cf a, cf b) { return {a.re + b.re, a.im + b.im}; }
__device__ __forceinline__ cf csub(cf a, cf b) { return {a.re - b.re, a.im - b.im}; }
__device__ __forceinline__ cf cmul(cf a, cf b) {
    return {__builtin_fmaf(a.re, b.re, -(a.im * b.im)), __builtin_fmaf(a.re, b.im, a.im * b.re)};
}
__device__ __forceinline__ cf rotj(cf a) { return {a.im, -a.re}; }
__device__ __forceinline__ void dft4(cf& x0, cf& x1, cf& x2, cf& x3) {
    cf a = cadd(x0, x2), b = csub(x0, x2), c = cadd(x1, x3), d = rotj(csub(x1, x3));
    x0 = cadd(a, c); x2 = csub(a, c); x1 = cadd(b, d); x3 = csub(b, d);
}
__device__ __forceinline__ void dft16(cf (&v)[16], const cf (&w)[16]) {
#pragma unroll
    for (int nb = 0; nb < 4; ++nb) dft4(v[nb], v[4 + nb], v[8 + nb], v[12 + nb]);
#pragma unroll
    for (int i = 5; i < 16; ++i) if ((i & 3) && (i >> 2)) v[i] = cmul(v[i], w[i]);
#pragma unroll
    for (int ka = 0; ka < 4; ++ka) dft4(v[4 * ka + 0], v[4 * ka + 1], v[4 * ka + 2], v[4 * ka + 3]);
}

typedef float f2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f2 pmul(f2 a, f2 b) { return __builtin_elementwise_fma(a.xx, b, a.yy * f2{-b.y, b.x}); }
__device__ __forceinline__ void pdft4(f2& x0, f2& x1, f2& x2, f2& x3) {
    f2 a = x0 + x2, b = x0 - x2, c = x1 + x3, z = x1 - x3;
    f2 d = f2{z.y, -z.x};
    x0 = a + c; x2 = a - c; x1 = b + d; x3 = b - d;
}
__device__ __forceinline__ void pdft16(f2 (&v)[16], const f2 (&w)[16]) {
#pragma unroll
    for (int nb = 0; nb < 4; ++nb) pdft4(v[nb], v[4 + nb], v[8 + nb], v[12 + nb]);
#pragma unroll
    for (int i = 5; i < 16; ++i) if ((i & 3) && (i >> 2)) v[i] = pmul(v[i], w[i]);
#pragma unroll
    for (int ka = 0; ka < 4; ++ka) pdft4(v[4 * ka + 0], v[4 * ka + 1], v[4 * ka + 2], v[4 * ka + 3]);
}
__global__ void __launch_bounds__(256) probe_pk(cf* out, const cf* tw, int iters) {
    extern __shared__ char pad[];
    f2 v[16], w[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        v[i] = f2{(float)(threadIdx.x + i), 1.0f};
        const cf t = tw[(threadIdx.x * 16 + i) & 1023];
        w[i] = f2{t.re, t.im};
    }
    for (int it = 0; it < iters; ++it) {
        pdft16(v, w);
#pragma unroll
        for (int i = 0; i < 16; ++i) v[i] = pmul(v[i], w[(i + 3) & 15]);
    }
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) s += v[i].x + v[i].y;
    if (s == 1234.5f) { out[threadIdx.x] = cf{v[0].x, v[0].y}; pad[0] = 1; }
}

__global__ void __launch_bounds__(256) probe(cf* out, const cf* tw, int iters) {
    extern __shared__ char pad[];
    cf v[16], w[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) { v[i] = cf{(float)(threadIdx.x + i), 1.0f}; w[i] = tw[(threadIdx.x * 16 + i) & 1023]; }
    for (int it = 0; it < iters; ++it) {
        dft16(v, w);
#pragma unroll
        for (int i = 0; i < 16; ++i) v[i] = cmul(v[i], w[(i + 3) & 15]);
    }
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) s += v[i].re + v[i].im;
    if (s == 1234.5f) { out[threadIdx.x] = v[0]; pad[0] = 1; }
}

int main() {
    hipDeviceProp_t p;
    hipGetDeviceProperties(&p, 0);
    const int cus = p.multiProcessorCount;
    cf *out, *tw;
    hipMalloc(&out, 4096 * sizeof(cf));
    hipMalloc(&tw, 1024 * sizeof(cf));
    hipMemset(tw, 0, 1024 * sizeof(cf));
    const int iters = 2000;
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    // blocks per CU via LDS: 160 KB / lds
    for (int pk = 0; pk < 2; ++pk)
    for (int bpc : {1, 2, 4}) {
        const size_t lds = (160 * 1024) / bpc - 1024;
        const int blocks = cus * bpc;
        auto k = pk ? probe_pk : probe;
        hipLaunchKernelGGL(k, dim3(blocks), dim3(256), lds, 0, out, tw, 10);
        hipDeviceSynchronize();
        hipEventRecord(e0);
        hipLaunchKernelGGL(k, dim3(blocks), dim3(256), lds, 0, out, tw, iters);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        // work per SIMD: bpc waves x iters iterations
        const double per_iter_ns = ms * 1e6 / ((double)bpc * iters);
        std::printf("%s waves/SIMD %d: %.3f ms, %.2f ns per wave-iteration per SIMD\n", pk ? "packed" : "scalar",
                    bpc, ms, per_iter_ns);
    }
    return 0;
}
