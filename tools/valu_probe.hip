// VALU issue-rate probe for gfx950 (calibration, not product): throughput of
// v_add_f32, v_fma_f32, v_pk_add_f32, v_pk_fma_f32, v_pk_mul_f32 over 8
// independent chains per lane, 4 waves per SIMD.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/_build/valu_probe tools/valu_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f2 __attribute__((ext_vector_type(2)));
constexpr int kIter = 4096;

template <int OP, int CH>
__global__ void __launch_bounds__(256) probe(float* out, float a0) {
    float s[8];
    f2 p[8];
    for (int i = 0; i < 8; ++i) { s[i] = a0 + i + threadIdx.x; p[i] = f2{s[i], s[i] + 1.0f}; }
    const float c = 1.0000001f;
    const f2 c2 = f2{c, c};
    for (int it = 0; it < kIter; ++it) {
#pragma unroll
        for (int i0 = 0; i0 < 8; ++i0) {
            const int i = i0 % CH;  // CH independent chains
            if constexpr (OP == 0) asm volatile("v_add_f32 %0, %0, %1" : "+v"(s[i]) : "v"(c));
            if constexpr (OP == 1) asm volatile("v_fma_f32 %0, %0, %1, %1" : "+v"(s[i]) : "v"(c));
            if constexpr (OP == 2) asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(p[i]) : "v"(c2));
            if constexpr (OP == 3) asm volatile("v_pk_fma_f32 %0, %0, %1, %1" : "+v"(p[i]) : "v"(c2));
            if constexpr (OP == 4) asm volatile("v_pk_mul_f32 %0, %0, %1" : "+v"(p[i]) : "v"(c2));
            if constexpr (OP == 5) asm volatile("v_mov_b32 %0, %1" : "=v"(s[i]) : "v"(s[(i + 1) & 7]));
            if constexpr (OP == 6) asm volatile("v_mul_f32 %0, %0, %1" : "+v"(s[i]) : "v"(c));
        }
    }
    float r = 0;
    for (int i = 0; i < 8; ++i) r += s[i] + p[i].x + p[i].y;
    if (r == 12345.0f) out[threadIdx.x] = r;
}

int main() {
    hipDeviceProp_t prop;
    hipGetDeviceProperties(&prop, 0);
    const int cus = prop.multiProcessorCount;
    float* out;
    hipMalloc(&out, 4096);
    const char* names[] = {"v_add_f32", "v_fma_f32", "v_pk_add_f32", "v_pk_fma_f32", "v_pk_mul_f32", "v_mov_b32",
                           "v_mul_f32"};
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (int ch : {8, 1}) {
        for (int wps : {4, 1}) {
            for (int op = 0; op < 7; ++op) {
                auto launch = [&] {
                    dim3 g(cus * wps), b(256);  // wps waves per SIMD
#define L_(O)                                                                              \
    if (ch == 8) hipLaunchKernelGGL((probe<O, 8>), g, b, 0, 0, out, 1.0f);                 \
    else hipLaunchKernelGGL((probe<O, 1>), g, b, 0, 0, out, 1.0f);
                    switch (op) {
                        case 0: L_(0) break;
                        case 1: L_(1) break;
                        case 2: L_(2) break;
                        case 3: L_(3) break;
                        case 4: L_(4) break;
                        case 5: L_(5) break;
                        case 6: L_(6) break;
                    }
                };
                launch();
                hipDeviceSynchronize();
                hipEventRecord(e0);
                for (int r = 0; r < 5; ++r) launch();
                hipEventRecord(e1);
                hipEventSynchronize(e1);
                float ms;
                hipEventElapsedTime(&ms, e0, e1);
                const double insts_per_simd = 5.0 * wps * kIter * 8;
                std::printf("chains %d waves/SIMD %d  %-14s %6.3f ns per wave-instruction per SIMD\n", ch, wps,
                            names[op], ms * 1e6 / insts_per_simd);
            }
        }
    }
    return 0;
}
