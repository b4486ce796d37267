// LDS bank-conflict probe for the cfg2 overlap-save image (calibration, not
// product): each kernel repeats ONE phase's LDS access pattern of
// fir_ols_os_kernel (kern_fir_ols_os.hip) on the same 34 KB image layout,
// element (r, c) at r * 272 + c + (c >> 4), 256 lanes, 4 workgroups per CU, so
// `rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS` reports
// the conflict cycles of each phase separately.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/_build/lds_probe tools/lds_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f2 __attribute__((ext_vector_type(2)));
constexpr int kRow = 272, kIter = 2000;

__device__ __forceinline__ int opaque0() {
    int z;
    asm volatile("v_mov_b32 %0, 0" : "=v"(z));
    return z;
}

template <int PH>
__global__ void __launch_bounds__(256, 4) probe(float* out) {
    __shared__ __attribute__((aligned(16))) f2 img[16 * kRow];
    const int t = threadIdx.x, hi4 = t >> 4, lo4 = t & 15;
    f2 acc = f2{0.0f, 0.0f};
    for (int i = t; i < 16 * kRow; i += 256) img[i] = f2{(float)i, 1.0f};
    __syncthreads();
    for (int it = 0; it < kIter; ++it) {
        const int z = opaque0();
        if constexpr (PH == 1) {  // P1: lane t writes column t, rows k
            f2* col = img + t + (t >> 4) + z;
#pragma unroll
            for (int k = 0; k < 16; ++k) col[k * kRow] = f2{(float)k, (float)it};
        } else if constexpr (PH == 2 || PH == 4) {  // P2 / P4: lane (hi4, lo4) touches (hi4, 16 j + lo4)
            f2* r2 = img + hi4 * kRow + lo4 + z;
#pragma unroll
            for (int j = 0; j < 16; ++j) {
                if constexpr (PH == 2) acc += r2[17 * j];
                else r2[17 * j] = f2{(float)j, (float)it};
            }
        } else if constexpr (PH == 3 || PH == 6) {  // P3: lane (hi4, lo4) touches (hi4, 16 lo4 + j)
            f2* r3 = img + hi4 * kRow + 17 * lo4 + z;
#pragma unroll
            for (int j = 0; j < 16; ++j) {
                if constexpr (PH == 3) acc += r3[j];
                else r3[j] = f2{(float)j, (float)it};
            }
        } else {  // P5: lane t reads column t
            const f2* col = img + t + (t >> 4) + z;
#pragma unroll
            for (int k = 0; k < 16; ++k) acc += col[k * kRow];
        }
    }
    if (acc.x == 1.2345e30f) out[t] = acc.y;
}
// distinct names for the profiler
int main() {
    hipDeviceProp_t prop;
    hipGetDeviceProperties(&prop, 0);
    float* out;
    hipMalloc(&out, 4096);
    const dim3 g(prop.multiProcessorCount * 4), b(256);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    auto run = [&](const char* name, void (*k)(float*)) {
        hipLaunchKernelGGL(k, g, b, 0, 0, out);
        hipEventRecord(e0);
        hipLaunchKernelGGL(k, g, b, 0, 0, out);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms = 0;
        hipEventElapsedTime(&ms, e0, e1);
        // 16 LDS instructions (64 lanes x 8 B) per wave per iteration
        const double waves = 4.0 * g.x, ins = waves * kIter * 16;
        std::printf("%-9s %8.3f ms  %6.2f CU-cycles per wave-instruction at 2.4 GHz\n", name, ms,
                    ms * 1e-3 * 2.4e9 * prop.multiProcessorCount / ins);
    };
    run("p1_write", probe<1>);
    run("p2_read", probe<2>);
    run("p2_write", probe<4>);
    run("p3_read", probe<3>);
    run("p3_write", probe<6>);
    run("p5_read", probe<5>);
    return hipDeviceSynchronize() == hipSuccess ? 0 : 1;
}
