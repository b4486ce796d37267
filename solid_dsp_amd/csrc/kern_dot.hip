// Batched DotProduct::execute (src/dot_product/mod.rs:153-171): for each of
// `batch` sample vectors s_b (stride `stride` samples),
//     out[b] = sum_{i < min(n, len)} c[i] * s_b[i]      (from zero, in order)
// with the coefficients stored FORWARD or REVERSE as DotProduct::new does
// (the host reverses them once).  One lane per vector, reference order, no FMA:
// bit-identical to the reference at the handle precision.
#include "sdsp_device.hpp"
#include "sdsp_kernels.hpp"

namespace sdsp {

template <typename C, typename I>
__global__ void __launch_bounds__(256)
dot_batched_kernel(const C* __restrict__ c, int it, const I* __restrict__ s, long long stride, long long batch,
                   I* __restrict__ out) {
    const long long b = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= batch) return;
    const I* v = s + b * stride;
    I acc = zero_v<I>();
    for (int i = 0; i < it; ++i) acc = add_(acc, mul_(c[i], v[i]));
    out[b] = acc;
}

template <typename C, typename I>
hipError_t launch_dot_t(const DotArgs& a, hipStream_t st) {
    dim3 grid((unsigned)((a.batch + 255) / 256));
    hipLaunchKernelGGL((dot_batched_kernel<C, I>), grid, dim3(256), 0, st, (const C*)a.coefs, a.it, (const I*)a.s,
                       (long long)a.stride, (long long)a.batch, (I*)a.out);
    return hipGetLastError();
}

hipError_t launch_dot(int dtype, const DotArgs& a, hipStream_t st) {
    if (a.batch == 0) return hipSuccess;
    switch (dtype) {
        case 0: return launch_dot_t<float, float>(a, st);
        case 1: return launch_dot_t<float, c32>(a, st);
        case 2: return launch_dot_t<c32, c32>(a, st);
        case 3: return launch_dot_t<double, double>(a, st);
        case 4: return launch_dot_t<double, c64>(a, st);
        case 5: return launch_dot_t<c64, c64>(a, st);
    }
    return hipErrorInvalidValue;
}

}  // namespace sdsp
