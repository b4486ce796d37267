// Single-sample step of the FIR / decimating FIR (gfx950): Filter::execute(sample)
// and DecimatingFIRFilter::push (src/filter/fir/mod.rs:209-212, decim.rs:127-131,
// 221-231) as ONE launch.  The sample travels as a kernel argument and the output
// is written straight to host-mapped memory followed by a system-scope release of
// a sequence flag the host polls, so a per-sample call costs one launch and the
// kernel's own time -- no host<->device copies, no stream synchronisation.  The dot product is
// the reference's: sum_{i<L} cr[i] x[n-i] from zero in increasing i, then * scale
// (this TU is built with -ffp-contract=off; EXACT keeps separate multiply and add),
// so the result is bit-identical to execute_block with n = 1.
#include "sdsp_device.hpp"
#include "sdsp_kernels.hpp"

namespace sdsp {

constexpr int kStepThreads = 256;
constexpr int kStepChunk = 1024;  // products staged in LDS per round

template <typename C, typename I, bool EXACT>
__global__ void __launch_bounds__(kStepThreads)
fir_step_kernel(I sample, const I* __restrict__ hist_in, I* __restrict__ hist_out, const C* __restrict__ cr, C scale,
                I* __restrict__ out, unsigned* __restrict__ flag, unsigned seq, int Lm1, int L, int emit) {
    __shared__ I prod[kStepChunk];
    const int t = threadIdx.x;
    // x[n - i]: the sample for i = 0, the delay line before it for i >= 1
    auto xs = [&](int i) -> I { return i == 0 ? sample : hist_in[Lm1 - i]; };
    if (emit) {
        I acc = zero_v<I>();
        if constexpr (EXACT) {
            // products are independent roundings: form them in parallel, then add them in the
            // reference order on one lane (identical to the sequential loop)
            for (int i0 = 0; i0 < L; i0 += kStepChunk) {
                const int m = L - i0 < kStepChunk ? L - i0 : kStepChunk;
                for (int k = t; k < m; k += kStepThreads) prod[k] = mul_(cr[i0 + k], xs(i0 + k));
                __syncthreads();
                if (t == 0)
                    for (int k = 0; k < m; ++k) acc = add_(acc, prod[k]);
                __syncthreads();
            }
        } else if (t == 0) {
            for (int i = 0; i < L; ++i) acc = mac<false>(acc, cr[i], xs(i));
        }
        if (t == 0) *out = mul_(acc, scale);
    }
    // the new delay line: the last Lm1 of (hist_in, sample)
    for (int k = t; k < Lm1; k += kStepThreads) hist_out[k] = k + 1 < Lm1 ? hist_in[k + 1] : sample;
    // every wave's delay-line stores happen before the flag (the host may start the next
    // device call as soon as it sees it): workgroup barrier, then a system-scope release
    __syncthreads();
    if (t == 0 && flag) __hip_atomic_store(flag, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

template <typename C, typename I>
hipError_t launch_fir_step_t(const FirStepArgs& a, hipStream_t s) {
    const I x = *reinterpret_cast<const I*>(a.sample);
    const C sc = a.scale ? *reinterpret_cast<const C*>(a.scale) : C{};
    if (a.exact)
        hipLaunchKernelGGL((fir_step_kernel<C, I, true>), dim3(1), dim3(kStepThreads), 0, s, x, (const I*)a.hist_in,
                           (I*)a.hist_out, (const C*)a.taps_rev, sc, (I*)a.out, a.flag, a.seq, a.Lm1, a.L,
                           a.emit ? 1 : 0);
    else
        hipLaunchKernelGGL((fir_step_kernel<C, I, false>), dim3(1), dim3(kStepThreads), 0, s, x, (const I*)a.hist_in,
                           (I*)a.hist_out, (const C*)a.taps_rev, sc, (I*)a.out, a.flag, a.seq, a.Lm1, a.L,
                           a.emit ? 1 : 0);
    return hipGetLastError();
}

hipError_t launch_fir_step(int dtype, const FirStepArgs& a, hipStream_t s) {
    switch (dtype) {
        case 0: return launch_fir_step_t<float, float>(a, s);
        case 1: return launch_fir_step_t<float, c32>(a, s);
        case 2: return launch_fir_step_t<c32, c32>(a, s);
        case 3: return launch_fir_step_t<double, double>(a, s);
        case 4: return launch_fir_step_t<double, c64>(a, s);
        case 5: return launch_fir_step_t<c64, c64>(a, s);
    }
    return hipErrorInvalidValue;
}

}  // namespace sdsp
