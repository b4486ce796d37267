// Lab translation unit for the one-shot overlap-save kernel (tools only, never
// part of libsdsp.so).  It compiles the lab copy of the kernel
// (tools/lab/ols_os_lab_kernel.hip: the product transform with every ablation and
// variant bit, ABL, documented at ols_os_segment; ABL 24 is the product's
// configuration), renaming its launcher, and adds a launcher that runs the
// compile-time variants selected by sdsp_lab_set_ols_variant -- the in-process A/B
// driver is tools/ols_lab.py.  tools/lab.mk links it in place of the product object.
#define SDSP_OLS_STAMPS 1
#define launch_fir_ols_os launch_fir_ols_os_product
#include "ols_os_lab_kernel.hip"
#undef launch_fir_ols_os

namespace sdsp {

static int g_lab_variant = 0, g_lab_lds = 0;

#define SDSP_OLS_LAB_VARIANTS(X) X(1) X(2) X(3) X(4) X(8) X(16) X(24) X(128) X(262168) X(2097176) X(4194328) X(132) X(256) X(260) X(512) X(768) X(772) X(1024) X(1028) X(2048) X(4096) X(6144) X(8192) X(8196) X(16384) X(16388) X(32768) X(49152) X(57344) X(131076) X(262144) X(524288) X(786432) X(2097152) X(4194304) X(6291456) X(16777216) X(18874368) X(18874880) X(33554432) X(35651584) X(67108888) X(268435480) X(65560) X(88) X(28) X(2072) X(8216) X(152)

hipError_t launch_fir_ols_os(const OlsPlan& p, const void* x, const void* hist, void* new_hist, void* y, size_t n,
                             int Lm1, size_t channels, hipStream_t s, bool wide) {
    if (wide && g_lab_variant == 0) return launch_fir_ols_os_t<524288>(p, x, hist, new_hist, y, n, Lm1, channels, s, 0);
#define SDSP_OLS_LAB_CASE(V) \
    if (g_lab_variant == V)  \
        return launch_fir_ols_os_t<V>(p, x, hist, new_hist, y, n, Lm1, channels, s, (size_t)g_lab_lds);
    SDSP_OLS_LAB_VARIANTS(SDSP_OLS_LAB_CASE)
#undef SDSP_OLS_LAB_CASE
    return launch_fir_ols_os_t<0>(p, x, hist, new_hist, y, n, Lm1, channels, s, (size_t)g_lab_lds);
}

}  // namespace sdsp

// variant (ABL bits), dynamic LDS bytes (pins occupancy); the third argument is unused
// (kept for tools/ols_lab.py)
extern "C" __attribute__((visibility("default"))) void sdsp_lab_set_ols_variant(int v, int lds, int) {
    sdsp::g_lab_variant = v;
    sdsp::g_lab_lds = lds;
}

// the clock stamps of the last variant-262144 dispatch (4 x 8192 u64: memtime, realtime at entry
// and exit of every 32nd workgroup; zero where no workgroup wrote)
extern "C" __attribute__((visibility("default"))) int sdsp_lab_ols_stamps(unsigned long long* out) {
    return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(sdsp::g_ols_stamps), sizeof(sdsp::g_ols_stamps), 0,
                                    hipMemcpyDeviceToHost);
}
extern "C" __attribute__((visibility("default"))) int sdsp_lab_ols_stamps_clear() {
    static unsigned long long z[4 * 8192];
    return (int)hipMemcpyToSymbol(HIP_SYMBOL(sdsp::g_ols_stamps), z, sizeof(z), 0, hipMemcpyHostToDevice);
}
