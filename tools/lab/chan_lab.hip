// Lab translation unit for the streaming channeliser (tools only, never part of
// libsdsp.so): the product source compiled unchanged (its launcher renamed) plus
// a launcher that runs chan1024_kernel<..., LAB> for the LAB value set by
// sdsp_lab_set_chan_ablation (tools/chan_ab.py).  LAB bits are documented at
// chan1024_kernel.  tools/lab.mk links it in place of the product object.
#define try_launch_chan1024 try_launch_chan1024_product
#define try_launch_fft1024_pass try_launch_fft1024_pass_product
#include "kern_chan1024.hip"
#undef try_launch_chan1024
#undef try_launch_fft1024_pass

namespace sdsp {

namespace {
// the column pass in 8-transform groups: two 512-thread workgroups per CU (VERDICT r05 #6;
// prefetch depth 0: at 4 or 8 the body spills at the 128 VGPRs two workgroups per CU allow).
// Measured 1266-1359 against 947-951 us for the 16-transform pass (profiles/r06/LAB.md)
template <bool INV, bool TW, int LA>
__global__ void __launch_bounds__(512, 4)
fft1024_pipe8_kernel(const cf* __restrict__ x, cf* __restrict__ y, const cf* __restrict__ tw,
                     const cf* __restrict__ twx, long long count, long long G, long long S0, long long S1,
                     long long Si, long long T1, long long So) {
    fft1024_pipe_body<INV, TW, true, true, 8, 0, LA, 0>(x, y, tw, twx, count, G, S0, S1, Si, T1, So);
}

// false: not the column pass (the caller falls through to the product launcher)
template <int LA>
bool launch_pipe8(const FftPass& p, hipStream_t s, hipError_t* err) {
    const bool wide = p.S1 == 1 && ((uintptr_t)p.x & 15) == 0 && (p.S0 & 1) == 0 && (p.Si & 1) == 0;
    if (p.L != 1024 || p.S1 != 1 || p.T1 != 1 || !wide || p.count % 16 != 0 || p.G % 16 != 0) return false;
    if (p.Ntw && (p.Ntw != (1LL << 20) || !p.twx)) return false;
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    const long long g8 = p.count / 8;
    const dim3 g3((unsigned)(g8 < 2LL * cus ? g8 : 2LL * cus));
#define SDSP_PIPE8(INV, TW)                                                                                          \
    hipLaunchKernelGGL((fft1024_pipe8_kernel<INV, TW, (LA | 16)>), g3, dim3(512), 0, s, (const cf*)p.x, (cf*)p.y, \
                       (const cf*)p.tw, (const cf*)p.twx, p.count, p.G, p.S0, p.S1, p.Si, p.T1, p.So)
    if (p.inverse) {
        if (p.Ntw) SDSP_PIPE8(true, true); else SDSP_PIPE8(true, false);
    } else {
        if (p.Ntw) SDSP_PIPE8(false, true); else SDSP_PIPE8(false, false);
    }
#undef SDSP_PIPE8
    *err = hipGetLastError();
    return true;
}
}  // namespace

static int g_chan_lab = 0;
static int g_fft_policy = 0;  // 4-step L = 1024 passes: bit 0 nontemporal loads, bit 1 nontemporal stores,
                              // bit 2 no inter-pass twiddle (ablation), 8 the pass skeleton
                              // (loads, staging, twiddle, stores; no FFT), 16 / 32 16-byte
                              // lanes on the strided side of the loads / stores (16: the
                              // product since r05u, so the same as 0), 64 XCD-ordered
                              // groups, 128 neighbouring groups paired on one XCD, 256 the
                              // column pass in 8-transform groups (two workgroups per CU),
                              // 384 both

bool try_launch_fft1024_pass(const FftPass& p_, hipStream_t s, hipError_t* err) {
    FftPass p = p_;
    if (g_fft_policy & 4) p.Ntw = 0;  // ablation: the column pass without its inter-pass twiddle (wrong results)
    switch (g_fft_policy & 251 & ~128) {
        case 1: return try_launch_fft1024_pass_t<2, 0>(p, s, err);
        case 2: return try_launch_fft1024_pass_t<0, 2>(p, s, err);
        case 3: return try_launch_fft1024_pass_t<2, 2>(p, s, err);
        case 8: return try_launch_fft1024_pass_t<8, 0>(p, s, err);  // skeleton: no FFT (timing only)
        case 16: return try_launch_fft1024_pass_t<16, 0>(p, s, err);
        case 32: return try_launch_fft1024_pass_t<0, 16>(p, s, err);
        case 48: return try_launch_fft1024_pass_t<16, 16>(p, s, err);
        case 56: return try_launch_fft1024_pass_t<24, 16>(p, s, err);
        case 64: return try_launch_fft1024_pass_t<32, 0>(p, s, err);
        case 72: return try_launch_fft1024_pass_t<40, 0>(p, s, err);
        case 112: return try_launch_fft1024_pass_t<48, 16>(p, s, err);
        case 120: return try_launch_fft1024_pass_t<56, 16>(p, s, err);
        default: break;
    }
    switch (g_fft_policy & 384) {
        case 128: return try_launch_fft1024_pass_t<64, 0>(p, s, err);
        case 256: return launch_pipe8<0>(p, s, err) || try_launch_fft1024_pass_t<0, 0>(p, s, err);
        case 384: return launch_pipe8<64>(p, s, err) || try_launch_fft1024_pass_t<64, 0>(p, s, err);
        default: return try_launch_fft1024_pass_t<0, 0>(p, s, err);
    }
}

bool try_launch_chan1024(const ChanArgs& a, hipStream_t s, hipError_t* err) {
    switch (g_chan_lab) {
        case 1: return try_launch_chan1024_t<1>(a, s, err);
        case 2: return try_launch_chan1024_t<2>(a, s, err);
        case 4: return try_launch_chan1024_t<4>(a, s, err);
        case 6: return try_launch_chan1024_t<6>(a, s, err);
        case 32: return try_launch_chan1024_t<32>(a, s, err);
        case 64: return try_launch_chan1024_t<64>(a, s, err);
        case 128: return try_launch_chan1024_t<128>(a, s, err);
        case 256: return try_launch_chan1024_t<256>(a, s, err);
        case 384: return try_launch_chan1024_t<384>(a, s, err);
        default: return try_launch_chan1024_t<0>(a, s, err);
    }
}

}  // namespace sdsp

// tools/chan_ab.py encoding: 1 no FFT, 2 no loads, 4 no stores, 8 plain stores,
// 16 nontemporal loads, 32 / 64 odd workgroups start ~6.8 / ~3.4 us late; bits from 128 up
// pass through as the kernel's LAB bits (128 write-through stores, 256 nontemporal round loads)
extern "C" __attribute__((visibility("default"))) void sdsp_lab_set_chan_ablation(int v) {
    sdsp::g_chan_lab = (v & 7) | ((v >> 2) & 24) | ((v & 8) ? 32 : 0) | ((v & 16) ? 64 : 0) | (v & ~127);
}

extern "C" __attribute__((visibility("default"))) void sdsp_lab_set_fft_policy(int v) { sdsp::g_fft_policy = v & 511; }
