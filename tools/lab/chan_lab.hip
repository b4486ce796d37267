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

static int g_chan_lab = 0;
static int g_fft_policy = 0;  // 4-step L = 1024 passes: bit 0 nontemporal loads, bit 1 nontemporal stores,
                              // bit 2 no inter-pass twiddle (ablation), 8 the pass skeleton
                              // (loads, staging, twiddle, stores; no FFT), 16 / 32 16-byte
                              // lanes on the strided side of the loads / stores (16: the
                              // product since r05u, so the same as 0), 64 XCD-ordered
                              // groups

bool try_launch_fft1024_pass(const FftPass& p_, hipStream_t s, hipError_t* err) {
    FftPass p = p_;
    if (g_fft_policy & 4) p.Ntw = 0;  // ablation: the column pass without its inter-pass twiddle (wrong results)
    switch (g_fft_policy & 123) {
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

extern "C" __attribute__((visibility("default"))) void sdsp_lab_set_fft_policy(int v) { sdsp::g_fft_policy = v & 127; }
