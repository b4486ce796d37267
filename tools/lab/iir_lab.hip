// Lab translation unit for the IIR wave scan (tools only, never part of
// libsdsp.so): the product source compiled unchanged (its launcher renamed) plus
// a launcher that runs sos_wscan_kernel<..., LAB> on real-f32 4-section warm-up
// scans (the cfg3 shape) for the ablation set by sdsp_lab_set_iir_ablation
// (tools/iir_ab.py).  LAB bits are documented at sos_wscan_kernel; bits 12-15 of
// the ablation value force the tiles per wave.  tools/lab.mk links it in place of
// the product object.
#define launch_iir_wscan launch_iir_wscan_product
#include "kern_iir_wscan.hip"
#undef launch_iir_wscan

namespace sdsp {

static int g_iir_lab = 0;

template <int CB, int LAB>
static hipError_t lab_cfg3(const IirArgs& a, hipStream_t st, int tpw) {
    return launch_wscan_t<float, float, 4, CB, 0, 0, LAB>(a, st, tpw);
}

template <int CB>
static hipError_t lab_cfg3_ab(const IirArgs& a, hipStream_t st, int ab, int tpw) {
    switch (ab) {
        case 1: return lab_cfg3<CB, 1>(a, st, tpw);
        case 5: return lab_cfg3<CB, 5>(a, st, tpw);
        case 6: return lab_cfg3<CB, 6>(a, st, tpw);
        case 2: return lab_cfg3<CB, 2>(a, st, tpw);
        case 4: return lab_cfg3<CB, 4>(a, st, tpw);
        case 7: return lab_cfg3<CB, 7>(a, st, tpw);
        case 8: return lab_cfg3<CB, 8>(a, st, tpw);
        case 16: return lab_cfg3<CB, 16>(a, st, tpw);
        case 24: return lab_cfg3<CB, 24>(a, st, tpw);
        case 32: return lab_cfg3<CB, 32>(a, st, tpw);
        case 64: return lab_cfg3<CB, 64>(a, st, tpw);
        case 128: return lab_cfg3<CB, 128>(a, st, tpw);
        case 136: return lab_cfg3<CB, 136>(a, st, tpw);
        case 256: return lab_cfg3<CB, 256>(a, st, tpw);
        case 280: return lab_cfg3<CB, 280>(a, st, tpw);
        case 512: return lab_cfg3<CB, 512>(a, st, tpw);
        case 1024: return lab_cfg3<CB, 1024>(a, st, tpw);
        case 2048: return lab_cfg3<CB, 2048>(a, st, tpw);
        // codes past the LAB bits (the value's low 12 bits): 3072 = the FORM 2 kernel (no register
        // prefetch) with the DPP lane shifts (LAB 2048: 116 VGPRs, 4 waves per SIMD)
        case 3072: return launch_wscan_t<float, float, 4, CB, 2, 0, 2048>(a, st, tpw);
        // 3073: LAB 4096 (the carry as the scan's element -1); 3074: LAB 4096 + 1024
        case 3073: return lab_cfg3<CB, 4096>(a, st, tpw);
        case 3074: return lab_cfg3<CB, 5120>(a, st, tpw);
        // 3075: LAB 4096 + 8192 (4 workgroups per CU)
        case 3075: return lab_cfg3<CB, 12288>(a, st, tpw);
        // 3076: LAB 16384 (blocks in launch order)
        case 3076: return lab_cfg3<CB, 16384>(a, st, tpw);
        // 3077: LAB 32768 (four-wave workgroups, the form before the one-wave product)
        case 3077: return lab_cfg3<CB, 32768>(a, st, tpw);
        default: return lab_cfg3<CB, 0>(a, st, tpw);
    }
}

hipError_t launch_iir_wscan(int dtype, const IirArgs& a, hipStream_t st) {
    const int ab = g_iir_lab & 4095, tpw = (g_iir_lab >> 12) & 15;
    if ((ab || tpw) && dtype == 0 && a.sections == 4 && a.Mi == 1 && a.Md == 1 && a.wc > 0 && a.n > 0) {
        if (a.ws_variant == 1) return lab_cfg3_ab<128>(a, st, ab, tpw);
        if (a.ws_variant == 0) return lab_cfg3_ab<256>(a, st, ab, tpw);
    }
    return launch_iir_wscan_product(dtype, a, st);
}

}  // namespace sdsp

extern "C" __attribute__((visibility("default"))) int sdsp_lab_set_iir_ablation(int v) {
    sdsp::g_iir_lab = v;
    return 0;
}
