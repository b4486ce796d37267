// One-shot, XCD-ordered overlap-save FIR for 32-bit complex streams (gfx950):
// the default interior-segment kernel of FIRFilter::execute_block for c32.
//
// Same filter as FIRFilter::execute (src/filter/fir/mod.rs:209-212),
//     y[n] = scale * sum_{i<L} h[L-1-i] x[n-i],
// per 4096-sample segment as a circular convolution with the zero-padded
// g[i] = scale h[L-1-i] (spectrum H/N precomputed in f64 on the host).
// Segment s reads x[s V - H, s V - H + 4096) and writes the V = 4096 - H
// outputs that do not wrap (H = 256 h2 >= L - 1).  The transform is the one of
// kern_fir_ols.hip / kern_fir_ols_pk.hip (three radix-16 passes each way,
// n = 256 n2 + 16 n1 + n0, k = k0 + 16 k1 + 256 k2, no bit reversal), in packed
// FP32 (sdsp_pk.hpp).  What differs is the shape, chosen for the HBM stream:
//
//  * one segment per 256-thread workgroup, one workgroup per segment (no
//    persistent loop): the dispatcher deals workgroup b to XCD b % 8, so
//    segment(b) = lo + (b % 8) q + b / 8 makes every XCD stream one contiguous
//    eighth of the call in order (the halo row of a segment is the tail its XCD
//    neighbour just read, an L2 hit).  Measured against the alternatives in
//    persistent grids (any order) and more or fewer workgroups per
//    CU are slower;
//  * 4 workgroups per CU (16 waves): 116 VGPRs and one 34 KB LDS image.  The
//    image is ALIASED across phases: in P2/P4 lane (k0, n0) owns the 16
//    positions (k0, 16 j + n0), in P3 lane (k0, k1) owns (k0, 16 k1 + j), in
//    P1/P5 lane t owns column t -- each lane reads and rewrites only its own
//    positions inside a phase, so one region suffices.  P2, P3 and P4 of wave w
//    touch only rows k0 = 4w .. 4w + 3, so only P1 -> P2 and P4 -> P5 need a
//    workgroup barrier;
//  * lane t owns column t in P1 / P5: 8-byte buffer loads and stores per row
//    (row offsets in SGPRs, no address arithmetic in VGPRs);
//  * no twiddle tables in LDS or per-lane tables in registers: W4096^(t k) =
//    D_{k>>2} C_{k&3} and W256^(l k) = F_{k>>2} E_{k&3} from per-lane bases
//    (C1, D1, E1, F1: two float4 from L2; C2 = C1 C1, C3 = C2 C1, ...), the
//    spectrum slice of P3 loaded from L2 in P2;
//  * nontemporal input loads and stores (the stream is read and written once).
//
// LDS image: element (r, c) at r * 272 + c + (c >> 4) (one 8-byte pad per
// 16-column block; rows 544 dwords apart, i.e. opposite halves of the 64
// banks).  Every access is a per-lane base plus a compile-time offset and is
// conflict-free except P5's reads (lanes 0 and 31 of a 32-lane group share a
// bank pair: SQ_LDS_BANK_CONFLICT counts 2 extra cycles per ds_read_b64,
// tools/lds_probe.hip).
//
// Numerics: bit-identical across calls and launch shapes; against the f64
// restatement rel-RMS ~1.8e-7 on the cfg2 taps (§8d tolerance 1e-6).
#include "sdsp_device.hpp"
#include "sdsp_kernels.hpp"
#include "sdsp_pk.hpp"

namespace sdsp {

using namespace pk;

namespace {

constexpr int kRow = 272;

// WAVE: the next phase reads only what this wave wrote (the LDS operations of one
// wave complete in order), so a compiler-level fence replaces the block barrier
template <bool WAVE> __device__ __forceinline__ void phase_sync() {
    if constexpr (WAVE) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    } else {
        __syncthreads();
    }
}

typedef unsigned int u2v __attribute__((ext_vector_type(2)));
constexpr int kBufWord3 = 0x00020000;  // raw buffer descriptor word 3 (gfx9 family)

// x = D_{k>>2} C_{k&3} for C_b = c[b-1], D_a = d[a-1] (k = 0 -> 1)
__device__ __forceinline__ f2 tw_pair(const f2 (&c)[3], const f2 (&d)[3], int k) {
    const int a = k >> 2, b = k & 3;
    if (a == 0) return b == 0 ? f2{1.0f, 0.0f} : c[b - 1];
    if (b == 0) return d[a - 1];
    return pmul(d[a - 1], c[b - 1]);
}

}  // namespace

// ABL selects compile-time variants of the segment transform.  The product kernel
// is ABL = 0; tools/lab/ols_lab.hip instantiates the others for in-process A/B runs
// (never part of libsdsp.so).  Bits: 1 block barriers at the wave-local phase
// boundaries; 2 no HBM traffic (ablation: outputs dropped); 4 HBM traffic only
// (ablation: no transform); 128 plain (not nontemporal) stores; 256 input rows
// loaded last to first; 512 output rows stored last to first; 1024 each XCD walks the
// even segments of its eighth, then the odd ones (a segment's halo row is then read
// long after its neighbour's tail: from HBM, not as a hit on an in-flight L2 miss);
// ablations of the per-segment table reads from L2: 2048 no spectrum loads, 4096 no
// twiddle-base loads (wrong results, timing only); 8192 write-through (sc1) stores; 16384
// plain (not nontemporal) input loads; 32768 all six twiddle bases loaded (the round-3 form;
// 49152 = the round-3 kernel); 131072 with 4: the HBM-only pattern in 16-byte lanes (the NCO
// kernel's shape).
template <int ABL>
__device__ __forceinline__ void ols_os_segment(const f2* __restrict__ x, const float4* __restrict__ Hs,
                                               const float4* __restrict__ tb, f2* __restrict__ y, long long base,
                                               int h2, f2* img, int t) {
    const int hi4 = t >> 4, lo4 = t & 15;
    const auto rx = __builtin_amdgcn_make_buffer_rsrc((void*)(x + base), (short)0, 32768, kBufWord3);
    const auto ry = __builtin_amdgcn_make_buffer_rsrc((void*)(y + base), (short)0, 32768, kBufWord3);
    const auto rt = __builtin_amdgcn_make_buffer_rsrc((void*)tb, (short)0, kOlsOsTabF4 * 16, kBufWord3);
    const auto rh = __builtin_amdgcn_make_buffer_rsrc((void*)Hs, (short)0, 2048 * 16, kBufWord3);
    f2 v[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        const int r = (ABL & 256) ? 15 - i : i;
        if constexpr ((ABL & 131072) != 0) v[r] = f2{0.0f, 0.0f};  // (the 16-byte-lane ablation loads its own)
        else if constexpr (ABL & 2) v[r] = f2{1e-3f * t + r, 1e-9f * (float)base};
        else if constexpr ((ABL & 16384) != 0)
            v[r] = __builtin_bit_cast(f2, __builtin_amdgcn_raw_buffer_load_b64(rx, 8 * t, 2048 * r, 0));
        else  // nontemporal (aux 2)
            v[r] = __builtin_bit_cast(f2, __builtin_amdgcn_raw_buffer_load_b64(rx, 8 * t, 2048 * r, 2));
    }
    if constexpr ((ABL & 4) && (ABL & 131072)) {
        // HBM-only with the NCO kernel's lane shape: the segment as eight 4 KB rows of 16-byte
        // lanes (lane t: bytes 16 t + 4096 k), the halo's bytes not stored
        typedef unsigned u4v __attribute__((ext_vector_type(4)));
        u4v w[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) w[k] = __builtin_bit_cast(u4v, __builtin_amdgcn_raw_buffer_load_b128(rx, 16 * t, 4096 * k, 2));
#pragma unroll
        for (int k = 0; k < 8; ++k) asm volatile("" : "+v"(w[k]));
#pragma unroll
        for (int k = 0; k < 8; ++k)
            if (4096 * k + 16 * t >= 2048 * h2) __builtin_amdgcn_raw_buffer_store_b128(w[k], ry, 16 * t, 4096 * k, 2);
        return;
    } else if constexpr (ABL & 4) {
        // every row's load in flight before the first store, as in the transform (without this
        // the compiler sinks each load into its store's `r >= h2` branch: one round trip per row)
#pragma unroll
        for (int r = 0; r < 16; ++r) asm volatile("" : "+v"(v[r]));
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const int r = (ABL & 512) ? 15 - i : i;
            if (r >= h2)
                __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u2v, v[r]), ry, 8 * t, 2048 * r,
                                                      (ABL & 8192) ? 16 : (ABL & 128) ? 0 : 2);
        }
        return;
    }
    // twiddle bases: column t of W4096, row lo4 of W256 (runtime.cpp ols_build)
    auto tab = [&](int lane, int off) {
        if constexpr ((ABL & 4096) != 0) {
            const float u = 1e-3f * (float)lane + 1e-6f * (float)off;
            return float4{u, 0.5f - u, 0.25f + u, 1.0f - u};
        } else {
            return __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rt, 16 * lane, off, 0));
        }
    };
    f2 Cb[3], Da[3], Eb[3], Fa[3];
    if constexpr ((ABL & (32768 | 4096)) == 0) {
        // the first power of each base from L2 ({C1, D1} per column, {E1, F1} per row: two
        // 16-byte loads where the six-base form takes six), the others as products (W^2 = W W,
        // W^3 = W^2 W): a third of the table traffic per segment, results within rounding of the
        // six-base form (rel-RMS 2.2e-7 between the two on cfg2)
        const float4 cd = tab(t, 16 * kOlsOsTabCD), ef = tab(lo4, 16 * kOlsOsTabEF);
        const f2 c1 = f2{cd.x, cd.y}, d1 = f2{cd.z, cd.w}, e1 = f2{ef.x, ef.y}, f1 = f2{ef.z, ef.w};
        const f2 c2 = pmul(c1, c1), d2 = pmul(d1, d1), e2 = pmul(e1, e1), f2_ = pmul(f1, f1);
        Cb[0] = c1, Cb[1] = c2, Cb[2] = pmul(c2, c1);
        Da[0] = d1, Da[1] = d2, Da[2] = pmul(d2, d1);
        Eb[0] = e1, Eb[1] = e2, Eb[2] = pmul(e2, e1);
        Fa[0] = f1, Fa[1] = f2_, Fa[2] = pmul(f2_, f1);
    } else {
        const float4 b0 = tab(t, 0), b1 = tab(t, 4096), b2 = tab(t, 8192);
        const float4 e0 = tab(lo4, 12288), e1 = tab(lo4, 12544), e2 = tab(lo4, 12800);
        Cb[0] = f2{b0.x, b0.y}, Cb[1] = f2{b0.z, b0.w}, Cb[2] = f2{b1.x, b1.y};
        Da[0] = f2{b1.z, b1.w}, Da[1] = f2{b2.x, b2.y}, Da[2] = f2{b2.z, b2.w};
        Eb[0] = f2{e0.x, e0.y}, Eb[1] = f2{e0.z, e0.w}, Eb[2] = f2{e1.x, e1.y};
        Fa[0] = f2{e1.z, e1.w}, Fa[1] = f2{e2.x, e2.y}, Fa[2] = f2{e2.z, e2.w};
    }
    f2* col = img + t + (t >> 4);  // (r, t) at col[r * kRow]

    // P1: DFT16 n2 -> k0, * W4096^(t k0) -> (k0, t)
    pdft16<false>(v);
#pragma unroll
    for (int k = 0; k < 16; ++k) col[k * kRow] = k == 0 ? v[0] : pmul(v[kout(k)], tw_pair(Cb, Da, k));
    __syncthreads();

    // P2: lane (k0 = hi4, n0 = lo4): DFT16 n1 -> k1, * W256^(n0 k1) -> (k0, 16 k1 + n0)
    f2* r2 = img + hi4 * kRow + lo4;  // (hi4, 16 j + lo4) at r2[17 j]
#pragma unroll
    for (int j = 0; j < 16; ++j) v[j] = r2[17 * j];
    float4 hq[8];  // spectrum slice of lane (k0, k1) = t for P3, k-pair major
#pragma unroll
    for (int p = 0; p < 8; ++p) {
        if constexpr ((ABL & 2048) != 0) hq[p] = float4{1e-3f * (float)t, (float)p, 0.5f, 1e-4f * (float)t};
        else hq[p] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rh, 16 * t, 4096 * p, 0));
    }
    f2 w2[16];  // W256^(lo4 k), used by P2 (n0 = lo4) and P3 (k1 = lo4)
#pragma unroll
    for (int k = 1; k < 16; ++k) w2[k] = tw_pair(Eb, Fa, k);
    pdft16<false>(v);
#pragma unroll
    for (int k = 0; k < 16; ++k) r2[17 * k] = k == 0 ? v[0] : pmul(v[kout(k)], w2[k]);
    phase_sync<!(ABL & 1)>();

    // P3: lane (k0 = hi4, k1 = lo4) over n0: DFT16 n0 -> k2, * H, IDFT16 k2 -> n0, * conj W256^(k1 n0)
    {
        f2* r3 = img + hi4 * kRow + 17 * lo4;  // (hi4, 16 lo4 + j) at r3[j]
#pragma unroll
        for (int j = 0; j < 16; ++j) v[j] = r3[j];
        pdft16<false>(v);
        f2 u[16];
#pragma unroll
        for (int p = 0; p < 8; ++p) {
            u[2 * p] = pmul(v[kout(2 * p)], f2{hq[p].x, hq[p].y});
            u[2 * p + 1] = pmul(v[kout(2 * p + 1)], f2{hq[p].z, hq[p].w});
        }
        pdft16<true>(u);
#pragma unroll
        for (int j = 0; j < 16; ++j) r3[j] = j == 0 ? u[kout(0)] : pmulc(u[kout(j)], w2[j]);
    }
    phase_sync<!(ABL & 1)>();

    // P4: lane (k0 = hi4, n0 = lo4): IDFT16 k1 -> n1 -> (k0, 16 n1 + n0)
#pragma unroll
    for (int j = 0; j < 16; ++j) v[j] = r2[17 * j];
    pdft16<true>(v);
#pragma unroll
    for (int k = 0; k < 16; ++k) r2[17 * k] = v[kout(k)];
    __syncthreads();

    // P5: lane t: * conj W4096^(t k0), IDFT16 k0 -> n2; row n2 at v[kout(n2)].  The bases are
    // made opaque first so the products are recomputed here rather than kept live from P1.
#pragma unroll
    for (int i = 0; i < 3; ++i) asm volatile("" : "+v"(Cb[i]), "+v"(Da[i]));
#pragma unroll
    for (int k = 0; k < 16; ++k) v[k] = k == 0 ? col[0] : pmulc(col[k * kRow], tw_pair(Cb, Da, k));
    pdft16<true>(v);
    if constexpr (ABL & 2) {  // outputs kept live, not stored
        f2 acc = v[0];
#pragma unroll
        for (int r = 1; r < 16; ++r) acc += v[r];
        if (acc.x == 1.2345e30f) __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u2v, acc), ry, 8 * t, 0, 0);
        return;
    }
    // nontemporal stores (3.14 -> 3.08 ms on cfg2, in-process A/B)
    constexpr int kStAux = (ABL & 8192) ? 16 : (ABL & 128) ? 0 : 2;  // 16: write-through (sc1), lab
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        const int r = (ABL & 512) ? 15 - i : i;
        if (r >= h2)
            __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u2v, v[kout(r)]), ry, 8 * t, 2048 * r, kStAux);
    }
}

template <int ABL>
__global__ void __launch_bounds__(256, 4)
fir_ols_os_kernel(const f2* __restrict__ x, const float4* __restrict__ Hs, const float4* __restrict__ tb,
                  f2* __restrict__ y, long long n, long long lo, long long hi, long long q, int h2) {
    __shared__ __attribute__((aligned(16))) f2 img[16 * kRow];
    const int xc = blockIdx.x & 7;
    long long j = blockIdx.x >> 3;
    if constexpr ((ABL & 1024) != 0) j = j < (q + 1) / 2 ? 2 * j : 2 * (j - (q + 1) / 2) + 1;
    const long long seg = lo + (long long)xc * q + j;
    const long long xe = lo + (long long)(xc + 1) * q;
    if (seg >= (xe < hi ? xe : hi)) return;  // uniform over the workgroup
    const int V = 4096 - 256 * h2;
    ols_os_segment<ABL>(x, Hs, tb, y, (long long)blockIdx.y * n + seg * V - 256 * h2, h2, img, threadIdx.x);
}

// interior segments [lo, hi) of every channel; ABL as above (0 = the product kernel)
template <int ABL>
hipError_t launch_fir_ols_os_t(const OlsPlan& p, const void* x, void* y, size_t n, size_t channels, hipStream_t s,
                               long long lo, long long hi, size_t dyn_lds) {
    if (hi <= lo) return hipSuccess;
    if (p.halo_rows < 1 || p.halo_rows > 15) return hipErrorInvalidValue;
    const long long q = (hi - lo + 7) / 8;
    const dim3 grid((unsigned)(8 * q), (unsigned)channels);
    hipLaunchKernelGGL(fir_ols_os_kernel<ABL>, grid, dim3(256), dyn_lds, s, (const f2*)x, (const float4*)p.d_pkt,
                       (const float4*)p.d_ostab, (f2*)y, (long long)n, lo, hi, q, p.halo_rows);
    return hipGetLastError();
}

hipError_t launch_fir_ols_os(const OlsPlan& p, const void* x, void* y, size_t n, size_t channels, hipStream_t s,
                             long long lo, long long hi) {
    return launch_fir_ols_os_t<0>(p, x, y, n, channels, s, lo, hi, 0);
}

}  // namespace sdsp
