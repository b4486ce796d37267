// ARCHIVE (lab only, never part of libsdsp.so): the round-3 overlap-save lab
// translation unit -- the product kernel of that round plus the persistent slot,
// staggered pair, trio, quad and queue kernels and the per-CU ticket experiments,
// all measured slower than the one-shot kernel (logs under
// profiles/r02/lab and profiles/r03/lab).  Frozen as it was built by tools/lab.mk
// in round 3 (-DSDSP_OLS_LAB resolved); `make -f tools/lab.mk archive_r03` builds
// tools/_build/libsdsp_lab_r03.so from it.
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
//  * 4 workgroups per CU (16 waves): 96 VGPRs and one 34 KB LDS image.  The
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
//    (3 + 3 float4 from L2), the spectrum slice of P3 loaded from L2 in P2.
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

// per-CU count of workgroups whose segment loads are in flight (lab bits 8/16/24)
__device__ unsigned int g_ols_cu_loading[8 * 256];

__device__ __forceinline__ unsigned int* cu_slot() {
    unsigned int xcc, hw;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    return g_ols_cu_loading + ((xcc & 7) << 8) + ((hw >> 8) & 255);
}

}  // namespace

// VAR = 0 is the product kernel; tools/lab.mk builds other values (SDSP_OLS_LAB)
// for in-process A/B runs -- they are never part of libsdsp.so.  Lab bits:
// 1 block barriers at the wave-local phase boundaries; 2 no HBM traffic
// (ablation: outputs dropped); 4 HBM traffic only (ablation: no transform);
// 8/16/24: at most 1/2/3 workgroups per CU with segment loads in flight (a
// per-CU ticket taken with vector atomics before the loads, returned once P1
// has consumed them); 32: high wave priority while issuing loads and stores; 128:
// plain (not nontemporal) stores.
// STG (lab, the staggered pair kernel): 0 one segment per workgroup; 1 / 2 the first /
// second half of a 512-lane workgroup running two segments, the second starting its
// loads at the barrier that ends the first half's P1 (three workgroup barriers per
// half: 1 = P1 | P4 | end, 2 = start | P1 | P4).  `active` false: no loads or stores,
// the barriers only (the last pair of a range with an odd count).
template <int VAR, int STG = 0>
__device__ __forceinline__ void ols_os_segment(const f2* __restrict__ x, const float4* __restrict__ Hs,
                                               const float4* __restrict__ tb, f2* __restrict__ y, long long base,
                                               int h2, f2* img, int t, bool active = true) {
    if constexpr (STG == 2) __syncthreads();  // the first half's P1 is done: its loads have landed
    const int hi4 = t >> 4, lo4 = t & 15;
    constexpr unsigned kLim = (VAR >> 3) & 3;
    unsigned int* slot = nullptr;
    bool held = false;  // lane 0 of wave 0 holds a ticket (bounded wait: a lab run can never hang on it)
    if constexpr (kLim != 0) {
        slot = cu_slot();
        if (t == 0) {
            for (int tries = 0; tries < 4096; ++tries) {
                if (__hip_atomic_fetch_add(slot, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < kLim) {
                    held = true;
                    break;
                }
                __hip_atomic_fetch_add(slot, 0xffffffffu, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __builtin_amdgcn_s_sleep(4);
            }
        }
        __syncthreads();
    }
    if constexpr (VAR & 32) __builtin_amdgcn_s_setprio(3);
    const auto rx = __builtin_amdgcn_make_buffer_rsrc((void*)(x + base), (short)0, 32768, kBufWord3);
    const auto ry = __builtin_amdgcn_make_buffer_rsrc((void*)(y + base), (short)0, 32768, kBufWord3);
    const auto rt = __builtin_amdgcn_make_buffer_rsrc((void*)tb, (short)0, kOlsOsTabF4 * 16, kBufWord3);
    const auto rh = __builtin_amdgcn_make_buffer_rsrc((void*)Hs, (short)0, 2048 * 16, kBufWord3);
    f2 v[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        if constexpr (VAR & 2) v[r] = f2{1e-3f * t + r, 1e-9f * (float)base};
        else if constexpr (STG != 0) v[r] = active ? __builtin_bit_cast(f2, __builtin_amdgcn_raw_buffer_load_b64(rx, 8 * t, 2048 * r, 0)) : f2{0.0f, 0.0f};
        else v[r] = __builtin_bit_cast(f2, __builtin_amdgcn_raw_buffer_load_b64(rx, 8 * t, 2048 * r, 0));
    }
    if constexpr (VAR & 32) __builtin_amdgcn_s_setprio(0);
    if constexpr (kLim != 0 && (VAR & 64)) {  // ticket back as soon as the loads have landed
#pragma unroll
        for (int r = 0; r < 16; ++r) asm volatile("" : "+v"(v[r]));
        __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
        __syncthreads();
        if (held) __hip_atomic_fetch_add(slot, 0xffffffffu, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        held = false;
    }
    if constexpr (VAR & 4) {
#pragma unroll
        for (int r = 0; r < 16; ++r)
            if (r >= h2)
                __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u2v, v[r]), ry, 8 * t, 2048 * r,
                                                      (VAR & 128) ? 0 : 2);
        if constexpr (kLim != 0) {
            __syncthreads();
            if (held) __hip_atomic_fetch_add(slot, 0xffffffffu, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        return;
    }
    // twiddle bases: column t of W4096, row lo4 of W256 (runtime.cpp ols_build)
    const float4 b0 = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rt, 16 * t, 0, 0));
    const float4 b1 = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rt, 16 * t, 4096, 0));
    const float4 b2 = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rt, 16 * t, 8192, 0));
    const float4 e0 = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rt, 16 * lo4, 12288, 0));
    const float4 e1 = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rt, 16 * lo4, 12544, 0));
    const float4 e2 = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rt, 16 * lo4, 12800, 0));
    f2 Cb[3] = {f2{b0.x, b0.y}, f2{b0.z, b0.w}, f2{b1.x, b1.y}};
    f2 Da[3] = {f2{b1.z, b1.w}, f2{b2.x, b2.y}, f2{b2.z, b2.w}};
    const f2 Eb[3] = {f2{e0.x, e0.y}, f2{e0.z, e0.w}, f2{e1.x, e1.y}};
    const f2 Fa[3] = {f2{e1.z, e1.w}, f2{e2.x, e2.y}, f2{e2.z, e2.w}};
    f2* col = img + t + (t >> 4);  // (r, t) at col[r * kRow]

    // P1: DFT16 n2 -> k0, * W4096^(t k0) -> (k0, t)
    pdft16<false>(v);
#pragma unroll
    for (int k = 0; k < 16; ++k) col[k * kRow] = k == 0 ? v[0] : pmul(v[kout(k)], tw_pair(Cb, Da, k));
    __syncthreads();
    if constexpr (kLim != 0) {
        if (held) __hip_atomic_fetch_add(slot, 0xffffffffu, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }

    // P2: lane (k0 = hi4, n0 = lo4): DFT16 n1 -> k1, * W256^(n0 k1) -> (k0, 16 k1 + n0)
    f2* r2 = img + hi4 * kRow + lo4;  // (hi4, 16 j + lo4) at r2[17 j]
#pragma unroll
    for (int j = 0; j < 16; ++j) v[j] = r2[17 * j];
    float4 hq[8];  // spectrum slice of lane (k0, k1) = t for P3, k-pair major
#pragma unroll
    for (int p = 0; p < 8; ++p) hq[p] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rh, 16 * t, 4096 * p, 0));
    f2 w2[16];  // W256^(lo4 k), used by P2 (n0 = lo4) and P3 (k1 = lo4)
#pragma unroll
    for (int k = 1; k < 16; ++k) w2[k] = tw_pair(Eb, Fa, k);
    pdft16<false>(v);
#pragma unroll
    for (int k = 0; k < 16; ++k) r2[17 * k] = k == 0 ? v[0] : pmul(v[kout(k)], w2[k]);
    phase_sync<!(VAR & 1)>();

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
    phase_sync<!(VAR & 1)>();

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
    if constexpr (VAR & 2) {  // outputs kept live, not stored
        f2 acc = v[0];
#pragma unroll
        for (int r = 1; r < 16; ++r) acc += v[r];
        if (acc.x == 1.2345e30f) __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u2v, acc), ry, 8 * t, 0, 0);
        return;
    }
    if constexpr (VAR & 32) __builtin_amdgcn_s_setprio(3);
    // nontemporal stores (3.14 -> 3.08 ms on cfg2, in-process A/B; lab bit 128: plain stores)
    constexpr int kStAux = (VAR & 128) ? 0 : 2;
#pragma unroll
    for (int r = 0; r < 16; ++r)
        if (r >= h2 && (STG == 0 || active))
            __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u2v, v[kout(r)]), ry, 8 * t, 2048 * r, kStAux);
    if constexpr (STG == 1) __syncthreads();  // the second half's P4 -> P5 barrier
}

// ---------------------------------------------------------------------------
// Slot kernel: the same segment transform (bit-identical to ols_os_segment<0>),
// persistent, one workgroup of SLOTS x 256 lanes per CU.  Slot s (waves
// 4s..4s+3) takes its segments one at a time from its XCD eighth's counter
// (workgroup b serves eighth b % 8; one returning device atomic per segment,
// fetched a segment ahead), so the chip-wide window of segments in flight stays
// as compact as the one-shot kernel's dispatch order.  What the shape buys: a
// slot issues the loads of its next segment BEFORE the stores of the current
// one (loads, stores and atomics retire in issue order per wave, so a wave that
// loads after storing waits for its stores), and the two cross-wave phase
// boundaries are slot-local LDS counters (no slot waits for another).
//
// Per-slot LDS: the 34 KB image of ols_os_segment.  Column t of the image is
// owned by lane t of the slot in P1 and P5, so segment i + 1's P1 may start
// while other waves of the slot still run segment i's P5.
template <int SLOTS>
struct OlsSlotShared {
    f2 img[SLOTS][16 * kRow];
    unsigned bar[SLOTS];      // slot barrier arrivals (monotonic)
    long long nxt[SLOTS][2];  // next segment of the slot, double-buffered by parity
    unsigned tk_next, tk_done;  // load tickets (FIFO): at most `tok` waves with segment loads in flight
};

__device__ __forceinline__ void tok_acquire(unsigned* next, const unsigned* done, int tok) {
    if (tok <= 0) return;
    unsigned my = 0;
    if ((threadIdx.x & 63) == 0) my = __hip_atomic_fetch_add(next, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    my = __builtin_amdgcn_readfirstlane(my);
    for (int spin = 0; __builtin_amdgcn_readfirstlane(__hip_atomic_load(done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) +
                               (unsigned)tok <= my && spin < (1 << 22);
         ++spin)
        __builtin_amdgcn_s_sleep(1);
    asm volatile("" ::: "memory");
}
__device__ __forceinline__ void tok_release(unsigned* done, int tok) {
    if (tok <= 0) return;
    if ((threadIdx.x & 63) == 0) __hip_atomic_fetch_add(done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// every wait is bounded (~2^22 x 64 cycles): a protocol error can never hang the GPU
constexpr int kSpinLimit = 1 << 22;

__device__ __forceinline__ unsigned lds_poll(const unsigned* p) {
    return __builtin_amdgcn_readfirstlane(__hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP));
}

// all 4 waves of a slot: this wave's LDS writes are complete before it arrives;
// no LDS access of the caller moves across the call.  false: the bounded wait ran
// out (a protocol error) -- the caller stops, it never goes on with unsynchronised data
__device__ __forceinline__ bool slot_barrier(unsigned* ctr, unsigned target) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if ((threadIdx.x & 63) == 0) __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    int spin = 0;
    for (; lds_poll(ctr) < target && spin < kSpinLimit; ++spin) __builtin_amdgcn_s_sleep(1);
    asm volatile("" ::: "memory");
    return spin < kSpinLimit;
}

// segment loads the compiler does not track (ABL 3): it then places no waits for them, and the
// one explicit wait lets the 16 younger stores of the previous segment stay in flight
typedef unsigned u4s __attribute__((ext_vector_type(4)));
__device__ __forceinline__ u4s rsrc_words(const void* base, unsigned bytes) {
    const unsigned long long a = (unsigned long long)base;
    return u4s{(unsigned)a, (unsigned)(a >> 32) & 0xffffu, bytes, (unsigned)kBufWord3};
}
__device__ __forceinline__ f2 ld_untracked(u4s rs, unsigned voff, unsigned soff) {
    f2 r;
    asm volatile("buffer_load_dwordx2 %0, %1, %2, %3 offen" : "=v"(r) : "v"(voff), "s"(rs), "s"(soff) : "memory");
    return r;
}
// wait for every vector-memory operation but the 16 youngest (the segment's stores, or the
// 16 dropped stores of the prologue); ties the loaded registers so nothing reads them earlier
__device__ __forceinline__ void wait_loads16(f2 (&v)[16]) {
    asm volatile("s_waitcnt vmcnt(16)"
                 : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3]), "+v"(v[4]), "+v"(v[5]), "+v"(v[6]), "+v"(v[7]),
                   "+v"(v[8]), "+v"(v[9]), "+v"(v[10]), "+v"(v[11]), "+v"(v[12]), "+v"(v[13]), "+v"(v[14]),
                   "+v"(v[15])
                 :
                 : "memory");
}

// ABL (lab builds only): 1 HBM traffic only (rows stored as loaded), 2 compute only (no loads, no stores),
// 3 full kernel with untracked segment loads
template <int SLOTS, int ABL = 0>
__global__ void __launch_bounds__(256 * SLOTS, 1)
fir_ols_slot_kernel(const f2* __restrict__ x, const float4* __restrict__ Hs, const float4* __restrict__ tb,
                    f2* __restrict__ y, long long n, long long lo, long long hi, long long q, int h2,
                    unsigned long long* __restrict__ queue, int tok) {
    __shared__ __attribute__((aligned(16))) OlsSlotShared<SLOTS> sh;
    const int slot = threadIdx.x >> 8, t = threadIdx.x & 255;
    const int hi4 = t >> 4, lo4 = t & 15;
    const int xc = blockIdx.x & 7;
    const long long s0 = lo + (long long)xc * q, xe0 = lo + (long long)(xc + 1) * q, xe = xe0 < hi ? xe0 : hi;
    const long long cnt = xe > s0 ? xe - s0 : 0;
    const int V = 4096 - 256 * h2;
    const long long chan = (long long)blockIdx.y * n;
    unsigned long long* qc = queue + 16 * (8 * blockIdx.y + xc);  // [channel][eighth], 128 bytes apart

    const auto rt = __builtin_amdgcn_make_buffer_rsrc((void*)tb, (short)0, kOlsOsTabF4 * 16, kBufWord3);
    const auto rh = __builtin_amdgcn_make_buffer_rsrc((void*)Hs, (short)0, 2048 * 16, kBufWord3);
    f2* img = sh.img[slot];
    f2* col = img + t + (t >> 4);
    f2* r2 = img + hi4 * kRow + lo4;
    unsigned* bar = &sh.bar[slot];
    unsigned nbar = 0;

    if (threadIdx.x < SLOTS) sh.bar[threadIdx.x] = 0;
    if (threadIdx.x == 0) sh.tk_next = sh.tk_done = 0;
    if (t == 0) sh.nxt[slot][0] = (long long)__hip_atomic_fetch_add(qc, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();  // the only workgroup barrier before the tail

    // loop-invariant twiddle bases: column t of W4096, row lo4 of W256 (runtime.cpp ols_build)
    const float4 b0 = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rt, 16 * t, 0, 0));
    const float4 b1 = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rt, 16 * t, 4096, 0));
    const float4 b2 = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rt, 16 * t, 8192, 0));
    f2 Cb[3] = {f2{b0.x, b0.y}, f2{b0.z, b0.w}, f2{b1.x, b1.y}};
    f2 Da[3] = {f2{b1.z, b1.w}, f2{b2.x, b2.y}, f2{b2.z, b2.w}};

    long long k = __builtin_amdgcn_readfirstlane((int)sh.nxt[slot][0]);  // index within the eighth
    if (k < 0) k = cnt;
    unsigned long long fetched = 0;
    if (t == 0) fetched = __hip_atomic_fetch_add(qc, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    f2 v[16];
    if (k < cnt) tok_acquire(&sh.tk_next, &sh.tk_done, tok);
    {
        const bool any = k < cnt;
        const auto rx = __builtin_amdgcn_make_buffer_rsrc((void*)(x + chan + (s0 + (any ? k : 0)) * V - 256 * h2),
                                                          (short)0, any ? 32768 : 0, kBufWord3);
        const u4s rxw = rsrc_words(x + chan + (s0 + (any ? k : 0)) * V - 256 * h2, any ? 32768u : 0u);
#pragma unroll
        for (int r = 0; r < 16; ++r)
            if constexpr (ABL == 2) v[r] = f2{1e-3f * t + r, 1e-9f * (float)k};
            else if constexpr (ABL == 3) v[r] = ld_untracked(rxw, 8 * t, 2048 * r);
            else v[r] = __builtin_bit_cast(f2, __builtin_amdgcn_raw_buffer_load_b64(rx, 8 * t, 2048 * r, 0));
        // 16 dropped stores (empty descriptor): the loop is entered with 16 vector-memory operations younger
        // than the segment loads on every path, so the waits at the top of the loop let a previous
        // segment's stores stay in flight (vmcnt counts loads and stores together, in issue order)
        const auto rz = __builtin_amdgcn_make_buffer_rsrc((void*)y, (short)0, 0, kBufWord3);
#pragma unroll
        for (int r = 0; r < 16; ++r) __builtin_amdgcn_raw_buffer_store_b64(u2v{0u, 0u}, rz, 8 * t, 2048 * r, 0);
        if constexpr (ABL == 3) wait_loads16(v);
    }
    for (long long it = 0; k < cnt; ++it) {  // k uniform over the slot
        const long long base = chan + (s0 + k) * V - 256 * h2;
        if constexpr (ABL == 1) {
#pragma unroll
            for (int r = 0; r < 16; ++r) asm volatile("" ::"v"(v[r]));  // the loads have landed
            tok_release(&sh.tk_done, tok);
            if (t == 0) sh.nxt[slot][(it + 1) & 1] = (long long)fetched;
            if (!slot_barrier(bar, 4 * ++nbar) || !slot_barrier(bar, 4 * ++nbar)) break;
        } else {
        // P1: DFT16 n2 -> k0, * W4096^(t k0) -> (k0, t)
        pdft16<false>(v);
        tok_release(&sh.tk_done, tok);  // the segment's loads have landed
#pragma unroll
        for (int kk = 0; kk < 16; ++kk) col[kk * kRow] = kk == 0 ? v[0] : pmul(v[kout(kk)], tw_pair(Cb, Da, kk));
        if (t == 0) sh.nxt[slot][(it + 1) & 1] = (long long)fetched;  // read after barrier 2
        if (!slot_barrier(bar, 4 * ++nbar)) break;

        // P2, P3, P4 (wave-local rows)
#pragma unroll
        for (int jj = 0; jj < 16; ++jj) v[jj] = r2[17 * jj];
        float4 hq[8];
#pragma unroll
        for (int p = 0; p < 8; ++p) hq[p] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rh, 16 * t, 4096 * p, 0));
        const float4 e0 = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rt, 16 * lo4, 12288, 0));
        const float4 e1 = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rt, 16 * lo4, 12544, 0));
        const float4 e2 = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rt, 16 * lo4, 12800, 0));
        const f2 Eb[3] = {f2{e0.x, e0.y}, f2{e0.z, e0.w}, f2{e1.x, e1.y}};
        const f2 Fa[3] = {f2{e1.z, e1.w}, f2{e2.x, e2.y}, f2{e2.z, e2.w}};
        f2 w2[16];
#pragma unroll
        for (int kk = 1; kk < 16; ++kk) w2[kk] = tw_pair(Eb, Fa, kk);
        pdft16<false>(v);
#pragma unroll
        for (int kk = 0; kk < 16; ++kk) r2[17 * kk] = kk == 0 ? v[0] : pmul(v[kout(kk)], w2[kk]);
        phase_sync<true>();
        {
            f2* r3 = img + hi4 * kRow + 17 * lo4;
#pragma unroll
            for (int jj = 0; jj < 16; ++jj) v[jj] = r3[jj];
            pdft16<false>(v);
            f2 u[16];
#pragma unroll
            for (int p = 0; p < 8; ++p) {
                u[2 * p] = pmul(v[kout(2 * p)], f2{hq[p].x, hq[p].y});
                u[2 * p + 1] = pmul(v[kout(2 * p + 1)], f2{hq[p].z, hq[p].w});
            }
            pdft16<true>(u);
#pragma unroll
            for (int jj = 0; jj < 16; ++jj) r3[jj] = jj == 0 ? u[kout(0)] : pmulc(u[kout(jj)], w2[jj]);
        }
        phase_sync<true>();
#pragma unroll
        for (int jj = 0; jj < 16; ++jj) v[jj] = r2[17 * jj];
        pdft16<true>(v);
#pragma unroll
        for (int kk = 0; kk < 16; ++kk) r2[17 * kk] = v[kout(kk)];
        if (!slot_barrier(bar, 4 * ++nbar)) break;

        // P5: * conj W4096^(t k0), IDFT16 k0 -> n2; row n2 at v[kout(n2)]
#pragma unroll
        for (int i = 0; i < 3; ++i) asm volatile("" : "+v"(Cb[i]), "+v"(Da[i]));
#pragma unroll
        for (int kk = 0; kk < 16; ++kk) v[kk] = kk == 0 ? col[0] : pmulc(col[kk * kRow], tw_pair(Cb, Da, kk));
        pdft16<true>(v);
        }
        // next segment: index, its loads and the fetch of the one after, issued before this segment's stores
        long long kn = __builtin_amdgcn_readfirstlane((int)sh.nxt[slot][(it + 1) & 1]);
        if (kn < 0) kn = cnt;
        if (t == 0 && kn < cnt) fetched = __hip_atomic_fetch_add(qc, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        f2 vn[16];
        if (kn < cnt) tok_acquire(&sh.tk_next, &sh.tk_done, tok);  // released after its P1
        {  // past the last segment: an empty descriptor (the loads return 0 without touching memory)
            const bool more = kn < cnt;
            const auto rx = __builtin_amdgcn_make_buffer_rsrc((void*)(x + chan + (s0 + (more ? kn : k)) * V - 256 * h2),
                                                              (short)0, more ? 32768 : 0, kBufWord3);
            const u4s rxw = rsrc_words(x + chan + (s0 + (more ? kn : k)) * V - 256 * h2, more ? 32768u : 0u);
#pragma unroll
            for (int r = 0; r < 16; ++r)
                if constexpr (ABL == 2) vn[r] = f2{1e-3f * t + r, 1e-9f * (float)kn};
                else if constexpr (ABL == 3) vn[r] = ld_untracked(rxw, 8 * t, 2048 * r);
                else vn[r] = __builtin_bit_cast(f2, __builtin_amdgcn_raw_buffer_load_b64(rx, 8 * t, 2048 * r, 0));
        }

        // halo rows (r < h2) go to an empty descriptor: the store is dropped, every row issues one store
        const auto ry = __builtin_amdgcn_make_buffer_rsrc((void*)(y + base), (short)0, 32768, kBufWord3);
        const auto rz = __builtin_amdgcn_make_buffer_rsrc((void*)(y + base), (short)0, 0, kBufWord3);
        if constexpr (ABL == 2) {
            f2 acc = v[0];
#pragma unroll
            for (int r = 1; r < 16; ++r) acc += v[r];
            if (acc.x == 1.2345e30f) __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u2v, acc), ry, 8 * t, 0, 0);
        } else {
#pragma unroll
            for (int r = 0; r < 16; ++r)
                __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u2v, v[ABL == 1 ? r : kout(r)]), r >= h2 ? ry : rz,
                                                      8 * t, 2048 * r, 0);
        }
        if constexpr (ABL == 3) wait_loads16(vn);
#pragma unroll
        for (int r = 0; r < 16; ++r) v[r] = vn[r];
        k = kn;
    }
    // the last workgroup to finish rewinds the counters for the next launch (stream order)
    __syncthreads();
    if (threadIdx.x == 0) {
        const unsigned long long total = (unsigned long long)gridDim.x * gridDim.y;
        unsigned long long* done = queue + 16 * 8 * gridDim.y;
        if (__hip_atomic_fetch_add(done, 1ull, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) == total - 1) {
            for (unsigned i = 0; i < 8 * gridDim.y; ++i)
                __hip_atomic_store(queue + 16 * i, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(done, 0ull, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}


__device__ unsigned long long g_ols_lab_queue[16 * 8 + 16];

template <int VAR>
__global__ void __launch_bounds__(256, 4)
fir_ols_os_kernel(const f2* __restrict__ x, const float4* __restrict__ Hs, const float4* __restrict__ tb,
                  f2* __restrict__ y, long long n, long long lo, long long hi, long long q, int h2) {
    __shared__ __attribute__((aligned(16))) f2 img[16 * kRow];
    const int xc = blockIdx.x & 7;
    const long long seg = lo + (long long)xc * q + (blockIdx.x >> 3);
    const long long xe = lo + (long long)(xc + 1) * q;
    if (seg >= (xe < hi ? xe : hi)) return;  // uniform over the workgroup
    const int V = 4096 - 256 * h2;
    ols_os_segment<VAR>(x, Hs, tb, y, (long long)blockIdx.y * n + seg * V - 256 * h2, h2, img, threadIdx.x);
}

// Staggered pair (lab): a 512-lane workgroup runs segments s and
// s + 1 of its XCD eighth in two 256-lane halves, the second half's loads issued only
// after the first half's P1 -- at most one segment's loads in flight per workgroup, two
// workgroups (16 waves) per CU, no atomics.
template <int VAR>
__global__ void __launch_bounds__(512, 2)
fir_ols_pair_kernel(const f2* __restrict__ x, const float4* __restrict__ Hs, const float4* __restrict__ tb,
                    f2* __restrict__ y, long long n, long long lo, long long hi, long long q, int h2) {
    __shared__ __attribute__((aligned(16))) f2 img[2][16 * kRow];
    const int xc = blockIdx.x & 7;
    const long long s0 = lo + (long long)xc * q + 2 * (long long)(blockIdx.x >> 3);
    const long long xe0 = lo + (long long)(xc + 1) * q, xe = xe0 < hi ? xe0 : hi;
    if (s0 >= xe) return;  // uniform over the workgroup
    const int V = 4096 - 256 * h2;
    const int half = threadIdx.x >> 8, t = threadIdx.x & 255;  // wave-uniform
    const long long seg = s0 + half;
    const long long base = (long long)blockIdx.y * n + (seg < xe ? seg : s0) * V - 256 * h2;
    if (half == 0) ols_os_segment<VAR, 1>(x, Hs, tb, y, base, h2, img[0], t, true);
    else ols_os_segment<VAR, 2>(x, Hs, tb, y, base, h2, img[1], t, seg < xe);
}

// Trio kernel (lab): one 768-lane workgroup per CU, three 256-lane slots, each
// running its segments through three stages; stages end at workgroup barriers
// (plain s_barrier, LDS waits only: loads and stores stay in flight):
//   S0  P5 and the stores of the current segment, then P1 of the next one
//       (lane-owned columns: P5's reads and P1's writes touch only the lane's own)
//   S1  P2 and the forward half of P3 (DFT16 n0 -> k2, * H)
//   S2  the inverse half of P3 and P4; the loads of the segment after are issued
// Slot s runs stage (t - s + 2) mod 3 at tick t (none before tick s): each tick
// one slot of the CU has segment loads in flight and one stores, while all 12
// waves compute.  Segments come from a per-XCD-eighth counter (one returning
// atomic per segment, fetched a stage before its loads): the segments a CU's
// XCD has in flight stay neighbours, as in the one-shot dispatch order.
struct OlsTrioShared {
    f2 img[3][16 * kRow];
    float4 hq[8][256];  // spectrum slices of P3, [k-pair][lane] (shared by the slots)
    int nidx[3];
};
__device__ unsigned long long g_ols_trio_q[2][8 * 16];

__device__ __forceinline__ void trio_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

__device__ __forceinline__ long long pick3(const long long (&a)[3], int s) { return s == 0 ? a[0] : s == 1 ? a[1] : a[2]; }

// ABL: 0 full, 1 HBM traffic only (rows stored as loaded), 2 compute only (no loads, stores dropped)
template <int ABL>
__global__ void __launch_bounds__(768, 1)
fir_ols_trio_kernel(const f2* __restrict__ x, const float4* __restrict__ Hs, const float4* __restrict__ tb,
                    f2* __restrict__ y, long long lo, long long hi, long long q, int h2, int par) {
    __shared__ __attribute__((aligned(16))) OlsTrioShared sh;
    const int slot = __builtin_amdgcn_readfirstlane(threadIdx.x >> 8);
    const int t = threadIdx.x & 255, hi4 = t >> 4, lo4 = t & 15;
    const int xc = blockIdx.x & 7, J = gridDim.x >> 3, jb = blockIdx.x >> 3;
    const long long s0 = lo + (long long)xc * q, se0 = s0 + q, se = se0 < hi ? se0 : hi;
    const int cnt = se > s0 ? (int)(se - s0) : 0;
    const int V = 4096 - 256 * h2;
    unsigned long long* ctr = &g_ols_trio_q[par][16 * xc];
    if (blockIdx.x == 0 && threadIdx.x < 8)  // the next launch's counters (the previous launch used them)
        __hip_atomic_store(&g_ols_trio_q[par ^ 1][16 * threadIdx.x], 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);

    const auto rt = __builtin_amdgcn_make_buffer_rsrc((void*)tb, (short)0, kOlsOsTabF4 * 16, kBufWord3);
    const auto rh = __builtin_amdgcn_make_buffer_rsrc((void*)Hs, (short)0, 2048 * 16, kBufWord3);
    const float4 b0 = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rt, 16 * t, 0, 0));
    const float4 b1 = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rt, 16 * t, 4096, 0));
    const float4 b2 = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rt, 16 * t, 8192, 0));
    f2 Cb[3] = {f2{b0.x, b0.y}, f2{b0.z, b0.w}, f2{b1.x, b1.y}};
    f2 Da[3] = {f2{b1.z, b1.w}, f2{b2.x, b2.y}, f2{b2.z, b2.w}};
    f2* img = sh.img[slot];
    f2* col = img + t + (t >> 4);
    f2* r2 = img + hi4 * kRow + lo4;
    f2* r3 = img + hi4 * kRow + 17 * lo4;

    // every wave tracks all three slots (uniform): current and next segment (cnt = none) and the
    // stage each slot runs in the current tick (-1 before its first tick; then 2, 0, 1, 2, 0, ...)
    int cur[3], nxt[3], ph[3];
#pragma unroll
    for (int s = 0; s < 3; ++s) {
        cur[s] = cnt;
        nxt[s] = 3 * jb + s < cnt ? 3 * jb + s : cnt;
        ph[s] = s == 0 ? 2 : -1;
    }
    const int myc0 = 0;
    (void)myc0;
    auto mine = [&](const int (&a)[3]) { return slot == 0 ? a[0] : slot == 1 ? a[1] : a[2]; };
    // a segment's buffer descriptors; none (num_records 0: loads return 0, stores are dropped) past the eighth
    auto seg_rsrc = [&](const f2* base, int k) {
        const bool ok = (unsigned)k < (unsigned)cnt;
        return __builtin_amdgcn_make_buffer_rsrc((void*)(base + (s0 + (ok ? k : 0)) * V - 256 * h2), (short)0,
                                                 ok ? 32768 : 0, kBufWord3);
    };
    // loop invariants: the spectrum slices in LDS, W256^(lo4 k) in registers
    for (int i = threadIdx.x; i < 8 * 256; i += 768)
        sh.hq[i >> 8][i & 255] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rh, 16 * (i & 255), 4096 * (i >> 8), 0));
    f2 w2[16];
    {
        const float4 e0 = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rt, 16 * lo4, 12288, 0));
        const float4 e1 = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rt, 16 * lo4, 12544, 0));
        const float4 e2 = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rt, 16 * lo4, 12800, 0));
        const f2 Eb[3] = {f2{e0.x, e0.y}, f2{e0.z, e0.w}, f2{e1.x, e1.y}};
        const f2 Fa[3] = {f2{e1.z, e1.w}, f2{e2.x, e2.y}, f2{e2.z, e2.w}};
        w2[0] = f2{1.0f, 0.0f};
#pragma unroll
        for (int k = 1; k < 16; ++k) w2[k] = tw_pair(Eb, Fa, k);
    }
    __syncthreads();
    f2 v[16], vn[16], u[16];
    unsigned long long got = 0;

    // S0: P5 and the stores of the current segment, then P1 of the next one (its loads were issued in S2)
    auto stage0 = [&]() {
        const auto ry = seg_rsrc(y, mine(cur));
        if constexpr (ABL == 1) {
            const auto rz = __builtin_amdgcn_make_buffer_rsrc((void*)y, (short)0, 0, kBufWord3);
#pragma unroll
            for (int r = 0; r < 16; ++r)
                __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u2v, v[r]), r >= h2 ? ry : rz, 8 * t, 2048 * r, 2);
#pragma unroll
            for (int r = 0; r < 16; ++r) v[r] = vn[r];
            return;
        }
        // P5: * conj W4096^(t k0), IDFT16 k0 -> n2
#pragma unroll
        for (int i = 0; i < 3; ++i) asm volatile("" : "+v"(Cb[i]), "+v"(Da[i]));
#pragma unroll
        for (int k = 0; k < 16; ++k) v[k] = k == 0 ? col[0] : pmulc(col[k * kRow], tw_pair(Cb, Da, k));
        pdft16<true>(v);
        if constexpr (ABL == 2) {
            f2 acc = v[0];
#pragma unroll
            for (int r = 1; r < 16; ++r) acc += v[r];
            if (acc.x == 1.2345e30f) __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u2v, acc), ry, 8 * t, 0, 0);
        } else {
            // every row issues one store (halo rows to an empty descriptor: dropped), so that the
            // count of memory operations younger than the next segment's loads is exact
            const auto rz = __builtin_amdgcn_make_buffer_rsrc((void*)y, (short)0, 0, kBufWord3);
#pragma unroll
            for (int r = 0; r < 16; ++r)
                __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u2v, v[kout(r)]), r >= h2 ? ry : rz, 8 * t, 2048 * r, 2);
        }
        // P1 of the next segment: DFT16 n2 -> k0, * W4096^(t k0) -> (k0, t)
#pragma unroll
        for (int r = 0; r < 16; ++r) v[r] = vn[r];
        pdft16<false>(v);
#pragma unroll
        for (int k = 0; k < 16; ++k) col[k * kRow] = k == 0 ? v[0] : pmul(v[kout(k)], tw_pair(Cb, Da, k));
    };
    // S1: P2 and the forward half of P3; the index of the segment after the next one
    auto stage1 = [&]() {
        if (t == 0 && mine(nxt) < cnt) got = __hip_atomic_fetch_add(ctr, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if constexpr (ABL == 1) return;
        // P2: lane (k0 = hi4, n0 = lo4): DFT16 n1 -> k1, * W256^(n0 k1)
#pragma unroll
        for (int j = 0; j < 16; ++j) v[j] = r2[17 * j];
        pdft16<false>(v);
#pragma unroll
        for (int k = 0; k < 16; ++k) r2[17 * k] = k == 0 ? v[0] : pmul(v[kout(k)], w2[k]);
        phase_sync<true>();
        // P3, forward half: DFT16 n0 -> k2, * H
#pragma unroll
        for (int j = 0; j < 16; ++j) v[j] = r3[j];
        pdft16<false>(v);
#pragma unroll
        for (int p = 0; p < 8; ++p) {
            const float4 h = sh.hq[p][t];
            u[2 * p] = pmul(v[kout(2 * p)], f2{h.x, h.y});
            u[2 * p + 1] = pmul(v[kout(2 * p + 1)], f2{h.z, h.w});
        }
    };
    // S2: publish the fetched index, issue the loads of the next segment, then the inverse half of
    // P3 and P4 of the current one
    auto stage2 = [&]() {
        const int mn = mine(nxt);
        if (t == 0) sh.nidx[slot] = mn < cnt && got < (unsigned long long)cnt ? (int)min((unsigned long long)cnt, 3ull * J + got) : cnt;
        const auto rx = seg_rsrc(x, mn);
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            if constexpr (ABL == 2) vn[r] = f2{1e-3f * t + r, 1e-9f * (float)mn};
            else vn[r] = __builtin_bit_cast(f2, __builtin_amdgcn_raw_buffer_load_b64(rx, 8 * t, 2048 * r, 0));
        }
        if constexpr (ABL == 1) return;
        pdft16<true>(u);
#pragma unroll
        for (int j = 0; j < 16; ++j) r3[j] = j == 0 ? u[kout(0)] : pmulc(u[kout(j)], w2[j]);
        phase_sync<true>();
        // P4: IDFT16 k1 -> n1
#pragma unroll
        for (int j = 0; j < 16; ++j) v[j] = r2[17 * j];
        pdft16<true>(v);
#pragma unroll
        for (int k = 0; k < 16; ++k) r2[17 * k] = v[kout(k)];
    };

    // a tick ends for every wave at one barrier; every slot that ran S0 in it moves on (the next
    // segment becomes current, the published index next)
    const int tick_cap = 3 * cnt + 16;  // a stale counter can only end the loop early, never hang it
    int tick = 0;
    auto end_tick = [&]() -> bool {
        trio_barrier();
        bool live = false;
#pragma unroll
        for (int s = 0; s < 3; ++s) {
            if (ph[s] == 0) {
                cur[s] = nxt[s];
                nxt[s] = nxt[s] < cnt ? __builtin_amdgcn_readfirstlane(sh.nidx[s]) : cnt;
            }
            ph[s] = ph[s] < 0 ? (tick + 1 == s ? 2 : -1) : (ph[s] == 2 ? 0 : ph[s] + 1);
            live = live || ph[s] < 0 || cur[s] < cnt || nxt[s] < cnt;
        }
        ++tick;
        return live && tick < tick_cap;
    };
    bool go = true;
    for (int i = 0; i < slot && go; ++i) go = end_tick();
    while (go) {
        stage2();
        if (!(go = end_tick())) break;
        stage0();
        if (!(go = end_tick())) break;
        stage1();
        go = end_tick();
    }
}

// Quad kernel (lab): the trio's schedule with four 256-lane slots (16 waves per CU, as
// many as the one-shot kernel) and four stages per segment:
//   S0  P1 (its loads were issued two stages earlier); the queue index of the segment
//       after the next
//   S1  P2 and the forward half of P3 (spectrum slice and W256 bases from L2); the index
//       is published in LDS
//   S2  loads of the next segment, the inverse half of P3, P4
//   S3  P5 and the stores
// Slot s runs stage (t - s + 2) mod 4 at tick t.  Memory operations per slot in issue
// order: S2 loads, S3 stores, S0 atomic, S1 table loads -- the only waits are P1's on
// its loads (the 16 stores stay in flight) and S1's on its table loads (which also
// drains the stores of two stages before).
struct OlsQuadShared {
    f2 img[4][16 * kRow];
    int nidx[4];
};
__device__ unsigned int g_ols_quad_q[2][8 * 32];

template <int ABL>
__global__ void __launch_bounds__(1024, 1)
fir_ols_quad_kernel(const f2* __restrict__ x, const float4* __restrict__ Hs, const float4* __restrict__ tb,
                    f2* __restrict__ y, long long lo, long long hi, long long q, int h2, int par) {
    __shared__ __attribute__((aligned(16))) OlsQuadShared sh;
    constexpr int NS = 4;
    const int slot = __builtin_amdgcn_readfirstlane(threadIdx.x >> 8);
    const int t = threadIdx.x & 255, hi4 = t >> 4, lo4 = t & 15;
    const int xc = blockIdx.x & 7, J = gridDim.x >> 3, jb = blockIdx.x >> 3;
    const long long s0 = lo + (long long)xc * q, se0 = s0 + q, se = se0 < hi ? se0 : hi;
    const int cnt = se > s0 ? (int)(se - s0) : 0;
    const int V = 4096 - 256 * h2;
    unsigned int* ctr = &g_ols_quad_q[par][32 * xc];
    if (blockIdx.x == 0 && threadIdx.x < 8)  // the next launch's counters (the previous launch used them)
        __hip_atomic_store(&g_ols_quad_q[par ^ 1][32 * threadIdx.x], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);

    const auto rt = __builtin_amdgcn_make_buffer_rsrc((void*)tb, (short)0, kOlsOsTabF4 * 16, kBufWord3);
    const auto rh = __builtin_amdgcn_make_buffer_rsrc((void*)Hs, (short)0, 2048 * 16, kBufWord3);
    const auto rz = __builtin_amdgcn_make_buffer_rsrc((void*)y, (short)0, 0, kBufWord3);
    const float4 b0 = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rt, 16 * t, 0, 0));
    const float4 b1 = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rt, 16 * t, 4096, 0));
    const float4 b2 = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rt, 16 * t, 8192, 0));
    f2 Cb[3] = {f2{b0.x, b0.y}, f2{b0.z, b0.w}, f2{b1.x, b1.y}};
    f2 Da[3] = {f2{b1.z, b1.w}, f2{b2.x, b2.y}, f2{b2.z, b2.w}};
    f2* img = sh.img[slot];
    f2* col = img + t + (t >> 4);
    f2* r2 = img + hi4 * kRow + lo4;
    f2* r3 = img + hi4 * kRow + 17 * lo4;

    // every wave tracks all slots (uniform): current and next segment (cnt = none) and the stage
    // each slot runs in the current tick (-1 before its first tick; then 2, 3, 0, 1, 2, ...)
    int cur[NS], nxt[NS], ph[NS];
#pragma unroll
    for (int s = 0; s < NS; ++s) {
        cur[s] = cnt;
        nxt[s] = NS * jb + s < cnt ? NS * jb + s : cnt;
        ph[s] = s == 0 ? 2 : -1;
    }
    auto mine = [&](const int (&a)[NS]) { return slot == 0 ? a[0] : slot == 1 ? a[1] : slot == 2 ? a[2] : a[3]; };
    auto seg_rsrc = [&](const f2* base, int k) {
        const bool ok = (unsigned)k < (unsigned)cnt;
        return __builtin_amdgcn_make_buffer_rsrc((void*)(base + (s0 + (ok ? k : 0)) * V - 256 * h2), (short)0,
                                                 ok ? 32768 : 0, kBufWord3);
    };
    f2 v[16], vn[16], u[16], Eb[3], Fa[3];
    float4 hq[8], e0, e1, e2;
    unsigned int got = 0;

    auto stage0 = [&]() {  // P1: DFT16 n2 -> k0, * W4096^(t k0) -> (k0, t); the queue fetch; S1's tables
#pragma unroll
        for (int p = 0; p < 8; ++p)
            hq[p] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rh, 16 * t, 4096 * p, 0));
        e0 = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rt, 16 * lo4, 12288, 0));
        e1 = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rt, 16 * lo4, 12544, 0));
        e2 = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rt, 16 * lo4, 12800, 0));
#pragma unroll
        for (int r = 0; r < 16; ++r) v[r] = vn[r];
        if constexpr (ABL == 1) return;
        pdft16<false>(v);
#pragma unroll
        for (int k = 0; k < 16; ++k) col[k * kRow] = k == 0 ? v[0] : pmul(v[kout(k)], tw_pair(Cb, Da, k));
    };
    auto stage1 = [&]() {  // P2, P3 forward half; publish the fetched index
        Eb[0] = f2{e0.x, e0.y}; Eb[1] = f2{e0.z, e0.w}; Eb[2] = f2{e1.x, e1.y};
        Fa[0] = f2{e1.z, e1.w}; Fa[1] = f2{e2.x, e2.y}; Fa[2] = f2{e2.z, e2.w};
        if constexpr (ABL == 1) {
#pragma unroll
            for (int j = 0; j < 16; ++j) u[j] = f2{0.0f, 0.0f};
            return;
        }
        f2 w2[16];  // W256^(lo4 k); recomputed in S2 (the bases, not the 15 products, live across)
        // P2: lane (k0 = hi4, n0 = lo4): DFT16 n1 -> k1, * W256^(n0 k1)
#pragma unroll
        for (int j = 0; j < 16; ++j) v[j] = r2[17 * j];
#pragma unroll
        for (int k = 1; k < 16; ++k) w2[k] = tw_pair(Eb, Fa, k);
        pdft16<false>(v);
#pragma unroll
        for (int k = 0; k < 16; ++k) r2[17 * k] = k == 0 ? v[0] : pmul(v[kout(k)], w2[k]);
        phase_sync<true>();
        // P3, forward half: DFT16 n0 -> k2, * H
#pragma unroll
        for (int j = 0; j < 16; ++j) v[j] = r3[j];
        pdft16<false>(v);
#pragma unroll
        for (int p = 0; p < 8; ++p) {
            u[2 * p] = pmul(v[kout(2 * p)], f2{hq[p].x, hq[p].y});
            u[2 * p + 1] = pmul(v[kout(2 * p + 1)], f2{hq[p].z, hq[p].w});
        }
    };
    auto stage2 = [&]() {  // loads of the next segment; P3 inverse half, P4
        const int mn = mine(nxt);
        // the queue index of the segment after: issued before the loads, so that S3 can wait for it
        // while the loads stay in flight
        if (t == 0 && mn < cnt) got = __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const auto rx = seg_rsrc(x, mn);
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            if constexpr (ABL == 2) vn[r] = f2{1e-3f * t + r, 1e-9f * (float)mn};
            else vn[r] = __builtin_bit_cast(f2, __builtin_amdgcn_raw_buffer_load_b64(rx, 8 * t, 2048 * r, 0));
        }
        if constexpr (ABL == 1) return;
        pdft16<true>(u);
#pragma unroll
        for (int j = 0; j < 16; ++j) r3[j] = j == 0 ? u[kout(0)] : pmulc(u[kout(j)], tw_pair(Eb, Fa, j));
        phase_sync<true>();
#pragma unroll
        for (int j = 0; j < 16; ++j) v[j] = r2[17 * j];
        pdft16<true>(v);
#pragma unroll
        for (int k = 0; k < 16; ++k) r2[17 * k] = v[kout(k)];
    };
    auto stage3 = [&]() {  // publish the fetched index; P5 and the stores (every row issues one: halo rows to an empty descriptor)
        // dynamic indices follow the static round; anything past the eighth reads as none
        if (t == 0) sh.nidx[slot] = mine(nxt) < cnt && got < (unsigned)cnt ? (int)min((unsigned)cnt, (unsigned)(NS * J) + got) : cnt;
        const auto ry = seg_rsrc(y, mine(cur));
        if constexpr (ABL != 1) {
#pragma unroll
            for (int i = 0; i < 3; ++i) asm volatile("" : "+v"(Cb[i]), "+v"(Da[i]));
#pragma unroll
            for (int k = 0; k < 16; ++k) v[k] = k == 0 ? col[0] : pmulc(col[k * kRow], tw_pair(Cb, Da, k));
            pdft16<true>(v);
        }
        if constexpr (ABL == 2) {
            f2 acc = v[0];
#pragma unroll
            for (int r = 1; r < 16; ++r) acc += v[r];
            if (acc.x == 1.2345e30f) __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u2v, acc), ry, 8 * t, 0, 0);
        } else {
#pragma unroll
            for (int r = 0; r < 16; ++r)
                __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u2v, v[ABL == 1 ? r : kout(r)]), r >= h2 ? ry : rz,
                                                      8 * t, 2048 * r, 2);
        }
    };

    const int tick_cap = 4 * cnt + 32;  // a stale counter can only end the loop early, never hang it
    int tick = 0;
    auto end_tick = [&]() -> bool {
        trio_barrier();
        bool live = false;
#pragma unroll
        for (int s = 0; s < NS; ++s) {
            if (ph[s] == 3) {  // slot s finished its segment: the next one becomes current
                cur[s] = nxt[s];
                nxt[s] = nxt[s] < cnt ? __builtin_amdgcn_readfirstlane(sh.nidx[s]) : cnt;
            }
            ph[s] = ph[s] < 0 ? (tick + 1 == s ? 2 : -1) : (ph[s] == 3 ? 0 : ph[s] + 1);
            live = live || ph[s] < 0 || cur[s] < cnt || nxt[s] < cnt;
        }
        ++tick;
        return live && tick < tick_cap;
    };
    bool go = true;
    for (int i = 0; i < slot && go; ++i) go = end_tick();
    while (go) {
        stage2();
        if (!(go = end_tick())) break;
        stage3();
        if (!(go = end_tick())) break;
        stage0();
        if (!(go = end_tick())) break;
        stage1();
        go = end_tick();
    }
}

// Queue kernel (lab): persistent 256-lane workgroups, three per CU, each running the
// one-shot kernel's segment transform (bit-identical) on a queue of segments with the
// next segment's loads in flight across the current one's P2-P5 (issued right after
// P1, into registers) -- no coupling between workgroups, so each CU's compute stays
// free-running, while a segment's loads are outstanding only for their latency rather
// than for a whole workgroup lifetime.  Segments from a per-XCD-eighth counter (one
// returning atomic per segment, issued before the loads so that waiting for it never
// waits for them); the index is published in LDS before the P4 -> P5 barrier.
__device__ unsigned int g_ols_queue_q[2][8 * 32];

template <int ABL>
__global__ void __launch_bounds__(256, 3)
fir_ols_queue_kernel(const f2* __restrict__ x, const float4* __restrict__ Hs, const float4* __restrict__ tb,
                     f2* __restrict__ y, long long lo, long long hi, long long q, int h2, int par) {
    __shared__ __attribute__((aligned(16))) f2 img[16 * kRow];
    __shared__ int nidx;
    const int t = threadIdx.x, hi4 = t >> 4, lo4 = t & 15;
    const int xc = blockIdx.x & 7, J = gridDim.x >> 3, jb = blockIdx.x >> 3;
    const long long s0 = lo + (long long)xc * q, se0 = s0 + q, se = se0 < hi ? se0 : hi;
    const int cnt = se > s0 ? (int)(se - s0) : 0;
    const int V = 4096 - 256 * h2;
    unsigned int* ctr = &g_ols_queue_q[par][32 * xc];
    if (blockIdx.x == 0 && t < 8)  // the next launch's counters (the previous launch used them)
        __hip_atomic_store(&g_ols_queue_q[par ^ 1][32 * t], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const auto rt = __builtin_amdgcn_make_buffer_rsrc((void*)tb, (short)0, kOlsOsTabF4 * 16, kBufWord3);
    const auto rh = __builtin_amdgcn_make_buffer_rsrc((void*)Hs, (short)0, 2048 * 16, kBufWord3);
    const auto rz = __builtin_amdgcn_make_buffer_rsrc((void*)y, (short)0, 0, kBufWord3);
    auto seg_rsrc = [&](const f2* base, int k) {  // none past the eighth: loads return 0, stores drop
        const bool ok = (unsigned)k < (unsigned)cnt;
        return __builtin_amdgcn_make_buffer_rsrc((void*)(base + (s0 + (ok ? k : 0)) * V - 256 * h2), (short)0,
                                                 ok ? 32768 : 0, kBufWord3);
    };
    auto next_index = [&](unsigned got) -> int {  // dynamic indices follow the static first round
        return got < (unsigned)cnt ? (int)min((unsigned)cnt, (unsigned)J + got) : cnt;
    };
    const float4 b0 = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rt, 16 * t, 0, 0));
    const float4 b1 = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rt, 16 * t, 4096, 0));
    const float4 b2 = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rt, 16 * t, 8192, 0));
    f2 Cb[3] = {f2{b0.x, b0.y}, f2{b0.z, b0.w}, f2{b1.x, b1.y}};
    f2 Da[3] = {f2{b1.z, b1.w}, f2{b2.x, b2.y}, f2{b2.z, b2.w}};
    f2* col = img + t + (t >> 4);
    f2* r2 = img + hi4 * kRow + lo4;
    f2* r3 = img + hi4 * kRow + 17 * lo4;

    int k = jb < cnt ? jb : cnt;  // uniform
    if (k >= cnt) return;
    unsigned got = 0;
    if (t == 0) got = __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    f2 v[16], vn[16];
    {
        const auto rx = seg_rsrc(x, k);
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            if constexpr (ABL == 2) v[r] = f2{1e-3f * t + r, 1e-9f * (float)k};
            else v[r] = __builtin_bit_cast(f2, __builtin_amdgcn_raw_buffer_load_b64(rx, 8 * t, 2048 * r, 0));
        }
    }
    // 16 dropped stores (empty descriptor): the loop is entered with 16 memory operations younger
    // than the segment's loads on every path, so P1's wait for them is vmcnt(16) on both
#pragma unroll
    for (int r = 0; r < 16; ++r) __builtin_amdgcn_raw_buffer_store_b64(u2v{0u, 0u}, rz, 8 * t, 2048 * r, 0);
    if (t == 0) nidx = next_index(got);
    trio_barrier();
    int kn = __builtin_amdgcn_readfirstlane(nidx);
    for (int it = 0; it <= cnt; ++it) {  // bounded: one segment per iteration
        // P1: DFT16 n2 -> k0, * W4096^(t k0) -> (k0, t)
        if constexpr (ABL != 1) {
            pdft16<false>(v);
#pragma unroll
            for (int kk = 0; kk < 16; ++kk) col[kk * kRow] = kk == 0 ? v[0] : pmul(v[kout(kk)], tw_pair(Cb, Da, kk));
        }
        // P2/P3's tables, the queue index of the segment after the next, then the next segment's
        // loads -- in this order, so that waiting for the tables or the index never waits for them
        float4 hq[8];
#pragma unroll
        for (int p = 0; p < 8; ++p) hq[p] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rh, 16 * t, 4096 * p, 0));
        const float4 e0 = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rt, 16 * lo4, 12288, 0));
        const float4 e1 = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rt, 16 * lo4, 12544, 0));
        const float4 e2 = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rt, 16 * lo4, 12800, 0));
        if (t == 0 && kn < cnt) got = __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        {
            const auto rx = seg_rsrc(x, kn);
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                if constexpr (ABL == 2) vn[r] = f2{1e-3f * t + r, 1e-9f * (float)kn};
                else vn[r] = __builtin_bit_cast(f2, __builtin_amdgcn_raw_buffer_load_b64(rx, 8 * t, 2048 * r, 0));
            }
        }
        if constexpr (ABL != 1) {
            trio_barrier();
            // P2: lane (k0 = hi4, n0 = lo4): DFT16 n1 -> k1, * W256^(n0 k1)
#pragma unroll
            for (int j = 0; j < 16; ++j) v[j] = r2[17 * j];
            const f2 Eb[3] = {f2{e0.x, e0.y}, f2{e0.z, e0.w}, f2{e1.x, e1.y}};
            const f2 Fa[3] = {f2{e1.z, e1.w}, f2{e2.x, e2.y}, f2{e2.z, e2.w}};
            f2 w2[16];
#pragma unroll
            for (int kk = 1; kk < 16; ++kk) w2[kk] = tw_pair(Eb, Fa, kk);
            pdft16<false>(v);
#pragma unroll
            for (int kk = 0; kk < 16; ++kk) r2[17 * kk] = kk == 0 ? v[0] : pmul(v[kout(kk)], w2[kk]);
            phase_sync<true>();
            // P3: DFT16 n0 -> k2, * H, IDFT16 k2 -> n0, * conj W256^(k1 n0)
            {
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
            phase_sync<true>();
            // P4: IDFT16 k1 -> n1
#pragma unroll
            for (int j = 0; j < 16; ++j) v[j] = r2[17 * j];
            pdft16<true>(v);
#pragma unroll
            for (int kk = 0; kk < 16; ++kk) r2[17 * kk] = v[kout(kk)];
        }
        if (t == 0) nidx = kn < cnt ? next_index(got) : cnt;  // read after the barrier below
        trio_barrier();
        const int knn = __builtin_amdgcn_readfirstlane(nidx);
        // P5: * conj W4096^(t k0), IDFT16 k0 -> n2, and the stores
        const auto ry = seg_rsrc(y, k);
        if constexpr (ABL != 1) {
#pragma unroll
            for (int i = 0; i < 3; ++i) asm volatile("" : "+v"(Cb[i]), "+v"(Da[i]));
#pragma unroll
            for (int kk = 0; kk < 16; ++kk) v[kk] = kk == 0 ? col[0] : pmulc(col[kk * kRow], tw_pair(Cb, Da, kk));
            pdft16<true>(v);
        }
        if constexpr (ABL == 2) {
            f2 acc = v[0];
#pragma unroll
            for (int r = 1; r < 16; ++r) acc += v[r];
            if (acc.x == 1.2345e30f) __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u2v, acc), ry, 8 * t, 0, 0);
        } else {
#pragma unroll
            for (int r = 0; r < 16; ++r)
                __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u2v, v[ABL == 1 ? r : kout(r)]), r >= h2 ? ry : rz,
                                                      8 * t, 2048 * r, 2);
        }
        if (kn >= cnt) break;  // uniform
#pragma unroll
        for (int r = 0; r < 16; ++r) v[r] = vn[r];
        k = kn;
        kn = knn;
        // P1 of the next segment rewrites the columns P5 just read: lane-owned, no barrier
    }
}

static int g_lab_variant = 0, g_lab_lds = 0, g_lab_tok = 0;
extern "C" __attribute__((visibility("default"))) void sdsp_lab_set_ols_variant(int v, int lds, int tok) {
    g_lab_variant = v;
    g_lab_lds = lds;
    g_lab_tok = v >= 256 && tok > 1 ? tok : 0;  // slot kernel: waves with loads in flight per CU (chunk field)
}
__global__ void ols_hwid_probe_kernel(unsigned int* out) {
    unsigned int xcc, hw;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    if (threadIdx.x == 0) {
        out[2 * blockIdx.x] = xcc;
        out[2 * blockIdx.x + 1] = hw;
    }
}
extern "C" __attribute__((visibility("default"))) int sdsp_lab_hwid_probe(unsigned int* d_out, int blocks) {
    hipLaunchKernelGGL(ols_hwid_probe_kernel, dim3(blocks), dim3(64), 40000, 0, d_out);
    return hipDeviceSynchronize() == hipSuccess ? 0 : 1;
}
#define SDSP_LAB_VARIANTS(X) X(1) X(2) X(3) X(4) X(8) X(16) X(24) X(12) X(20) X(28) X(32) X(36) X(48) X(80) X(88) X(84) X(92) X(128) X(132)

hipError_t launch_fir_ols_os(const OlsPlan& p, const void* x, void* y, size_t n, size_t channels, hipStream_t s,
                             long long lo, long long hi) {
    if (hi <= lo) return hipSuccess;
    if (p.halo_rows < 1 || p.halo_rows > 15) return hipErrorInvalidValue;
    const long long q = (hi - lo + 7) / 8;
    const dim3 grid((unsigned)(8 * q), (unsigned)channels);
    if (g_lab_variant >= 2048 && g_lab_variant < 2051) {  // queue kernel (+ ablation); lds field = workgroups per XCD
        static int par = 0;
        int cus = 256;
        (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
        const int J = g_lab_lds > 0 ? g_lab_lds : 3 * cus / 8;
        if (channels != 1) return hipErrorInvalidValue;
        const dim3 gq(8 * J);
        const int abl = g_lab_variant - 2048;
        if (abl == 0)
            hipLaunchKernelGGL(fir_ols_queue_kernel<0>, gq, dim3(256), 0, s, (const f2*)x, (const float4*)p.d_pkt,
                               (const float4*)p.d_ostab, (f2*)y, lo, hi, q, p.halo_rows, par);
        else if (abl == 1)
            hipLaunchKernelGGL(fir_ols_queue_kernel<1>, gq, dim3(256), 0, s, (const f2*)x, (const float4*)p.d_pkt,
                               (const float4*)p.d_ostab, (f2*)y, lo, hi, q, p.halo_rows, par);
        else
            hipLaunchKernelGGL(fir_ols_queue_kernel<2>, gq, dim3(256), 0, s, (const f2*)x, (const float4*)p.d_pkt,
                               (const float4*)p.d_ostab, (f2*)y, lo, hi, q, p.halo_rows, par);
        par ^= 1;
        return hipGetLastError();
    }
    if (g_lab_variant >= 1028 && g_lab_variant < 1031) {  // quad kernel (+ ablation)
        static int par = 0;
        int cus = 256;
        (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
        const int J = g_lab_lds > 0 ? g_lab_lds : cus / 8;
        if (channels != 1) return hipErrorInvalidValue;
        const dim3 g4(8 * J);
        const int abl = g_lab_variant - 1028;
        if (abl == 0)
            hipLaunchKernelGGL(fir_ols_quad_kernel<0>, g4, dim3(1024), 0, s, (const f2*)x, (const float4*)p.d_pkt,
                               (const float4*)p.d_ostab, (f2*)y, lo, hi, q, p.halo_rows, par);
        else if (abl == 1)
            hipLaunchKernelGGL(fir_ols_quad_kernel<1>, g4, dim3(1024), 0, s, (const f2*)x, (const float4*)p.d_pkt,
                               (const float4*)p.d_ostab, (f2*)y, lo, hi, q, p.halo_rows, par);
        else
            hipLaunchKernelGGL(fir_ols_quad_kernel<2>, g4, dim3(1024), 0, s, (const f2*)x, (const float4*)p.d_pkt,
                               (const float4*)p.d_ostab, (f2*)y, lo, hi, q, p.halo_rows, par);
        par ^= 1;
        return hipGetLastError();
    }
    if (g_lab_variant >= 1024 && g_lab_variant < 1027) {  // trio kernel (+ ablation)
        static int par = 0;
        int cus = 256;
        (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
        const int J = g_lab_lds > 0 ? g_lab_lds : cus / 8;
        if (channels != 1) return hipErrorInvalidValue;
        const dim3 g3(8 * J);
        const int abl = g_lab_variant - 1024;
        if (abl == 0)
            hipLaunchKernelGGL(fir_ols_trio_kernel<0>, g3, dim3(768), 0, s, (const f2*)x, (const float4*)p.d_pkt,
                               (const float4*)p.d_ostab, (f2*)y, lo, hi, q, p.halo_rows, par);
        else if (abl == 1)
            hipLaunchKernelGGL(fir_ols_trio_kernel<1>, g3, dim3(768), 0, s, (const f2*)x, (const float4*)p.d_pkt,
                               (const float4*)p.d_ostab, (f2*)y, lo, hi, q, p.halo_rows, par);
        else
            hipLaunchKernelGGL(fir_ols_trio_kernel<2>, g3, dim3(768), 0, s, (const f2*)x, (const float4*)p.d_pkt,
                               (const float4*)p.d_ostab, (f2*)y, lo, hi, q, p.halo_rows, par);
        par ^= 1;
        return hipGetLastError();
    }
    if (g_lab_variant == 512) {  // staggered pair kernel
        const long long q2 = (q + 1) / 2;
        hipLaunchKernelGGL(fir_ols_pair_kernel<0>, dim3((unsigned)(8 * q2), (unsigned)channels), dim3(512), 0, s,
                           (const f2*)x, (const float4*)p.d_pkt, (const float4*)p.d_ostab, (f2*)y, (long long)n, lo,
                           hi, q, p.halo_rows);
        return hipGetLastError();
    }
    if (g_lab_variant >= 256 && g_lab_variant < 512) {  // slot kernel: 256 + 16 ablation + SLOTS (3 or 4); lds field = workgroups per eighth
        const int slots = g_lab_variant & 15;
        const int J = g_lab_lds > 0 ? g_lab_lds : 32;
        const dim3 g2(8 * J, (unsigned)channels);
        if (channels != 1) return hipErrorInvalidValue;
        unsigned long long* qp = nullptr;
        hipGetSymbolAddress((void**)&qp, HIP_SYMBOL(g_ols_lab_queue));
        const int abl = (g_lab_variant >> 4) & 3;
        if (slots == 4 && abl == 1)
            hipLaunchKernelGGL((fir_ols_slot_kernel<4, 1>), g2, dim3(1024), 0, s, (const f2*)x, (const float4*)p.d_pkt,
                               (const float4*)p.d_ostab, (f2*)y, (long long)n, lo, hi, q, p.halo_rows, qp, g_lab_tok);
        else if (slots == 4 && abl == 3)
            hipLaunchKernelGGL((fir_ols_slot_kernel<4, 3>), g2, dim3(1024), 0, s, (const f2*)x, (const float4*)p.d_pkt,
                               (const float4*)p.d_ostab, (f2*)y, (long long)n, lo, hi, q, p.halo_rows, qp, g_lab_tok);
        else if (slots == 4 && abl == 2)
            hipLaunchKernelGGL((fir_ols_slot_kernel<4, 2>), g2, dim3(1024), 0, s, (const f2*)x, (const float4*)p.d_pkt,
                               (const float4*)p.d_ostab, (f2*)y, (long long)n, lo, hi, q, p.halo_rows, qp, g_lab_tok);
        else if (slots == 4)
            hipLaunchKernelGGL((fir_ols_slot_kernel<4>), g2, dim3(1024), 0, s, (const f2*)x, (const float4*)p.d_pkt,
                               (const float4*)p.d_ostab, (f2*)y, (long long)n, lo, hi, q, p.halo_rows, qp, g_lab_tok);
        else if (slots == 3)
            hipLaunchKernelGGL((fir_ols_slot_kernel<3>), g2, dim3(768), 0, s, (const f2*)x, (const float4*)p.d_pkt,
                               (const float4*)p.d_ostab, (f2*)y, (long long)n, lo, hi, q, p.halo_rows, qp, g_lab_tok);
        else
            return hipErrorInvalidValue;
        return hipGetLastError();
    }
#define SDSP_LAB_CASE(V)                                                                                       \
    if (g_lab_variant == V) {                                                                                  \
        hipLaunchKernelGGL(fir_ols_os_kernel<V>, grid, dim3(256), g_lab_lds, s, (const f2*)x,                  \
                           (const float4*)p.d_pkt,                                                             \
                           (const float4*)p.d_ostab, (f2*)y, (long long)n, lo, hi, q, p.halo_rows);            \
        return hipGetLastError();                                                                              \
    }
    SDSP_LAB_VARIANTS(SDSP_LAB_CASE)
    hipLaunchKernelGGL(fir_ols_os_kernel<0>, grid, dim3(256), 0, s, (const f2*)x, (const float4*)p.d_pkt,
                       (const float4*)p.d_ostab, (f2*)y, (long long)n, lo, hi, q, p.halo_rows);
    return hipGetLastError();
}

}  // namespace sdsp
