// Persistent overlap-save FIR, N = 4096, in packed FP32 arithmetic (gfx950):
// the alternative interior-segment kernel of the c32 overlap-save path
// (SDSP_TUNE_OLS_KERNEL = SDSP_OLS_PERSISTENT; the default is the one-shot
// kernel of kern_fir_ols_os.hip).
//
// Same transform and data flow as fir_ols4096_kernel in kern_fir_ols.hip
// (P1..P5, three radix-16 passes each way, two LDS regions, four barriers per
// segment), with every complex operation a v_pk_* instruction (sdsp_pk.hpp) and
// the same IEEE operation sequence per component, so the two kernels agree bit
// for bit.  The twiddle rows and the lane's spectrum slice live in registers
// (96 VGPRs, loaded once per workgroup); each workgroup walks `per` consecutive
// interior segments (boundary segments run in fir_ols4096_edge_kernel).
//
// 16-byte global accesses: lane t owns column col(t) = 32 (t >> 5) + 2 (t & 15)
// + ((t >> 4) & 1).  A lane loads two adjacent columns (X, X + 1) of one row
// (rows 2i / 2i + 1 for the lower / upper 16 lanes of each 32) and one
// v_permlane16_swap per dword turns the pair into its column over rows 2i,
// 2i + 1; stores swap back.  HBM issue schedule: the next segment's row-pair
// loads and the previous segment's deferred stores are spread over the
// segment's phases (load chunk i at hook kLoadAt[i], store chunk i at
// kStoreAt[i]; hooks 0 loop head, 1 after P1's LDS writes, 3 after P2's, 5 after
// P3's, 7 after P4's) instead of one burst after P1 (7-8 % faster).
#include "sdsp_device.hpp"
#include "sdsp_kernels.hpp"
#include "sdsp_pk.hpp"

namespace sdsp {

using namespace pk;

namespace {

constexpr int kRowA = 272;           // A image: 16 rows of 256 (+16 pad) samples
constexpr int kRegion = 16 * kRowA;  // samples per LDS region
// A image: column c sits at acol(c) = c ^ bit 4 of c; B image: row r at r ^ bit 4 of r,
// its 16-byte pairs XOR-swizzled by r & 7 (bank-conflict free for every access of P1..P5)
__device__ __forceinline__ int acol(int c) { return c ^ ((c >> 4) & 1); }
__device__ __forceinline__ int brow(int r) { return r ^ ((r >> 4) & 1); }
__device__ __forceinline__ int bidx(int r, int c) { return brow(r) * 16 + ((((c >> 1) ^ r) & 7) << 1) + (c & 1); }

template <int B> struct Hook { static constexpr int value = B; };
constexpr int kLoadAt[8] = {0, 0, 1, 1, 3, 3, 5, 5};
constexpr int kStoreAt[8] = {1, 1, 3, 3, 5, 5, 7, 7};

}  // namespace

template <int H2>
__global__ void __launch_bounds__(256, 2)
fir_ols4096_pk_kernel(const f2* __restrict__ x, const f2* __restrict__ Hs, const f2* __restrict__ tw1,
                      const f2* __restrict__ tw2, f2* __restrict__ y, long long n, long long seg_lo,
                      long long seg_hi, long long per, long long xm) {
    __shared__ __attribute__((aligned(16))) f2 lds[2 * kRegion];
    f2* const rA = lds;
    f2* const rB = lds + kRegion;
    const int ch = blockIdx.y;
    x += (long long)ch * n;
    y += (long long)ch * n;
    const int t = threadIdx.x;
    const int hi4 = t >> 4, lo4 = t & 15;
    const int up = (t >> 4) & 1;
    const int colX = 32 * (t >> 5) + 2 * (t & 15);
    const int col = colX + up;
    constexpr int V = 4096 - 256 * H2;
    // `per` consecutive segments per workgroup; workgroup b runs on XCD b % 8, so chunk
    // (b % 8) xm + b / 8 keeps each XCD on one contiguous part of the stream
    const long long b = (long long)(blockIdx.x % 8) * xm + blockIdx.x / 8;
    long long seg = seg_lo + b * per;
    if (seg + per < seg_hi) seg_hi = seg + per;

    f2 w1[16], w2[16], Hr[16];
    // k-pair major tables (OlsPlan::d_pkt): one coalesced 16-byte access per lane and pair
    auto load_tables = [&] {
#pragma unroll
        for (int k = 0; k < 16; k += 2) {
            const float4 a = reinterpret_cast<const float4*>(tw1)[(k / 2) * 256 + col];
            const float4 c = reinterpret_cast<const float4*>(tw2)[(k / 2) * 16 + lo4];
            const float4 e = reinterpret_cast<const float4*>(Hs)[(k / 2) * 256 + t];
            w1[k] = f2{a.x, a.y};
            w1[k + 1] = f2{a.z, a.w};
            w2[k] = f2{c.x, c.y};
            w2[k + 1] = f2{c.z, c.w};
            Hr[k] = f2{e.x, e.y};
            Hr[k + 1] = f2{e.z, e.w};
        }
    };
    float4 nq[8];  // row 2i + up, columns colX, colX + 1
    auto load = [&](long long sg, auto sel) {
        const float4* xb = reinterpret_cast<const float4*>(x + sg * V - 256 * H2 + 256 * up + colX);
#pragma unroll
        for (int i = 0; i < 8; ++i)
            if (sel(i)) nq[i] = xb[256 * i];
    };
    // stores are deferred by one segment: segment s's outputs go out during segment s + 1,
    // ahead of the loads for segment s + 2, so the loop-head wait for those loads never
    // covers freshly issued stores
    f2 ov[16];
    long long oseg = -1;
    auto store_out = [&](auto sel) {
        float4* yb = reinterpret_cast<float4*>(y + oseg * V - 256 * H2 + 256 * up + colX);
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            if (!sel(i)) continue;
            if (2 * i + 1 < H2) continue;  // both rows are halo
            float4 q = make_float4(ov[2 * i].x, ov[2 * i].y, ov[2 * i + 1].x, ov[2 * i + 1].y);
            swap16(q.x, q.z);
            swap16(q.y, q.w);
            if (2 * i >= H2 || up) yb[256 * i] = q;  // row 2i is halo when 2i < H2
        }
    };
    auto segment = [&] {
        f2 v[16];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            float4 q = nq[i];
            swap16(q.x, q.z);
            swap16(q.y, q.w);
            v[2 * i] = f2{q.x, q.y};
            v[2 * i + 1] = f2{q.z, q.w};
        }
        const long long nxt = seg + 1 < seg_hi ? seg + 1 : seg;
        auto hook = [&](auto pt) {
            constexpr int P = decltype(pt)::value;
            if (oseg >= 0) store_out([](int i) { return kStoreAt[i] == P; });
            load(nxt, [](int i) { return kLoadAt[i] == P; });
        };
        hook(Hook<0>{});
        // P1: DFT over n2 -> k0, twiddle, A[k0][col]
        pdft16<false>(v);
#pragma unroll
        for (int k = 0; k < 16; ++k) rA[k * kRowA + acol(col)] = pmul(v[kout(k)], w1[k]);
        hook(Hook<1>{});
        __syncthreads();
        // P2: lane (k0=hi4, n0=lo4) reads n1
#pragma unroll
        for (int k = 0; k < 16; ++k) v[k] = rA[hi4 * kRowA + 16 * k + (lo4 ^ (k & 1))];
        pdft16<false>(v);
#pragma unroll
        for (int k = 0; k < 16; ++k) rB[bidx(16 * hi4 + k, lo4)] = pmul(v[kout(k)], w2[k]);
        hook(Hook<3>{});
        __syncthreads();
        // P3: lane (k0=hi4, k1=lo4) reads its row over n0
        {
            const float4* row = reinterpret_cast<const float4*>(rB + brow(t) * 16);
#pragma unroll
            for (int p = 0; p < 8; ++p) {
                const float4 q = row[(p ^ t) & 7];
                v[2 * p] = f2{q.x, q.y};
                v[2 * p + 1] = f2{q.z, q.w};
            }
        }
        pdft16<false>(v);
        f2 u[16];
#pragma unroll
        for (int k = 0; k < 16; ++k) u[k] = pmul(v[kout(k)], Hr[k]);
        pdft16<true>(u);
        {
            float4* row = reinterpret_cast<float4*>(rA + brow(t) * 16);
#pragma unroll
            for (int p = 0; p < 8; ++p) {
                const f2 a = pmulc(u[kout(2 * p)], w2[2 * p]);
                const f2 c = pmulc(u[kout(2 * p + 1)], w2[2 * p + 1]);
                row[(p ^ t) & 7] = make_float4(a.x, a.y, c.x, c.y);
            }
        }
        hook(Hook<5>{});
        __syncthreads();
        // P4: lane (k0=hi4, n0=lo4) reads k1
#pragma unroll
        for (int k = 0; k < 16; ++k) v[k] = rA[bidx(16 * hi4 + k, lo4)];
        pdft16<true>(v);
#pragma unroll
        for (int k = 0; k < 16; ++k) rB[hi4 * kRowA + 16 * k + (lo4 ^ (k & 1))] = v[kout(k)];
        hook(Hook<7>{});
        __syncthreads();
        // P5: lane col reads k0
#pragma unroll
        for (int k = 0; k < 16; ++k) v[k] = pmulc(rB[k * kRowA + acol(col)], w1[k]);
        pdft16<true>(v);
#pragma unroll
        for (int k = 0; k < 16; ++k) ov[k] = v[kout(k)];
        oseg = seg;
        // tables opaque once per segment: swizzled copies of them are not hoisted out of the loop
#pragma unroll
        for (int k = 0; k < 16; ++k) asm volatile("" : "+v"(w1[k]), "+v"(w2[k]), "+v"(Hr[k]));
        // the next segment's P1 writes region A: every lane has finished reading
        // region A (P4) before the barrier that precedes P5.
    };
    if (seg < seg_hi) load(seg, [](int) { return true; });
    load_tables();  // after the first segment's loads: a short run waits for tables only at P1
    for (; seg < seg_hi; ++seg) segment();
    if (oseg >= 0) store_out([](int) { return true; });
}

hipError_t launch_fir_ols_pk(const OlsPlan& p, const void* x, void* y, size_t n, size_t channels, hipStream_t s,
                             long long lo, long long hi) {
    if (hi <= lo) return hipSuccess;
    const float4* const pkt = reinterpret_cast<const float4*>(p.d_pkt);
    const long long per = kOlsSegsPerBlock;
    const long long xm = ((hi - lo + per - 1) / per + 7) / 8;
    const dim3 grid((unsigned)(8 * xm), (unsigned)channels);
#define SDSP_OLS_PK(HV)                                                                                           \
    hipLaunchKernelGGL((fir_ols4096_pk_kernel<HV>), grid, dim3(256), 0, s, (const f2*)x, (const f2*)pkt,          \
                       (const f2*)(pkt + 2048), (const f2*)(pkt + 4096), (f2*)y, (long long)n, lo, hi, per, xm)
    switch (p.halo_rows) {
        case 1: SDSP_OLS_PK(1); break;
        case 2: SDSP_OLS_PK(2); break;
        case 3: SDSP_OLS_PK(3); break;
        case 4: SDSP_OLS_PK(4); break;
        default: return hipErrorInvalidValue;
    }
#undef SDSP_OLS_PK
    return hipGetLastError();
}

}  // namespace sdsp
