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
//    eighth of the call in order (a one-shot copy in that order runs at copy
//    speed, profiles/r01/pattern_probe_7.log; the halo row of a segment is
//    the tail its XCD neighbour just read, an L2 hit);
//  * resources for 4 workgroups per CU (16 waves): <= 128 VGPRs and one 34 KB
//    LDS image + 2 KB twiddle row table.  The image is ALIASED across phases:
//    in P2/P4 lane (k0, n0) owns the 16 positions (k0, 16 j + n0), in P3 lane
//    (k0, k1) owns (k0, 16 k1 + j), in P1/P5 lane c owns (k, c) -- each lane
//    reads and rewrites only its own positions inside a phase, so one region
//    with the four phase barriers suffices (no second image, no extra barrier);
//  * no per-lane tables in registers: W4096^(c k) = D_{k>>2} C_{k&3} from six
//    per-lane bases (C_b = W^(b c), D_a = W^(4 a c)), W256 rows from LDS, the
//    lane's spectrum slice loaded from L2 during P2 for P3.
//
// LDS image: element (r, c) (r = row 0..15, c = 0..255, block b = c >> 4,
// e = c & 15) at r*272 + 16 b + 2 ((e >> 1 ^ b) & 7) + (e & 1).  Rows are 544
// dwords apart (opposite halves of the 64 banks); the 16-byte pair swizzle by
// the block index keeps P3's ds_read_b128 / ds_write_b128 and every 8-byte
// access of P2..P5 conflict-free (P1's ds_write_b64 is 2-way).
#include "sdsp_device.hpp"
#include "sdsp_kernels.hpp"
#include "sdsp_pk.hpp"

namespace sdsp {

using namespace pk;

namespace {

constexpr int kRow = 272;

__device__ __forceinline__ int opos(int r, int c) {
    const int b = c >> 4, e = c & 15;
    return r * kRow + 16 * b + ((((e >> 1) ^ b) & 7) << 1) + (e & 1);
}

}  // namespace

__global__ void __launch_bounds__(256, 4)
fir_ols_os_kernel(const f2* __restrict__ x, const float4* __restrict__ Hs, const float4* __restrict__ tb,
                  f2* __restrict__ y, long long n, long long lo, long long hi, long long q, int h2) {
    __shared__ __attribute__((aligned(16))) f2 img[16 * kRow];
    __shared__ float4 sw2[128];
    const int t = threadIdx.x;
    const int xc = blockIdx.x & 7;
    const long long seg = lo + (long long)xc * q + (blockIdx.x >> 3);
    const long long xe = lo + (long long)(xc + 1) * q;
    if (seg >= (xe < hi ? xe : hi)) return;  // uniform over the workgroup
    const int V = 4096 - 256 * h2;
    const long long base = (long long)blockIdx.y * n + seg * V - 256 * h2;
    const int up = (t >> 4) & 1;
    const int colX = 32 * (t >> 5) + 2 * (t & 15);
    const int col = colX + up;
    const int hi4 = t >> 4, lo4 = t & 15;

    // the segment: lane loads columns colX, colX + 1 of rows 2i + up (16-byte rows)
    float4 nq[8];
    {
        const float4* xb = reinterpret_cast<const float4*>(x + base + 256 * up + colX);
#pragma unroll
        for (int i = 0; i < 8; ++i) nq[i] = xb[256 * i];
    }
    // twiddle bases of column col, and the W256 row table into LDS (row r, pair p at r*8 + (p ^ r/2))
    const float4 b0 = tb[col], b1 = tb[256 + col], b2 = tb[512 + col];
    if (t < 128) {
        const int r = t >> 3, p = t & 7;
        sw2[r * 8 + (p ^ (r >> 1))] = tb[768 + t];
    }
    f2 Cb[3] = {f2{b0.x, b0.y}, f2{b0.z, b0.w}, f2{b1.x, b1.y}};
    f2 Da[3] = {f2{b1.z, b1.w}, f2{b2.x, b2.y}, f2{b2.z, b2.w}};
    // W4096^(col k) = D_{k>>2} C_{k&3}
    auto w1 = [&](int k) -> f2 {
        const int a = k >> 2, b = k & 3;
        if (a == 0) return b == 0 ? f2{1.0f, 0.0f} : Cb[b - 1];
        if (b == 0) return Da[a - 1];
        return pmul(Da[a - 1], Cb[b - 1]);
    };

    f2 v[16];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        float4 r = nq[i];
        swap16(r.x, r.z);
        swap16(r.y, r.w);
        v[2 * i] = f2{r.x, r.y};
        v[2 * i + 1] = f2{r.z, r.w};
    }
    // P1: DFT16 n2 -> k0, * W4096^(col k0) -> (k0, col)
    pdft16<false>(v);
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        if (k == 0) img[opos(0, col)] = v[0];
        else img[opos(k, col)] = pmul(v[kout(k)], w1(k));
    }
    __syncthreads();

    // P2: lane (k0 = hi4, n0 = lo4): DFT16 n1 -> k1, * W256^(n0 k1) -> (k0, 16 k1 + n0)
#pragma unroll
    for (int j = 0; j < 16; ++j) v[j] = img[opos(hi4, 16 * j + lo4)];
    float4 hq[8];  // spectrum slice of lane (k0, k1) = t for P3, k-pair major
#pragma unroll
    for (int p = 0; p < 8; ++p) hq[p] = Hs[p * 256 + t];
    pdft16<false>(v);
    const float4* w2row = sw2 + lo4 * 8;
#pragma unroll
    for (int p = 0; p < 8; ++p) {
        const float4 w = w2row[p ^ (lo4 >> 1)];
        img[opos(hi4, 16 * (2 * p) + lo4)] = p == 0 ? v[0] : pmul(v[kout(2 * p)], f2{w.x, w.y});
        img[opos(hi4, 16 * (2 * p + 1) + lo4)] = pmul(v[kout(2 * p + 1)], f2{w.z, w.w});
    }
    __syncthreads();

    // P3: lane (k0 = hi4, k1 = lo4) over n0: DFT16 n0 -> k2, * H, IDFT16 k2 -> n0, * conj W256^(k1 n0)
    {
        float4* row = reinterpret_cast<float4*>(img + hi4 * kRow + 16 * lo4);
#pragma unroll
        for (int p = 0; p < 8; ++p) {
            const float4 r = row[(p ^ lo4) & 7];
            v[2 * p] = f2{r.x, r.y};
            v[2 * p + 1] = f2{r.z, r.w};
        }
        pdft16<false>(v);
        f2 u[16];
#pragma unroll
        for (int p = 0; p < 8; ++p) {
            u[2 * p] = pmul(v[kout(2 * p)], f2{hq[p].x, hq[p].y});
            u[2 * p + 1] = pmul(v[kout(2 * p + 1)], f2{hq[p].z, hq[p].w});
        }
        pdft16<true>(u);
#pragma unroll
        for (int p = 0; p < 8; ++p) {
            const float4 w = w2row[p ^ (lo4 >> 1)];
            const f2 a = p == 0 ? u[kout(0)] : pmulc(u[kout(2 * p)], f2{w.x, w.y});
            const f2 c = pmulc(u[kout(2 * p + 1)], f2{w.z, w.w});
            row[(p ^ lo4) & 7] = make_float4(a.x, a.y, c.x, c.y);
        }
    }
    __syncthreads();

    // P4: lane (k0 = hi4, n0 = lo4): IDFT16 k1 -> n1 -> (k0, 16 n1 + n0)
#pragma unroll
    for (int j = 0; j < 16; ++j) v[j] = img[opos(hi4, 16 * j + lo4)];
    pdft16<true>(v);
#pragma unroll
    for (int k = 0; k < 16; ++k) img[opos(hi4, 16 * k + lo4)] = v[kout(k)];
    __syncthreads();

    // P5: lane col: * conj W4096^(col k0), IDFT16 k0 -> n2; row n2 at v[kout(n2)].  The bases
    // are made opaque first so the products are recomputed here rather than kept live from P1.
#pragma unroll
    for (int i = 0; i < 3; ++i) asm volatile("" : "+v"(Cb[i]), "+v"(Da[i]));
#pragma unroll
    for (int k = 0; k < 16; ++k) v[k] = k == 0 ? img[opos(0, col)] : pmulc(img[opos(k, col)], w1(k));
    pdft16<true>(v);
    float4* yb = reinterpret_cast<float4*>(y + base + 256 * up + colX);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const f2 a = v[kout(2 * i)], c = v[kout(2 * i + 1)];
        float4 r = make_float4(a.x, a.y, c.x, c.y);
        swap16(r.x, r.z);
        swap16(r.y, r.w);
        if (2 * i + up >= h2) yb[256 * i] = r;  // rows below h2 are the halo
    }
}

hipError_t launch_fir_ols_os(const OlsPlan& p, const void* x, void* y, size_t n, size_t channels, hipStream_t s,
                             long long lo, long long hi) {
    if (hi <= lo) return hipSuccess;
    if (p.halo_rows < 1 || p.halo_rows > 15) return hipErrorInvalidValue;
    const long long q = (hi - lo + 7) / 8;
    const dim3 grid((unsigned)(8 * q), (unsigned)channels);
    hipLaunchKernelGGL(fir_ols_os_kernel, grid, dim3(256), 0, s, (const f2*)x, (const float4*)p.d_pkt,
                       (const float4*)p.d_ostab, (f2*)y, (long long)n, lo, hi, q, p.halo_rows);
    return hipGetLastError();
}

}  // namespace sdsp
