// IIR kernels (gfx950): second-order-section cascades and direct-form-II
// filters, plain / decimating / interpolating.
//
// Reference semantics (src/filter/iir/sos.rs:92-114, mod.rs:270-289):
//   per section, coefficients divided by a0 once (in the Coef type):
//     d = (0 + a1 w1) + a2 w2;  w = x - d;  y = ((0 + b0 w) + b1 w1) + b2 w2;
//     w2 <- w1; w1 <- w;  the cascade feeds y of section s into section s+1.
//   Normal DF-II (mod.rs:272-279), window of cap = max(nb, na):
//     d = sum_{i<na-1} (a[i+1]/a0) w[n-1-i];  w = x - d;  y = sum_{i<nb} (b[i]/a0) w[n-i]
//   DecimatingIIRFilter (decim.rs:190-233): runs on every input, emits when
//     (index+1) % M == 0;  InterpolatingIIRFilter (interp.rs:184-221): input
//     x followed by M-1 zeros.
//
// Two algorithms:
//   * serial: one lane per channel walks the stream in the reference's exact
//     operation order (bit-identical to the reference algorithm at the
//     handle's precision).  Right for many channels or short blocks.
//   * scan (SOS cascades): the recurrence is linear in its 2S-dim state
//     S[n+1] = A S[n] + B x[n].  A block stages T*B samples in LDS; lane t
//     (1) runs its B-sample chunk from zero state -> local final state s_t,
//     (2) a Hillis-Steele scan with the host-precomputed P_k = A^(B 2^k)
//         gives every lane its true initial state  I_t = sum_{j<t} A^(B(t-1-j)) s_j,
//     (3) reruns its chunk from I_t and writes the outputs back through LDS
//         for coalesced stores.
//     Across blocks each block first runs `wc` warm-up chunks of the
//     preceding input: the carried-in state is multiplied by A^(wc*B), which
//     the host makes < 1e-9 (f32) / 1e-17 (f64) in infinity norm before it
//     selects this path (stable cascades only; otherwise the serial path).
//     Block 0 of a call injects the exact carried state as the warm-up
//     result, and the lane holding the call's last sample writes the exact
//     final state for the next call.
#include "sdsp_device.hpp"
#include "sdsp_kernels.hpp"

namespace sdsp {

// ---------------------------------------------------------------- arithmetic
template <bool EXACT, typename C, typename I>
__device__ __forceinline__ I dot2(C a1, I w1, C a2, I w2) {  // (0 + a1 w1) + a2 w2
    if constexpr (EXACT) return add_(add_(zero_v<I>(), mul_(a1, w1)), mul_(a2, w2));
    else return fmac_(mul_(a1, w1), a2, w2);
}
template <bool EXACT, typename C, typename I>
__device__ __forceinline__ I dot3(C b0, I w, C b1, I w1, C b2, I w2) {  // ((0 + b0 w) + b1 w1) + b2 w2
    if constexpr (EXACT) return add_(add_(add_(zero_v<I>(), mul_(b0, w)), mul_(b1, w1)), mul_(b2, w2));
    else return fmac_(fmac_(mul_(b0, w), b1, w1), b2, w2);
}

// coefficient layout (Coef type): section s at [5s..5s+4] = b0, b1, b2, a1, a2 (all / a0)
template <bool EXACT, int S, typename C, typename I>
__device__ __forceinline__ I sos_step(const C* __restrict__ c, I x, I (&w1)[S], I (&w2)[S]) {
    I v = x;
#pragma unroll
    for (int s = 0; s < S; ++s) {
        const I d = dot2<EXACT>(c[5 * s + 3], w1[s], c[5 * s + 4], w2[s]);
        const I w = sub_(v, d);
        v = dot3<EXACT>(c[5 * s + 0], w, c[5 * s + 1], w1[s], c[5 * s + 2], w2[s]);
        w2[s] = w1[s];
        w1[s] = w;
    }
    return v;
}

// domain sample k of an interpolating stream (x then Mi-1 zeros)
template <typename I>
__device__ __forceinline__ I domain_in(const I* __restrict__ x, long long k, int Mi) {
    if (Mi == 1) return x[k];
    return (k % Mi) == 0 ? x[k / Mi] : zero_v<I>();
}

// ---------------------------------------------------------------- serial SOS
// state layout per channel: [w1_0, w2_0, w1_1, w2_1, ...]
template <int S, typename C, typename I>
__global__ void __launch_bounds__(64)
sos_serial_kernel(const I* __restrict__ x, I* __restrict__ y, const C* __restrict__ coefs,
                  const I* __restrict__ st_in, I* __restrict__ st_out, long long n, long long nout, int Mi, int Md,
                  long long phase, int channels) {
    const int ch = blockIdx.x * blockDim.x + threadIdx.x;
    if (ch >= channels) return;
    x += (long long)ch * n;
    y += (long long)ch * nout;
    I w1[S], w2[S];
#pragma unroll
    for (int s = 0; s < S; ++s) {
        w1[s] = st_in[(long long)ch * 2 * S + 2 * s];
        w2[s] = st_in[(long long)ch * 2 * S + 2 * s + 1];
    }
    const long long nd = n * Mi;
    long long o = 0, idx = phase;
    for (long long k = 0; k < nd; ++k) {
        const I v = sos_step<true, S>(coefs, domain_in(x, k, Mi), w1, w2);
        idx = idx + 1 == Md ? 0 : idx + 1;
        if (idx == 0) y[o++] = v;
    }
#pragma unroll
    for (int s = 0; s < S; ++s) {
        st_out[(long long)ch * 2 * S + 2 * s] = w1[s];
        st_out[(long long)ch * 2 * S + 2 * s + 1] = w2[s];
    }
}

// ---------------------------------------------------------------- serial SOS, LDS-staged
// bytes per channel and tile: 1 KB runs per channel (cfg11: 1.72 -> 1.47 ms against 256-byte runs,
// 512-byte runs 1.74 ms; alternating whole bench lines, profiles/r05/lab/r05zk_libab_cfg11.log).  The
// 64 KB tile leaves room for two workgroups per CU and the prefetched tile holds 256 VGPRs per lane;
// the longer runs, not the occupancy, are what the HBM stream rewards (a -D override builds the
// A/B libraries)
#ifndef SDSP_SERIAL_LDS_RUN
#define SDSP_SERIAL_LDS_RUN 1024
#endif
// The same recurrence (lane = channel, reference order, bit-identical) for banks of
// >= 64 channels without rate change: a one-wave workgroup serves 64 channels and
// moves them through LDS in tiles of SDSP_SERIAL_LDS_RUN bytes per channel, so HBM sees coalesced
// runs instead of one element per lane 8n bytes apart (measured 2.4x the
// algorithmic traffic on the active_lag bank), with the next tile's loads in flight
// while the current one runs.
#ifndef SDSP_SERIAL_LD_AUX
#define SDSP_SERIAL_LD_AUX 2   // tile loads: nontemporal
#endif
#ifndef SDSP_SERIAL_ST_AUX
#define SDSP_SERIAL_ST_AUX 16  // tile stores: write-through (sc1)
#endif
template <int S, typename C, typename I>
__global__ void __launch_bounds__(64)
sos_serial_lds_kernel(const I* __restrict__ x, I* __restrict__ y, const C* __restrict__ coefs,
                      const I* __restrict__ st_in, I* __restrict__ st_out, long long n, int channels, bool vec_ok) {
    using v4u = unsigned __attribute__((ext_vector_type(4)));
    constexpr int kRun = SDSP_SERIAL_LDS_RUN, E = 16 / (int)sizeof(I), T = kRun / (int)sizeof(I), kRow = kRun + 16;
    constexpr int NV = kRun / 16;  // 16-byte vectors per channel and tile
    constexpr int kLogNV = __builtin_ctz(NV);
    static_assert((NV & (NV - 1)) == 0, "power-of-two tiles");
    __shared__ __attribute__((aligned(16))) char lds[64 * kRow];
    const int lane = threadIdx.x;
    const long long c0 = (long long)blockIdx.x * 64;
    const int nch = channels - c0 < 64 ? (int)(channels - c0) : 64;
    const int ch = (int)c0 + lane;
    I w1[S], w2[S];
#pragma unroll
    for (int s = 0; s < S; ++s) {
        w1[s] = lane < nch ? st_in[(long long)ch * 2 * S + 2 * s] : zero_v<I>();
        w2[s] = lane < nch ? st_in[(long long)ch * 2 * S + 2 * s + 1] : zero_v<I>();
    }
    // vector v of a tile: channel v >> kLogNV, 16-byte part v & (NV - 1)
    auto vaddr = [&](long long k0, int v) -> long long { return (c0 + (v >> kLogNV)) * n + k0 + (long long)(v & (NV - 1)) * E; };
    v4u pre[NV];
    // the pipelined path takes whole workgroups only: its per-vector offsets are a lane offset plus a
    // scalar offset, and rows past the last channel are not left to the descriptor's range check
    // (the partial last workgroup of a bank runs the element-wise loop below)
    const bool fast = vec_ok && nch == 64;
    long long kstart = 0;
    if (fast && (unsigned long long)n * 64ull * sizeof(I) < (1ull << 32)) {
        // whole tiles, pipelined without branches around memory operations: buffer loads and stores
        // through a descriptor that is empty past the last whole tile (no traffic), the
        // loop rotated so each tile is staged in the iteration that loaded it -- the compiler's wait
        // for the loads then sits behind only that iteration's stores
        const long long nfull = n / T * T;
        // vector v = lane + 64 j sits at channel (lane >> kLogNV) + j (64 / NV), part lane & (NV - 1):
        // one per-lane offset plus a wave-uniform j (64 / NV) n sizeof(I) (the instruction's scalar
        // offset), so the tile's NV offsets hold no registers
        const unsigned off0 = (unsigned)(((long long)(lane >> kLogNV) * n + (long long)(lane & (NV - 1)) * E) *
                                         (long long)sizeof(I));
        const int jstride = (int)((64 / NV) * n * (long long)sizeof(I));
        auto rsrc = [&](const void* base, long long k0) {
            const bool ok = k0 < nfull;
            const unsigned nrec = ok ? (unsigned)(((long long)nch * n - k0) * (long long)sizeof(I)) : 0u;
            return __builtin_amdgcn_make_buffer_rsrc((void*)((const I*)base + c0 * n + (ok ? k0 : 0)), (short)0, nrec,
                                                     0x00020000);
        };
        auto ld = [&](long long k0) {
            const auto r = rsrc(x, k0);
#pragma unroll
            for (int j = 0, so = 0; j < NV; ++j, so += jstride) {
                asm volatile("" : "+s"(so));  // formed here: not NV values hoisted into (spilled) SGPRs
                pre[j] = __builtin_bit_cast(v4u, __builtin_amdgcn_raw_buffer_load_b128(r, off0, so, SDSP_SERIAL_LD_AUX));
            }
        };
        auto stage = [&] {
#pragma unroll
            for (int j = 0; j < NV; ++j) {
                const int v = lane + 64 * j;
                *reinterpret_cast<v4u*>(lds + (v >> kLogNV) * kRow + (v & (NV - 1)) * 16) = pre[j];
            }
        };
        if (nfull > 0) {
            ld(0);
            stage();
            for (long long k0 = 0; k0 < nfull; k0 += T) {
                ld(k0 + T);  // past the last whole tile: an empty descriptor, no traffic
                __builtin_amdgcn_s_waitcnt(0xC07F);
                __builtin_amdgcn_wave_barrier();
                I* row = reinterpret_cast<I*>(lds + lane * kRow);
                for (int e = 0; e < T; ++e) row[e] = sos_step<true, S>(coefs, row[e], w1, w2);
                __builtin_amdgcn_s_waitcnt(0xC07F);
                __builtin_amdgcn_wave_barrier();
                const auto r = rsrc(y, k0);
#pragma unroll
                for (int j = 0, so = 0; j < NV; ++j, so += jstride) {
                    const int v = lane + 64 * j;
                    asm volatile("" : "+s"(so));
                    __builtin_amdgcn_raw_buffer_store_b128(
                        *reinterpret_cast<const v4u*>(lds + (v >> kLogNV) * kRow + (v & (NV - 1)) * 16), r, off0, so,
                        SDSP_SERIAL_ST_AUX);
                }
                __builtin_amdgcn_s_waitcnt(0xC07F);
                __builtin_amdgcn_wave_barrier();
                stage();
            }
        }
        kstart = nfull;  // the ragged tail (if any) below
    }
    // the ragged tail, a partial workgroup, or calls past 32-bit buffer offsets: whole tiles copied
    // through LDS without a prefetch, partial ones element by element
    for (long long k0 = kstart; k0 < n; k0 += T) {
        const bool full = fast && k0 + T <= n;
        if (full) {
#pragma unroll 4
            for (int j = 0; j < NV; ++j) {
                const int v = lane + 64 * j;
                *reinterpret_cast<v4u*>(lds + (v >> kLogNV) * kRow + (v & (NV - 1)) * 16) =
                    *reinterpret_cast<const v4u*>(x + vaddr(k0, v));
            }
        } else {
            for (int i = lane; i < 64 * T; i += 64) {
                const int cl = i / T, e = i % T;
                *reinterpret_cast<I*>(lds + cl * kRow + e * (int)sizeof(I)) =
                    (cl < nch && k0 + e < n) ? x[(c0 + cl) * n + k0 + e] : zero_v<I>();
            }
        }
        __builtin_amdgcn_s_waitcnt(0xC07F);
        __builtin_amdgcn_wave_barrier();
        const int cnt = n - k0 < T ? (int)(n - k0) : T;
        I* row = reinterpret_cast<I*>(lds + lane * kRow);
        for (int e = 0; e < cnt; ++e) row[e] = sos_step<true, S>(coefs, row[e], w1, w2);
        __builtin_amdgcn_s_waitcnt(0xC07F);
        __builtin_amdgcn_wave_barrier();
        if (full) {
#pragma unroll 4
            for (int j = 0; j < NV; ++j) {
                const int v = lane + 64 * j;
                *reinterpret_cast<v4u*>(y + vaddr(k0, v)) =  // plain: nontemporal +1.7 % (cfg11)
                    *reinterpret_cast<const v4u*>(lds + (v >> kLogNV) * kRow + (v & (NV - 1)) * 16);
            }
        } else {
            for (int i = lane; i < 64 * T; i += 64) {
                const int cl = i / T, e = i % T;
                if (cl < nch && k0 + e < n)
                    y[(c0 + cl) * n + k0 + e] = *reinterpret_cast<const I*>(lds + cl * kRow + e * (int)sizeof(I));
            }
        }
        __builtin_amdgcn_s_waitcnt(0xC07F);
        __builtin_amdgcn_wave_barrier();
    }
    if (lane < nch) {
#pragma unroll
        for (int s = 0; s < S; ++s) {
            st_out[(long long)ch * 2 * S + 2 * s] = w1[s];
            st_out[(long long)ch * 2 * S + 2 * s + 1] = w2[s];
        }
    }
}

// ---------------------------------------------------------------- serial Normal DF-II
// hh[i] = w[n-1-i] for i < cap-1 (newest first; the window's oldest slot is
// never read by either dot product, src/filter/iir/mod.rs:272-279).
// coefs: num[0..nb) = b/a0 then den[0..na-1) = a[1..]/a0
template <int CAP, typename C, typename I>
__global__ void __launch_bounds__(64)
normal_serial_kernel(const I* __restrict__ x, I* __restrict__ y, const C* __restrict__ num, int nb,
                     const C* __restrict__ den, int nd1, const I* __restrict__ st_in, I* __restrict__ st_out,
                     long long n, long long nout, int Mi, int Md, long long phase, int channels, int cap) {
    const int ch = blockIdx.x * blockDim.x + threadIdx.x;
    if (ch >= channels) return;
    x += (long long)ch * n;
    y += (long long)ch * nout;
    I hh[CAP];
#pragma unroll
    for (int i = 0; i < CAP; ++i) hh[i] = (i < cap - 1) ? st_in[(long long)ch * (cap - 1) + i] : zero_v<I>();
    const long long ndom = n * Mi;
    long long o = 0, idx = phase;
    for (long long k = 0; k < ndom; ++k) {
        I d = zero_v<I>();
#pragma unroll
        for (int i = 0; i < CAP; ++i)
            if (i < nd1) d = add_(d, mul_(den[i], hh[i]));
        const I v = sub_(domain_in(x, k, Mi), d);
        I out = add_(zero_v<I>(), mul_(num[0], v));
#pragma unroll
        for (int i = 1; i < CAP + 1; ++i)
            if (i < nb) out = add_(out, mul_(num[i], hh[i - 1]));
#pragma unroll
        for (int i = CAP - 1; i > 0; --i) hh[i] = hh[i - 1];
        hh[0] = v;
        idx = idx + 1 == Md ? 0 : idx + 1;
        if (idx == 0) y[o++] = out;
    }
    for (int i = 0; i < cap - 1; ++i) st_out[(long long)ch * (cap - 1) + i] = hh[i];
}

// ---------------------------------------------------------------- scan SOS
template <typename I> struct scan_chunk { static constexpr int B = sizeof(I) == 4 ? 64 : (sizeof(I) == 8 ? 32 : 16); };
constexpr int kScanT = 256;

// y = P x for a D x D real matrix (row-major) and a vector of I
template <int D, typename R, typename I>
__device__ __forceinline__ void matvec(const R* __restrict__ P, const I (&x)[D], I (&y)[D]) {
#pragma unroll
    for (int r = 0; r < D; ++r) {
        I acc = mul_(P[r * D + 0], x[0]);
#pragma unroll
        for (int c = 1; c < D; ++c) acc = fmac_(acc, P[r * D + c], x[c]);
        y[r] = acc;
    }
}

template <int S, typename C, typename I>
__global__ void __launch_bounds__(kScanT)
sos_scan_kernel(const I* __restrict__ x, I* __restrict__ y, const C* __restrict__ coefs,
                const C* __restrict__ P /* [8][D][D] */, const I* __restrict__ st_in, I* __restrict__ st_out,
                long long n, long long nout, int Mi, int Md, long long phase, int wc) {
    constexpr int D = 2 * S;
    constexpr int B = scan_chunk<I>::B;
    constexpr int RS = B + 1;  // padded chunk stride in LDS (odd in 4-byte words for 4-byte I)
    extern __shared__ __attribute__((aligned(16))) char lds_raw[];
    I* buf = reinterpret_cast<I*>(lds_raw);                     // [T][RS] samples
    I* sv = reinterpret_cast<I*>(lds_raw + sizeof(I) * kScanT * RS);  // [T][D] scan exchange

    const int ch = blockIdx.y;
    x += (long long)ch * n;
    y += (long long)ch * nout;
    st_in += (long long)ch * D;
    st_out += (long long)ch * D;
    const int t = threadIdx.x;
    const long long nd = n * Mi;                     // domain samples in this call
    const long long per_blk = (long long)(kScanT - wc) * B;
    const long long kb = (long long)blockIdx.x * per_blk - (long long)wc * B;  // domain index of lane 0 sample 0

    // stage T*B domain samples (negative indices: zero)
    for (int f = t; f < kScanT * B; f += kScanT) {
        const long long k = kb + f;
        buf[(f / B) * RS + (f % B)] = (k >= 0 && k < nd) ? domain_in(x, k, Mi) : zero_v<I>();
    }
    __syncthreads();

    const long long k0 = kb + (long long)t * B;  // my first domain sample
    int cnt = 0;                                  // valid samples in my chunk
    if (k0 < nd && k0 + B > 0) cnt = (int)min<long long>(B, nd - k0);

    // (1) local zero-state run
    I s[D];
    {
        I w1[S], w2[S];
#pragma unroll
        for (int q = 0; q < S; ++q) { w1[q] = zero_v<I>(); w2[q] = zero_v<I>(); }
        const bool inject = blockIdx.x == 0 && t == wc - 1;
        if (k0 >= 0) {
            for (int i = 0; i < cnt; ++i) (void)sos_step<false, S>(coefs, buf[t * RS + i], w1, w2);
        }
#pragma unroll
        for (int q = 0; q < S; ++q) {
            s[2 * q] = inject ? st_in[2 * q] : w1[q];
            s[2 * q + 1] = inject ? st_in[2 * q + 1] : w2[q];
        }
    }
    // (2) inclusive Hillis-Steele scan: G_t = sum_{j<=t} A^(B(t-j)) s_j
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const int off = 1 << k;
#pragma unroll
        for (int d = 0; d < D; ++d) sv[t * D + d] = s[d];
        __syncthreads();
        if (t >= off) {
            I prev[D], add[D];
#pragma unroll
            for (int d = 0; d < D; ++d) prev[d] = sv[(t - off) * D + d];
            matvec<D>(P + k * D * D, prev, add);
#pragma unroll
            for (int d = 0; d < D; ++d) s[d] = add_(s[d], add[d]);
        }
        __syncthreads();
    }
    // initial state of my chunk: G_{t-1}
#pragma unroll
    for (int d = 0; d < D; ++d) sv[t * D + d] = s[d];
    __syncthreads();
    I w1[S], w2[S];
#pragma unroll
    for (int q = 0; q < S; ++q) {
        w1[q] = t > 0 ? sv[(t - 1) * D + 2 * q] : zero_v<I>();
        w2[q] = t > 0 ? sv[(t - 1) * D + 2 * q + 1] : zero_v<I>();
    }
    // (3) rerun and write outputs in place
    if (t >= wc && k0 >= 0) {
        for (int i = 0; i < cnt; ++i) buf[t * RS + i] = sos_step<false, S>(coefs, buf[t * RS + i], w1, w2);
        if (cnt > 0 && k0 + cnt == nd) {
#pragma unroll
            for (int q = 0; q < S; ++q) {
                st_out[2 * q] = w1[q];
                st_out[2 * q + 1] = w2[q];
            }
        }
    }
    __syncthreads();
    // coalesced store of this block's outputs (domain k -> output index when it is emitted)
    const long long j0 = (Md - 1 - phase) % Md;  // first emitting domain index
    for (int f = wc * B + t; f < kScanT * B; f += kScanT) {
        const long long k = kb + f;
        if (k < 0 || k >= nd) continue;
        if (Md == 1) {
            y[k] = buf[(f / B) * RS + (f % B)];
        } else if (k >= j0 && (k - j0) % Md == 0) {
            y[(k - j0) / Md] = buf[(f / B) * RS + (f % B)];
        }
    }
}

// ---------------------------------------------------------------- launchers
template <typename C, typename I, int S>
hipError_t launch_sos_t(const IirArgs& a, hipStream_t st) {
    if (a.algo_scan) {
        constexpr int B = scan_chunk<I>::B;
        constexpr int D = 2 * S;
        const long long nd = (long long)a.n * a.Mi;
        const long long per_blk = (long long)(kScanT - a.wc) * B;
        const long long nblk = (nd + per_blk - 1) / per_blk;
        const size_t lds = sizeof(I) * kScanT * (B + 1) + sizeof(I) * kScanT * D;
        dim3 grid((unsigned)nblk, (unsigned)a.channels);
        hipLaunchKernelGGL((sos_scan_kernel<S, C, I>), grid, dim3(kScanT), lds, st, (const I*)a.x, (I*)a.y,
                           (const C*)a.coefs, (const C*)a.P, (const I*)a.st_in, (I*)a.st_out, (long long)a.n,
                           (long long)a.nout, a.Mi, a.Md, (long long)a.phase, a.wc);
    } else if (a.Mi == 1 && a.Md == 1 && a.channels >= 64) {
        dim3 grid((unsigned)((a.channels + 63) / 64));
        const bool vec_ok = reinterpret_cast<uintptr_t>(a.x) % 16 == 0 && reinterpret_cast<uintptr_t>(a.y) % 16 == 0 &&
                            (a.n * sizeof(I)) % 16 == 0;
        hipLaunchKernelGGL((sos_serial_lds_kernel<S, C, I>), grid, dim3(64), 0, st, (const I*)a.x, (I*)a.y,
                           (const C*)a.coefs, (const I*)a.st_in, (I*)a.st_out, (long long)a.n, (int)a.channels,
                           vec_ok);
    } else {
        dim3 grid((unsigned)((a.channels + 63) / 64));
        hipLaunchKernelGGL((sos_serial_kernel<S, C, I>), grid, dim3(64), 0, st, (const I*)a.x, (I*)a.y,
                           (const C*)a.coefs, (const I*)a.st_in, (I*)a.st_out, (long long)a.n, (long long)a.nout,
                           a.Mi, a.Md, (long long)a.phase, (int)a.channels);
    }
    return hipGetLastError();
}

template <typename C, typename I>
hipError_t launch_sos_dt(const IirArgs& a, hipStream_t st) {
    switch (a.sections) {
        case 1: return launch_sos_t<C, I, 1>(a, st);
        case 2: return launch_sos_t<C, I, 2>(a, st);
        case 3: return launch_sos_t<C, I, 3>(a, st);
        case 4: return launch_sos_t<C, I, 4>(a, st);
        case 5: return launch_sos_t<C, I, 5>(a, st);
        case 6: return launch_sos_t<C, I, 6>(a, st);
        case 7: return launch_sos_t<C, I, 7>(a, st);
        case 8: return launch_sos_t<C, I, 8>(a, st);
    }
    return hipErrorInvalidValue;
}

template <typename C, typename I>
hipError_t launch_normal_dt(const IirArgs& a, hipStream_t st) {
    dim3 grid((unsigned)((a.channels + 63) / 64));
#define SDSP_NORMAL(CAPV)                                                                                        \
    hipLaunchKernelGGL((normal_serial_kernel<CAPV, C, I>), grid, dim3(64), 0, st, (const I*)a.x, (I*)a.y,          \
                       (const C*)a.coefs, a.nb, (const C*)a.coefs + a.nb, a.na - 1, (const I*)a.st_in,            \
                       (I*)a.st_out, (long long)a.n, (long long)a.nout, a.Mi, a.Md, (long long)a.phase,            \
                       (int)a.channels, a.cap)
    if (a.cap <= 4) SDSP_NORMAL(4);
    else if (a.cap <= 8) SDSP_NORMAL(8);
    else if (a.cap <= 16) SDSP_NORMAL(16);
    else if (a.cap <= 32) SDSP_NORMAL(32);
    else return hipErrorInvalidValue;
#undef SDSP_NORMAL
    return hipGetLastError();
}

int iir_scan_chunk(int dtype) {
    switch (dtype) {
        case 0: return scan_chunk<float>::B;
        case 1: return scan_chunk<c32>::B;
        case 3: return scan_chunk<double>::B;
        case 4: return scan_chunk<c64>::B;
    }
    return 0;
}

hipError_t launch_iir(int dtype, const IirArgs& a, hipStream_t st) {
    if (a.n == 0) return hipSuccess;
    if (a.sections > 0) {
        switch (dtype) {
            case 0: return launch_sos_dt<float, float>(a, st);
            case 1: return launch_sos_dt<float, c32>(a, st);
            case 3: return launch_sos_dt<double, double>(a, st);
            case 4: return launch_sos_dt<double, c64>(a, st);
        }
    } else {
        switch (dtype) {
            case 0: return launch_normal_dt<float, float>(a, st);
            case 1: return launch_normal_dt<float, c32>(a, st);
            case 3: return launch_normal_dt<double, double>(a, st);
            case 4: return launch_normal_dt<double, c64>(a, st);
        }
    }
    return hipErrorInvalidValue;
}

}  // namespace sdsp
