// Column-parallel polyphase decimator (gfx950), SDSP_ALGO_FMA path.
//
// DecimatingFIRFilter (src/filter/fir/decim.rs:115-118, 221-228) emits
//     y[m] = scale * sum_{i<L} cr[i] * ext(j0 + m*M - i),   cr[i] = h[L-1-i]
// With L = K*M, write i = k*M + p and q = M-1-p.  Row rho of the stream is the
// M contiguous samples X[rho][q] = ext(j0 + rho*M - (M-1) + q), so
//     y[m] = scale * sum_{k<K} sum_{q<M} h[(K-1-k)*M + q] * X[m-k][q].
//
// A group of M lanes walks rows in stream order: lane q loads X[rho][q] (one
// coalesced M-sample load per row), keeps its K taps in registers and adds
// tap[k]*X[rho][q] into a ring of K per-output accumulators (output rho+k).
// After row rho the lane's partial for output rho is final; the partials of a
// chunk of CH rows go through an LDS tile [CH][M]; P = M/CH lanes sum one row
// (CH columns each) and combine by lane exchange, so every input sample is read
// from HBM once, touches LDS twice and costs K fused multiply-adds.  Each
// group owns `seg` consecutive outputs and starts K rows early (warm-up,
// outputs discarded); a wave holds G = 64/M groups.
//
// Summation order differs from the reference (phase-major partials, fused
// multiply-add), so this is the FMA path; SDSP_ALGO_EXACT keeps the
// reference-order kernel in kern_fir_direct.hip.
#include "sdsp_device.hpp"
#include "sdsp_kernels.hpp"

namespace sdsp {

namespace {

constexpr int kPolyThreads = 256;
constexpr int kPolyWaves = kPolyThreads / 64;

template <typename I>
__device__ __forceinline__ I ext_at(const I* __restrict__ x, const I* __restrict__ hist, long long j, long long n,
                                    int Lm1) {
    if (j >= 0) return j < n ? x[j] : zero_v<I>();
    const long long h = (long long)Lm1 + j;
    return h >= 0 ? hist[h] : zero_v<I>();
}

__device__ __forceinline__ float shfl_xor_v(float v, int d) { return __shfl_xor(v, d); }
__device__ __forceinline__ double shfl_xor_v(double v, int d) { return __shfl_xor(v, d); }
template <typename T> __device__ __forceinline__ cpx<T> shfl_xor_v(cpx<T> v, int d) {
    return {__shfl_xor(v.re, d), __shfl_xor(v.im, d)};
}

// streaming (non-temporal) load of a 4/8/16-byte value: the input is read once
template <typename T> __device__ __forceinline__ T nt_load(const T* p) {
    typedef unsigned u1v __attribute__((ext_vector_type(1)));
    typedef unsigned u2v __attribute__((ext_vector_type(2)));
    typedef unsigned u4v __attribute__((ext_vector_type(4)));
    T out;
    if constexpr (sizeof(T) == 16) {
        const u4v v = __builtin_nontemporal_load(reinterpret_cast<const u4v*>(p));
        __builtin_memcpy(&out, &v, 16);
    } else if constexpr (sizeof(T) == 8) {
        const u2v v = __builtin_nontemporal_load(reinterpret_cast<const u2v*>(p));
        __builtin_memcpy(&out, &v, 8);
    } else {
        static_assert(sizeof(T) == 4, "nt_load size");
        const u1v v = __builtin_nontemporal_load(reinterpret_cast<const u1v*>(p));
        __builtin_memcpy(&out, &v, 4);
    }
    return out;
}

// V adjacent columns per lane: one 16-byte load per lane and row when the row
// start is 16-byte aligned (V = 16 / sizeof(I)), else one sample per lane.
template <typename I, int V> struct alignas(V * sizeof(I)) IVec {
    I e[V];
};

template <typename I, int M, int K, int V> struct PolyGeom {
    static constexpr int MV = M / V;                      // lanes per group
    static constexpr int G = 64 / MV;                     // groups per wave
    static constexpr int CH = K > MV / 4 ? K : MV / 4;    // rows per reduction chunk
    static constexpr int P = MV > CH ? MV / CH : 1;       // lanes per output in the reduction (<= 4)
    static constexpr int RPL = CH > MV ? CH / MV : 1;     // outputs per lane when CH >= MV
    // one 8-byte slot of padding per row: lane (r, part) of the reduction reads
    // slot r*(MV*sizeof(I)/8 + 1) + part*CH*sizeof(I)/8, distinct mod 32 within a group
    static constexpr int RB = MV * (int)sizeof(I) + 8;
    static constexpr int LDS_WAVE = G * CH * RB;
};

template <typename C, typename I, int M, int K, int V, bool INTERIOR>
__device__ __forceinline__ void poly_group(const I* __restrict__ x, const I* __restrict__ hist,
                                           const C (&tap)[K][V], C scale, I* __restrict__ y,
                                           char* __restrict__ tile, long long n, int Lm1, long long j0,
                                           long long m_begin, long long m_end, int q) {
    using Geo = PolyGeom<I, M, K, V>;
    constexpr int CH = Geo::CH, MV = Geo::MV, RB = Geo::RB;
    constexpr int SPC = CH / K;  // K-row steps per chunk
    const long long nchunks = (m_end - m_begin + CH - 1) / CH;
    const long long nsteps = 1 + nchunks * SPC;
    const long long rho0 = m_begin - K;
    // sample index of X[rho][q*V] = jq + rho*M
    const long long jq = j0 - (M - 1) + q * V;

    using Vec = IVec<I, V>;
    I acc[K];
    Vec cur[K], nxt[K];
#pragma unroll
    for (int k = 0; k < K; ++k) acc[k] = zero_v<I>();

    auto load = [&](Vec (&v)[K], long long rho) {
#pragma unroll
        for (int u = 0; u < K; ++u) {
            const long long j = jq + (rho + u) * M;
            if constexpr (INTERIOR) {
                v[u] = nt_load(reinterpret_cast<const Vec*>(x + j));
            } else {
#pragma unroll
                for (int e = 0; e < V; ++e) v[u].e[e] = ext_at(x, hist, j + e, n, Lm1);
            }
        }
    };

    load(cur, rho0);
    for (long long s = 0; s < nsteps; ++s) {
        if (s + 1 < nsteps) load(nxt, rho0 + (s + 1) * K);
        const int trow = (int)((s - 1) % SPC) * K;  // tile row of this step's first row (s >= 1)
#pragma unroll
        for (int u = 0; u < K; ++u) {
#pragma unroll
            for (int k = 0; k < K; ++k)
#pragma unroll
                for (int e = 0; e < V; ++e) acc[(u + k) % K] = fmac_(acc[(u + k) % K], tap[k][e], cur[u].e[e]);
            if (s > 0) *reinterpret_cast<I*>(tile + (trow + u) * RB + q * (int)sizeof(I)) = acc[u];
            acc[u] = zero_v<I>();
        }
        if (s > 0 && s % SPC == 0) {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            const long long c = m_begin + (s / SPC - 1) * CH;
            if constexpr (CH >= MV) {
                // lane q sums whole rows q, q + MV, ...
#pragma unroll
                for (int t = 0; t < Geo::RPL; ++t) {
                    const int r = q + t * MV;
                    const I* row = reinterpret_cast<const I*>(tile + r * RB);
                    I sum = row[0];
#pragma unroll
                    for (int e = 1; e < MV; ++e) sum = add_(sum, row[e]);
                    if (c + r < m_end) y[c + r] = mul_(sum, scale);
                }
            } else {
                // output r = q % CH: lane part q / CH sums columns [part*CH, part*CH+CH),
                // then the P parts combine across lanes q ^ CH, q ^ 2CH
                const int r = q % CH, part = q / CH;
                const I* row = reinterpret_cast<const I*>(tile + r * RB) + part * CH;
                I sum = row[0];
#pragma unroll
                for (int e = 1; e < CH; ++e) sum = add_(sum, row[e]);
#pragma unroll
                for (int d = CH; d < MV; d *= 2) sum = add_(sum, shfl_xor_v(sum, d));
                if (part == 0 && c + r < m_end) y[c + r] = mul_(sum, scale);
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        }
#pragma unroll
        for (int u = 0; u < K; ++u) cur[u] = nxt[u];
    }
}

template <typename C, typename I, int M, int K, int V>
__global__ void __launch_bounds__(kPolyThreads)
decim_poly_kernel(const I* __restrict__ x, const I* __restrict__ hist, const C* __restrict__ cr, C scale,
                  I* __restrict__ y, long long n, long long nout, long long j0, long long seg) {
    using Geo = PolyGeom<I, M, K, V>;
    constexpr int G = Geo::G, CH = Geo::CH, MV = Geo::MV;
    constexpr int L = K * M;
    extern __shared__ __attribute__((aligned(16))) char lds[];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int g = lane / MV, q = lane % MV;
    const int ch = blockIdx.y;
    x += (long long)ch * n;
    y += (long long)ch * nout;
    hist += (long long)ch * (L - 1);

    const long long wave_id = (long long)xcd_order(blockIdx.x, gridDim.x) * kPolyWaves + wave;  // XCD-ordered
    const long long gid = wave_id * G + g;
    const long long m_begin = gid * seg;
    if (m_begin >= nout) return;
    const long long m_end = m_begin + seg < nout ? m_begin + seg : nout;

    C tap[K][V];
#pragma unroll
    for (int k = 0; k < K; ++k)
#pragma unroll
        for (int e = 0; e < V; ++e) tap[k][e] = cr[k * M + (M - 1 - (q * V + e))];

    char* tile = lds + (wave * G + g) * CH * Geo::RB;
    // wave-uniform interior test over all groups of this wave (rows warm-up .. last chunk)
    const long long first_j = j0 - (M - 1) + (wave_id * G * seg - K) * M;
    const long long last_row = (wave_id * G + G - 1) * seg + (seg + CH - 1) / CH * CH - 1;
    const long long last_j = j0 + last_row * M;
    if (first_j >= 0 && last_j < n)
        poly_group<C, I, M, K, V, true>(x, hist, tap, scale, y, tile, n, L - 1, j0, m_begin, m_end, q);
    else
        poly_group<C, I, M, K, V, false>(x, hist, tap, scale, y, tile, n, L - 1, j0, m_begin, m_end, q);
}

template <typename C, typename I, int M, int K, int V>
hipError_t launch_poly_t(const FirArgs& a, hipStream_t s) {
    using Geo = PolyGeom<I, M, K, V>;
    const long long nout = (long long)a.nout;
    // outputs per group: a multiple of CH.  64-256 measured fastest on cfg4; 256 keeps the
    // K warm-up rows per group (re-read input) to ~3% of the traffic
    long long seg = a.seg > 0 ? a.seg : (nout + 8191) / 8192;
    if (a.seg <= 0 && seg > 256) seg = 256;
    seg = (seg + Geo::CH - 1) / Geo::CH * Geo::CH;
    if (seg < Geo::CH) seg = Geo::CH;
    const long long groups = (nout + seg - 1) / seg;
    const long long waves = (groups + Geo::G - 1) / Geo::G;
    dim3 grid((unsigned)((waves + kPolyWaves - 1) / kPolyWaves), (unsigned)a.channels);
    const size_t lds = (size_t)kPolyWaves * Geo::LDS_WAVE;
    const C scale = *reinterpret_cast<const C*>(a.scale);
    hipLaunchKernelGGL((decim_poly_kernel<C, I, M, K, V>), grid, dim3(kPolyThreads), lds, s, (const I*)a.x,
                       (const I*)a.hist, (const C*)a.taps_rev, scale, (I*)a.y, (long long)a.n, nout,
                       (long long)a.j0, seg);
    return hipGetLastError();
}

template <typename C, typename I, int M, int K>
hipError_t poly_by_v(const FirArgs& a, hipStream_t s) {
    constexpr int VW = sizeof(I) >= 16 ? 1 : 16 / (int)sizeof(I);
    if constexpr (VW > 1) {
        // 16-byte rows: every row start j0 - (M-1) + rho*M a multiple of VW, and 16-byte
        // aligned channel bases
        const bool aligned = (a.j0 + 1) % VW == 0 && (a.channels == 1 || a.n % VW == 0) &&
                             reinterpret_cast<uintptr_t>(a.x) % 16 == 0;
        if (aligned) return launch_poly_t<C, I, M, K, VW>(a, s);
    }
    return launch_poly_t<C, I, M, K, 1>(a, s);
}

template <typename C, typename I, int M>
bool poly_by_k(const FirArgs& a, hipStream_t s, hipError_t* err) {
    switch (a.L / M) {
        case 2: *err = poly_by_v<C, I, M, 2>(a, s); return true;
        case 4: *err = poly_by_v<C, I, M, 4>(a, s); return true;
        case 8: *err = poly_by_v<C, I, M, 8>(a, s); return true;
        case 16: *err = poly_by_v<C, I, M, 16>(a, s); return true;
    }
    return false;
}

template <typename C, typename I>
bool poly_by_m(const FirArgs& a, hipStream_t s, hipError_t* err) {
    constexpr int sz = (int)sizeof(I);
    switch (a.M) {
        case 8: if constexpr (8 * sz >= 32 && 8 * sz <= 256) return poly_by_k<C, I, 8>(a, s, err); break;
        case 16: if constexpr (16 * sz >= 32 && 16 * sz <= 256) return poly_by_k<C, I, 16>(a, s, err); break;
        case 32: if constexpr (32 * sz >= 32 && 32 * sz <= 256) return poly_by_k<C, I, 32>(a, s, err); break;
        case 64: if constexpr (64 * sz >= 32 && 64 * sz <= 256) return poly_by_k<C, I, 64>(a, s, err); break;
    }
    return false;
}

}  // namespace

// true when the column-parallel kernel handles this decimator (FMA path,
// L = K*M with K in {2,4,8,16}, M in {8..64} with an M-sample row of 32..256 bytes)
bool try_launch_decim_poly(int dtype, const FirArgs& a, hipStream_t s, hipError_t* err) {
    if (a.exact || a.M < 8 || a.L % a.M != 0) return false;
    switch (dtype) {
        case 0: return poly_by_m<float, float>(a, s, err);
        case 1: return poly_by_m<float, c32>(a, s, err);
        case 2: return poly_by_m<c32, c32>(a, s, err);
        case 3: return poly_by_m<double, double>(a, s, err);
        case 4: return poly_by_m<double, c64>(a, s, err);
        case 5: return poly_by_m<c64, c64>(a, s, err);
    }
    return false;
}

}  // namespace sdsp
