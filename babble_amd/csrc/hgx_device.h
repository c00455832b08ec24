// Device helpers shared by the libhgx HIP translation units (gfx950, wave64).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace hgx {

__device__ __forceinline__ int lane_id() { return (int)(threadIdx.x & 63); }

// Strongly-see count of 8-bit rebased coordinates, 4 per dword: window bytes hold LA' in [0, 126], the
// candidate's bytes nf = 128 - FD' with FD' in [1, 127] (127 = none), so LA' + nf lies in [1, 253]: no
// carry leaves a byte, and bit 7 is set exactly when LA' >= FD'. With no carries the add may span 64
// bits (one v_lshl_add_u64 per 8 coordinates instead of a v_sub per 4).
template <int HD>
__device__ __forceinline__ uint32_t swar_ge_count(const uint32_t (&v)[HD], const uint32_t (&nf)[HD]) {
    uint32_t c = 0;
    if constexpr (HD % 2 == 0) {
        // one chain of v_bcnt_u32_b32 with its accumulate operand (the empty asm keeps the compiler from
        // re-associating the sum into bcnt(x, 0) + v_add3 trees: 2.5 instead of 3 VALU per dword)
#pragma unroll
        for (int i = 0; i < HD / 2; i++) {
            const uint64_t s = ((((uint64_t)v[2 * i + 1]) << 32) | v[2 * i]) + ((((uint64_t)nf[2 * i + 1]) << 32) | nf[2 * i]);
            c = __builtin_popcount((uint32_t)s & 0x80808080u) + c;
            asm volatile("" : "+v"(c));
            c = __builtin_popcount((uint32_t)(s >> 32) & 0x80808080u) + c;
            asm volatile("" : "+v"(c));
        }
    } else {
#pragma unroll
        for (int d = 0; d < HD; d++) c += __builtin_popcount((v[d] + nf[d]) & 0x80808080u);
    }
    return c;
}
// a candidate row dword (bytes FD' with the validity bit cleared) as its nf bytes (128 - FD'); 127 = none -> 1
__device__ __forceinline__ uint32_t swar_nf(uint32_t fd7) { return 0x80808080u - fd7; }

__device__ __forceinline__ uint64_t group_mask(int gs, int grp) {
    return (gs >= 64) ? ~0ull : (((1ull << gs) - 1ull) << (gs * grp));
}

// Storage of the coordinate arrays LA / FDT. int32_t: the raw values
// (lastAncestors -1 = none, firstDescendants MaxInt32 = none). uint16_t ("compact",
// every Index < 65534 and n even): LA stored as value + 1 (none = 0, so the encoding
// is order-preserving and max() works on it directly), FD stored as is with
// none = 0xFFFF. Kernels decode to int32 before comparing with raw values.
template <typename CT>
struct Coord;
template <>
struct Coord<int32_t> {
    static constexpr int32_t kLaNone = -1;
    __device__ __forceinline__ static int32_t la(int32_t v) { return v; }
    __device__ __forceinline__ static int32_t enc_la(int32_t v) { return v; }
    __device__ __forceinline__ static int32_t fd(int32_t v) { return v; }
    __device__ __forceinline__ static int32_t enc_fd(int32_t v) { return v; }
};
template <>
struct Coord<uint16_t> {
    static constexpr int32_t kLaNone = 0;
    __device__ __forceinline__ static int32_t la(uint32_t v) { return (int32_t)v - 1; }
    __device__ __forceinline__ static uint16_t enc_la(int32_t v) { return (uint16_t)(v + 1); }
    __device__ __forceinline__ static int32_t fd(uint32_t v) { return v == 0xFFFFu ? 2147483647 : (int32_t)v; }
    __device__ __forceinline__ static uint16_t enc_fd(int32_t v) { return v >= 0xFFFF ? (uint16_t)0xFFFF : (uint16_t)v; }
};

// order LDS accesses of one wave (lanes exchange data through LDS without a block barrier)
__device__ __forceinline__ void wave_lds_fence() {
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
}

__device__ __forceinline__ uint64_t wave_min_u64(uint64_t x) {
    for (int o = 32; o >= 1; o >>= 1) {
        const uint64_t y = __shfl_xor(x, o);
        x = y < x ? y : x;
    }
    return x;
}

__device__ __forceinline__ uint64_t wave_max_u64(uint64_t x) {
    for (int o = 32; o >= 1; o >>= 1) {
        const uint64_t y = __shfl_xor(x, o);
        x = y > x ? y : x;
    }
    return x;
}

// Wave-cooperative exact selection: the K-th smallest (0-based) of the valid values
// held by the wave (CPL per lane). Radix select on (v - min) with 8-bit buckets from
// the top set bit of the range down: each pass histograms the still-active values in
// a 256-entry LDS scratch owned by this wave, finds the bucket holding rank K by a
// wave prefix scan and keeps only that bucket. ceil(bits(range)/8) passes (<= 8).
// Requires 0 <= K < #valid. Every lane returns the result.
template <int CPL>
__device__ uint64_t wave_select_kth(const uint64_t (&v)[CPL], const bool (&ok)[CPL], int K,
                                    uint32_t* __restrict__ hist) {
    const int lane = lane_id();
    uint64_t lo = ~0ull, hi = 0;
#pragma unroll
    for (int q = 0; q < CPL; q++)
        if (ok[q]) { lo = v[q] < lo ? v[q] : lo; hi = v[q] > hi ? v[q] : hi; }
    lo = wave_min_u64(lo);
    hi = wave_max_u64(hi);
    bool act[CPL];
#pragma unroll
    for (int q = 0; q < CPL; q++) act[q] = ok[q];
    uint64_t base = lo;
    uint64_t range = hi - lo;
    int k = K;
    while (range != 0) {
        int bits = 64 - __clzll((long long)range);
        const int shift = bits > 8 ? bits - 8 : 0;
#pragma unroll
        for (int t = 0; t < 4; t++) hist[lane * 4 + t] = 0;
        wave_lds_fence();
#pragma unroll
        for (int q = 0; q < CPL; q++)
            if (act[q]) atomicAdd(&hist[(uint32_t)((v[q] - base) >> shift)], 1u);
        wave_lds_fence();
        uint32_t h[4], s = 0;
#pragma unroll
        for (int t = 0; t < 4; t++) { h[t] = hist[lane * 4 + t]; s += h[t]; }
        uint32_t incl = s;   // inclusive prefix over lanes
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = __shfl_up(incl, o);
            if (lane >= o) incl += y;
        }
        const uint32_t excl = incl - s;
        // the lane whose [excl, incl) holds k owns the bucket
        int bucket = -1;
        uint32_t below = 0;
        if ((uint32_t)k >= excl && (uint32_t)k < incl) {
            uint32_t acc = excl;
#pragma unroll
            for (int t = 0; t < 4; t++) {
                if (bucket < 0 && (uint32_t)k < acc + h[t]) { bucket = lane * 4 + t; below = acc; }
                acc += h[t];
            }
        }
        const uint64_t bm = __ballot(bucket >= 0);
        const int src = __ffsll((unsigned long long)bm) - 1;
        bucket = __shfl(bucket, src);
        below = __shfl(below, src);
        wave_lds_fence();
        k -= (int)below;
        const uint64_t nb = base + ((uint64_t)bucket << shift);
#pragma unroll
        for (int q = 0; q < CPL; q++) act[q] = act[q] && ((v[q] - base) >> shift) == (uint64_t)bucket;
        if (shift == 0) return nb;
        const uint64_t top = nb + ((1ull << shift) - 1);
        base = nb;
        range = (top < hi ? top : hi) - nb;
        // shrink to the actual active values for a tighter next pass
        uint64_t alo = ~0ull, ahi = 0;
#pragma unroll
        for (int q = 0; q < CPL; q++)
            if (act[q]) { alo = v[q] < alo ? v[q] : alo; ahi = v[q] > ahi ? v[q] : ahi; }
        alo = wave_min_u64(alo);
        ahi = wave_max_u64(ahi);
        base = alo;
        range = ahi - alo;
    }
    return base;
}

// Inclusive wave scans in lane order on DPP (GFX9 row_shr 1/2/4/8 within rows of 16,
// then row_bcast 15 / 31 across rows): a few VALU ops instead of ds_bpermute shuffles.
// Lanes without a DPP source keep the identity `id`.
#define HGX_DPP_SCAN(x, id, OP)                                                                  \
    do {                                                                                         \
        x = OP(x, (uint32_t)__builtin_amdgcn_update_dpp((int)(id), (int)(x), 0x111, 0xf, 0xf, false)); \
        x = OP(x, (uint32_t)__builtin_amdgcn_update_dpp((int)(id), (int)(x), 0x112, 0xf, 0xf, false)); \
        x = OP(x, (uint32_t)__builtin_amdgcn_update_dpp((int)(id), (int)(x), 0x114, 0xf, 0xf, false)); \
        x = OP(x, (uint32_t)__builtin_amdgcn_update_dpp((int)(id), (int)(x), 0x118, 0xf, 0xf, false)); \
        x = OP(x, (uint32_t)__builtin_amdgcn_update_dpp((int)(id), (int)(x), 0x142, 0xa, 0xf, false)); \
        x = OP(x, (uint32_t)__builtin_amdgcn_update_dpp((int)(id), (int)(x), 0x143, 0xc, 0xf, false)); \
    } while (0)
#define HGX_OP_ADD(a, b) ((a) + (b))
#define HGX_OP_MIN(a, b) min((a), (b))
#define HGX_OP_MAX(a, b) max((a), (b))

__device__ __forceinline__ uint32_t wave_scan_add_u32(uint32_t x) { HGX_DPP_SCAN(x, 0u, HGX_OP_ADD); return x; }
// wave-wide min / max of a u32, returned in an SGPR (lane 63 of the inclusive scan)
__device__ __forceinline__ uint32_t wave_reduce_min_u32(uint32_t x) {
    HGX_DPP_SCAN(x, 0xffffffffu, HGX_OP_MIN);
    return (uint32_t)__builtin_amdgcn_readlane((int)x, 63);
}
__device__ __forceinline__ uint32_t wave_reduce_max_u32(uint32_t x) {
    HGX_DPP_SCAN(x, 0u, HGX_OP_MAX);
    return (uint32_t)__builtin_amdgcn_readlane((int)x, 63);
}

// 32-bit k-th smallest for the common case (values already rebased): radix select with
// 8-bit digits from the top set bit of the range. Reductions and the bucket scan run on
// DPP, the chosen bucket is read from the owning lane with readlane, and the wave's
// 256-bin histogram (16-B aligned, lane l owns bins 4l..4l+3) is zeroed and read as one
// 16-B access per lane. Requires 0 <= K < #valid; every lane returns the result.
template <int CPL>
__device__ uint32_t wave_select_kth32(const uint32_t (&v)[CPL], const bool (&ok)[CPL], int K,
                                      uint32_t* __restrict__ hist) {
    const int lane = lane_id();
    uint32_t lo = 0xffffffffu, hi = 0;
#pragma unroll
    for (int q = 0; q < CPL; q++)
        if (ok[q]) { lo = min(lo, v[q]); hi = max(hi, v[q]); }
    lo = wave_reduce_min_u32(lo);
    hi = wave_reduce_max_u32(hi);
    const uint32_t range = hi - lo;
    if (range == 0) return lo;
    const int bits = 32 - __clz((int)range);
    uint32_t d[CPL];
    bool act[CPL];
#pragma unroll
    for (int q = 0; q < CPL; q++) { d[q] = v[q] - lo; act[q] = ok[q]; }
    uint4* __restrict__ h4 = (uint4*)hist;
    uint32_t prefix = 0;
    uint32_t k = (uint32_t)K;
    for (int shift = ((bits - 1) / 8) * 8; shift >= 0; shift -= 8) {
        h4[lane] = make_uint4(0u, 0u, 0u, 0u);
        wave_lds_fence();
#pragma unroll
        for (int q = 0; q < CPL; q++)
            if (act[q]) atomicAdd(&hist[(d[q] >> shift) & 255u], 1u);
        wave_lds_fence();
        const uint4 h = h4[lane];
        const uint32_t sum = h.x + h.y + h.z + h.w;
        const uint32_t incl = wave_scan_add_u32(sum);
        const uint32_t excl = incl - sum;
        // bucket of the k-th value inside this lane's 4 bins (meaningful in one lane)
        const uint32_t a1 = excl + h.x, a2 = a1 + h.y, a3 = a2 + h.z;
        const int bt = (k < a1) ? 0 : (k < a2) ? 1 : (k < a3) ? 2 : 3;
        const uint32_t below = (k < a1) ? excl : (k < a2) ? a1 : (k < a3) ? a2 : a3;
        const uint64_t bm = __ballot(k >= excl && k < incl);
        const int src = (int)__builtin_ctzll(bm);
        const uint32_t bucket = (uint32_t)__builtin_amdgcn_readlane(lane * 4 + bt, src);
        k -= (uint32_t)__builtin_amdgcn_readlane((int)below, src);
        wave_lds_fence();
        prefix |= bucket << shift;
#pragma unroll
        for (int q = 0; q < CPL; q++) act[q] = act[q] && ((d[q] >> shift) & 255u) == bucket;
    }
    return lo + prefix;
}

// The same k-th smallest by bisection on the value: each step counts the valid values <= mid with
// CPL compares whose ballots are popcounted in SGPRs (no LDS, no atomics). For rows whose values
// crowd into a few buckets (the witnesses' lastAncestors of one chain in k_threshold span a few
// dozen indices), the radix select's LDS atomics hit the same bins from most lanes and serialise;
// here a step costs CPL VALU compares and a handful of scalar ops, log2(range) steps.
template <int CPL>
__device__ uint32_t wave_select_kth32_bisect(const uint32_t (&v)[CPL], const bool (&ok)[CPL], int K) {
    uint32_t lo = 0xffffffffu, hi = 0;
#pragma unroll
    for (int q = 0; q < CPL; q++)
        if (ok[q]) { lo = min(lo, v[q]); hi = max(hi, v[q]); }
    lo = wave_reduce_min_u32(lo);
    hi = wave_reduce_max_u32(hi);
    uint32_t a = 0, b = hi - lo;   // answer in [a, b]: the smallest t with #(v - lo <= t) > K
    uint32_t d[CPL];
#pragma unroll
    for (int q = 0; q < CPL; q++) d[q] = ok[q] ? v[q] - lo : 0xffffffffu;   // (invalid: above every t < 2^32 - 1)
    while (a < b) {
        const uint32_t mid = a + ((b - a) >> 1);
        int cnt = 0;
#pragma unroll
        for (int q = 0; q < CPL; q++) cnt += __popcll(__ballot(d[q] <= mid));
        if (cnt > K) b = mid;
        else a = mid + 1;
    }
    return lo + a;
}

}  // namespace hgx
