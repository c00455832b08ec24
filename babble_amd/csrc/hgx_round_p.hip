// Persistent round recurrence: one resident workgroup per chain runs every round of a
// DivideRounds in ONE launch (RoundInc, hashgraph.go:285-305; StronglySee :170-198;
// DivideRounds :616-646). DESIGN.md §3.3.
//
// Round s of chain c finds Bm[s+1][c] = the first offset k >= Bm[s][c] whose event strongly
// sees >= SM candidates of W'_s (the first event of each chain with round >= s), exactly as
// k_round_k does (same per-candidate binary search over a window of 31 probe rows, same 8-bit
// SWAR compare, same K(w) histogram). What changes is how the rounds are chained:
//  * the workgroup of chain c stays resident for all rounds. Its own boundary is the start of
//    its next window, so the window's raw lastAncestors rows and firstDescendants columns are
//    staged by LDS-DMA right after the boundary is known, while the other chains finish;
//  * the only data a round needs from other workgroups is W'_s: for each chain its boundary
//    and its candidate's rebased firstDescendants row. The producer (the workgroup that found
//    the candidate) stores the row and an 8-byte granule {tag = s + 1, boundary | flags}, both
//    write-through (sc1), without a drain in between: both are self-validating. The granule
//    carries its round tag; the row's bytes are rebased values in [1, 127], so bit 7 of every
//    byte is free and carries a validity bit v(s) = (s >> 2) & 1, with the rows of round s in
//    buffer s % 4: the previous contents of that buffer are round s - 4's rows, whose v is the
//    opposite. A consumer wave loads the granules and the rows of ITS candidates together (sc1
//    loads, one hop), and reloads until every granule carries tag s + 1 and every row of a
//    candidate that exists has every bit 7 equal to v(s) (4-byte stores are single-copy atomic,
//    so a dword is old or new as a whole); a wave whose candidates arrived early searches while
//    the last producers still run. These are MI355X_MICROARCH.md's data-tagged granules
//    (handoff-1to1): no producer drain, no separate flag hop; one workgroup per CU, hipMalloc
//    memory, sc1 stores and loads of every handed-off byte;
//  * no grid barrier and no kernel boundary per round; every wait is bounded (s_memrealtime),
//    a workgroup that gives up raises the abort word, every workgroup then leaves, and the
//    host reruns the rounds with the per-launch step (k_round_k).
// A candidate row that does not fit 8 bits is flagged in its granule and that candidate alone
// is counted with exact int32 compares (k_round_k flags the whole round instead).
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

#include "hgx_device.h"
#include "hgx_kernels.h"

namespace hgx {

typedef __attribute__((address_space(1))) uint64_t gu64;
typedef __attribute__((address_space(1))) uint32_t gu32;
typedef __attribute__((address_space(3))) void* lds_ptr_t;

constexpr int kRpP = 31;       // probes per window (K in [0, 31], 5 binary-search levels)
constexpr int kRpSlots = 4;    // granule ring slots (a slot is rewritten 4 rounds later)
constexpr uint32_t kRpEx = 1u << 31, kRpOv = 1u << 30, kRpBm = (1u << 30) - 1;

// Optional phase clocks (-DHGX_STEP_PROF, build variant "prof"): thread 0 of each workgroup adds
// s_memtime deltas per phase of every round, flushed once at the end of the launch.
#ifdef HGX_STEP_PROF
// slots: 0 rebase, 1 poll, 2 rows, 3 search, 4 boundary, 5 granule, 6 outputs, 7 staging wait,
// 8 staging issue, 9 row build + stores; 15 = block-rounds
__device__ unsigned long long hgx_rp_prof[16];
#define RP_PROF_BEGIN() long long _pt = clock64(); unsigned long long _pa[16] = {}
#define RP_PROF(i)                                                \
    do {                                                          \
        if (threadIdx.x == 0) {                                   \
            const long long _t = clock64();                       \
            _pa[i] += (unsigned long long)(_t - _pt);             \
            _pt = _t;                                             \
            if ((i) == 6) _pa[15] += 1;                           \
        }                                                         \
    } while (0)
#define RP_PROF_COUNT(i)                                          \
    do {                                                          \
        if (threadIdx.x == 0) _pa[i] += 1;                        \
    } while (0)
#define RP_PROF_END()                                                              \
    do {                                                                           \
        if (threadIdx.x == 0)                                                      \
            for (int _i = 0; _i < 16; _i++)                                        \
                if (_pa[_i]) atomicAdd(&hgx_rp_prof[_i], _pa[_i]);                 \
    } while (0)
void round_p_prof_dump() {
    unsigned long long h[16];
    if (hipMemcpyFromSymbol(h, HIP_SYMBOL(hgx_rp_prof), sizeof(h)) != hipSuccess) return;
    const double r = h[15] ? (double)h[15] : 1.0;
    fprintf(stderr, "[hgx] k_round_p clk per block-round (thread 0): staging-wait %.0f barrier %.0f rebase %.0f poll %.0f "
            "rows %.0f search-levels %.0f search-barrier %.0f boundary %.0f staging-issue %.0f row-build %.0f granule %.0f "
            "outputs %.0f | block-rounds %llu, synchronous stagings %llu, later windows %llu\n",
            h[7] / r, h[12] / r, h[0] / r, h[1] / r, h[2] / r, h[13] / r, h[3] / r, h[4] / r, h[8] / r, h[9] / r, h[5] / r,
            h[6] / r, h[15], h[10], h[11]);
    unsigned long long z[16] = {};
    (void)hipMemcpyToSymbol(HIP_SYMBOL(hgx_rp_prof), z, sizeof(z));
}
#else
#define RP_PROF_BEGIN() (void)0
#define RP_PROF(i) (void)0
#define RP_PROF_END() (void)0
#define RP_PROF_COUNT(i) (void)0
void round_p_prof_dump() {}
#endif

// ---- write-through hand-off primitives (MI355X_MICROARCH.md, Valid forms, row 1) ----------
__device__ __forceinline__ uint64_t rp_ld_gran(const uint64_t* p) {
    return __hip_atomic_load((gu64*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);   // sc1 load
}
__device__ __forceinline__ void rp_st_gran(uint64_t* p, uint64_t v) {
    __hip_atomic_store((gu64*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);      // sc1 store
}
__device__ __forceinline__ void rp_st_sc1(uint32_t* p, uint32_t v) {
    asm volatile("global_store_dword %0, %1, off sc1" ::"v"(p), "v"(v) : "memory");
}
__device__ __forceinline__ uint32_t rp_ld_abort(const int32_t* p) {
    return (uint32_t)__hip_atomic_load((gu32*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void rp_vm_drain() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
__device__ __forceinline__ void rp_lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// HD dwords of this lane's part of a candidate row, sc1 loads (every load of handed-off bytes)
template <int HD>
__device__ __forceinline__ void rp_ld_row(const uint32_t* p, uint32_t (&v)[HD]) {
    if constexpr (HD >= 4) {
#pragma unroll
        for (int k = 0; k < HD / 4; k++) {
            uint4 x;
            asm volatile("global_load_dwordx4 %0, %1, off sc1" : "=v"(x) : "v"(p + 4 * k) : "memory");
            v[4 * k] = x.x; v[4 * k + 1] = x.y; v[4 * k + 2] = x.z; v[4 * k + 3] = x.w;
        }
    } else if constexpr (HD == 2) {
        uint2 x;
        asm volatile("global_load_dwordx2 %0, %1, off sc1" : "=v"(x) : "v"(p) : "memory");
        v[0] = x.x; v[1] = x.y;
    } else {
        uint32_t x;
        asm volatile("global_load_dword %0, %1, off sc1" : "=v"(x) : "v"(p) : "memory");
        v[0] = x;
    }
}

// HD dwords of an LDS row, all reads in flight before one wait (16-byte reads when HD % 4 == 0)
template <int HD>
__device__ __forceinline__ void rp_lds_row(const uint32_t* p, uint32_t (&v)[HD]) {
    const uint32_t a = (uint32_t)(uintptr_t)p;
    if constexpr (HD % 4 == 0) {
        typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
        u32x4 r[HD / 4];
#pragma unroll
        for (int k = 0; k < HD / 4; k++) asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(r[k]) : "v"(a), "i"(16 * k));
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
        for (int k = 0; k < HD / 4; k++) {
            asm volatile("" : "+v"(r[k]));
            v[4 * k] = r[k].x; v[4 * k + 1] = r[k].y; v[4 * k + 2] = r[k].z; v[4 * k + 3] = r[k].w;
        }
    } else if constexpr (HD == 2) {
        uint64_t r;
        asm volatile("ds_read_b64 %0, %1" : "=v"(r) : "v"(a));
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        asm volatile("" : "+v"(r));
        v[0] = (uint32_t)r; v[1] = (uint32_t)(r >> 32);
    } else {
        uint32_t r;
        asm volatile("ds_read_b32 %0, %1" : "=v"(r) : "v"(a));
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        asm volatile("" : "+v"(r));
        v[0] = r;
    }
}

// sum over the Q adjacent lanes of a candidate (DPP: quad_perm xor 1, xor 2, half-row mirror)
template <int Q>
__device__ __forceinline__ uint32_t rp_combine(uint32_t x) {
    if constexpr (Q >= 2) x += (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0xB1, 0xf, 0xf, false);
    if constexpr (Q >= 4) x += (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x4E, 0xf, 0xf, false);
    if constexpr (Q >= 8) x += (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x141, 0xf, 0xf, false);
    return x;
}

constexpr int rp_part_stride(int hd) {   // smallest stride >= hd that is 8 or 24 (mod 32)
    int ps = hd;
    while (ps % 32 != 8 && ps % 32 != 24) ps++;
    return ps;
}

// geometry of one instantiation: n <= 4 NDW chains per graph; candidate j's row is split over
// Q adjacent lanes (HD dwords each); T threads
template <typename CT, int NDW, int Q>
struct RpCfg {
    static constexpr int NC = 4 * NDW;
    static constexpr int HD = NDW / Q;
    static constexpr int T = (NC * Q < 64) ? 64 : NC * Q;
    static constexpr int NW = T / 64;
    // 8-bit window rows: part q of a row (HD dwords, what one lane of a candidate compares) at
    // q * PS with PS = 8 or 24 (mod 32), so the Q lanes of a candidate read disjoint bank groups,
    // and rows RS = Q * PS + 4 dwords apart (consecutive rows shifted by 4 banks)
    static constexpr int PS = rp_part_stride(HD);
    static constexpr int WS = Q * PS + 4;                      // row stride (dwords)
    static constexpr int CSZ = (int)sizeof(CT);
    // staging ring: NSEG segments of SEG positions (64 bytes of one firstDescendants column) of
    // the chain's rows; segment m (positions [SEG m, SEG m + SEG) from the chain's start) sits in
    // slot m % NSEG
    static constexpr int SEG = 64 / CSZ, NSEG = 4, RR = SEG * NSEG;
    static constexpr int SEG_RAW = SEG * NC * CSZ;               // bytes: raw lastAncestors rows of a segment
    static constexpr int KR16 = (SEG_RAW / 16 + T - 1) / T;      // 16-byte DMA per lane per segment
    static constexpr int CW = 16;                                // dwords per staged FD column (SEG positions)
    static constexpr int CPI = 4;                                // FD columns per DMA instruction (a group)
    static constexpr int KF = (NDW + NW - 1) / NW;               // groups per wave per segment
    static constexpr int SEG_FD = NDW * 65 * 4;                  // bytes: groups of 64 dwords + 1 pad
    // LDS carve (bytes, 16-aligned)
    static constexpr int O_WIN = 0;
    static constexpr int O_RAW = O_WIN + ((kRpP * WS * 4 + 15) & ~15);   // [RR][n] raw rows
    static constexpr int O_FD = O_RAW + NSEG * SEG_RAW;                   // [NSEG][NDW groups][65]
    static constexpr int O_CB = O_FD + NSEG * SEG_FD;                     // c_base[NC]
    static constexpr int O_CO = O_CB + NC * 4;                           // c_off[NC]
    static constexpr int O_BM0 = O_CO + NC * 4;                          // Bm of the candidates, by round parity
    static constexpr int O_BM1 = O_BM0 + NC * 4;
    static constexpr int O_HIST = O_BM1 + NC * 4;                        // 32 bins
    static constexpr int SBW = (NC / 32 + 4 + 3) & ~3;                   // S row words per buffer
    static constexpr int O_SB = O_HIST + 32 * 4;                         // S row bits [2][SBW], by round parity
    static constexpr int O_MISC = O_SB + 2 * SBW * 4;                    // [0] B, [1] tot, [2] any, [3] fail
    static constexpr int USED = O_MISC + 64;
    // at least 82 KB: one workgroup per CU (the hand-off rule's geometry), whatever fits
    static constexpr int LDS = USED > 84 * 1024 ? USED : 84 * 1024;
    static_assert(USED <= 160 * 1024, "k_round_p: LDS carve exceeds a CU's 160 KB");
};

struct RoundPArgs {
    RoundArgs A;
    uint32_t* FD8p;     // [4][C][ndw] rebased candidate rows, row-major (round s: buffer s % 4, bit 7 of
                        // every byte = v(s) = (s >> 2) & 1)
    uint64_t* gran;     // [kRpSlots][C]
    int32_t* st;        // [0] abort, [1] max over graphs of the round each stopped at, [2] graphs that
                        // finished (W'_s empty) in this launch, [3] rows counted exactly (over 8 bits)
    int32_t* fin;       // [G] the round at which graph g found W'_s empty (-1: not yet, this call)
    int r0, r_end;      // rounds [r0, r_end) at most
    long long tmo;      // one wait's budget in s_memrealtime ticks (100 MHz)
};

template <typename CT, int NDW, int Q>
__global__ void __launch_bounds__((4 * NDW * Q < 64) ? 64 : 4 * NDW * Q) k_round_p(RoundPArgs P) {
    typedef RpCfg<CT, NDW, Q> K;
    constexpr int HD = K::HD, T = K::T, WS = K::WS;
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    const RoundArgs& A = P.A;
    const int n = A.n, C = A.C, sm = A.sm;
    const int t = threadIdx.x, lane = lane_id(), wave = __builtin_amdgcn_readfirstlane(t >> 6);
    const int gc = blockIdx.x, g = gc / n, cl = gc % n, g0 = g * n;
    const int j = t / Q, q = t % Q;              // candidate slot and row part of this lane
    const bool jv = j < n && t < K::NC * Q;      // a real chain of the graph
    uint32_t* win = (uint32_t*)(lds + K::O_WIN);
    int32_t* cbase = (int32_t*)(lds + K::O_CB);
    int32_t* coff = (int32_t*)(lds + K::O_CO);
    int32_t* hist = (int32_t*)(lds + K::O_HIST);
    uint32_t* sbits_all = (uint32_t*)(lds + K::O_SB);
    int32_t* misc = (int32_t*)(lds + K::O_MISC);

    if (P.fin[g] >= 0) return;   // the graph finished in an earlier launch of this DivideRounds
    const int len = A.c_len[gc], off = A.c_off[gc];
    for (int i = t; i < n; i += T) {
        cbase[i] = A.c_base[g0 + i];
        coff[i] = A.c_off[g0 + i];
        // Bm of round r0 - 1 (bases of round r0's window), written by earlier launches
        ((int32_t*)(lds + (((P.r0 - 1) & 1) ? K::O_BM1 : K::O_BM0)))[i] = P.r0 > 0 ? A.Bm[(size_t)(P.r0 - 1) * C + g0 + i] : 0;
    }
    int b = A.Bm[(size_t)P.r0 * C + gc];

    // ---- staging ring (LDS-DMA, fixed instruction counts per wave): segment m = the raw
    // lastAncestors rows and firstDescendants columns at positions [SEG m, SEG m + SEG) of the
    // chain; chain offsets are multiples of 32 (hgx_engine.cpp layout), so every segment is
    // 64-byte aligned in both arrays. Rows past the chain's end lie in its slot's slack (read,
    // never used).
    constexpr int SEG = K::SEG, NSEG = K::NSEG, RR = K::RR;
    const int last_seg = len > 0 ? (len - 1) / SEG : -1;
    int seg_hi = -1;   // highest segment staged (uniform); [seg_hi - NSEG + 1, seg_hi] are resident
    auto stage_seg = [&](int m) {
        const int slot = m % NSEG;
        const uint32_t* __restrict__ src = (const uint32_t*)((const uint8_t*)A.LA + ((size_t)off + (size_t)m * SEG) * n * K::CSZ);
        uint32_t* raw_w = (uint32_t*)(lds + K::O_RAW + slot * SEG * n * K::CSZ);   // rows (p % RR) * n
        const int nch = SEG * n * K::CSZ / 16;   // 16-byte chunks
#pragma unroll
        for (int k = 0; k < K::KR16; k++) {
            const int c0 = wave * 64 + k * T;    // this wave instruction's first chunk
            if (c0 + lane < nch)
                __builtin_amdgcn_global_load_lds((const void*)(src + 4 * (c0 + lane)), (lds_ptr_t)(raw_w + 4 * c0), 16, 0, 0);
        }
        // columns: lane = (column % 4, dword); one instruction = one group of 4 columns
        const int icol = lane >> 4, pcol = lane & 15;
        const uint32_t* __restrict__ fsrc = (const uint32_t*)((const uint8_t*)A.FDT + ((size_t)off + (size_t)m * SEG) * K::CSZ) + pcol;
        const size_t cstride = (size_t)A.Pcap * K::CSZ / 4;   // dwords between columns
        uint32_t* fd_w = (uint32_t*)(lds + K::O_FD + slot * K::SEG_FD);
#pragma unroll
        for (int k = 0; k < K::KF; k++) {
            const int grp = min(wave + k * K::NW, NDW - 1);
            const int i = min(grp * 4 + icol, n - 1);
            __builtin_amdgcn_global_load_lds((const void*)(fsrc + (size_t)i * cstride), (lds_ptr_t)(fd_w + grp * 65), 4, 0, 0);
        }
    };
    // segments [max(seg_hi + 1, lo), hi] (hi <= lo + NSEG - 1: a slot is reused only when its
    // segment is below lo)
    auto stage_range = [&](int lo, int hi) {
        for (int m = max(seg_hi + 1, lo); m <= hi; m++) stage_seg(m);
        seg_hi = max(seg_hi, hi);
    };
    auto fd_at = [&](int i, int p) -> CT {   // staged FD of coordinate i at chain offset p
        const uint8_t* fd_w = lds + K::O_FD + ((p / SEG) % NSEG) * K::SEG_FD;
        return *(const CT*)(fd_w + ((i >> 2) * 65 + (i & 3) * 16) * 4 + (p % SEG) * K::CSZ);
    };
    auto raw_at = [&](int p, int i) -> CT {   // staged lastAncestors row of chain offset p
        return ((const CT*)(lds + K::O_RAW))[(p % RR) * n + i];
    };
    // rebased 8-bit window rows (0x80 | clamp(LA - base + 1, 0, 126)) of the window [kb, kb + np)
    typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
    auto rebase = [&](int kb, int np, const int32_t* bmp) {
        constexpr int RS = T / NDW > 0 ? T / NDW : 1;   // rows per pass
        for (int d = t % NDW; d < NDW; d += T) {
            const int i0 = 4 * d;
            int32_t bq[4];
#pragma unroll
            for (int u = 0; u < 4; u++) bq[u] = (i0 + u < n) ? cbase[i0 + u] + bmp[i0 + u] : 0;
            for (int p = t / NDW; p < np; p += RS) {
                uint32_t w;
                if constexpr (K::CSZ == 2) {
                    const uint32_t* rp = (const uint32_t*)(lds + K::O_RAW) + (((kb + p) % RR) * n + i0) / 2;
                    const uint32_t r01 = i0 < n ? rp[0] : 0u, r23 = i0 + 2 < n ? rp[1] : 0u;
                    const u16x2 b01 = {(unsigned short)bq[0], (unsigned short)bq[1]};
                    const u16x2 b23 = {(unsigned short)bq[2], (unsigned short)bq[3]};
                    const u16x2 cap = {126, 126};
                    const u16x2 y01 = __builtin_elementwise_min(__builtin_elementwise_sub_sat(__builtin_bit_cast(u16x2, r01), b01), cap);
                    const u16x2 y23 = __builtin_elementwise_min(__builtin_elementwise_sub_sat(__builtin_bit_cast(u16x2, r23), b23), cap);
                    w = __builtin_amdgcn_perm(__builtin_bit_cast(uint32_t, y23), __builtin_bit_cast(uint32_t, y01), 0x06040200u) |
                        0x80808080u;
                } else {
                    w = 0x80808080u;
#pragma unroll
                    for (int u = 0; u < 4; u++) {
                        if (i0 + u < n) {
                            const int32_t x = Coord<CT>::la(raw_at(kb + p, i0 + u)) - bq[u] + 1;
                            w |= (uint32_t)min(max(x, 0), 126) << (8 * u);
                        }
                    }
                }
                win[p * WS + (d / HD) * K::PS + d % HD] = w;
            }
        }
    };

    // round r's outputs (the per-launch step writes the same): rounds of the chain's events
    // [o_b, o_kstar), wstat / wflag / Bm, the new candidate's WLA / WFD rows (its segment stays
    // staged: o_kstar is the next window's start) and its S row (sbits buffer r & 1)
    int o_b = 0, o_kstar = 0;
    auto outputs = [&](int r, int tid, int nthr) {   // by threads [0, nthr) (tid = this thread's)
        const bool o_have = o_b < len, o_nx = o_kstar < len;
        for (int k = o_b + tid; k < o_kstar; k += nthr) A.p_round[off + k] = r;
        if (tid == 0) {
            A.wstat[(size_t)r * C + gc] = o_have ? ((o_kstar > o_b) ? 2 : 1) : 0;
            A.wflag[(size_t)(r + 1) * C + gc] = o_nx ? 1 : 0;
            A.Bm[(size_t)(r + 1) * C + gc] = o_kstar;
            if (o_nx) A.active[r] = 1;
        }
        if (o_nx) {
            const size_t nrow = ((size_t)(r + 1) * C + gc) * n;
            for (int i = tid; i < n; i += nthr) {
                A.WLA[nrow + i] = Coord<CT>::la(raw_at(o_kstar, i));
                const CT f = fd_at(i, o_kstar);
                if constexpr (K::CSZ == 2) ((uint16_t*)A.WFD)[nrow + i] = f;
                else A.WFD[nrow + i] = f;
            }
            const uint32_t* sb = sbits_all + (r & 1) * K::SBW;
            const size_t srow = ((size_t)(r + 1) * C + gc) * A.nw;
            for (int wd = tid; wd < A.nw; wd += nthr)
                A.Smat[srow + wd] = (uint64_t)sb[2 * wd] | ((2 * wd + 1 < K::NC / 32 + 1 ? (uint64_t)sb[2 * wd + 1] : 0) << 32);
        }
    };
    RP_PROF_BEGIN();
    int s = P.r0;
    bool failed = false;
    for (;; s++) {
        if (s >= P.r_end) break;   // capacity: the host continues from round s
        const int32_t* bm_prev = (const int32_t*)(lds + (((s - 1) & 1) ? K::O_BM1 : K::O_BM0));
        int32_t* bm_cur = (int32_t*)(lds + ((s & 1) ? K::O_BM1 : K::O_BM0));
        const bool have = b < len;   // block-uniform
        int kb = b, np = have ? min(kRpP, len - b) : 0;
        // (a) the first load of this lane's candidate granule and row part (W'_s) goes out first
        // and is in flight while this round's window (staged at the end of the previous round,
        // before these loads) lands and is rebased to base(s). Every lane issues them (a clamped
        // address for the lanes past n), so the vmcnt below covers exactly the staging.
        const uint64_t* gp = P.gran + (size_t)(s % kRpSlots) * C + g0 + (jv ? j : 0);
        const uint32_t* rowp = P.FD8p + ((size_t)(s & (kRoundPBufs - 1)) * C + g0 + (jv ? j : 0)) * NDW + q * HD;
        const uint32_t vbit = ((s >> 2) & 1) ? 0x80808080u : 0u;
        uint64_t gv = rp_ld_gran(gp);
        uint32_t fd[HD];
        rp_ld_row<HD>(rowp, fd);
        // No wait here: the window's segments were staged two rounds ago or earlier, and every
        // wave's poll drain of the previous round waited for them (the end-of-round barrier then
        // covers every wave). Waiting here would also wait for the previous round's stores.
        uint32_t* sbits = sbits_all + (s & 1) * K::SBW;
        if (have && min((b + kRpP - 1) / SEG, last_seg) > seg_hi) {
            // the window is not staged yet (the first round of a launch, or a chain that advanced
            // by more than the ring's lookahead): stage it now and wait for it
            stage_range(b / SEG, min(b / SEG + NSEG - 1, last_seg));
            rp_vm_drain();
            RP_PROF_COUNT(10);
        }
        RP_PROF(7);
        if (t < 32) hist[t] = 0;
        if (t == 0) { misc[2] = 0; misc[3] = 0; }
        if (t < K::NC / 32 + 1) sbits[t] = 0;
        rp_lds_barrier();
        RP_PROF(12);
        if (have) rebase(b, np, bm_prev);
        rp_lds_barrier();
        RP_PROF(0);

        // (b) until every candidate of this wave is published: its granule carries tag s + 1 and,
        // when the candidate exists, every byte of its row part carries v(s); reload otherwise
        bool wfail = false;
        {
            const long long tw = __builtin_amdgcn_s_memrealtime();
            for (int spins = 0;; spins++) {
                rp_vm_drain();
#pragma unroll
                for (int d = 0; d < HD; d++) asm volatile("" : "+v"(fd[d]));
                uint32_t bad = 0;
#pragma unroll
                for (int d = 0; d < HD; d++) bad |= (fd[d] ^ vbit) & 0x80808080u;
                const bool tag_ok = (uint32_t)(gv >> 32) == (uint32_t)(s + 1);
                const bool ok = !jv || (tag_ok && (!((uint32_t)gv & kRpEx) || bad == 0));
                if (__all(ok)) break;
                if ((spins & 31) == 31) {
                    const long long now = __builtin_amdgcn_s_memrealtime();
                    if (now - tw > P.tmo || rp_ld_abort(P.st) != 0) { wfail = true; break; }
                }
                __builtin_amdgcn_s_sleep(1);
                if (!ok) {
                    gv = rp_ld_gran(gp);
                    rp_ld_row<HD>(rowp, fd);
                }
            }
        }
        RP_PROF(1);
        const uint32_t gval = (uint32_t)gv;
        const bool cand = jv && !wfail && (gval & kRpEx);
        const bool ov = cand && (gval & kRpOv);
        const int bmj = (int)(gval & kRpBm);
        if (jv && q == 0 && !wfail) bm_cur[j] = bmj;
        if (cand && have) {
#pragma unroll
            for (int d = 0; d < HD; d++) fd[d] &= 0x7F7F7F7Fu;   // the validity bits off: rebased values
        } else {
#pragma unroll
            for (int d = 0; d < HD; d++) fd[d] = 0x7F7F7F7Fu;   // never seen
        }
        if (wfail && lane == 0) misc[3] = 1;
        if (cand && q == 0) misc[2] = 1;   // (same value from every writer)
        // the ring ahead: segments up to b / SEG + NSEG - 1, landing behind the search, the
        // publish and the outputs (the next round's first wait covers them; a window after a
        // first-window boundary lies below b / SEG + 3)
        if (have) stage_range(b / SEG, min(b / SEG + NSEG - 1, last_seg));
        RP_PROF(2);

        // (c) search, window after window until the boundary is found (a later window is rare)
        int kstar = len, B = -1, K_last = kRpP, carried = 0;
        bool done = false;
        const bool wave_cand = __any(cand) && have;
        for (; have;) {
            int lo = 0, hi = kRpP;
            if (wave_cand) {
#pragma unroll 1
                for (int it = 0; it < 5; it++) {
                    const int mid = (lo + hi) >> 1;
                    uint32_t cnt = 0;
                    if (!ov) {
                        uint32_t v[HD];
                        rp_lds_row<HD>(win + mid * WS + q * K::PS, v);
#pragma unroll
                        for (int d = 0; d < HD; d++) cnt += __builtin_popcount((v[d] - fd[d]) & 0x80808080u);
                    } else if (!done && mid < np) {
                        // exact int32 compares of this part of the row (hashgraph.go:191-197)
                        const int i_lo = q * HD * 4, i_hi = min(n, (q + 1) * HD * 4);
                        const size_t pos = (size_t)coff[j] + bmj;
                        for (int i = i_lo; i < i_hi; i++) {
                            const int32_t fdv = Coord<CT>::fd(((const CT*)A.FDT)[(size_t)i * A.Pcap + pos]);
                            const int32_t lav = min(Coord<CT>::la(raw_at(kb + mid, i)), kMaxI32 - 1);
                            cnt += lav >= fdv ? 1u : 0u;
                        }
                    }
                    cnt = rp_combine<Q>(cnt);
                    const bool seen = done || mid >= np || ((int)cnt >= sm && !(j == cl && kb + mid == b));
                    if (seen) hi = mid; else lo = mid + 1;
                }
            }
            const int Kw = lo;
            RP_PROF(13);
            if (cand && q == 0 && !done && Kw < np) atomicAdd(&hist[Kw], 1);
            rp_lds_barrier();
            RP_PROF(3);
            if (wave == 0) {   // boundary: first probe where #{K <= p} (+ seen in earlier windows) >= SM
                const uint32_t v = lane < np ? (uint32_t)hist[lane] : 0u;
                const uint32_t inc = wave_scan_add_u32(v) + (uint32_t)carried;
                const uint64_t m = __ballot(lane < np && (int)inc >= sm);
                const int tot = __builtin_amdgcn_readlane((int)inc, 63);
                if (lane == 0) { misc[0] = m ? (int)__builtin_ctzll(m) : -1; misc[1] = tot; }
            }
            rp_lds_barrier();
            B = misc[0];
            K_last = Kw;
            if (B >= 0 || misc[2] == 0 || misc[3] != 0) {
                if (B >= 0) kstar = kb + B;
                break;
            }
            // no boundary in this window: the next one (synchronous staging)
            RP_PROF_COUNT(11);
            carried = misc[1];
            if (cand && Kw < np) done = true;
            kb += np;
            if (kb >= len) break;
            np = min(kRpP, len - kb);
            if (t < 32) hist[t] = 0;
            if (min((kb + kRpP - 1) / SEG, last_seg) > seg_hi) stage_range(kb / SEG, min(kb / SEG + NSEG - 1, last_seg));
            rp_vm_drain();
            __syncthreads();
            rebase(kb, np, bm_prev);
            rp_lds_barrier();
        }
        if (!have) rp_lds_barrier();   // the pollers' any / fail words
        RP_PROF(4);
        if (misc[3] != 0) { failed = true; break; }
        if (misc[2] == 0) break;       // W'_s is empty: no round s (every workgroup of the graph agrees)

        // (d) wave 0 publishes W'_{s+1} of chain c: its rebased row (base(s+1) = c_base + Bm[s],
        // bit 7 of every byte = v(s + 1)) and its granule, written through with no drain in between
        // (both self-validating)
        const bool nx = kstar < len;
        RP_PROF(8);
        bool of = false;
        if (wave == 0 && nx) {
            const uint32_t vb1 = (((s + 1) >> 2) & 1) ? 0x80808080u : 0u;
            uint32_t* dst = P.FD8p + ((size_t)((s + 1) & (kRoundPBufs - 1)) * C + gc) * NDW;
            for (int d = lane; d < NDW; d += 64) {
                uint32_t w = 0;
#pragma unroll
                for (int u = 0; u < 4; u++) {
                    const int i = 4 * d + u;
                    uint32_t v = 127u;
                    if (i < n) {
                        const int32_t f = Coord<CT>::fd(fd_at(i, kstar));
                        if (f != kMaxI32) {
                            const int32_t x = f - (cbase[i] + bm_cur[i]) + 1;
                            if (x > 126) of = true;
                            else v = (uint32_t)x;
                        }
                    }
                    w |= v << (8 * u);
                }
                rp_st_sc1(dst + d, w | vb1);
            }
        }
        RP_PROF(9);
        if (wave == 0) {
            of = __any(of);
            if (lane == 0)
                rp_st_gran(P.gran + (size_t)((s + 1) % kRpSlots) * C + gc,
                           ((uint64_t)(uint32_t)(s + 2) << 32) | (uint32_t)kstar | (nx ? kRpEx : 0u) | (of ? kRpOv : 0u));
            if (of && lane == 0) atomicAdd(&P.st[3], 1);   // rows counted exactly (instrumentation)
        }
        RP_PROF(5);
        // (e) the S row of the new candidate, then the round's outputs
        if (have && nx && cand && q == 0 && (done || K_last <= B)) atomicOr(&sbits[j >> 5], 1u << (j & 31));
        o_b = b;
        o_kstar = kstar;
        rp_lds_barrier();   // the S row bits are complete
        outputs(s, t, T);
        b = kstar;
        rp_lds_barrier();   // every read of this round's LDS is done
        RP_PROF(6);
    }

    rp_vm_drain();   // no LDS-DMA outlives the workgroup
    RP_PROF_END();
    if (failed) {
        // the first workgroup to give up records its chain and round (st[3] then holds the
        // round, not the exact-row count: the launch is redone anyway)
        if (t == 0 && atomicCAS((int32_t*)P.st, 0, gc + 1) == 0) atomicExch(&P.st[3], s);
        return;
    }
    if (t == 0) {
        if (s < P.r_end) {   // W'_s empty: round s has no events (the per-launch step's outputs)
            A.wstat[(size_t)s * C + gc] = 0;
            A.wflag[(size_t)(s + 1) * C + gc] = 0;
            A.Bm[(size_t)(s + 1) * C + gc] = len;
            if (cl == 0) {
                P.fin[g] = s;
                atomicAdd(&P.st[2], 1);
            }
        }
        if (cl == 0) atomicMax(&P.st[1], s);
    }
}

// W'_{r} rows (row-major, rebased to base(r), bit 7 = v(r)) and their granules before the first
// launch of a DivideRounds, from the WFD rows k_round_gather wrote; the chain's rows in the three
// other buffers get the invalid bit for the rounds r + 1 .. r + 3 that will use them (they may
// hold an earlier call's rows of those very rounds). One workgroup per chain.
template <typename CT>
__global__ void __launch_bounds__(64) k_round_p_init(RoundPArgs P, int ndw) {
    const RoundArgs& A = P.A;
    const int gc = blockIdx.x, n = A.n, C = A.C, g = gc / n, r = P.r0;
    const int b = A.Bm[(size_t)r * C + gc];
    const bool have = b < A.c_len[gc];
    bool of = false;
    const CT* __restrict__ row = (const CT*)A.WFD + ((size_t)r * C + gc) * n;
    for (int d = threadIdx.x; d < ndw; d += 64) {
        uint32_t w = 0;
        for (int u = 0; u < 4; u++) {
            const int i = 4 * d + u;
            uint32_t v = 127u;
            if (have && i < n) {
                const int32_t f = Coord<CT>::fd(row[i]);
                if (f != kMaxI32) {
                    const int32_t bs = A.c_base[g * n + i] + (r > 0 ? A.Bm[(size_t)(r - 1) * C + g * n + i] : 0);
                    const int32_t x = f - bs + 1;
                    if (x > 126) of = true;
                    else v = (uint32_t)x;
                }
            }
            w |= v << (8 * u);
        }
        P.FD8p[((size_t)(r & (kRoundPBufs - 1)) * C + gc) * ndw + d] = w | ((((r >> 2) & 1) ? 0x80808080u : 0u));
        for (int k = 1; k < kRoundPBufs; k++)
            P.FD8p[((size_t)((r + k) & (kRoundPBufs - 1)) * C + gc) * ndw + d] =
                (((r + k) >> 2) & 1) ? 0x7F7F7F7Fu : 0xFFFFFFFFu;   // bit 7 = !v(r + k)
    }
    of = __any(of);
    if (threadIdx.x == 0)
        P.gran[(size_t)(r % kRpSlots) * C + gc] =
            ((uint64_t)(uint32_t)(r + 1) << 32) | (uint32_t)b | (have ? kRpEx : 0u) | (of ? kRpOv : 0u);
}

template <typename CT, int NDW, int Q>
static hipError_t rp_launch(hipStream_t st, const RoundPArgs& P, int num_cus) {
    typedef RpCfg<CT, NDW, Q> K;
    const void* f = (const void*)k_round_p<CT, NDW, Q>;
    static bool attr = false;
    static int per_cu = 0;
    if (!attr) {
        hipError_t e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, K::LDS);
        if (e != hipSuccess) return e;
        e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, f, K::T, K::LDS);
        if (e != hipSuccess) return e;
        attr = true;
    }
    // every workgroup must be resident at once (they wait for each other): one per CU
    if (per_cu < 1 || P.A.C > num_cus * per_cu) return hipErrorCooperativeLaunchTooLarge;
    hipLaunchKernelGGL((k_round_p<CT, NDW, Q>), dim3(P.A.C), dim3(K::T), K::LDS, st, P);
    return hipGetLastError();
}

template <typename CT>
static hipError_t rp_launch_t(hipStream_t st, const RoundPArgs& P, int num_cus) {
    switch (round_k_ndw(P.A.n)) {
        case 2: return rp_launch<CT, 2, 2>(st, P, num_cus);
        case 4: return rp_launch<CT, 4, 4>(st, P, num_cus);
        case 8: return rp_launch<CT, 8, 2>(st, P, num_cus);
        case 16: return rp_launch<CT, 16, 4>(st, P, num_cus);
        case 32: return rp_launch<CT, 32, 4>(st, P, num_cus);
        case 64: return rp_launch<CT, 64, 4>(st, P, num_cus);
        default: return hipErrorInvalidValue;
    }
}

bool round_p_ok(int n, int C, int num_cus) { return n >= 1 && n <= 256 && C <= num_cus; }

// rounds (fin[g], r_last] of the graphs that finished before r_last: empty rows, as the
// per-launch step writes them for every chain of every round
__global__ void k_round_p_tail(RoundArgs A, const int32_t* __restrict__ fin, int r_last) {
    const int gc = blockIdx.x * blockDim.x + threadIdx.x;
    if (gc >= A.C) return;
    const int len = A.c_len[gc];
    for (int r = fin[gc / A.n] + 1; r <= r_last; r++) {
        A.wstat[(size_t)r * A.C + gc] = 0;
        A.wflag[(size_t)(r + 1) * A.C + gc] = 0;
        A.Bm[(size_t)(r + 1) * A.C + gc] = len;
    }
}

void launch_round_p_tail(hipStream_t st, const RoundArgs& A, const int32_t* fin, int r_last) {
    hipLaunchKernelGGL(k_round_p_tail, dim3((A.C + 255) / 256), dim3(256), 0, st, A, fin, r_last);
}

hipError_t launch_round_p(hipStream_t st, const RoundArgs& A, uint32_t* FD8p, uint64_t* gran, int32_t* status,
                          int32_t* fin, int r0, int r_end, int init, int num_cus) {
    RoundPArgs P{};
    P.A = A;
    P.FD8p = FD8p;
    P.gran = gran;
    P.st = status;
    P.fin = fin;
    P.r0 = r0;
    P.r_end = r_end;
    P.tmo = 5000000;   // 50 ms per wait (a round takes microseconds)
    if (init) {
        if (A.compact) hipLaunchKernelGGL(k_round_p_init<uint16_t>, dim3(A.C), dim3(64), 0, st, P, round_k_ndw(A.n));
        else hipLaunchKernelGGL(k_round_p_init<int32_t>, dim3(A.C), dim3(64), 0, st, P, round_k_ndw(A.n));
        const hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    return A.compact ? rp_launch_t<uint16_t>(st, P, num_cus) : rp_launch_t<int32_t>(st, P, num_cus);
}

}  // namespace hgx
