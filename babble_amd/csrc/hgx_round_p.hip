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

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "hgx_device.h"
#include "hgx.h"
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
// slots: 1 poll, 2 post-poll barrier + S row of the previous round, 13 search levels, 3 vm drain +
// histogram barrier, 4 scan + later windows, 5 publish / next-window rebase / outputs / staging /
// next poll issue;
// 10 synchronous stagings, 11 later windows; 15 = block-rounds
__device__ unsigned long long hgx_rp_prof[16];
// per (round, chain) s_memrealtime stamps (100 MHz, low 32 bits) of wave 0 (thread 0) and of
// wave 1 (thread 64): poll done, boundary known, publish issued (wave 0) / next window rebased
// (wave 1), end of round; rounds < 4096, chains < 256
constexpr int kRpTrR = 4096, kRpTrC = 256, kRpTrW = 8;
__device__ uint32_t hgx_rp_trace[kRpTrR * kRpTrC * kRpTrW];
// every wave's poll-done and end-of-round stamps for rounds [100, 164): [64][256][16][2]
__device__ uint32_t hgx_rp_trace2[64 * 256 * 16 * 2];
#define RP_TRACE_W(r, k)                                                                           \
    do {                                                                                           \
        if (lane == 0 && (r) >= 100 && (r) < 164 && gc < 256 && wave < 16)                        \
            hgx_rp_trace2[((((r) - 100) * 256 + gc) * 16 + wave) * 2 + (k)] = (uint32_t)__builtin_amdgcn_s_memrealtime(); \
    } while (0)
#define RP_TRACE(k) const uint32_t _tr##k = (uint32_t)__builtin_amdgcn_s_memrealtime()
#define RP_TRACE_STORE(r)                                                                        \
    do {                                                                                         \
        if ((threadIdx.x == 0 || threadIdx.x == 64) && (r) < kRpTrR && gc < kRpTrC) {            \
            uint32_t* _p = hgx_rp_trace + ((size_t)(r) * kRpTrC + gc) * kRpTrW + (threadIdx.x ? 4 : 0); \
            _p[0] = _tr0; _p[1] = _tr1; _p[2] = _tr2; _p[3] = (uint32_t)__builtin_amdgcn_s_memrealtime(); \
        }                                                                                        \
    } while (0)
#ifndef HGX_PROF_T
#define HGX_PROF_T 0   // the profiled thread (64: wave 1, a rebasing wave)
#endif
#define RP_PROF_BEGIN() long long _pt = clock64(); unsigned long long _pa[16] = {}
#define RP_PROF(i)                                                \
    do {                                                          \
        if (threadIdx.x == HGX_PROF_T) {                          \
            const long long _t = clock64();                       \
            _pa[i] += (unsigned long long)(_t - _pt);             \
            _pt = _t;                                             \
            if ((i) == 5) _pa[15] += 1;                           \
        }                                                         \
    } while (0)
#define RP_PROF_COUNT(i)                                          \
    do {                                                          \
        if (threadIdx.x == HGX_PROF_T) _pa[i] += 1;               \
    } while (0)
#define RP_PROF_END()                                                              \
    do {                                                                           \
        if (threadIdx.x == HGX_PROF_T)                                             \
            for (int _i = 0; _i < 16; _i++)                                        \
                if (_pa[_i]) atomicAdd(&hgx_rp_prof[_i], _pa[_i]);                 \
    } while (0)
void round_p_prof_dump() {
    unsigned long long h[16];
    if (hipMemcpyFromSymbol(h, HIP_SYMBOL(hgx_rp_prof), sizeof(h)) != hipSuccess) return;
    const double r = h[15] ? (double)h[15] : 1.0;
    fprintf(stderr, "[hgx] k_round_p clk per block-round (thread 0): poll %.0f bases+flags %.0f S row %.0f staging issue %.0f "
            "search-levels %.0f drain+barrier %.0f scan %.0f publish %.0f slice %.0f end barrier %.0f | block-rounds %llu, "
            "synchronous stagings %llu, later windows %llu\n",
            h[1] / r, h[6] / r, h[7] / r, h[2] / r, h[13] / r, h[3] / r, h[4] / r, h[8] / r, h[9] / r, h[5] / r, h[15], h[10],
            h[11]);
    unsigned long long z[16] = {};
    (void)hipMemcpyToSymbol(HIP_SYMBOL(hgx_rp_prof), z, sizeof(z));
    if (const char* path = getenv("HGX_RP_TRACE_FILE")) {
        std::vector<uint32_t> tr((size_t)kRpTrR * kRpTrC * kRpTrW);
        if (hipMemcpyFromSymbol(tr.data(), HIP_SYMBOL(hgx_rp_trace), tr.size() * 4) == hipSuccess) {
            if (FILE* f = fopen(path, "wb")) {
                fwrite(tr.data(), 4, tr.size(), f);
                fclose(f);
            }
            std::vector<uint32_t> t2((size_t)64 * 256 * 16 * 2);
            if (hipMemcpyFromSymbol(t2.data(), HIP_SYMBOL(hgx_rp_trace2), t2.size() * 4) == hipSuccess)
                if (FILE* f = fopen((std::string(path) + ".waves").c_str(), "wb")) {
                    fwrite(t2.data(), 4, t2.size(), f);
                    fclose(f);
                }
        }
    }
}
#else
#define RP_PROF_BEGIN() (void)0
#define RP_TRACE(k) (void)0
#define RP_TRACE_STORE(r) (void)0
#define RP_TRACE_W(r, k) (void)0
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
// the same into a window on another device (peer mapping): system scope
__device__ __forceinline__ void rp_st_sys(uint32_t* p, uint32_t v) {
    asm volatile("global_store_dword %0, %1, off sc0 sc1" ::"v"(p), "v"(v) : "memory");
}
// 16-byte forms (a write-through store is one fabric write per lane: per byte a dword store costs
// ~6x a dwordx4 one, MI355X_MICROARCH.md)
__device__ __forceinline__ void rp_st4_sc1(uint32_t* p, uint4 v) {
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    const u32x4 x = {v.x, v.y, v.z, v.w};
    asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(p), "v"(x) : "memory");
}
__device__ __forceinline__ void rp_st4_sys(uint32_t* p, uint4 v) {
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    const u32x4 x = {v.x, v.y, v.z, v.w};
    asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1" ::"v"(p), "v"(x) : "memory");
}
// a wave's row dwords w (lane d = dword d) as 16-byte pieces: lane l < 16 gets dwords 4l .. 4l + 3
__device__ __forceinline__ uint4 rp_gather4(uint32_t w) {
    const int src = (4 * lane_id()) & 63;
    return make_uint4((uint32_t)__shfl((int)w, src), (uint32_t)__shfl((int)w, src + 1),
                      (uint32_t)__shfl((int)w, src + 2), (uint32_t)__shfl((int)w, src + 3));
}
__device__ __forceinline__ void rp_st_gran_sys(uint64_t* p, uint64_t v) {
    __hip_atomic_store((gu64*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ uint32_t rp_ld_abort(const int32_t* p) {
    return (uint32_t)__hip_atomic_load((gu32*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void rp_vm_drain() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
__device__ __forceinline__ void rp_lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// The rows' layout in a buffer, chunk-major: part q of candidate gc (HD dwords, what lane q of the
// candidate compares) in chunks of CS = min(4, HD) dwords, chunk k of (gc, q) at ((k C + gc) Q + q) CS.
// A poll instruction's 64 lanes (64 / Q candidates, chunk k of every part) then read one contiguous
// 1 KB instead of 16-byte pieces of 16 rows (the request rate of the polls, k_round_pb's lesson);
// HD <= 4 is plain row-major.
__host__ __device__ constexpr int rp_q_of(int ndw) { return ndw == 2 || ndw == 8 ? 2 : 4; }
__host__ __device__ constexpr size_t rp_chunk_off(int k, int gc, int q, int C, int Q, int CS) {
    return (((size_t)k * C + gc) * Q + q) * CS;
}

// A candidate's granule and this lane's HD dwords of its row (chunk k at p + k cst dwords), sc1 loads
// (every load of handed-off bytes), issued AND waited for in ONE asm statement: an asm load's
// destination registers are written when the data returns, so a load left in flight across
// compiler-visible code lets the register allocator copy (or reuse) them before the data lands.
template <int HD>
__device__ __forceinline__ void rp_ld_cand(const uint64_t* gp, const uint32_t* p, size_t cst, uint64_t& gv,
                                           uint32_t (&v)[HD]) {
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    if constexpr (HD == 16) {
        u32x4 a, b, c, d;
        const uint32_t *p1 = p + cst, *p2 = p + 2 * cst, *p3 = p + 3 * cst;
        asm volatile(
            "global_load_dwordx2 %0, %5, off sc1\n\t"
            "global_load_dwordx4 %1, %6, off sc1\n\t"
            "global_load_dwordx4 %2, %7, off sc1\n\t"
            "global_load_dwordx4 %3, %8, off sc1\n\t"
            "global_load_dwordx4 %4, %9, off sc1\n\t"
            "s_waitcnt vmcnt(0)"
            : "=&v"(gv), "=&v"(a), "=&v"(b), "=&v"(c), "=&v"(d) : "v"(gp), "v"(p), "v"(p1), "v"(p2), "v"(p3) : "memory");
        const u32x4 q4[4] = {a, b, c, d};
#pragma unroll
        for (int k = 0; k < 4; k++) { v[4 * k] = q4[k].x; v[4 * k + 1] = q4[k].y; v[4 * k + 2] = q4[k].z; v[4 * k + 3] = q4[k].w; }
    } else if constexpr (HD == 8) {
        u32x4 a, b;
        const uint32_t* p1 = p + cst;
        asm volatile(
            "global_load_dwordx2 %0, %3, off sc1\n\t"
            "global_load_dwordx4 %1, %4, off sc1\n\t"
            "global_load_dwordx4 %2, %5, off sc1\n\t"
            "s_waitcnt vmcnt(0)"
            : "=&v"(gv), "=&v"(a), "=&v"(b) : "v"(gp), "v"(p), "v"(p1) : "memory");
        v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
    } else if constexpr (HD == 4) {
        u32x4 a;
        asm volatile(
            "global_load_dwordx2 %0, %2, off sc1\n\t"
            "global_load_dwordx4 %1, %3, off sc1\n\t"
            "s_waitcnt vmcnt(0)"
            : "=&v"(gv), "=&v"(a) : "v"(gp), "v"(p) : "memory");
        v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
    } else {
        static_assert(HD == 1, "rp_ld_cand: HD in {1, 4, 8, 16}");
        uint32_t x;
        asm volatile(
            "global_load_dwordx2 %0, %2, off sc1\n\t"
            "global_load_dword %1, %3, off sc1\n\t"
            "s_waitcnt vmcnt(0)"
            : "=&v"(gv), "=&v"(x) : "v"(gp), "v"(p) : "memory");
        v[0] = x;
    }
}

// HD dwords of an LDS row: every read and its wait in one asm statement (16-byte reads when
// HD % 4 == 0)
template <int HD>
__device__ __forceinline__ void rp_lds_row(const uint32_t* p, uint32_t (&v)[HD]) {
    const uint32_t a = (uint32_t)(uintptr_t)p;
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    if constexpr (HD == 16) {
        u32x4 r0, r1, r2, r3;
        asm volatile(
            "ds_read_b128 %0, %4\n\tds_read_b128 %1, %4 offset:16\n\tds_read_b128 %2, %4 offset:32\n\t"
            "ds_read_b128 %3, %4 offset:48\n\ts_waitcnt lgkmcnt(0)"
            : "=&v"(r0), "=&v"(r1), "=&v"(r2), "=&v"(r3) : "v"(a) : "memory");
        const u32x4 q4[4] = {r0, r1, r2, r3};
#pragma unroll
        for (int k = 0; k < 4; k++) { v[4 * k] = q4[k].x; v[4 * k + 1] = q4[k].y; v[4 * k + 2] = q4[k].z; v[4 * k + 3] = q4[k].w; }
    } else if constexpr (HD == 8) {
        u32x4 r0, r1;
        asm volatile("ds_read_b128 %0, %2\n\tds_read_b128 %1, %2 offset:16\n\ts_waitcnt lgkmcnt(0)"
                     : "=&v"(r0), "=&v"(r1) : "v"(a) : "memory");
        v[0] = r0.x; v[1] = r0.y; v[2] = r0.z; v[3] = r0.w; v[4] = r1.x; v[5] = r1.y; v[6] = r1.z; v[7] = r1.w;
    } else if constexpr (HD == 4) {
        u32x4 r0;
        asm volatile("ds_read_b128 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=&v"(r0) : "v"(a) : "memory");
        v[0] = r0.x; v[1] = r0.y; v[2] = r0.z; v[3] = r0.w;
    } else if constexpr (HD == 2) {
        uint64_t r;
        asm volatile("ds_read_b64 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=&v"(r) : "v"(a) : "memory");
        v[0] = (uint32_t)r; v[1] = (uint32_t)(r >> 32);
    } else {
        uint32_t r;
        asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=&v"(r) : "v"(a) : "memory");
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
    // firstDescendants columns: one 16-byte DMA instruction = 16 columns x 64 bytes (lane k:
    // column k / 4, 16-byte chunk k % 4), groups FDG = 1040 bytes apart (16-byte pad: the 16
    // groups start on different banks)
    static constexpr int FDG = 1040;
    static constexpr int NG = (NC + 15) / 16;                    // column groups of a segment
    static constexpr int KF = (NG + NW - 1) / NW;                // groups per wave per segment
    static constexpr int SEG_FD = NG * FDG;                      // bytes
    // LDS carve (bytes, 16-aligned)
    static constexpr int O_WIN = 0;
    static constexpr int O_RAW = O_WIN + ((kRpP * WS * 4 + 15) & ~15);   // [RR][n] raw rows
    static constexpr int O_FD = O_RAW + NSEG * SEG_RAW;                   // [NSEG][NG groups][FDG]
    static constexpr int O_CB = O_FD + NSEG * SEG_FD;                     // c_base[NC]
    static constexpr int O_CO = O_CB + NC * 4;                           // c_off[NC]
    static constexpr int O_BS0 = O_CO + NC * 4;                          // bases c_base + Bm[r], by round parity
    static constexpr int O_BS1 = O_BS0 + NC * 4;
    static constexpr int O_HIST = O_BS1 + NC * 4;                        // [2][32] bins, by round parity
    static constexpr int O_SL = O_HIST + 2 * 32 * 4;                     // S row slices [2][NW] u64, by round parity
    static constexpr int O_MISC = O_SL + 2 * NW * 8;                     // [2][8] by parity: [2] any, [3] fail
    static constexpr int USED = O_MISC + 64;
    // at least 82 KB: one workgroup per CU (the hand-off rule's geometry), whatever fits
    static constexpr int LDS = USED > 84 * 1024 ? USED : 84 * 1024;
    static_assert(USED <= 160 * 1024, "k_round_p: LDS carve exceeds a CU's 160 KB");
};

struct RoundPArgs {
    RoundArgs A;
    uint32_t* FD8p;     // [4][C ndw] rebased candidate rows, chunk-major (rp_chunk_off; round s: buffer s % 4, bit 7 of
                        // every byte = v(s) = (s >> 2) & 1)
    uint64_t* gran;     // [kRpSlots][C]
    int32_t* st;        // [0] abort, [1] max over graphs of the round each stopped at, [2] graphs that
                        // finished (W'_s empty) in this launch, [3] rows counted exactly (over 8 bits)
    int32_t* fin;       // [G] the round at which graph g found W'_s empty (-1: not yet, this call)
    int r0, r_end;      // rounds [r0, r_end) at most
    long long tmo;      // one wait's budget in s_memrealtime ticks (100 MHz)
    int c_lo;           // this launch's first chain (a shard's chain block)
    // the windows every candidate row and granule is written to (device memory; nwin = 1: FD8p / gran
    // alone, Wd unused). Kept out of the kernel arguments: the loop's SGPRs are already spilled, and
    // more arguments made the compiler reload arguments inside the round loop (c2 rounds +0.9 ms)
    int nwin;
    const RoundPWindows* Wd;
};

// One round s of chain c, in the order of its critical path:
//  (a) poll: every lane waits for its candidate's granule and row part (W'_s, published by the
//      other chains in round s - 1), writes base(s+1)[j] = c_base[j] + Bm[s][j];
//  (b) the outputs of round s - 1 (plain stores) and the staging ring ahead (LDS-DMA) are issued
//      behind the poll: they land during the search, nothing waits for them until (d);
//  (c) search of the window [b, b + 31), rebased to base(s) in round s - 1;
//  (d) K(w) histogram, one barrier, every wave scans it (the boundary B, no second barrier);
//  (e) wave 0 publishes W'_{s+1} of chain c (row rebased to base(s+1), granule) at once, while the
//      other waves rebase the next window [kstar, kstar + 31) to base(s+1); one barrier; the poll
//      loads of round s + 1 go out.
// SH: a shard's launch of a chain-sharded group (W windows); the plain launch over every
// chain is a separate instantiation, so its loop keeps the code (and registers) it had without windows
template <typename CT, int NDW, int Q, bool SH>
__global__ void __launch_bounds__((4 * NDW * Q < 64) ? 64 : 4 * NDW * Q) k_round_p(RoundPArgs P) {
    typedef RpCfg<CT, NDW, Q> K;
    constexpr int HD = K::HD, T = K::T, WS = K::WS, NW = K::NW;
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    const RoundArgs& A = P.A;
    const int n = A.n, C = A.C, sm = A.sm;
    const int t = threadIdx.x, lane = lane_id(), wave = __builtin_amdgcn_readfirstlane(t >> 6);
    const int gc = P.c_lo + (int)blockIdx.x, g = gc / n, cl = gc % n, g0 = g * n;
    const int j = t / Q, q = t % Q;              // candidate slot and row part of this lane
    const bool jv = j < n && t < K::NC * Q;      // a real chain of the graph
    uint32_t* win = (uint32_t*)(lds + K::O_WIN);
    int32_t* cbase = (int32_t*)(lds + K::O_CB);
    int32_t* coff = (int32_t*)(lds + K::O_CO);
    auto bases = [&](int r) { return (int32_t*)(lds + ((r & 1) ? K::O_BS1 : K::O_BS0)); };   // c_base + Bm[r]
    auto hist_of = [&](int r) { return (int32_t*)(lds + K::O_HIST) + (r & 1) * 32; };
    auto misc_of = [&](int r) { return (int32_t*)(lds + K::O_MISC) + (r & 1) * 8; };

    if (P.fin[g] >= 0) return;   // the graph finished in an earlier launch of this DivideRounds
    const int len = A.c_len[gc], off = A.c_off[gc];
    for (int i = t; i < n; i += T) {
        const int32_t cb = A.c_base[g0 + i];
        cbase[i] = cb;
        coff[i] = A.c_off[g0 + i];
        // bases of round r0's window: c_base + Bm[r0 - 1], written by earlier launches
        bases(P.r0 - 1)[i] = cb + (P.r0 > 0 ? A.Bm[(size_t)(P.r0 - 1) * C + g0 + i] : 0);
    }
    if (t < 64) hist_of(0)[t] = 0;
    if (t < 16) misc_of(t >> 3)[t & 7] = 0;
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
        const int raw_w = K::O_RAW + slot * SEG * n * K::CSZ;   // rows (p % RR) * n
        const int nch = SEG * n * K::CSZ / 16;   // 16-byte chunks
#pragma unroll
        for (int k = 0; k < K::KR16; k++) {
            const int c0 = wave * 64 + k * T;    // this wave instruction's first chunk
            if (c0 + lane < nch)
                __builtin_amdgcn_global_load_lds((const void*)(src + 4 * (c0 + lane)), (lds_ptr_t)(lds + raw_w + 16 * c0), 16, 0, 0);
        }
        // columns: lane = (column % 16 via lane / 4, 16-byte chunk lane % 4); one instruction =
        // one group of 16 columns
        const int icol = lane >> 2, pch = lane & 3;
        const uint8_t* __restrict__ fsrc = (const uint8_t*)A.FDT + ((size_t)off + (size_t)m * SEG) * K::CSZ + pch * 16;
        const size_t cstride = (size_t)A.Pcap * K::CSZ;   // bytes between columns
        const int fd_w = K::O_FD + slot * K::SEG_FD;
#pragma unroll
        for (int k = 0; k < K::KF; k++) {
            const int grp = wave + k * NW;
            if (grp < K::NG) {
                const int i = min(grp * 16 + icol, n - 1);
                __builtin_amdgcn_global_load_lds((const void*)(fsrc + (size_t)i * cstride), (lds_ptr_t)(lds + fd_w + grp * K::FDG), 16, 0, 0);
            }
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
        return *(const CT*)(fd_w + (i >> 4) * K::FDG + (i & 15) * 64 + (p % SEG) * K::CSZ);
    };
    auto raw_at = [&](int p, int i) -> CT {   // staged lastAncestors row of chain offset p
        return ((const CT*)(lds + K::O_RAW))[(p % RR) * n + i];
    };
    // rebased 8-bit window rows (clamp(LA - base + 1, 0, 126), swar_ge_count) of the window [kb, kb + np),
    // by threads [0, nthr) (tid = this thread's), bases bq = c_base + Bm of the previous round
    typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
    auto rebase = [&](int kb, int np, const int32_t* bsp, int tid, int nthr) {
        const int RS = nthr / NDW > 0 ? nthr / NDW : 1;   // rows per pass
        for (int d = tid % NDW; d < NDW && tid < RS * NDW; d += nthr) {
            const int i0 = 4 * d;
            int32_t bq[4];
#pragma unroll
            for (int u = 0; u < 4; u++) bq[u] = (i0 + u < n) ? bsp[i0 + u] : 0;
            for (int p = tid / NDW; p < np; p += RS) {
                uint32_t w;
                if constexpr (K::CSZ == 2) {
                    const uint32_t* rp = (const uint32_t*)(lds + K::O_RAW) + (((kb + p) % RR) * n + i0) / 2;
                    const uint32_t r01 = i0 < n ? rp[0] : 0u, r23 = i0 + 2 < n ? rp[1] : 0u;
                    const u16x2 b01 = {(unsigned short)bq[0], (unsigned short)bq[1]};
                    const u16x2 b23 = {(unsigned short)bq[2], (unsigned short)bq[3]};
                    const u16x2 cap = {126, 126};
                    const u16x2 y01 = __builtin_elementwise_min(__builtin_elementwise_sub_sat(__builtin_bit_cast(u16x2, r01), b01), cap);
                    const u16x2 y23 = __builtin_elementwise_min(__builtin_elementwise_sub_sat(__builtin_bit_cast(u16x2, r23), b23), cap);
                    w = __builtin_amdgcn_perm(__builtin_bit_cast(uint32_t, y23), __builtin_bit_cast(uint32_t, y01), 0x06040200u);
                } else {
                    w = 0u;
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

    // Round r's outputs: only Bm[r + 1] (the chain's next boundary) and the new candidate's S row
    // are written in the loop, by wave 0 behind round r + 1's poll (a wave's vm counter is in
    // order: stores before a poll hold its loads back). The rest (rounds of the chain's events,
    // wstat / wflag / active, the candidates' WLA rows) follows from Bm alone and is written after
    // the launch by k_round_p_post, coalesced.
    // round r's S row from the waves' slices (LDS buffer r & 1) and its Bm, by wave 0 after the
    // barrier that follows them
    constexpr int CPW = 64 / Q;   // candidates per wave
    // (the output columns' addresses once, outside the loop: the kernel-argument reloads they took
    // inside it sat on wave 0's path between its poll and its search)
    int32_t* const bm_col = A.Bm + gc;
    const int nw_s = A.nw;
    uint64_t* const sm_row = A.Smat + (size_t)gc * nw_s;
    const size_t sm_stride = (size_t)C * nw_s;
    auto s_row = [&](int r, int kst) {
        if (lane == 0) bm_col[(size_t)(r + 1) * C] = kst;
        if (kst >= len) return;   // no new candidate: no S row
        const uint64_t* sl = (const uint64_t*)(lds + K::O_SL) + (r & 1) * NW;
        constexpr int WPW = 64 / CPW;   // waves per 64-bit word
        if (lane < nw_s) {
            uint64_t w = 0;
#pragma unroll
            for (int k = 0; k < WPW; k++)
                if (lane * WPW + k < NW) w |= sl[lane * WPW + k] << (k * CPW);
            sm_row[(size_t)(r + 1) * sm_stride + lane] = w;
        }
    };
    RP_PROF_BEGIN();
    // prologue: round r0's window staged and rebased to base(r0) = c_base + Bm[r0 - 1]
    if (b < len) stage_range(b / SEG, min(b / SEG + NSEG - 1, last_seg));
    rp_vm_drain();
    rp_lds_barrier();
    if (b < len) rebase(b, min(kRpP, len - b), bases(P.r0 - 1), t, T);
    rp_lds_barrier();   // the first window is rebased (every later round: the barrier ending (e))
    // the first poll's loads (each round issues the next round's)
    // (this lane's poll addresses and the publish's bases once, outside the loop: see bm_col)
    constexpr int CS = HD < 4 ? HD : 4;   // chunk dwords (rp_chunk_off)
    static_assert(rp_q_of(NDW) == Q, "k_round_p: Q as rp_q_of");
    const size_t cst = (size_t)C * Q * CS;   // chunk stride (dwords)
    const uint64_t* const gran_lane = P.gran + g0 + (jv ? j : 0);
    const uint32_t* const row_lane =
        P.FD8p + (HD <= 4 ? (size_t)(g0 + (jv ? j : 0)) * NDW + q * HD : rp_chunk_off(0, g0 + (jv ? j : 0), q, C, Q, CS));
    uint32_t* const fd8_out = P.FD8p;
    uint64_t* const gran_out = P.gran + gc;
    auto gran_at = [&](int r) { return gran_lane + (size_t)(r % kRpSlots) * C; };
    auto row_at = [&](int r) { return row_lane + (size_t)(r & (kRoundPBufs - 1)) * C * NDW; };
    int s = P.r0;
    bool failed = false;
    int s_r = -1, s_k = 0;   // the round whose Bm / S row is still to be written (by wave 0, after the next barrier)
    for (;; s++) {
        if (s >= P.r_end) break;   // capacity: the host continues from round s
        int32_t* hist = hist_of(s);
        int32_t* misc = misc_of(s);
        const bool have = b < len;   // block-uniform
        int kb = b, np = have ? min(kRpP, len - b) : 0;

        // (a) this lane's candidate granule and row part (W'_s): reload until the granule carries
        // tag s + 1 and, when the candidate exists, every byte of the row part carries v(s)
        const uint32_t vbit = ((s >> kRoundPShift) & 1) ? 0x80808080u : 0u;
        bool wfail = false;
        uint64_t gv = 0;
        uint32_t fd[HD];
        {
            const uint64_t* gp = gran_at(s);
            const uint32_t* rowp = row_at(s);
            const long long tw = __builtin_amdgcn_s_memrealtime();
            bool ok = false;
            // the poll at the top priority: the waves whose candidates arrived search meanwhile, and
            // the youngest waves (last in the age order) would otherwise issue their loads last
            // (without it: c3 round_search 15.80 -> 16.41-16.49 ms)
            __builtin_amdgcn_s_setprio(3);
            for (int spins = 0;; spins++) {
                if (!ok) rp_ld_cand<HD>(gp, rowp, cst, gv, fd);   // (a lane whose candidate is complete keeps it)
                uint32_t bad = 0;
#pragma unroll
                for (int d = 0; d < HD; d++) bad |= (fd[d] ^ vbit) & 0x80808080u;
                const bool tag_ok = (uint32_t)(gv >> 32) == (uint32_t)(s + 1);
                ok = !jv || (tag_ok && (!((uint32_t)gv & kRpEx) || bad == 0));
                if (__all(ok)) break;
                if ((spins & 31) == 31) {
                    const long long now = __builtin_amdgcn_s_memrealtime();
                    if (now - tw > P.tmo || rp_ld_abort(P.st) != 0) { wfail = true; break; }
                }
                __builtin_amdgcn_s_sleep(1);
            }
            __builtin_amdgcn_s_setprio(0);
        }
        RP_PROF(1);
        RP_TRACE(0);
        RP_TRACE_W(s, 0);
        const uint32_t gval = (uint32_t)gv;
        const bool cand = jv && !wfail && (gval & kRpEx);
        const bool ov = cand && (gval & kRpOv);
        const int bmj = (int)(gval & kRpBm);
        if (jv && q == 0 && !wfail) bases(s)[j] = cbase[j] + bmj;   // base(s + 1)[j]
        if (cand && have) {
#pragma unroll
            for (int d = 0; d < HD; d++) fd[d] = swar_nf(fd[d] & 0x7F7F7F7Fu);   // validity bits off, as 128 - FD'

        } else {
#pragma unroll
            for (int d = 0; d < HD; d++) fd[d] = 0x01010101u;   // never seen (FD' = 127)
        }
        if (wfail && lane == 0) misc[3] = 1;
        if (cand && q == 0) misc[2] = 1;   // (same value from every writer)
        // (no barrier here: the window was rebased before the barrier ending round s - 1, and each
        // wave searches as soon as its own candidates arrived; c3 rounds 20.7 -> 19.3 ms)
        // round s + 1's histogram and flags start empty: their buffers were last read in round
        // s - 1 (before this barrier) and are next written in round s + 1's poll (after round s's
        // histogram barrier)
        if (t >= T - 32) hist_of(s + 1)[t - (T - 32)] = 0;
        if (t < 8) misc_of(s + 1)[t] = 0;
        RP_PROF(6);
        if (s_r >= 0) {   // round s - 1's S row: every wave set its slice before this barrier
            if (wave == 0) s_row(s_r, s_k);
            s_r = -1;
        }
        RP_PROF(7);
        // the ring ahead (segments up to b / SEG + NSEG - 1), behind the poll (a wave's loads return
        // in order: staging issued before the poll would hold it back) and behind the LDS writes
        // above (the compiler waits for an LDS-DMA before the next LDS access it cannot tell
        // apart); it lands during the search, and the histogram wait covers it before the next
        // window's rebase reads it
        if (have) stage_range(b / SEG, min(b / SEG + NSEG - 1, last_seg));
        RP_PROF(2);

        // (c) search, window after window until the boundary is found (a later window is rare)
        int kstar = len, B = -1, K_last = kRpP, carried = 0;
        bool done = false, any = false;
        const bool wave_cand = __any(cand) && have;
        // VALU and memory issue go to the older waves of a SIMD first, so with 4 waves per SIMD the
        // youngest finished the search ~1.3 us after the oldest and everyone waited for it at the
        // histogram barrier: the younger half searches at a higher priority (c3 rounds 22.9 ->
        // 21.2 ms; graded priorities by age measured the same, priority kept through the publish
        // and the poll 7x slower)
        // (without it: c3 round_search 15.80 -> 16.64-16.74 ms)
        if (NW >= 8 && wave >= NW / 2) __builtin_amdgcn_s_setprio(2);
        for (;;) {
            int lo = 0, hi = kRpP;
            if (wave_cand) {
#pragma unroll 1
                for (int it = 0; it < 5; it++) {
                    const int mid = (lo + hi) >> 1;
                    uint32_t cnt = 0;
                    if (!ov) {
                        uint32_t v[HD];
                        rp_lds_row<HD>(win + mid * WS + q * K::PS, v);
                        cnt = swar_ge_count<HD>(v, fd);
                    } else if (!done && mid < np) {
                        // exact int32 compares of this part of the row (hashgraph.go:191-197)
                        const int i_lo = q * HD * 4, i_hi = min(n, (q + 1) * HD * 4);
                        const size_t pos = (size_t)coff[j] + bmj;
                        // candidate j's firstDescendants are its owner shard's (valid for that
                        // shard's chains only; a peer-mapped read when it lies on another device)
                        const CT* __restrict__ fdt = (const CT*)A.FDT;
                        if (SH) {
                            int ow = 0;
                            while (ow + 1 < P.nwin && g0 + j >= P.Wd->c_split[ow + 1]) ow++;
                            fdt = (const CT*)P.Wd->FDT[ow];
                        }
                        for (int i = i_lo; i < i_hi; i++) {
                            const int32_t fdv = Coord<CT>::fd(fdt[(size_t)i * A.Pcap + pos]);
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
            if (NW >= 8) __builtin_amdgcn_s_setprio(0);
            RP_PROF(13);
            if (cand && q == 0 && !done && Kw < np) atomicAdd(&hist[Kw], 1);
            // (d) the histogram is complete (and the staging issued in round s - 1 has landed: the
            // next window's rebase reads it); every wave scans it (the boundary: first probe where
            // #{K <= p} (+ seen in earlier windows) >= SM)
            rp_vm_drain();
            rp_lds_barrier();
            RP_PROF(3);
            int tot;
            {
                const uint32_t v = lane < np ? (uint32_t)hist[lane] : 0u;
                const uint32_t inc = wave_scan_add_u32(v) + (uint32_t)carried;
                const uint64_t m = __ballot(lane < np && (int)inc >= sm);
                tot = __builtin_amdgcn_readlane((int)inc, 63);
                B = m ? (int)__builtin_ctzll(m) : -1;
            }
            any = misc[2] != 0;
            K_last = Kw;
            if (B >= 0 || !any || misc[3] != 0 || !have) {
                if (B >= 0) kstar = kb + B;
                break;
            }
            // no boundary in this window: the next one (synchronous staging)
            RP_PROF_COUNT(11);
            carried = tot;
            if (cand && Kw < np) done = true;
            kb += np;
            if (kb >= len) break;
            np = min(kRpP, len - kb);
            rp_lds_barrier();   // every wave has scanned the histogram
            if (t < 32) hist[t] = 0;
            if (min((kb + kRpP - 1) / SEG, last_seg) > seg_hi) stage_range(kb / SEG, min(kb / SEG + NSEG - 1, last_seg));
            rp_vm_drain();
            rp_lds_barrier();
            rebase(kb, np, bases(s - 1), t, T);
            rp_lds_barrier();
        }
        RP_PROF(4);
        RP_TRACE(1);
        if (misc[3] != 0) { failed = true; break; }
        if (!any) break;       // W'_s is empty: no round s (every workgroup of the graph agrees)

        // (e) wave 0 publishes W'_{s+1} of chain c at once: its row rebased to base(s+1) =
        // c_base + Bm[s] (bit 7 of every byte = v(s + 1)) and its granule, written through with no
        // drain in between (both self-validating); the other waves rebase the next window to the
        // same bases and write round s's outputs; then every wave stages the ring ahead and issues
        // the next poll's loads
        const bool nx = kstar < len;
        if (nx && min((kstar + kRpP - 1) / SEG, last_seg) > seg_hi) {
            // the next window is not staged (int32 coordinates, or a boundary past the first window)
            stage_range(kstar / SEG, min(kstar / SEG + NSEG - 1, last_seg));
            rp_vm_drain();
            rp_lds_barrier();
            RP_PROF_COUNT(10);
        }
        const int32_t* bs1 = bases(s);
        const int np1 = nx ? min(kRpP, len - kstar) : 0;
        if (wave == 0) {
            bool of = false;
            if (nx) {
                const uint32_t vb1 = (((s + 1) >> kRoundPShift) & 1) ? 0x80808080u : 0u;
                const size_t roff = ((size_t)((s + 1) & (kRoundPBufs - 1)) * C + gc) * NDW;   // (row-major: HD < 4)
                // lane l's 16 bytes (dwords 4l .. 4l + 3): chunk (4l % HD) / 4 of part 4l / HD
                const size_t boff = (size_t)((s + 1) & (kRoundPBufs - 1)) * C * NDW;
                const size_t coff = HD > 4 ? boff + rp_chunk_off((4 * lane % HD) / 4, gc, 4 * lane / HD, C, Q, 4)
                                           : roff + 4 * lane;   // (HD <= 4: row-major)
                static_assert(NDW <= 64, "k_round_p: one row dword per lane of wave 0");
                const int d = lane;
                uint32_t w = 0;
                if (d < NDW) {
                    // every LDS read first (4 firstDescendants, 4 bases), then the byte arithmetic
                    CT f[4];
#pragma unroll
                    for (int u = 0; u < 4; u++) f[u] = fd_at(min(4 * d + u, n - 1), kstar);
                    const int4 bq = *(const int4*)(bs1 + 4 * d);
                    const int32_t bqa[4] = {bq.x, bq.y, bq.z, bq.w};
#pragma unroll
                    for (int u = 0; u < 4; u++) {
                        const int32_t fv = Coord<CT>::fd(f[u]);
                        const bool real = 4 * d + u < n && fv != kMaxI32;
                        const int32_t x = fv - bqa[u] + 1;
                        of |= real && x > 126;
                        w |= (real && x <= 126 ? (uint32_t)x : 127u) << (8 * u);
                    }
                }
                w |= vb1;
                // into every shard's window (one: the launch's own buffers, whose address the kernel
                // arguments hold in SGPRs: no scalar load ahead of the store), 16 bytes per lane
                if constexpr (NDW % 4 == 0) {
                    const uint4 w4 = rp_gather4(w);
                    if (lane < NDW / 4) {
                        if (!SH) {
                            rp_st4_sc1(fd8_out + coff, w4);
                        } else {
                            const RoundPWindows* __restrict__ Wd = P.Wd;
                            for (int wi = 0; wi < P.nwin; wi++) {
                                if ((Wd->remote >> wi) & 1u) rp_st4_sys(Wd->FD8p[wi] + coff, w4);
                                else rp_st4_sc1(Wd->FD8p[wi] + coff, w4);
                            }
                        }
                    }
                } else if (d < NDW) {
                    if (!SH) {
                        rp_st_sc1(fd8_out + roff + d, w);
                    } else {
                        const RoundPWindows* __restrict__ Wd = P.Wd;
                        for (int wi = 0; wi < P.nwin; wi++) {
                            if ((Wd->remote >> wi) & 1u) rp_st_sys(Wd->FD8p[wi] + roff + d, w);
                            else rp_st_sc1(Wd->FD8p[wi] + roff + d, w);
                        }
                    }
                }
            }
            of = __any(of);
            if (lane == 0) {
                const uint64_t gw = ((uint64_t)(uint32_t)(s + 2) << 32) | (uint32_t)kstar | (nx ? kRpEx : 0u) | (of ? kRpOv : 0u);
                const size_t go = (size_t)((s + 1) % kRpSlots) * C + gc;
                if (!SH) {
                    rp_st_gran(gran_out + (go - gc), gw);
                } else {
                    const RoundPWindows* __restrict__ Wd = P.Wd;
                    for (int wi = 0; wi < P.nwin; wi++) {
                        if ((Wd->remote >> wi) & 1u) rp_st_gran_sys(Wd->gran[wi] + go, gw);
                        else rp_st_gran(Wd->gran[wi] + go, gw);
                    }
                }
            }
            if (of && lane == 0) atomicAdd(&P.st[3], 1);   // rows counted exactly (instrumentation)
        }
        RP_PROF(8);
        if (NW == 1) {
            if (nx) rebase(kstar, np1, bs1, t, T);
        } else if (wave > 0) {
            if (nx) rebase(kstar, np1, bs1, t - 64, T - 64);
        }
        RP_TRACE(2);
        {
            // the new candidate's S row (DecideFame, hashgraph.go:688-705): bit j = it strongly sees
            // candidate j of W'_s. The Q lanes of a candidate agree, so each wave's ballot holds its
            // 64 / Q candidates' bits every Q-th lane; the wave parks its slice in LDS and wave 0
            // writes the row (and Bm) after the next barrier
            const uint64_t m = __ballot(have && nx && cand && (done || K_last <= B));
            uint64_t x = 0;
#pragma unroll
            for (int k = 0; k < CPW; k++) x |= ((m >> (k * Q)) & 1ull) << k;
            if (lane == 0) ((uint64_t*)(lds + K::O_SL))[(s & 1) * NW + wave] = x;
            s_r = s;
            s_k = kstar;
        }
        b = kstar;
        RP_PROF(9);
        // the next window's rebase, the S-row slices and the publish are complete before any wave
        // polls: each wave then searches as soon as its own candidates arrived (no barrier between
        // the poll and the search; the histogram barrier joins the waves)
        rp_lds_barrier();
        RP_PROF(5);
        RP_TRACE_W(s, 1);
        RP_TRACE_STORE(s);
    }

    rp_vm_drain();   // no LDS-DMA outlives the workgroup
    rp_lds_barrier();
    if (!failed && s_r >= 0 && wave == 0) s_row(s_r, s_k);   // the last round's Bm and S row
    RP_PROF_END();
    if (failed) {
        // the first workgroup to give up records its chain and round (st[3] then holds the
        // round, not the exact-row count: the launch is redone anyway)
        if (t == 0 && atomicCAS((int32_t*)P.st, 0, gc + 1) == 0) {
            atomicExch(&P.st[3], s);
            // every other shard gives up too (its workgroups wait for this shard's granules)
            for (int wi = 0; SH && wi < P.nwin; wi++)
                if (P.Wd->st[wi] != P.st)
                    __hip_atomic_store((gu32*)P.Wd->st[wi], (uint32_t)(gc + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
        return;
    }
    // the launch's first workgroup of a graph reports (a shard's chain block starts mid-graph)
    const bool rep = cl == 0 || (SH && gc == P.c_lo);
    if (t == 0) {
        if (s < P.r_end) {   // W'_s empty: round s has no events (the per-launch step's outputs)
            A.wstat[(size_t)s * C + gc] = 0;
            A.wflag[(size_t)(s + 1) * C + gc] = 0;
            A.Bm[(size_t)(s + 1) * C + gc] = len;
            if (rep) {
                P.fin[g] = s;
                atomicAdd(&P.st[2], 1);
            }
        }
        if (rep) atomicMax(&P.st[1], s);
    }
}

// W'_{r} rows (row-major, rebased to base(r), bit 7 = v(r)) and their granules before the first
// launch of a DivideRounds, from the WFD rows k_round_gather wrote; the chain's rows in the three
// other buffers get the invalid bit for the rounds r + 1 .. r + 3 that will use them (they may
// hold an earlier call's rows of those very rounds). One workgroup per chain.
template <typename CT>
__global__ void __launch_bounds__(64) k_round_p_init(RoundPArgs P, int ndw) {
    const RoundArgs& A = P.A;
    const int gc = P.c_lo + (int)blockIdx.x, n = A.n, C = A.C, g = gc / n, r = P.r0;
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
        // into every shard's window (write-through; the launches that read them start after this
        // kernel has completed on every shard), dword d at its place in the chunk-major layout
        const int Q = rp_q_of(ndw), HD = ndw / Q, CS = HD < 4 ? HD : 4;
        const size_t dof = rp_chunk_off((d % HD) / CS, gc, d / HD, C, Q, CS) + (d % HD) % CS;
        for (int wi = 0; wi < P.nwin; wi++) {
            const bool rem = P.nwin > 1 && ((P.Wd->remote >> wi) & 1u);
            uint32_t* fw = P.nwin > 1 ? P.Wd->FD8p[wi] : P.FD8p;
            const uint32_t v0 = w | ((((r >> kRoundPShift) & 1) ? 0x80808080u : 0u));
            uint32_t* p0 = fw + (size_t)(r & (kRoundPBufs - 1)) * C * ndw + dof;
            if (rem) rp_st_sys(p0, v0); else rp_st_sc1(p0, v0);
            for (int k = 1; k < kRoundPBufs; k++) {
                uint32_t* pk = fw + (size_t)((r + k) & (kRoundPBufs - 1)) * C * ndw + dof;
                const uint32_t vk = (((r + k) >> kRoundPShift) & 1) ? 0x7F7F7F7Fu : 0xFFFFFFFFu;   // bit 7 = !v(r + k)
                if (rem) rp_st_sys(pk, vk); else rp_st_sc1(pk, vk);
            }
        }
    }
    of = __any(of);
    if (threadIdx.x == 0) {
        const uint64_t gw = ((uint64_t)(uint32_t)(r + 1) << 32) | (uint32_t)b | (have ? kRpEx : 0u) | (of ? kRpOv : 0u);
        for (int wi = 0; wi < P.nwin; wi++) {
            uint64_t* gw_p = (P.nwin > 1 ? P.Wd->gran[wi] : P.gran) + (size_t)(r % kRpSlots) * C + gc;
            if (P.nwin > 1 && ((P.Wd->remote >> wi) & 1u)) rp_st_gran_sys(gw_p, gw);
            else rp_st_gran(gw_p, gw);
        }
    }
}

template <typename CT, int NDW, int Q, bool SH>
static hipError_t rp_launch(hipStream_t st, const RoundPArgs& P, int num_cus, int nblk) {
    typedef RpCfg<CT, NDW, Q> K;
    const void* f = (const void*)k_round_p<CT, NDW, Q, SH>;
    int per_cu = 0;
    hipError_t e = ensure_lds_limit(f, K::LDS);
    if (e == hipSuccess) e = blocks_per_cu(f, K::T, K::LDS, &per_cu);
    if (e != hipSuccess) return e;
    // every workgroup must be resident at once (they wait for each other): one per CU
    if (per_cu < 1 || P.A.C > num_cus * per_cu) return hipErrorCooperativeLaunchTooLarge;
    hipLaunchKernelGGL((k_round_p<CT, NDW, Q, SH>), dim3(nblk), dim3(K::T), K::LDS, st, P);
    return hipGetLastError();
}

template <typename CT, bool SH>
static hipError_t rp_launch_t(hipStream_t st, const RoundPArgs& P, int num_cus, int nblk) {
    switch (round_k_ndw(P.A.n)) {
        case 2: return rp_launch<CT, 2, 2, SH>(st, P, num_cus, nblk);
        case 4: return rp_launch<CT, 4, 4, SH>(st, P, num_cus, nblk);
        case 8: return rp_launch<CT, 8, 2, SH>(st, P, num_cus, nblk);
        case 16: return rp_launch<CT, 16, 4, SH>(st, P, num_cus, nblk);
        case 32: return rp_launch<CT, 32, 4, SH>(st, P, num_cus, nblk);
        case 64: return rp_launch<CT, 64, 4, SH>(st, P, num_cus, nblk);
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

// After the persistent launches of a DivideRounds: what the per-launch step writes besides Bm
// and the S rows, for rounds [r_lo, r_hi] of every chain, from Bm alone: the rounds of the chain's
// events [Bm[r], Bm[r+1]), wstat[r], wflag[r+1], active[r] and the new candidate's WLA row (the
// lastAncestors row at Bm[r+1]). One wave per (chain, 64 rounds), lane = round: a round
// holds a few events per chain, so a block per (chain, rounds) left most of its threads idle
// (c4: 0.42 ms for 8 192 chains x 139 rounds).
template <typename CT>
__global__ void __launch_bounds__(256) k_round_p_post(RoundArgs A, int r_lo, int r_hi) {
    const int gc = (int)blockIdx.x * 4 + (int)(threadIdx.x >> 6), lane = (int)(threadIdx.x & 63);
    if (gc >= A.C) return;
    const int n = A.n, C = A.C, len = A.c_len[gc], off = A.c_off[gc];
    const CT* __restrict__ LA = (const CT*)A.LA;
    {
        const int r0 = r_lo + 64 * (int)blockIdx.y;   // this wave's 64 rounds
        const int r = r0 + lane;
        int k = len;
        if (r <= r_hi) {
            const int b = A.Bm[(size_t)r * C + gc];
            k = A.Bm[(size_t)(r + 1) * C + gc];
            for (int x = b; x < k; x++) A.p_round[off + x] = r;
            A.wstat[(size_t)r * C + gc] = b < len ? ((k > b) ? 2 : 1) : 0;
            A.wflag[(size_t)(r + 1) * C + gc] = k < len ? 1 : 0;
            if (k < len) A.active[r] = 1;
        }
        // the WLA rows of these rounds, each by the whole wave (coalesced at any n)
        for (int q = 0; q < 64 && r0 + q <= r_hi; q++) {
            const int kq = __shfl(k, q);
            if (kq >= len) continue;   // (wave-uniform)
            const CT* row = LA + (size_t)(off + kq) * n;
            int32_t* dst = A.WLA + ((size_t)(r0 + q + 1) * C + gc) * n;
            if (sizeof(CT) == 2 && (n & 1) == 0) {   // compact: two coordinates per lane (4-byte loads, 8-byte stores)
                const uint32_t* row2 = (const uint32_t*)row;
                for (int i = lane; i < n / 2; i += 64) {
                    const uint32_t v = row2[i];
                    *(int2*)(dst + 2 * i) = make_int2(Coord<CT>::la(v & 0xFFFFu), Coord<CT>::la(v >> 16));
                }
            } else {
                for (int i = lane; i < n; i += 64) dst[i] = Coord<CT>::la(row[i]);
            }
        }
    }
}

void launch_round_p_post(hipStream_t st, const RoundArgs& A, int r_lo, int r_hi) {
    if (r_hi < r_lo) return;
    const dim3 grid((A.C + 3) / 4, (r_hi - r_lo + 64) / 64);
    if (A.compact) hipLaunchKernelGGL(k_round_p_post<uint16_t>, grid, dim3(256), 0, st, A, r_lo, r_hi);
    else hipLaunchKernelGGL(k_round_p_post<int32_t>, grid, dim3(256), 0, st, A, r_lo, r_hi);
}

void launch_round_p_tail(hipStream_t st, const RoundArgs& A, const int32_t* fin, int r_last) {
    hipLaunchKernelGGL(k_round_p_tail, dim3((A.C + 255) / 256), dim3(256), 0, st, A, fin, r_last);
}

hipError_t launch_round_p(hipStream_t st, const RoundArgs& A, uint32_t* FD8p, uint64_t* gran, int32_t* status,
                          int32_t* fin, int r0, int r_end, int init, int num_cus, int c_lo, int c_hi,
                          const RoundPWindows* win_dev, int nwin) {
    if (c_hi < 0) c_hi = A.C;
    if (c_lo < 0 || c_hi > A.C || c_lo >= c_hi) return hipErrorInvalidValue;
    RoundPArgs P{};
    P.c_lo = c_lo;
    if (nwin > kMaxShards || (nwin > 1 && !win_dev)) return hipErrorInvalidValue;
    P.nwin = nwin > 1 ? nwin : 1;   // 1: one launch over every chain, its own buffers
    P.Wd = nwin > 1 ? win_dev : nullptr;
    P.A = A;
    P.FD8p = FD8p;
    P.gran = gran;
    P.st = status;
    P.fin = fin;
    P.r0 = r0;
    P.r_end = r_end;
    P.tmo = 5000000;   // 50 ms per wait (a round takes microseconds)
    if (init) {
        const dim3 grid(c_hi - c_lo);
        if (A.compact) hipLaunchKernelGGL(k_round_p_init<uint16_t>, grid, dim3(64), 0, st, P, round_k_ndw(A.n));
        else hipLaunchKernelGGL(k_round_p_init<int32_t>, grid, dim3(64), 0, st, P, round_k_ndw(A.n));
        const hipError_t e = hipGetLastError();
        if (e != hipSuccess || init == 2) return e;   // (2: the initial rows only)
    }
    if (P.nwin > 1)
        return A.compact ? rp_launch_t<uint16_t, true>(st, P, num_cus, c_hi - c_lo)
                         : rp_launch_t<int32_t, true>(st, P, num_cus, c_hi - c_lo);
    return A.compact ? rp_launch_t<uint16_t, false>(st, P, num_cus, c_hi - c_lo)
                     : rp_launch_t<int32_t, false>(st, P, num_cus, c_hi - c_lo);
}

// ---- the recurrence's exchange floor (bench.py roofline.latency) --------------------------------
// k_round_p with the search taken out: C resident workgroups (one per CU, the recurrence's LDS carve)
// and per round s every workgroup publishes an NDW-dword row (16-byte write-through stores, chunk-major,
// every dword = s + 1) and an 8-byte granule {s + 1}, then every lane polls its candidate's granule and
// row part (Q lanes per candidate, HD = NDW / Q dwords each, sc1 loads issued and waited for together,
// rp_ld_cand) until all of them carry s + 1, then one workgroup barrier. Rows in 4 buffers by s % 4, as
// the recurrence's. The time per round is the all-to-all hand-off a round of the recurrence cannot go
// below (C = 2: one 1-to-1 hand-off each way). Every wait is bounded (st[0] = 1: gave up).
template <int NDW, int Q>
__global__ void __launch_bounds__(4 * NDW * Q) k_xchg_floor(int C, int rounds, uint32_t* __restrict__ rows,
                                                            uint64_t* __restrict__ gran, int32_t* __restrict__ st,
                                                            long long tmo) {
    constexpr int HD = NDW / Q, CS = HD < 4 ? HD : 4;
    const int c = blockIdx.x, t = threadIdx.x, lane = t & 63, wave = t >> 6;
    const int j = t / Q, q = t % Q;
    const size_t buf = (size_t)C * NDW, cst = (size_t)C * Q * CS;
    bool failed = false;
    for (int s = 0; s < rounds && !failed; s++) {
        const uint32_t tag = (uint32_t)(s + 1);
        uint32_t* rb = rows + (size_t)(s & 3) * buf;
        uint64_t* gb = gran + (size_t)(s & 3) * C;
        if (wave == 0) {   // publish: lane l < NDW / 4 writes 16 bytes, (q, k) = its part and chunk
            if (lane < NDW / 4) {
                const int pq = lane / (HD / CS > 0 ? HD / CS : 1), pk = lane % (HD / CS > 0 ? HD / CS : 1);
                rp_st4_sc1(rb + rp_chunk_off(pk, c, pq, C, Q, CS), make_uint4(tag, tag, tag, tag));
            }
            if (lane == 0) rp_st_gran(gb + c, (uint64_t)tag << 32);
        }
        if (j < C) {
            const long long t0 = __builtin_amdgcn_s_memrealtime();
            for (;;) {
                uint64_t gv;
                uint32_t v[HD];
                rp_ld_cand<HD>(gb + j, rb + rp_chunk_off(0, j, q, C, Q, CS), cst, gv, v);
                bool ok = (uint32_t)(gv >> 32) == tag;
#pragma unroll
                for (int d = 0; d < HD; d++) ok = ok && v[d] == tag;
                if (ok) break;
                if (__builtin_amdgcn_s_memrealtime() - t0 > tmo || rp_ld_abort(st) != 0) {
                    failed = true;
                    break;
                }
            }
        }
        if (failed) __hip_atomic_store((gu32*)st, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __syncthreads();
        failed = rp_ld_abort(st) != 0;
    }
}

template <int NDW, int Q>
static hipError_t xchg_launch(hipStream_t s, int C, int rounds, uint32_t* rows, uint64_t* gran, int32_t* st) {
    const void* f = (const void*)k_xchg_floor<NDW, Q>;
    const size_t lds = 84 * 1024;   // one workgroup per CU, as k_round_p
    const hipError_t e = ensure_lds_limit(f, lds);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL((k_xchg_floor<NDW, Q>), dim3(C), dim3(4 * NDW * Q), lds, s, C, rounds, rows, gran, st,
                       (long long)2000000);
    return hipGetLastError();
}

hipError_t launch_xchg_floor(hipStream_t s, int C, int n, int rounds, uint32_t* rows, uint64_t* gran, int32_t* st) {
    switch (round_k_ndw(n)) {   // the geometry k_round_p takes at this n
        case 16: return xchg_launch<16, 4>(s, C, rounds, rows, gran, st);
        case 32: return xchg_launch<32, 4>(s, C, rounds, rows, gran, st);
        case 64: return xchg_launch<64, 4>(s, C, rounds, rows, gran, st);
        default: return hipErrorInvalidValue;
    }
}

}  // namespace hgx

// Measurement entry for bench.py (roofline.latency): the exchange floor of a recurrence round with
// `chains` workgroups of k_round_p's geometry at n coordinates (16 < n <= 256), one warm-up launch, then
// one timed launch of `rounds` rounds (HIP events on the launch stream). HGX_ERR_DEVICE when a
// workgroup gave up waiting (not all resident) or on any HIP error.
extern "C" int32_t hgx_exchange_floor_bench(int32_t device, int32_t chains, int32_t n, int32_t rounds,
                                            double* us_per_round) {
    if (chains < 2 || chains > 1024 || n <= 16 || n > 256 || rounds < 1 || !us_per_round) return HGX_ERR_INVALID;
    int prev = 0, cus = 0;
    (void)hipGetDevice(&prev);
    if (hipSetDevice(device) != hipSuccess) return HGX_ERR_DEVICE;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || chains > cus) {
        (void)hipSetDevice(prev);
        return HGX_ERR_INVALID;   // one resident workgroup per CU
    }
    const int ndw = hgx::round_k_ndw(n);
    uint32_t* rows = nullptr;
    uint64_t* gran = nullptr;
    int32_t* st = nullptr;
    hipStream_t s = nullptr;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    int32_t h_st = 0;
    float ms = 0.f;
    hipError_t e = hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipEventCreate(&e0);
    if (e == hipSuccess) e = hipEventCreate(&e1);
    if (e == hipSuccess) e = hipMalloc((void**)&rows, (size_t)4 * chains * ndw * 4);
    if (e == hipSuccess) e = hipMalloc((void**)&gran, (size_t)4 * chains * 8);
    if (e == hipSuccess) e = hipMalloc((void**)&st, 16);
    for (int it = 0; it < 2 && e == hipSuccess; it++) {   // (a warm-up launch, then the timed one)
        e = hipMemsetAsync(rows, 0, (size_t)4 * chains * ndw * 4, s);
        if (e == hipSuccess) e = hipMemsetAsync(gran, 0, (size_t)4 * chains * 8, s);
        if (e == hipSuccess) e = hipMemsetAsync(st, 0, 16, s);
        if (e == hipSuccess && it) e = hipEventRecord(e0, s);
        if (e == hipSuccess) e = hgx::launch_xchg_floor(s, chains, n, it ? rounds : std::min(rounds, 64), rows, gran, st);
        if (e == hipSuccess && it) e = hipEventRecord(e1, s);
        if (e == hipSuccess) e = hipMemcpyAsync(&h_st, st, 4, hipMemcpyDeviceToHost, s);
        if (e == hipSuccess) e = hipStreamSynchronize(s);
        if (e == hipSuccess && h_st != 0) e = hipErrorLaunchTimeOut;
    }
    if (e == hipSuccess) e = hipEventElapsedTime(&ms, e0, e1);
    if (rows) (void)hipFree(rows);
    if (gran) (void)hipFree(gran);
    if (st) (void)hipFree(st);
    if (e0) (void)hipEventDestroy(e0);
    if (e1) (void)hipEventDestroy(e1);
    if (s) (void)hipStreamDestroy(s);
    (void)hipSetDevice(prev);
    if (e != hipSuccess) return HGX_ERR_DEVICE;
    *us_per_round = (double)ms * 1e3 / rounds;
    return HGX_OK;
}
