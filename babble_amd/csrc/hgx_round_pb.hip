// Persistent round recurrence for 256 < n <= 1024 (one graph): the k_round_p design (every round in
// one launch, candidate rows and granules handed over write-through and self-validating; RoundInc
// hashgraph.go:285-305, StronglySee :170-198) for candidate rows too large for one workgroup's
// registers. DESIGN.md §3.3.
//
//  * one workgroup of 1 024 threads per PP = 3 chains WITH events (the "probers"; silent chains have
//    no candidate in any round and no workgroup, their granules are never polled). Every prober's
//    31-probe window lives in LDS rebased to 8 bits (as k_round_p);
//  * 8 lanes per candidate (each holds a 1/8 part of the candidate's 8-bit rebased row, the counts
//    combined by DPP inside the wave), so a pass covers 128 candidates: the candidates come in chunks
//    of 128 (8 at n = 1 024), each chunk polled, validated and then searched against the PP windows
//    at once (three binary searches per loaded row). A candidate row crosses the fabric once per
//    workgroup and round: with one prober per workgroup the polls of c5 moved ~700 MB per round and
//    took 190 us of the ~350 us round (tools/probe, prof build);
//  * per (prober, candidate) its K(w) and "seen in an earlier window" bit go to LDS (the S row is
//    assembled from them once the boundary is known); per prober a K(w) histogram gives the boundary;
//  * the windows' raw lastAncestors rows and the new candidates' firstDescendants come straight from
//    HBM (at n = 1 024 a 32-position staging segment is 64 KB).
#include <hip/hip_runtime.h>

#include <cstdint>

#include "hgx_device.h"
#include "hgx_kernels.h"

namespace hgx {

namespace {

typedef __attribute__((address_space(1))) uint64_t gu64;
typedef __attribute__((address_space(1))) uint32_t gu32;

// kst bytes: K(w) (0..63) | seen in an earlier window | candidate
constexpr uint8_t kPbKM = 63, kPbDone = 64, kPbCand = 128;
constexpr int kPbSlots = 4;
constexpr int kPbPP = 3;   // probers (chains) per workgroup
constexpr uint32_t kPbEx = 1u << 31, kPbOv = 1u << 30, kPbBm = (1u << 30) - 1;

__device__ __forceinline__ void pb_st_sc1(uint32_t* p, uint32_t v) {
    asm volatile("global_store_dword %0, %1, off sc1" ::"v"(p), "v"(v) : "memory");
}
__device__ __forceinline__ void pb_st4_sc1(uint32_t* p, uint4 v) {
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    const u32x4 x = {v.x, v.y, v.z, v.w};
    asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(p), "v"(x) : "memory");
}
__device__ __forceinline__ void pb_st_gran(uint64_t* p, uint64_t v) {
    __hip_atomic_store((gu64*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint32_t pb_ld_abort(const int32_t* p) {
    return (uint32_t)__hip_atomic_load((gu32*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void pb_vm_drain() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
__device__ __forceinline__ void pb_lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// Candidate rows CHUNK-MAJOR (as k_round_p's rp_chunk_off): part q (HD dwords, lane q of the candidate)
// of chain gc in 16-byte chunks, chunk k at ((k C + gc) Q + q) x 16 bytes of the round's buffer, so a poll
// instruction's 64 lanes (8 candidates x 8 parts, chunk k of each) read one contiguous KB.
__host__ __device__ constexpr size_t pb_chunk_off(int k, int gc, int q, int C) { return (((size_t)k * C + gc) * 8 + q) * 4; }

// a wave-uniform pointer held in SGPRs (the base of a chunk's loads)
__device__ __forceinline__ const uint32_t* pb_uniform(const uint32_t* p) {
    const uint64_t a = (uint64_t)(uintptr_t)p;
    return (const uint32_t*)(uintptr_t)(((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(a >> 32)) << 32) |
                                        (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)a));
}

// a candidate's granule and this lane's HD dwords of its row: chunk k at sb + k cst (SGPR base, uniform)
// + vo bytes (this lane's (gc, q) offset), sc1 loads issued and waited for in one asm statement (see
// rp_ld_cand, hgx_round_p.hip)
template <int HD>
__device__ __forceinline__ void pb_ld_cand(const uint64_t* gp, const uint32_t* sb, size_t cst, uint32_t vo, uint64_t& gv,
                                           uint32_t (&v)[HD]) {
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    static_assert(HD == 16 || HD == 24 || HD == 32, "pb_ld_cand: HD in {16, 24, 32}");
    const uint32_t *s0 = pb_uniform(sb), *s1 = pb_uniform(sb + cst), *s2 = pb_uniform(sb + 2 * cst), *s3 = pb_uniform(sb + 3 * cst);
    u32x4 a, b, c, d;
    asm volatile(
        "global_load_dwordx2 %0, %5, off sc1\n\t"
        "global_load_dwordx4 %1, %6, %7 sc1\n\t"
        "global_load_dwordx4 %2, %6, %8 sc1\n\t"
        "global_load_dwordx4 %3, %6, %9 sc1\n\t"
        "global_load_dwordx4 %4, %6, %10 sc1\n\t"
        "s_waitcnt vmcnt(0)"
        : "=&v"(gv), "=&v"(a), "=&v"(b), "=&v"(c), "=&v"(d) : "v"(gp), "v"(vo), "s"(s0), "s"(s1), "s"(s2), "s"(s3) : "memory");
    const u32x4 q4[4] = {a, b, c, d};
#pragma unroll
    for (int k = 0; k < 4; k++) { v[4 * k] = q4[k].x; v[4 * k + 1] = q4[k].y; v[4 * k + 2] = q4[k].z; v[4 * k + 3] = q4[k].w; }
    if constexpr (HD == 32) {
        const uint32_t *s4 = pb_uniform(sb + 4 * cst), *s5 = pb_uniform(sb + 5 * cst), *s6 = pb_uniform(sb + 6 * cst),
                       *s7 = pb_uniform(sb + 7 * cst);
        u32x4 e, f, g, h;
        asm volatile(
            "global_load_dwordx4 %0, %4, %5 sc1\n\t"
            "global_load_dwordx4 %1, %4, %6 sc1\n\t"
            "global_load_dwordx4 %2, %4, %7 sc1\n\t"
            "global_load_dwordx4 %3, %4, %8 sc1\n\t"
            "s_waitcnt vmcnt(0)"
            : "=&v"(e), "=&v"(f), "=&v"(g), "=&v"(h) : "v"(vo), "s"(s4), "s"(s5), "s"(s6), "s"(s7) : "memory");
        const u32x4 r4[4] = {e, f, g, h};
#pragma unroll
        for (int k = 0; k < 4; k++) { v[16 + 4 * k] = r4[k].x; v[17 + 4 * k] = r4[k].y; v[18 + 4 * k] = r4[k].z; v[19 + 4 * k] = r4[k].w; }
    } else if constexpr (HD == 24) {
        const uint32_t *s4 = pb_uniform(sb + 4 * cst), *s5 = pb_uniform(sb + 5 * cst);
        u32x4 e, f;
        asm volatile(
            "global_load_dwordx4 %0, %2, %3 sc1\n\t"
            "global_load_dwordx4 %1, %2, %4 sc1\n\t"
            "s_waitcnt vmcnt(0)"
            : "=&v"(e), "=&v"(f) : "v"(vo), "s"(s4), "s"(s5) : "memory");
        const u32x4 r4[2] = {e, f};
#pragma unroll
        for (int k = 0; k < 2; k++) { v[16 + 4 * k] = r4[k].x; v[17 + 4 * k] = r4[k].y; v[18 + 4 * k] = r4[k].z; v[19 + 4 * k] = r4[k].w; }
    }
}

__device__ __forceinline__ uint32_t pb_combine8(uint32_t x) {   // sum over the 8 lanes of a candidate
    x += (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0xB1, 0xf, 0xf, false);    // quad_perm xor 1
    x += (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x4E, 0xf, 0xf, false);    // quad_perm xor 2
    x += (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x141, 0xf, 0xf, false);   // half-row mirror
    return x;
}

// Rows are COMPRESSED to the chains with events: coordinate slot i < na is chain amap[i] (c5's 341
// silent peers, whose coordinates are "none" everywhere and never count, take no bytes: 768 instead of
// 1 024 coordinate slots per row).
template <int HD_, int NP_>
struct PbCfg {
    static constexpr int Q = 8, T = 1024, NW = T / 64, PP = kPbPP;
    // probes per window (31: 5 search levels; 63: 6): c5's chains have ~38 events per round, so a
    // 31-probe window rarely held the boundary and most rounds searched two windows
    static constexpr int NP = NP_, LV = NP_ == 31 ? 5 : 6;
    static_assert(NP_ == 31 || NP_ == 63, "k_round_pb: windows of 31 or 63 probes");
    static constexpr int HD = HD_;              // row dwords per lane (16, 24 or 32)
    static constexpr int NDW = Q * HD;          // row dwords (4 coordinate slots each)
    static constexpr int CPB = T / Q;           // candidates per pass (128)
    static constexpr int NC = 1024;             // chains (bases, K, map)
    // window rows: dword 8h + e of part q (what lane q of a candidate compares) at h * 64 + 8 q + e, so
    // part q lies in banks 8q .. 8q + 7 of every row whatever the row; a ds_read_b128 lane group holds
    // two candidates per part, which read the part's two halves in opposite orders (the candidates
    // 2, 3 (mod 4) of a wave high half first): conflict-free whatever rows they probe
    static constexpr int WS = NDW;              // window row stride (dwords)
    static constexpr int WIN = NP * WS;         // window (dwords)
    // LDS (bytes)
    static constexpr int O_WIN = 0;                       // [PP][NP][WS] rebased probes
    static constexpr int O_BS = O_WIN + PP * WIN * 4;     // [2][NC] c_base + Bm, by round parity
    static constexpr int O_KST = O_BS + 2 * NC * 4;       // [PP][NC] bytes: K | done << 5 | cand << 6
    static constexpr int O_HIST = O_KST + PP * NC;        // [PP][64]
    static constexpr int O_POF = O_HIST + PP * 64 * 4;    // [PP] the published row's overflow flag
    static constexpr int O_MISC = O_POF + PP * 4;         // [8]: [2] any, [3] fail
    static constexpr int O_AMAP = O_MISC + 32;            // [NC] the chains with events (candidates)
    static constexpr int LDS = O_AMAP + NC * 4;
    static_assert(LDS <= 160 * 1024, "k_round_pb: LDS carve exceeds a CU's 160 KB");
};

struct RoundPbArgs {
    RoundArgs A;
    uint32_t* FD8p;   // [4][C][ndw], bit 7 of every byte = v(s) = (s >> 2) & 1 (round s: buffer s % 4)
    uint64_t* gran;   // [4][C]
    int32_t* st;      // [0] abort, [1] max round stopped, [2] finished, [3] rows counted exactly
    int32_t* fin;     // [1]
    const int32_t* amap;   // [na] the chains with events
    int na;
    int r0, r_end;
    long long tmo;
};

}  // namespace

// Optional phase clocks (-DHGX_STEP_PROF, build variant "prof"): thread 0 of each workgroup adds
// clock deltas per phase: 1 polls, 2 searches (both summed over the chunks), 3 histogram barrier,
// 4 scan + later windows, 5 publish + S rows, 6 publish barrier, 7 next windows' rebase + end barrier;
// 15 = block-rounds
#ifdef HGX_STEP_PROF
__device__ unsigned long long hgx_pb_prof[16];
#define PB_PROF_BEGIN() long long _pt = clock64(); unsigned long long _pa[16] = {}
#define PB_PROF(i)                                    \
    do {                                              \
        if (threadIdx.x == 0) {                       \
            const long long _t = clock64();           \
            _pa[i] += (unsigned long long)(_t - _pt); \
            _pt = _t;                                 \
            if ((i) == 7) _pa[15] += 1;               \
        }                                             \
    } while (0)
#define PB_PROF_END()                                              \
    do {                                                           \
        if (threadIdx.x == 0)                                      \
            for (int _i = 0; _i < 16; _i++)                        \
                if (_pa[_i]) atomicAdd(&hgx_pb_prof[_i], _pa[_i]); \
    } while (0)
void round_pb_prof_dump() {
    unsigned long long h[16];
    if (hipMemcpyFromSymbol(h, HIP_SYMBOL(hgx_pb_prof), sizeof(h)) != hipSuccess) return;
    if (!h[15]) return;
    const double r = (double)h[15];
    fprintf(stderr, "[hgx] k_round_pb clk per block-round (thread 0): polls %.0f searches %.0f hist-barrier %.0f "
            "scan+windows %.0f publish: gathers+store %.0f window loads %.0f S rows %.0f pub-barrier %.0f "
            "granules %.0f rebase k=0 %.0f k=1 %.0f k=2 %.0f end barrier %.0f | block-rounds %llu\n",
            h[1] / r, h[2] / r, h[3] / r, h[4] / r, h[8] / r, h[9] / r, h[5] / r, h[6] / r, h[10] / r, h[11] / r,
            h[12] / r, h[13] / r, h[7] / r, h[15]);
    unsigned long long z[16] = {};
    (void)hipMemcpyToSymbol(HIP_SYMBOL(hgx_pb_prof), z, sizeof(z));
}
#else
#define PB_PROF_BEGIN() (void)0
#define PB_PROF(i) (void)0
#define PB_PROF_END() (void)0
void round_pb_prof_dump() {}
#endif

template <typename CT, int HD_, int NP_>
__global__ void __launch_bounds__(1024) k_round_pb(RoundPbArgs P) {
    typedef PbCfg<HD_, NP_> K;
    constexpr int kPbP = K::NP;
    constexpr int Q = K::Q, T = K::T, NW = K::NW, PP = K::PP, HD = K::HD, WS = K::WS, CPB = K::CPB, NDW = K::NDW;
    constexpr int NC = K::NC;
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    const RoundArgs& A = P.A;
    const int n = A.n, C = A.C, sm = A.sm;
    const int t = threadIdx.x, lane = lane_id(), wave = __builtin_amdgcn_readfirstlane(t >> 6);
    const int jl = t / Q, q = t % Q;   // candidate slot in a pass, row part
    const int hsw = (jl >> 1) & 1;     // this candidate reads each 8-dword piece high half first
    auto winp = [&](int k) { return (uint32_t*)(lds + K::O_WIN) + k * K::WIN; };
    auto bpar = [&](int r) { return (int32_t*)(lds + K::O_BS) + (r & 1) * NC; };   // c_base + Bm[r]
    auto kstp = [&](int k) { return lds + K::O_KST + k * NC; };
    auto histp = [&](int k) { return (int32_t*)(lds + K::O_HIST) + k * 64; };
    int32_t* pof = (int32_t*)(lds + K::O_POF);
    int32_t* misc = (int32_t*)(lds + K::O_MISC);
    int32_t* amapl = (int32_t*)(lds + K::O_AMAP);
    if (P.fin[0] >= 0) return;   // finished in an earlier launch of this DivideRounds
    const CT* __restrict__ LA = (const CT*)A.LA;
    const CT* __restrict__ FDT = (const CT*)A.FDT;
    // the probers (block-uniform)
    int gcs[PP], lens[PP], offs[PP], bs[PP];
    bool valid[PP];
#pragma unroll
    for (int k = 0; k < PP; k++) {
        const int a = (int)blockIdx.x * PP + k;
        valid[k] = a < P.na;
        gcs[k] = __builtin_amdgcn_readfirstlane(valid[k] ? P.amap[a] : 0);
        lens[k] = __builtin_amdgcn_readfirstlane(valid[k] ? A.c_len[gcs[k]] : 0);
        offs[k] = __builtin_amdgcn_readfirstlane(A.c_off[gcs[k]]);
        bs[k] = __builtin_amdgcn_readfirstlane(valid[k] ? A.Bm[(size_t)P.r0 * C + gcs[k]] : 0);
    }
    for (int i = t; i < NC; i += T) {
        // (a silent chain's Bm rows are written after the launches: 0 = its length; its bases never
        // change and its candidate bits stay 0: only the chains with events are polled)
        const bool li = i < n && A.c_len[i] > 0;
        const int32_t cb = i < n ? A.c_base[i] : 0;
        bpar(P.r0 - 1)[i] = cb + (P.r0 > 0 && li ? A.Bm[(size_t)(P.r0 - 1) * C + i] : 0);
        if (!li) bpar(P.r0)[i] = cb;
        if (i < P.na) amapl[i] = P.amap[i];
    }
    for (int i = t; i < PP * NC; i += T) lds[K::O_KST + i] = 0;
    if (t < PP * 64) ((int32_t*)(lds + K::O_HIST))[t] = 0;
    if (t < PP) pof[t] = 0;
    if (t < 8) misc[t] = 0;
    // rebased 8-bit window rows of prober k's positions [kb, kb + np) against bases bq, straight from
    // HBM: rb_load issues a thread's raw loads, rb_store rebases them into the window. A thread takes
    // GS = 16 bytes of coordinate slots (8 compact, 4 int32: 2 or 1 window dwords) of rows
    // p = t / NG + k RPP; threads past RPP rows idle. Where its slots are GS consecutive chains from an
    // aligned one (c5: every slot), a row's slots are ONE 16-byte load (the per-slot gathers issued 26
    // dword loads per thread and window and took ~20 us per window at c5, the memory pipeline's
    // request rate, not its bytes); otherwise one gather per slot
    constexpr int GS = 16 / (int)sizeof(CT);       // slots per thread
    constexpr int GD = GS / 4;                     // window dwords per thread
    constexpr int NG = NDW / GD;                   // threads per row
    constexpr int RPP = T / NG;                    // rows per pass
    constexpr int PER = (kPbP + RPP - 1) / RPP;    // passes
    typedef uint32_t RawRows[PER][4];
    const int ge = t % NG, gp0 = t / NG;           // slot group, first row
    int g_c0;                                      // first chain of an aligned run (vector loads), else -1
    {
        const int i0 = GS * ge;
        bool vec = i0 < P.na && n % GS == 0;
        const int c0 = vec ? P.amap[i0] : -1;
        vec = vec && c0 % GS == 0;
#pragma unroll
        for (int u = 1; u < GS; u++) vec = vec && (i0 + u >= P.na || P.amap[i0 + u] == c0 + u);
        g_c0 = vec ? c0 : -1;
    }
    auto slot_chain = [&](int u) __attribute__((always_inline)) -> int {   // chain of slot GS ge + u (-1: no coordinate)
        const int i = GS * ge + u;
        return i < P.na ? (g_c0 >= 0 ? g_c0 + u : amapl[i]) : -1;
    };
    auto rb_load = [&](RawRows& raw, int off, int kb, int np) __attribute__((always_inline)) {
#pragma unroll
        for (int k = 0; k < PER; k++) {
            const int p = gp0 + k * RPP;
#pragma unroll
            for (int u = 0; u < 4; u++) raw[k][u] = 0u;
            if (gp0 < RPP && p < np) {
                const CT* row = LA + (size_t)(off + kb + p) * n;
                if (g_c0 >= 0) {
                    const uint4 v = *(const uint4*)(row + g_c0);
                    raw[k][0] = v.x; raw[k][1] = v.y; raw[k][2] = v.z; raw[k][3] = v.w;
                } else {
#pragma unroll
                    for (int u = 0; u < GS; u++) {
                        const int ch = slot_chain(u);
                        const uint32_t a = ch >= 0 ? (uint32_t)row[ch] : 0u;
                        if constexpr (sizeof(CT) == 2) raw[k][u >> 1] |= a << (16 * (u & 1));
                        else raw[k][u] = a;
                    }
                }
            }
        }
    };
    auto rb_store = [&](const RawRows& raw, uint32_t* win, int np, const int32_t* bq) __attribute__((always_inline)) {
        if (gp0 >= RPP || gp0 >= np) return;
        int32_t bqv[GS];
        bool sv[GS];
#pragma unroll
        for (int u = 0; u < GS; u++) {
            const int ch = slot_chain(u);
            sv[u] = ch >= 0;
            bqv[u] = ch >= 0 ? bq[ch] : 0;
        }
        const int d = GD * ge;   // first window dword (GD consecutive ones share an 8-dword piece)
        const int wa = ((d % HD) >> 3) * 64 + (d / HD) * 8 + (d & 7);
#pragma unroll
        for (int k = 0; k < PER; k++) {
            const int p = gp0 + k * RPP;
            if (p >= np) continue;
            uint32_t w[GD];
#pragma unroll
            for (int x = 0; x < GD; x++) w[x] = 0u;   // (swar_ge_count's window bytes)
#pragma unroll
            for (int u = 0; u < GS; u++) {
                int32_t la;
                if constexpr (sizeof(CT) == 2) la = (int32_t)((raw[k][u >> 1] >> (16 * (u & 1))) & 0xFFFFu) - 1;
                else la = (int32_t)raw[k][u];
                const int32_t x = la - bqv[u] + 1;
                if (sv[u]) w[u >> 2] |= (uint32_t)min(max(x, 0), 126) << (8 * (u & 3));
            }
            if constexpr (GD == 2) *(uint2*)(win + p * WS + wa) = make_uint2(w[0], w[1]);
            else win[p * WS + wa] = w[0];
        }
    };
    auto rebase = [&](uint32_t* win, int off, int kb, int np, const int32_t* bq) __attribute__((always_inline)) {
        RawRows raw;
        rb_load(raw, off, kb, np);
        rb_store(raw, win, np, bq);
    };
    pb_lds_barrier();   // the bases (a rebase reads other threads' entries)
#pragma unroll
    for (int k = 0; k < PP; k++)
        if (valid[k] && bs[k] < lens[k]) rebase(winp(k), offs[k], bs[k], min(kPbP, lens[k] - bs[k]), bpar(P.r0 - 1));
    pb_lds_barrier();
    PB_PROF_BEGIN();
    int s = P.r0;
    bool failed = false;
    for (;; s++) {
        if (s >= P.r_end) break;
        bool have[PP], act[PP];
        int kb[PP], np[PP], kstar[PP], B[PP], carried[PP];
#pragma unroll
        for (int k = 0; k < PP; k++) {
            have[k] = valid[k] && bs[k] < lens[k];
            act[k] = have[k];
            kb[k] = bs[k];
            np[k] = have[k] ? min(kPbP, lens[k] - bs[k]) : 0;
            kstar[k] = lens[k];
            B[k] = -1;
            carried[k] = 0;
        }
        const uint32_t vbit = ((s >> kRoundPShift) & 1) ? 0x80808080u : 0u;
        // the firstDescendants lines (and address translations) the publish will gather: the round's
        // new candidate lies in the window, whose middle position's column entries share a page and
        // mostly a line with it (each coordinate's column is its own 2 MB page: without this the
        // publish's 1 024 gathers per prober each took a translation miss, 26 us per c5 round); the
        // loads complete behind this round's first poll, which waits for the candidates anyway
        uint32_t pfx = 0;
        if (t < P.na) {
            const int ch = amapl[t];
#pragma unroll
            for (int k = 0; k < PP; k++)
                if (have[k]) pfx += (uint32_t)FDT[(size_t)ch * A.Pcap + offs[k] + min(bs[k] + kPbP / 2, lens[k] - 1)];
        }
        bool any = false;
        for (int w_it = 0;; w_it++) {
            // every chunk of 128 candidates: poll (reload in a later window), search every active window
            // (chunks over the chains with events only: c5's 341 silent peers cost no chunk slots). A wave
            // takes its chunks in the order their candidates arrive: a chunk whose rows are not complete
            // yet is passed over and retried after the others, so a late candidate delays its own chunk's
            // search only, not the searches of the chunks after it (with the chunks in order, the wave
            // holding the round's last candidate searched every later chunk after it arrived)
            const int nch = (P.na + CPB - 1) / CPB;
            uint32_t pend = (1u << nch) - 1u;   // (nch <= 8)
            const long long tw = __builtin_amdgcn_s_memrealtime();
            bool wfail_w = false;
            for (int spins = 0; pend; spins++) {
              if (spins > 0) {   // a pass with nothing new: a pause and the bounded-wait checks
                if ((spins & 7) == 7) {
                    const long long now = __builtin_amdgcn_s_memrealtime();
                    if (now - tw > P.tmo || pb_ld_abort(P.st) != 0) {
                        wfail_w = true;
                        if (lane == 0) misc[3] = 1;
                    }
                }
                __builtin_amdgcn_s_sleep(1);
              }
              for (int ch = 0; ch < nch; ch++) {
                if (!((pend >> ch) & 1u)) continue;
                const int ja = ch * CPB + jl;
                const bool jv = ja < P.na;
                const int j = jv ? amapl[ja] : 0;   // candidate chain
                const bool live = jv;
                uint64_t gv = 0;
                uint32_t fd[HD];
                const uint64_t* gp = P.gran + (size_t)(s % kPbSlots) * C + (live ? j : 0);
                // (chunk-major: the buffer's base in SGPRs, this lane's (chain, part) offset in bytes)
                const uint32_t* rsb = P.FD8p + (size_t)(s & (kRoundPBufs - 1)) * C * NDW;
                const uint32_t rvo = (uint32_t)(pb_chunk_off(0, live ? j : 0, q, C) * 4);
                // (a wave of this workgroup gave up: no further waits)
                bool wfail = wfail_w || *(volatile int32_t*)&misc[3] != 0;
                if (!wfail && __any(live)) {
                    pb_ld_cand<HD>(gp, rsb, (size_t)C * 8 * 4, rvo, gv, fd);
                    uint32_t bad = 0;
#pragma unroll
                    for (int d = 0; d < HD; d++) bad |= (fd[d] ^ vbit) & 0x80808080u;
                    const bool tag_ok = (uint32_t)(gv >> 32) == (uint32_t)(s + 1);
                    const bool ok = !live || (tag_ok && (!((uint32_t)gv & kPbEx) || bad == 0));
                    if (!__all(ok)) continue;   // not complete yet: the next pending chunk
                }
                pend &= ~(1u << ch);
                spins = 0;
                PB_PROF(1);
                const uint32_t gval = (uint32_t)gv;
                const bool cand = live && !wfail && (gval & kPbEx);
                const bool ov = cand && (gval & kPbOv);
                if (w_it == 0 && jv && q == 0 && !wfail) bpar(s)[j] = A.c_base[j] + (live ? (int)(gval & kPbBm) : 0);
                if (wfail && lane == 0) misc[3] = 1;
                if (cand && q == 0) misc[2] = 1;
#pragma unroll
                for (int d = 0; d < HD; d++) fd[d] = cand ? swar_nf(fd[d] & 0x7F7F7F7Fu) : 0x01010101u;   // 128 - FD'

                // (candidates 2, 3 (mod 4) read each 8-dword piece high half first: their registers too)
                if (hsw) {
#pragma unroll
                    for (int h = 0; h < HD / 8; h++)
#pragma unroll
                        for (int e = 0; e < 4; e++) {
                            const uint32_t x = fd[8 * h + e];
                            fd[8 * h + e] = fd[8 * h + 4 + e];
                            fd[8 * h + 4 + e] = x;
                        }
                }
                bool done[PP], srch[PP];
                int lo[PP], hi[PP];
                const bool wc = __any(cand);
#pragma unroll
                for (int k = 0; k < PP; k++) {
                    done[k] = w_it > 0 && jv && (kstp(k)[j] & kPbDone);   // seen in an earlier window
                    srch[k] = act[k] && wc;
                    lo[k] = 0;
                    hi[k] = kPbP;
                }
                bool srch_any = false;
#pragma unroll
                for (int k = 0; k < PP; k++) srch_any |= srch[k];
#pragma unroll 1
                for (int it = 0; it < (srch_any ? K::LV : 0); it++) {
                    int mid[PP];
                    uint32_t cnt[PP];
#pragma unroll
                    for (int k = 0; k < PP; k++) {
                        mid[k] = (lo[k] + hi[k]) >> 1;
                        cnt[k] = 0;
                    }
                    if (!ov) {
                        // this lane's part of each active window's probe row, 8 dwords at a time
#pragma unroll
                        for (int k = 0; k < PP; k++) {
                            if (!srch[k]) continue;
                            const uint4* rp = (const uint4*)(winp(k) + mid[k] * WS + q * 8) + hsw;
#pragma unroll
                            for (int h = 0; h < HD / 8; h++) {
                                const uint4 v0 = rp[16 * h], v1 = rp[16 * h + 1 - 2 * hsw];
                                const uint32_t v8[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
                                const uint32_t f8[8] = {fd[8 * h], fd[8 * h + 1], fd[8 * h + 2], fd[8 * h + 3],
                                                        fd[8 * h + 4], fd[8 * h + 5], fd[8 * h + 6], fd[8 * h + 7]};
                                cnt[k] += swar_ge_count<8>(v8, f8);
                            }
                        }
                    } else {
                        // exact int32 compares of this part of the row (hashgraph.go:191-197)
                        // (this lane's coordinate slots, each a chain with events)
                        const int i_lo = q * HD * 4, i_hi = min(P.na, (q + 1) * HD * 4);
                        const size_t pos = (size_t)A.c_off[j] + (gval & kPbBm);
#pragma unroll
                        for (int k = 0; k < PP; k++) {
                            if (!srch[k] || done[k] || mid[k] >= np[k]) continue;
                            for (int i = i_lo; i < i_hi; i++) {
                                const int ch = amapl[i];
                                const int32_t fdv = Coord<CT>::fd(FDT[(size_t)ch * A.Pcap + pos]);
                                const int32_t lav =
                                    min(Coord<CT>::la(LA[(size_t)(offs[k] + kb[k] + mid[k]) * n + ch]), kMaxI32 - 1);
                                cnt[k] += lav >= fdv ? 1u : 0u;
                            }
                        }
                    }
#pragma unroll
                    for (int k = 0; k < PP; k++) {
                        if (!srch[k]) continue;
                        const uint32_t c8 = pb_combine8(cnt[k]);
                        const bool seen = done[k] || mid[k] >= np[k] || ((int)c8 >= sm && !(j == gcs[k] && kb[k] + mid[k] == bs[k]));
                        if (seen) hi[k] = mid[k]; else lo[k] = mid[k] + 1;
                    }
                }
                PB_PROF(2);
#pragma unroll
                for (int k = 0; k < PP; k++) {
                    if (!act[k]) continue;   // (a prober whose boundary is known keeps its K)
                    const int Kw = srch[k] ? lo[k] : 0;
                    if (cand && q == 0 && !done[k] && Kw < np[k]) atomicAdd(&histp(k)[Kw], 1);
                    // K of this window, seen-earlier bit, candidate bit (the S row's inputs)
                    if (jv && q == 0) kstp(k)[j] = (uint8_t)(min(Kw, (int)kPbKM) | (done[k] ? kPbDone : 0) | (cand ? kPbCand : 0));
                }
              }
            }
            // the histograms are complete: every wave scans them (the boundary: first probe where
            // #{K <= p} (+ seen in earlier windows) >= SM)
            pb_lds_barrier();
            PB_PROF(3);
            any = misc[2] != 0;
            const bool fail = misc[3] != 0;
            bool more = false, nxt[PP];
            int tot[PP];
#pragma unroll
            for (int k = 0; k < PP; k++) {
                nxt[k] = false;
                tot[k] = 0;
                if (!act[k]) continue;
                const uint32_t v = lane < np[k] ? (uint32_t)histp(k)[lane] : 0u;
                const uint32_t inc = wave_scan_add_u32(v) + (uint32_t)carried[k];
                const uint64_t m = __ballot(lane < np[k] && (int)inc >= sm);
                tot[k] = __builtin_amdgcn_readlane((int)inc, 63);
                B[k] = __builtin_amdgcn_readfirstlane(m ? (int)__builtin_ctzll(m) : -1);
                if (B[k] >= 0) kstar[k] = kb[k] + B[k];
                // no boundary in this window (rare): the next one, if the chain has more events
                nxt[k] = B[k] < 0 && any && !fail && kb[k] + np[k] < lens[k];
                more |= nxt[k];
            }
            if (!more) break;
            pb_lds_barrier();   // every wave has scanned the histograms and read kst
#pragma unroll
            for (int k = 0; k < PP; k++) {
                if (!nxt[k]) {
                    act[k] = false;
                    continue;
                }
                // the candidates seen in this window are seen at every later probe
                uint8_t* ks = kstp(k);
                for (int jj = t; jj < n; jj += T) {
                    const uint8_t k8 = ks[jj];
                    if ((k8 & kPbCand) && (k8 & kPbKM) < np[k]) ks[jj] = (uint8_t)(k8 | kPbDone);
                }
                if (t < 64) histp(k)[t] = 0;
                carried[k] = tot[k];
                kb[k] += np[k];
                np[k] = min(kPbP, lens[k] - kb[k]);
                rebase(winp(k), offs[k], kb[k], np[k], bpar(s - 1));
            }
            pb_lds_barrier();
        }
        PB_PROF(4);
        if (misc[3] != 0) { failed = true; break; }
        if (!any) break;   // W'_s is empty: no round s
        // W'_{s+1} of each prober: the firstDescendants row of position kstar rebased to
        // base(s+1) = c_base + Bm[s] (bit 7 = v(s + 1)), straight from the FDT columns; then the next
        // windows' raw rows (compact coordinates: every prober's loads at once; int32 rows are loaded
        // after the barrier, one prober at a time)
        // (63-probe windows: prober 0's rows now, the others' after the barrier, one row set in registers)
        constexpr bool kMerged = sizeof(CT) == 2 && kPbP == 31;
        constexpr bool kPipe = sizeof(CT) == 2 && kPbP == 63;
        constexpr int kPipeBufs = 1;   // (two row sets in flight spilled and measured no faster)
        RawRows rawn[kMerged ? PP : kPipe ? kPipeBufs : 1];
        int np1[PP];
        {
            const int k = t / NDW, d = t % NDW;
            int kk = -1;   // (a register-indexed prober: its scalars by an unrolled select)
#pragma unroll
            for (int x = 0; x < PP; x++)
                if (k == x && valid[x] && kstar[x] < lens[x]) kk = x;
            int off = 0, kst_ = 0, gc = 0;
#pragma unroll
            for (int x = 0; x < PP; x++)
                if (kk == x) { off = offs[x]; kst_ = kstar[x]; gc = gcs[x]; }
            if (kk >= 0) {
                int dch[4];   // the chains of this dword's 4 coordinate slots (-1: none)
#pragma unroll
                for (int u = 0; u < 4; u++) dch[u] = 4 * d + u < P.na ? amapl[4 * d + u] : -1;
                CT f[4];
#pragma unroll
                for (int u = 0; u < 4; u++) f[u] = FDT[(size_t)(dch[u] >= 0 ? dch[u] : 0) * A.Pcap + off + kst_];
                const uint32_t vb1 = (((s + 1) >> kRoundPShift) & 1) ? 0x80808080u : 0u;
                const int32_t* bs1 = bpar(s);
                uint32_t w = 0;
                bool of = false;
#pragma unroll
                for (int u = 0; u < 4; u++) {
                    const int32_t fv = Coord<CT>::fd(f[u]);
                    const bool real = dch[u] >= 0 && fv != kMaxI32;
                    const int32_t x = fv - (real ? bs1[dch[u]] : 0) + 1;
                    of |= real && x > 126;
                    w |= (real && x <= 126 ? (uint32_t)x : 127u) << (8 * u);
                }
                // (16 bytes per lane: a prober's NDW threads fill whole waves, so its 64 consecutive dwords of
                // a wave go out as 16 dwordx4 write-through stores, ~6x cheaper per byte than dword ones)
                static_assert(NDW % 64 == 0, "k_round_pb: a prober's row dwords fill whole waves");
                const int src = (4 * lane) & 63;
                const uint32_t wv = w | vb1;
                const uint4 w4 = make_uint4((uint32_t)__shfl((int)wv, src), (uint32_t)__shfl((int)wv, src + 1),
                                            (uint32_t)__shfl((int)wv, src + 2), (uint32_t)__shfl((int)wv, src + 3));
                if (lane < 16)
                    pb_st4_sc1(P.FD8p + (size_t)((s + 1) & (kRoundPBufs - 1)) * C * NDW +
                                   pb_chunk_off(((d - lane + 4 * lane) % HD) / 4, gc, (d - lane + 4 * lane) / HD, C), w4);
                if (of) pof[kk] = 1;
            }
            PB_PROF(8);
            // (the next windows' rows: issued after the publish, which waits for its gathers alone, and
            // in flight behind the S rows, the barrier and the granules)
#pragma unroll
            for (int x = 0; x < PP; x++) {
                np1[x] = valid[x] && kstar[x] < lens[x] ? min(kPbP, lens[x] - kstar[x]) : 0;
                if constexpr (kMerged) rb_load(rawn[x], offs[x], kstar[x], np1[x]);
            }
            if constexpr (kPipe) rb_load(rawn[0], offs[0], kstar[0], np1[0]);
            PB_PROF(9);
        }
        // the S rows (DecideFame, hashgraph.go:688-705): bit j = the new candidate strongly sees
        // candidate j of W'_s, i.e. j was seen in an earlier window or K(j) <= B
        constexpr int WPR = NC / 64;   // 64-bit words per S row
        for (int task = wave; task < PP * WPR; task += NW) {
            const int k = task / WPR, w = task % WPR;
            int Bk = -1, gc = 0;
            bool nx = false;
#pragma unroll
            for (int x = 0; x < PP; x++)
                if (k == x) { Bk = B[x]; gc = gcs[x]; nx = valid[x] && kstar[x] < lens[x]; }
            if (!nx || w >= A.nw) continue;   // (wave-uniform)
            const int jj = w * 64 + lane;
            const uint8_t k8 = jj < n ? kstp(k)[jj] : 0;
            const uint64_t m = __ballot((k8 & kPbCand) && ((k8 & kPbDone) || (int)(k8 & kPbKM) <= Bk));
            if (lane == 0) A.Smat[((size_t)(s + 1) * C + gc) * A.nw + w] = m;
        }
#pragma unroll
        for (int k = 0; k < PP; k++)
            if (t == k && valid[k]) A.Bm[(size_t)(s + 1) * C + gcs[k]] = kstar[k];
        PB_PROF(5);
        pb_lds_barrier();   // the rows' overflow flags, every search read of the windows, kst reads
        PB_PROF(6);
#pragma unroll
        for (int k = 0; k < PP; k++) {
            if (t == k && valid[k]) {
                const bool of = pof[k] != 0;
                const bool nx = kstar[k] < lens[k];
                pb_st_gran(P.gran + (size_t)((s + 1) % kPbSlots) * C + gcs[k],
                           ((uint64_t)(uint32_t)(s + 2) << 32) | (uint32_t)kstar[k] | (nx ? kPbEx : 0u) |
                               (of ? kPbOv : 0u));
                if (of) atomicAdd(&P.st[3], 1);
                pof[k] = 0;   // (same thread: read before)
            }
        }
        if (t >= 64 && t < 64 + PP * 64) ((int32_t*)(lds + K::O_HIST))[t - 64] = 0;
        if (t == 200) misc[2] = 0;
        PB_PROF(10);
#pragma unroll
        for (int k = 0; k < PP; k++) {
            if constexpr (kMerged) {
                rb_store(rawn[k], winp(k), np1[k], bpar(s));
            } else if constexpr (kPipe) {
                if (kPipeBufs == 2) {
                    if (k + 1 < PP) rb_load(rawn[(k + 1) % kPipeBufs], offs[k + 1], kstar[k + 1], np1[k + 1]);
                    rb_store(rawn[k % kPipeBufs], winp(k), np1[k], bpar(s));
                } else {
                    if (k > 0) rb_load(rawn[0], offs[k], kstar[k], np1[k]);
                    rb_store(rawn[0], winp(k), np1[k], bpar(s));
                }
            } else if (np1[k] > 0) {
                rebase(winp(k), offs[k], kstar[k], np1[k], bpar(s));
            }
            bs[k] = kstar[k];
            PB_PROF(11 + k);
        }
        if (pfx == 0xFFFFFFFFu) misc[7] = 1;   // (the prefetch's use: never true, keeps the loads)
        pb_lds_barrier();
        PB_PROF(7);
    }
    PB_PROF_END();
    pb_vm_drain();
    if (failed) {
        if (t == 0 && atomicCAS((int32_t*)P.st, 0, gcs[0] + 1) == 0) atomicExch(&P.st[3], s);
        return;
    }
#pragma unroll
    for (int k = 0; k < PP; k++) {
        if (t != k || !valid[k]) continue;
        const bool rep = blockIdx.x == 0 && k == 0;
        if (s < P.r_end) {   // W'_s empty: round s has no events (the per-launch step's outputs)
            A.wstat[(size_t)s * C + gcs[k]] = 0;
            A.wflag[(size_t)(s + 1) * C + gcs[k]] = 0;
            A.Bm[(size_t)(s + 1) * C + gcs[k]] = lens[k];
            if (rep) {
                P.fin[0] = s;
                atomicAdd(&P.st[2], 1);
            }
        }
        if (rep) atomicMax(&P.st[1], s);
    }
}

// W'_{r0}'s compressed rows (rebased to base(r0), bit 7 = v(r0)) and granules of the chains with events,
// from the WFD rows of launch_round_gather (k_round_p_init's job, for the compressed slots); the three
// other buffers get the invalid bit for the rounds r0 + 1 .. r0 + 3 that will use them. One workgroup per
// chain with events.
template <typename CT>
__global__ void __launch_bounds__(64) k_round_pb_init(RoundPbArgs P, int ndw) {
    const RoundArgs& A = P.A;
    const int gc = P.amap[blockIdx.x], n = A.n, C = A.C, r = P.r0;
    const int b = A.Bm[(size_t)r * C + gc];
    const bool have = b < A.c_len[gc];
    bool of = false;
    const CT* __restrict__ row = (const CT*)A.WFD + ((size_t)r * C + gc) * n;
    for (int d = threadIdx.x; d < ndw; d += 64) {
        uint32_t w = 0;
        for (int u = 0; u < 4; u++) {
            const int i = 4 * d + u;
            uint32_t v = 127u;
            if (have && i < P.na) {
                const int ch = P.amap[i];
                const int32_t f = Coord<CT>::fd(row[ch]);
                if (f != kMaxI32) {
                    const int32_t bs = A.c_base[ch] + (r > 0 ? A.Bm[(size_t)(r - 1) * C + ch] : 0);
                    const int32_t x = f - bs + 1;
                    if (x > 126) of = true;
                    else v = (uint32_t)x;
                }
            }
            w |= v << (8 * u);
        }
        // (chunk-major, pb_chunk_off: dword d is dword (d % HD) % 4 of chunk (d % HD) / 4 of part d / HD)
        const int hd = ndw / 8;
        const size_t dof = pb_chunk_off((d % hd) / 4, gc, d / hd, C) + (d % hd) % 4;
        pb_st_sc1(P.FD8p + (size_t)(r & (kRoundPBufs - 1)) * C * ndw + dof,
                  w | (((r >> kRoundPShift) & 1) ? 0x80808080u : 0u));
        for (int k = 1; k < kRoundPBufs; k++)
            pb_st_sc1(P.FD8p + (size_t)((r + k) & (kRoundPBufs - 1)) * C * ndw + dof,
                      (((r + k) >> kRoundPShift) & 1) ? 0x7F7F7F7Fu : 0xFFFFFFFFu);   // bit 7 = !v(r + k)
    }
    of = __any(of);
    if (threadIdx.x == 0)
        pb_st_gran(P.gran + (size_t)(r % kPbSlots) * C + gc,
                   ((uint64_t)(uint32_t)(r + 1) << 32) | (uint32_t)b | (have ? kPbEx : 0u) | (of ? kPbOv : 0u));
}

// the rows of silent chains (no events, no workgroup) for rounds [r_lo, r_hi]: Bm = 0 (= len)
__global__ void k_round_pb_silent(RoundArgs A, int r_lo, int r_hi) {
    const int gc = blockIdx.x * blockDim.x + threadIdx.x;
    if (gc >= A.C || A.c_len[gc] != 0) return;
    for (int r = r_lo; r <= r_hi + 1; r++) A.Bm[(size_t)r * A.C + gc] = 0;
}

namespace {
template <typename CT, int HD, int NP>
hipError_t pb_launch(hipStream_t st, const RoundPbArgs& P, int num_cus, bool init) {
    typedef PbCfg<HD, NP> K;
    const void* f = (const void*)k_round_pb<CT, HD, NP>;
    int per_cu = 0;
    hipError_t e = ensure_lds_limit(f, K::LDS);
    if (e == hipSuccess) e = blocks_per_cu(f, K::T, K::LDS, &per_cu);
    if (e != hipSuccess) return e;
    const int nblk = (P.na + K::PP - 1) / K::PP;
    // every workgroup must be resident at once (they wait for each other)
    if (per_cu < 1 || nblk > num_cus * per_cu) return hipErrorCooperativeLaunchTooLarge;
    if (init) {
        hipLaunchKernelGGL(k_round_pb_init<CT>, dim3(P.na), dim3(64), 0, st, P, K::NDW);
        e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL((k_round_pb<CT, HD, NP>), dim3(nblk), dim3(K::T), K::LDS, st, P);
    return hipGetLastError();
}
}  // namespace

bool round_pb_ok(int n, int G) { return G == 1 && n > 256 && n <= 1024; }

hipError_t launch_round_pb(hipStream_t st, const RoundArgs& A, uint32_t* FD8p, uint64_t* gran, int32_t* status,
                           int32_t* fin, const int32_t* amap, int na, int r0, int r_end, int num_cus, bool init) {
    if (!round_pb_ok(A.n, A.C / A.n) || na < 1) return hipErrorInvalidValue;
    RoundPbArgs P{};
    P.A = A;
    P.FD8p = FD8p;
    P.gran = gran;
    P.st = status;
    P.fin = fin;
    P.amap = amap;
    P.na = na;
    P.r0 = r0;
    P.r_end = r_end;
    P.tmo = 5000000;   // 50 ms per wait
    // row dwords per lane by the chains with events (coordinate slots = 32 HD)
    if (na > 1024) return hipErrorInvalidValue;
    const int hd = na <= 512 ? 16 : na <= 768 ? 24 : 32;
    // (63-probe windows where three fit the LDS with compact coordinates)
    // (31-probe windows at every width: c5 6.0 -> 8.1 ms)
    if (A.compact)
        return hd == 16 ? pb_launch<uint16_t, 16, 63>(st, P, num_cus, init)
                        : hd == 24 ? pb_launch<uint16_t, 24, 63>(st, P, num_cus, init) : pb_launch<uint16_t, 32, 31>(st, P, num_cus, init);
    return hd == 16 ? pb_launch<int32_t, 16, 31>(st, P, num_cus, init)
                    : hd == 24 ? pb_launch<int32_t, 24, 31>(st, P, num_cus, init) : pb_launch<int32_t, 32, 31>(st, P, num_cus, init);
}

void launch_round_pb_silent(hipStream_t st, const RoundArgs& A, int r_lo, int r_hi) {
    if (r_hi < r_lo) return;
    hipLaunchKernelGGL(k_round_pb_silent, dim3((A.C + 255) / 256), dim3(256), 0, st, A, r_lo, r_hi);
}

}  // namespace hgx
