// Round step with one lane per candidate (RoundInc, hashgraph.go:285-305; StronglySee
// hashgraph.go:170-198). DESIGN.md §3.3.
//
// Step s finds, for chain c, the boundary Bm[s+1][c] = first offset k >= Bm[s][c] whose
// event strongly sees >= SM candidates w of W'_s (the first event of each chain with round
// >= s; its own candidate does not count at the probe that is itself). Strongly seeing w is
// monotone along the chain (lastAncestors only grow), so every candidate has a first
// strongly-seeing probe K(w) in a window of P probe rows, and the boundary is the SM-th
// smallest K(w): each lane binary-searches its own candidate's K(w), an LDS histogram of
// the K(w) gives the boundary. No barrier per search level, and the per-(probe, candidate)
// count never leaves the lane.
//
// The count #{i : LA[x][i] >= FD[w][i]} runs on 8-bit SWAR: every coordinate is rebased
// per round to base_i = Index of the candidate of round s-1 on chain i (c_base + Bm[s-1][i]).
// A candidate of round s has FD[w][i] >= base_i (its descendants have round >= s, so they sit
// at or after Bm[s][i] >= Bm[s-1][i]), so FD' = FD - base + 1 is in [1, 126] when the
// candidate's first descendants are within 125 events of base (127 = none), and the probe
// values are LA' = clamp(LA - base + 1, 0, 126) with the byte's top bit set: per byte,
// (0x80 | LA') - FD' never borrows and its bit 7 is [LA' >= FD'] = [LA >= FD]. One v_sub,
// one v_and, one v_bcnt per 4 coordinates. The producer of a candidate row (the step that
// found it) writes it rebased and flags the round if a value does not fit; a flagged round
// runs the exact int32 compare instead (same search, slower).
//
// The step also writes what the next step needs: the new candidate's rows (WLA, raw WFD,
// rebased FD8) and its strongly-seen bitmask, DecideFame's S row (hashgraph.go:688-705).
//
// Memory: every step reads all candidates' rebased rows (64 KB at n = 256), written by the
// previous step on every XCD. They are laid out so that a wave's 64 lanes (64 candidates) load
// consecutive 16-byte groups (fd8_at); all head loads are issued before one explicit wait,
// and barriers wait for LDS only, so no barrier drains the window staging early.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

#include "hgx_device.h"
#include "hgx_kernels.h"

namespace hgx {

// Optional phase clocks (-DHGX_STEP_PROF, build variant "prof"): thread 0 of each block adds
// s_memtime deltas per phase to hgx_rk_prof[] once, at the end of the step.
#ifdef HGX_STEP_PROF
__device__ unsigned long long hgx_rk_prof[8];
#define RK_PROF_BEGIN() long long _pt = clock64(); unsigned long long _pa[8] = {0, 0, 0, 0, 0, 0, 0, 0}
#define RK_PROF(i)                                                \
    do {                                                          \
        if (threadIdx.x == 0) {                                   \
            const long long _t = clock64();                       \
            _pa[i] += (unsigned long long)(_t - _pt);             \
            _pt = _t;                                             \
        }                                                         \
    } while (0)
#define RK_PROF_END()                                                              \
    do {                                                                           \
        if (threadIdx.x == 0) {                                                    \
            _pa[7] += 1;                                                           \
            for (int _i = 0; _i < 8; _i++)                                         \
                if (_pa[_i]) atomicAdd(&hgx_rk_prof[_i], _pa[_i]);                 \
        }                                                                          \
    } while (0)
void round_k_prof_dump() {
    unsigned long long h[8];
    if (hipMemcpyFromSymbol(h, HIP_SYMBOL(hgx_rk_prof), sizeof(h)) != hipSuccess) return;
    fprintf(stderr, "[hgx] k_round_k phases (clk sums): head %llu window %llu convert %llu search %llu boundary %llu "
            "outputs: S row %llu, candidate rows %llu | block-steps %llu\n", h[0], h[1], h[2], h[3], h[4], h[6], h[5],
            h[7]);
}
#else
#define RK_PROF_BEGIN() (void)0
#define RK_PROF(i) (void)0
#define RK_PROF_END() (void)0
void round_k_prof_dump() {}
#endif

constexpr int kWinP = 31;   // probes per window: K in [0, 31], 5 binary-search levels

// window row stride in dwords: even (8-byte reads) and == 2 mod 4, so that 32 lanes reading
// 32 different rows at the same column hit 32 distinct bank pairs (MI355X_MICROARCH.md, LDS)
__host__ __device__ constexpr int win_stride(int ndw) { return (ndw % 4 == 0) ? ndw + 2 : ndw + 4; }
__host__ __device__ constexpr int win_dwords(int ndw) { return kWinP * win_stride(ndw); }

// LDS-DMA instruction counts of one wave, fixed at compile time (every lane active, sources
// clamped into the valid range, destinations padded), so that explicit `s_waitcnt vmcnt(N)`
// can wait for the loads issued before a staging and leave the staging in flight
template <int NDW, int GW, int CSZ>
struct RkDma {
    static constexpr int WD = win_dwords(NDW);
    static constexpr int RAWD = kWinP * NDW * CSZ;                        // raw dwords at n = 4 * NDW
    static constexpr int KR16 = (RAWD + GW * 256 - 1) / (GW * 256);       // raw rows, 16 B per lane
    static constexpr int KR4 = (RAWD + GW * 64 - 1) / (GW * 64);          // raw rows, 4 B per lane
    static constexpr int CPI = (CSZ == 2) ? 4 : 2;                        // FD columns per instruction
    static constexpr int KF = (4 * NDW + GW * CPI - 1) / (GW * CPI);      // FD columns
    static constexpr int WIN_LDS = WD;                                    // dwords
    static constexpr int RAW_LDS = (KR16 * GW * 256 > KR4 * GW * 64) ? KR16 * GW * 256 : KR4 * GW * 64;
    static constexpr int FDC_LDS = KF * GW * 65;                          // groups of 64 + 1 pad dword
};

// FD8 layout: per (parity, graph) the n candidate rows as [NDW / GWD][n][GWD] dwords, so that
// the 64 lanes of a wave (64 candidates) load one GWD-dword group each from consecutive
// addresses (row-major rows put every lane of a load on its own cache line: 64 lines per
// instruction). GWD = 4 when a wave's share of a row (HD dwords) is whole 16-byte groups.
__host__ __device__ constexpr int fd8_gwd(int hd) { return (hd % 4 == 0) ? 4 : 2; }
__host__ __device__ inline size_t fd8_at(int par, int C, int n, int ndw, int gwd, int g, int j, int d) {
    return (size_t)par * C * ndw + ((size_t)g * ndw / gwd + d / gwd) * n * gwd + (size_t)j * gwd + d % gwd;
}

struct RoundKLds {
    int win, raw, fdc, base, bm1, hist, total;
};

// one chain group's LDS: rebased byte window | raw LA rows | FD columns (stg) | bases | histogram
template <int NDW, int GW, int CSZ>
__host__ __device__ inline RoundKLds round_k_lds(bool stg) {
    typedef RkDma<NDW, GW, CSZ> D;
    RoundKLds L{};
    int o = 0;
    L.win = o;
    o += D::WIN_LDS * 4;
    L.raw = o;
    if (stg) o += D::RAW_LDS * 4;
    L.fdc = o;
    if (stg) o += D::FDC_LDS * 4;
    L.base = o;
    o += 4 * NDW * 4;
    L.bm1 = o;
    o += 4 * NDW * 4;
    L.hist = o;
    o += 32 * 4;
    L.total = (o + 15) & ~15;
    return L;
}

// s_waitcnt vmcnt(N) for a compile-time N; N > 63 (the counter's range) waits for more
template <int N>
__device__ __forceinline__ void wait_vm() {
    asm volatile("s_waitcnt vmcnt(%0)" ::"i"(N < 63 ? N : 63) : "memory");
}
// workgroup barrier for LDS only: __syncthreads() would also wait for every outstanding
// global load, the staging DMA included
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// HD dwords of an LDS row as plain ds_read_b64 (2 cycles, 256 B/clk, 64-bank rule), all in
// flight before one wait. Left to itself the compiler fuses pairs into ds_read2_b64 (8 cycles,
// 128 B/clk, 32-bank rule: rows 16 apart conflict), which halves the search's LDS bandwidth
// (MI355X_MICROARCH.md, LDS table).
template <int HD>
__device__ __forceinline__ void lds_read_row(const uint32_t* p, uint32_t (&v)[HD]) {
    static_assert(HD % 2 == 0 && HD <= 64, "row width");
    const uint32_t a = (uint32_t)(uintptr_t)p;   // LDS byte address
    uint64_t r[HD / 2];
#define RK_RD(k) asm volatile("ds_read_b64 %0, %1 offset:%2" : "=v"(r[k]) : "v"(a), "i"(8 * (k)))
    RK_RD(0);
    if constexpr (HD >= 4) RK_RD(1);
    if constexpr (HD >= 8) { RK_RD(2); RK_RD(3); }
    if constexpr (HD >= 16) { RK_RD(4); RK_RD(5); RK_RD(6); RK_RD(7); }
    if constexpr (HD >= 32) { RK_RD(8); RK_RD(9); RK_RD(10); RK_RD(11); RK_RD(12); RK_RD(13); RK_RD(14); RK_RD(15); }
    if constexpr (HD >= 64) {
        RK_RD(16); RK_RD(17); RK_RD(18); RK_RD(19); RK_RD(20); RK_RD(21); RK_RD(22); RK_RD(23);
        RK_RD(24); RK_RD(25); RK_RD(26); RK_RD(27); RK_RD(28); RK_RD(29); RK_RD(30); RK_RD(31);
    }
#undef RK_RD
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
    for (int k = 0; k < HD / 2; k++) {
        asm volatile("" : "+v"(r[k]));   // the values exist only after the wait
        v[2 * k] = (uint32_t)r[k];
        v[2 * k + 1] = (uint32_t)(r[k] >> 32);
    }
}

// Loads the compiler does not see as loads: it would otherwise move the first use of a
// uniform value (a readfirstlane) right behind its load and wait there, serialising the head
// of the step. Their values exist only after ld_wait(), which waits for every load issued so
// far (the compiler's own waits only get stronger from the extra outstanding loads).
__device__ __forceinline__ int32_t ld_i32(const int32_t* p) {
    int32_t v;
    asm volatile("global_load_dword %0, %1, off" : "=v"(v) : "v"(p) : "memory");
    return v;
}
__device__ __forceinline__ uint4 ld_u32x4(const uint32_t* p) {
    uint4 v;
    asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(v) : "v"(p) : "memory");
    return v;
}
__device__ __forceinline__ uint2 ld_u32x2(const uint32_t* p) {
    uint2 v;
    asm volatile("global_load_dwordx2 %0, %1, off" : "=v"(v) : "v"(p) : "memory");
    return v;
}
__device__ __forceinline__ uint32_t ld_u8(const uint8_t* p) {
    uint32_t v;
    asm volatile("global_load_ubyte %0, %1, off" : "=v"(v) : "v"(p) : "memory");
    return v;
}

// CG waves of 64 candidates each; every candidate's row is split over H waves (coordinate
// dwords [h*NDW/H, (h+1)*NDW/H)), whose partial counts meet in LDS once per search level, so
// that two waves share each SIMD; GPB chain groups per block when a group is one wave.
template <typename CT, int NDW, int CG, int H, int GPB, bool STG, int NCH>
__global__ void __launch_bounds__(64 * CG * H * GPB) k_round_k(RoundArgs A, int s) {
    constexpr int P = kWinP;
    constexpr int GW = CG * H;           // waves of one chain group
    constexpr int GL = 64 * GW;          // threads of one chain group
    constexpr int HD = NDW / H;          // candidate-row dwords per wave
    constexpr int WS = win_stride(NDW);
    constexpr int FDW = P / 2 + 1;       // dwords per compact FD column (32 positions from an even start)
    constexpr int CW = (sizeof(CT) == 2) ? FDW : 32;   // dwords per staged FD column
    constexpr int CPI = 64 / CW;                        // FD columns per LDS-DMA wave instruction
    typedef RkDma<NDW, GW, sizeof(CT) == 2 ? 2 : 4> D;
    static_assert(D::CPI == CPI, "FD column groups");
    // vector-memory instructions a wave issues between the boundary load and the staging
    constexpr int GWD = fd8_gwd(HD);
    constexpr int NFD8 = HD / GWD;
    constexpr int BPT = (4 * NDW + GL - 1) / GL;   // base coordinates per thread (n <= 4 NDW)
    constexpr int NSMALL = 2 + 3 * BPT;   // after the candidate rows: root floor, ovf, bases
    static_assert(GPB == 1 || GW == 1, "several chain groups per block only with one-wave groups");
    static_assert(NDW % (2 * H) == 0, "row split");
    static_assert(NCH == 1 || (GPB == 1 && NCH <= 12), "candidate chunks: one chain group per block");
    typedef __attribute__((address_space(3))) void* lds_ptr_t;
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    __shared__ int s_B[GPB], s_tot[GPB];
    __shared__ int pc[(H > 1) ? 2 * H * 64 * CG : 1];   // partial counts by level parity

    const int n = A.n, C = A.C, sm = A.sm;
    const int lane = lane_id(), wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int grp = wave / GW, wh = wave % GW, h = wh / CG, cw = wh % CG;
    const int gt = wh * 64 + lane;       // thread within the chain group
    const int gc = blockIdx.x * GPB + grp;
    if (gc >= C) return;   // group-uniform; block barriers are only used when GPB == 1
    RK_PROF_BEGIN();
    const RoundKLds L = round_k_lds<NDW, GW, sizeof(CT) == 2 ? 2 : 4>(STG);
    uint8_t* gl = lds + (size_t)grp * L.total;
    uint32_t* win = (uint32_t*)(gl + L.win);
    CT* raw = (CT*)(gl + L.raw);
    CT* fdc = (CT*)(gl + L.fdc);
    int32_t* base = (int32_t*)(gl + L.base);
    int32_t* bm1 = (int32_t*)(gl + L.bm1);
    int32_t* hist = (int32_t*)(gl + L.hist);
    auto gsync = [&]() {   // LDS only: every wait for global loads is explicit
        if constexpr (GW == 1) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        else lds_barrier();
    };

    const int g = gc / n, cl = gc % n;
    const int par = s & 1;
    const size_t wrow = (size_t)s * C + (size_t)g * n;
    // Every load of the step is issued before any is waited on, and none sits behind a branch:
    // the boundary, the chain's extent and the forwarded window's tag first, then this lane's
    // part of its candidate's rebased row (written by the step that found the candidate), the
    // window the previous step forwarded (both at fixed addresses), the flags and the bases.
    int b = ld_i32(A.Bm + (size_t)s * C + gc);
    int len = ld_i32(A.c_len + gc), off = ld_i32(A.c_off + gc);
    // candidates come in NCH chunks of 64 * CG (one chunk unless n > 256): lane (cw, lane) holds
    // candidate ch * 64 * CG + jl of chunk ch, coordinate dwords [h * HD, (h + 1) * HD) of its row
    const int jl = cw * 64 + lane;
    auto load_chunk = [&](int ch, uint32_t (&dst)[HD], uint32_t& wf) {
        const int jc = ch * 64 * CG + jl;
        const int jcc = jc < n ? jc : 0;
        const uint32_t* __restrict__ row = A.FD8 + fd8_at(par, C, n, NDW, GWD, g, jcc, h * HD);
        if constexpr (GWD == 4) {
#pragma unroll
            for (int d = 0; d < HD; d += 4) {
                const uint4 v = ld_u32x4(row + (size_t)(d / 4) * n * 4);
                dst[d] = v.x; dst[d + 1] = v.y; dst[d + 2] = v.z; dst[d + 3] = v.w;
            }
        } else {
#pragma unroll
            for (int d = 0; d < HD; d += 2) {
                const uint2 v = ld_u32x2(row + (size_t)(d / 2) * n * 2);
                dst[d] = v.x; dst[d + 1] = v.y;
            }
        }
        wf = ld_u8(A.wflag + wrow + jcc);
    };
    uint32_t fd[HD], wfl;
    load_chunk(0, fd, wfl);
    // root floor (after hgx_reset): offsets >= gk have round >= s+1 whatever they strongly see
    // (gB is a valid array without roots too: an unconditional load)
    const bool rootr = s + 1 <= A.gmax;
    int gkv = ld_i32(A.gB + (rootr ? (size_t)(s + 1) * C + gc : 0));
    int ovf_s = ld_i32(A.ovf + s);
    int cbv[BPT], bmp[BPT], bmc[BPT];
    const size_t prow = s > 0 ? wrow - C : wrow;
#pragma unroll
    for (int u = 0; u < BPT; u++) {
        const int i = gt + u * GL;
        const int ii = i < n ? i : 0;
        cbv[u] = ld_i32(A.c_base + g * n + ii);
        bmp[u] = ld_i32(A.Bm + prow + ii);
        bmc[u] = ld_i32(A.Bm + wrow + ii);
    }
    wait_vm<NFD8 + 1 + NSMALL>();   // the boundary and the chain's extent have landed
    asm volatile("" : "+v"(b), "+v"(len), "+v"(off));
    b = __builtin_amdgcn_readfirstlane(b);
    len = __builtin_amdgcn_readfirstlane(len);
    off = __builtin_amdgcn_readfirstlane(off);
    if (b >= len) {
        __builtin_amdgcn_s_waitcnt(0);   // no LDS-DMA outlives the block
        if (gt == 0) {
            A.wstat[(size_t)s * C + gc] = 0;
            A.wflag[(size_t)(s + 1) * C + gc] = 0;
            A.Bm[(size_t)(s + 1) * C + gc] = len;
        }
        return;
    }

    // staging: raw LA rows [kbase, kbase + min(2P, len - kbase)) (contiguous; the window and
    // the next step's) and the window's FD columns (the new candidate's FD row comes from
    // there), by LDS-DMA with a fixed instruction count per wave; then wait for everything
    // issued before it, leaving the staging in flight
    int fsh = 0;
    auto stage_and_wait_rest = [&](int kbase, int np) {
        if constexpr (STG) {
            const int nraw = min(kWinP, len - kbase);
            const int nel = (int)((size_t)nraw * n * sizeof(CT) / 4);
            const uint32_t* __restrict__ src = (const uint32_t*)A.LA + (size_t)(off + kbase) * n * sizeof(CT) / 4;
            uint32_t* raw_w = (uint32_t*)raw;
            // FD columns: one wave instruction stages CPI columns of CW dwords each (positions
            // [kbase, kbase+np) for int32; the 2*FDW positions from the even start below kbase for
            // uint16) into a 64-dword group; groups are 65 dwords apart (bank spread)
            uint32_t* fd_w = (uint32_t*)fdc;
            const int pcol = lane % CW, icol = lane / CW;
            const uint32_t* __restrict__ fsrc;
            size_t cstride;
            if constexpr (sizeof(CT) == 4) {
                fsrc = (const uint32_t*)A.FDT + off + kbase + min(pcol, np - 1);
                cstride = (size_t)A.Pcap;
            } else {
                const int64_t p0 = (off + kbase) & ~1;
                fsh = (off + kbase) & 1;
                fsrc = (const uint32_t*)((const CT*)A.FDT + p0) + pcol;
                cstride = (size_t)(A.Pcap / 2);
            }
            auto fd_cols = [&]() {
#pragma unroll
                for (int k = 0; k < D::KF; k++) {
                    const int i0 = wh * CPI + k * GW * CPI;
                    const int i = min(i0 + icol, n - 1);
                    __builtin_amdgcn_global_load_lds((const void*)(fsrc + (size_t)i * cstride),
                                                     (lds_ptr_t)(fd_w + (size_t)(i0 / CPI) * 65), 4, 0, 0);
                }
            };
            if (((n * (int)sizeof(CT)) & 15) == 0) {
#pragma unroll
                for (int k = 0; k < D::KR16; k++) {
                    const int c0 = wh * 256 + k * GW * 256;
                    __builtin_amdgcn_global_load_lds((const void*)(src + min(c0 + lane * 4, nel - 4)),
                                                     (lds_ptr_t)(raw_w + c0), 16, 0, 0);
                }
                fd_cols();
                wait_vm<D::KR16 + D::KF>();
            } else {
#pragma unroll
                for (int k = 0; k < D::KR4; k++) {
                    const int c0 = wh * 64 + k * GW * 64;
                    __builtin_amdgcn_global_load_lds((const void*)(src + min(c0 + lane, nel - 1)),
                                                     (lds_ptr_t)(raw_w + c0), 4, 0, 0);
                }
                fd_cols();
                wait_vm<D::KR4 + D::KF>();
            }
        } else {
            __builtin_amdgcn_s_waitcnt(0);
        }
    };
    auto la_at = [&](int kbase, int p, int i) -> int32_t {   // decoded lastAncestors of staged row p
        if constexpr (STG) return Coord<CT>::la(raw[p * n + i]);
        else return Coord<CT>::la(((const CT*)A.LA)[(size_t)(off + kbase + p) * n + i]);
    };
    // rebased byte rows: (0x80 | LA') per coordinate against bases bs[], padding coordinates
    // LA' = 0, for staged rows [p0, p0 + np); a thread keeps one dword column d (4 coordinates,
    // their bases in registers) over the rows and hands each word to put(p, d, word)
    typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
    auto rebase_rows = [&](int kbase, int p0, int np, const int32_t* bs, auto&& put) {
        constexpr int RS = (GL >= NDW) ? GL / NDW : 1;   // rows per pass
        constexpr int NP = (P + RS - 1) / RS;              // passes (fixed trip count)
        for (int d = gt % NDW; d < NDW; d += GL) {
            const int i0 = 4 * d;
            if constexpr (sizeof(CT) == 2) {
                // packed: LA' = min(sat(raw - base), 126) on coordinate pairs (raw = LA + 1); the raw
                // rows from LDS (staged) or straight from HBM (big n: the rows do not fit in LDS)
                u16x2 b01 = {0, 0}, b23 = {0, 0};
                if (i0 < n) b01 = u16x2{(unsigned short)bs[i0], (unsigned short)bs[i0 + 1]};
                if (i0 + 2 < n) b23 = u16x2{(unsigned short)bs[i0 + 2], (unsigned short)bs[i0 + 3]};
                const u16x2 cap = {126, 126};
                uint32_t g01[STG ? 1 : NP], g23[STG ? 1 : NP];
                if constexpr (!STG) {   // every pass's HBM loads in flight before the first is used
                    const int ic = i0 < n ? i0 : 0;
#pragma unroll
                    for (int u = 0; u < NP; u++) {
                        const int p = min(gt / NDW + u * RS, np - 1);   // (n even: dword-aligned pairs)
                        const uint32_t* rp =
                            (const uint32_t*)((const CT*)A.LA + (size_t)(off + kbase + p0 + p) * n + ic);
                        g01[u] = rp[0];
                        g23[u] = rp[i0 + 2 < n ? 1 : 0];
                    }
                }
#pragma unroll
                for (int u = 0; u < NP; u++) {
                    const int p = gt / NDW + u * RS;
                    if (p < np) {
                        uint32_t r01 = 0u, r23 = 0u;
                        if constexpr (STG) {
                            const uint32_t* rp = (const uint32_t*)(raw + (p0 + p) * n + i0);
                            r01 = i0 < n ? rp[0] : 0u;
                            r23 = i0 + 2 < n ? rp[1] : 0u;
                        } else if (i0 < n) {
                            r01 = g01[u];
                            r23 = i0 + 2 < n ? g23[u] : 0u;
                        }
                        const u16x2 y01 = __builtin_elementwise_min(
                            __builtin_elementwise_sub_sat(__builtin_bit_cast(u16x2, r01), b01), cap);
                        const u16x2 y23 = __builtin_elementwise_min(
                            __builtin_elementwise_sub_sat(__builtin_bit_cast(u16x2, r23), b23), cap);
                        const uint32_t w = __builtin_amdgcn_perm(__builtin_bit_cast(uint32_t, y23),
                                                                 __builtin_bit_cast(uint32_t, y01), 0x06040200u);
                        put(p, d, w | 0x80808080u);
                    }
                }
            } else {
                int32_t bq[4];
#pragma unroll
                for (int q = 0; q < 4; q++) bq[q] = (i0 + q < n) ? bs[i0 + q] : 0;
                for (int p = gt / NDW; p < np; p += RS) {
                    uint32_t w = 0x80808080u;
#pragma unroll
                    for (int q = 0; q < 4; q++) {
                        const int i = i0 + q;
                        if (i < n) {
                            const int32_t x = la_at(kbase, p0 + p, i) - bq[q] + 1;
                            w |= (uint32_t)min(max(x, 0), 126) << (8 * q);
                        }
                    }
                    put(p, d, w);
                }
            }
        }
    };
    // total count over the H waves of this candidate (partial counts meet in LDS)
    auto combine = [&](uint32_t part, int it) -> uint32_t {
        if constexpr (H == 1) {
            return part;
        } else {
            int* pcb = pc + (it & 1) * (H * 64 * CG);
            pcb[h * 64 * CG + jl] = (int)part;
            gsync();
            uint32_t t = 0;
#pragma unroll
            for (int q = 0; q < H; q++) t += (uint32_t)pcb[q * 64 * CG + jl];
            return t;
        }
    };

    int kbase = b, np = min(P, len - b);
    stage_and_wait_rest(kbase, np);   // everything before the staging has landed
    asm volatile("" : "+v"(gkv), "+v"(wfl), "+v"(ovf_s));
#pragma unroll
    for (int d = 0; d < HD; d++) asm volatile("" : "+v"(fd[d]));
#pragma unroll
    for (int u = 0; u < BPT; u++) asm volatile("" : "+v"(cbv[u]), "+v"(bmp[u]), "+v"(bmc[u]));
    const int gk = rootr ? gkv : len;
    const bool exact = ovf_s != 0;   // a candidate row of this round did not fit 8 bits
#pragma unroll
    for (int u = 0; u < BPT; u++) {
        const int i = gt + u * GL;
        if (i < n) {
            base[i] = cbv[u] + (s > 0 ? bmp[u] : 0);   // base(s): Index of round s-1's candidate on chain i
            bm1[i] = cbv[u] + bmc[u];                  // base(s+1)
        }
    }
    if (gt < 32) hist[gt] = 0;
    RK_PROF(0);

    int kstar = len, carried = 0, B = -1;
    // per chunk (bit / 5-bit field ch): the lane's candidate exists, was seen in an earlier
    // window (seen at every later probe), and its first seeing probe K in the current window
    uint32_t cand_bits = 0, done_bits = 0;
    uint64_t k_bits = 0;
    uint32_t fdn[NCH > 1 ? HD : 1], wfln = 0;   // the next chunk's rows, in flight during a search
    for (int w_it = 0;; w_it++) {
        if (w_it > 0) stage_and_wait_rest(kbase, np);   // a later window (rare)
        __builtin_amdgcn_s_waitcnt(0);
        gsync();
        RK_PROF(1);
        rebase_rows(kbase, 0, np, base, [&](int p, int d, uint32_t w) { win[p * WS + d] = w; });
        gsync();
        RK_PROF(2);
#pragma unroll 1
        for (int ch = 0; ch < NCH; ch++) {
            if (ch * 64 * CG >= n) break;   // (block-uniform) no candidate in this chunk
            if constexpr (NCH > 1) {
                if (ch > 0 || w_it > 0) {
                    if (ch == 0) load_chunk(0, fdn, wfln);   // a later window: the first chunk again
                    __builtin_amdgcn_s_waitcnt(0);
#pragma unroll
                    for (int d = 0; d < HD; d++) {
                        asm volatile("" : "+v"(fdn[d]));
                        fd[d] = fdn[d];
                    }
                    asm volatile("" : "+v"(wfln));
                    wfl = wfln;
                }
                if (ch + 1 < NCH) load_chunk(ch + 1, fdn, wfln);
            }
            const int jc = ch * 64 * CG + jl;
            const bool cand = jc < n && wfl == 1;
            if (cand) cand_bits |= 1u << ch;
            const bool done = (done_bits >> ch) & 1u;
            // first probe of the window that strongly sees this lane's candidate (np: none);
            // probes past the window's end count as seeing (keeps the predicate monotone)
            int lo = 0, hi = P;
            // a wave whose 64 candidates are all absent (silent chains) only keeps the barriers
            const bool wave_cand = __ballot(cand) != 0;
            if (!exact) {
#pragma unroll
                for (int d = 0; d < HD; d++) fd[d] = cand ? fd[d] : 0x7F7F7F7Fu;   // never seen
#pragma unroll
                for (int it = 0; it < 5; it++) {
                    const int mid = (lo + hi) >> 1;
                    const uint32_t* row = win + mid * WS + h * HD;
                    uint32_t c4[4] = {0, 0, 0, 0};
                    if (wave_cand) {
                    // big n (several chunks, the next chunk's rows in flight): the row in two halves,
                    // fewer live registers (one block of 16 waves per CU)
                    constexpr int RH = (NCH > 1 && HD >= 32) ? HD / 2 : HD;
#pragma unroll
                    for (int r0 = 0; r0 < HD; r0 += RH) {
                        uint32_t v[RH];
                        lds_read_row<RH>(row + r0, v);
#pragma unroll
                        for (int d = 0; d < RH; d++) c4[d & 3] += __builtin_popcount((v[d] - fd[r0 + d]) & 0x80808080u);
                    }
                    }
                    uint32_t cnt = (c4[0] + c4[1]) + (c4[2] + c4[3]);
                    cnt = combine(cnt, it);
                    const bool seen = done || mid >= np || ((int)cnt >= sm && !(jc == cl && kbase + mid == b));
                    if (seen) hi = mid; else lo = mid + 1;
                }
            } else {
                // exact int32 compares against the raw candidate row (rounds flagged by the producer)
                const int i_lo = h * HD * 4, i_hi = min(n, (h + 1) * HD * 4);
                const size_t jrow = (wrow + (jc < n ? jc : 0)) * n;
                for (int it = 0; it < 5; it++) {
                    const int mid = (lo + hi) >> 1;
                    uint32_t cnt = 0;
                    if (cand && !done && mid < np) {
                        for (int i = i_lo; i < i_hi; i++) {
                            const int32_t fdv = (sizeof(CT) == 2) ? Coord<uint16_t>::fd(((const uint16_t*)A.WFD)[jrow + i])
                                                                  : A.WFD[jrow + i];
                            const int32_t lav = min(la_at(kbase, mid, i), kMaxI32 - 1);
                            cnt += lav >= fdv ? 1u : 0u;
                        }
                    }
                    cnt = combine(cnt, it);
                    const bool seen = done || mid >= np || (cand && (int)cnt >= sm && !(jc == cl && kbase + mid == b));
                    if (seen) hi = mid; else lo = mid + 1;
                }
            }
            const int K = lo;
            k_bits = (k_bits & ~(31ull << (5 * ch))) | ((uint64_t)K << (5 * ch));
            // earlier windows' candidates are in `carried`
            if (h == 0 && K < np && cand && !done) atomicAdd(&hist[K], 1);
        }
        RK_PROF(3);
        gsync();
        if (wh == 0) {   // boundary: first probe where #{K <= p} (+ candidates seen earlier) >= SM
            const uint32_t v = lane < np ? (uint32_t)hist[lane] : 0u;
            const uint32_t inc = wave_scan_add_u32(v) + (uint32_t)carried;
            const uint64_t m = __ballot(lane < np && ((int)inc >= sm || kbase + lane >= gk));
            const int tot = __builtin_amdgcn_readlane((int)inc, 63);
            if (lane == 0) {
                s_B[grp] = m ? (int)__builtin_ctzll(m) : -1;
                s_tot[grp] = tot;
            }
        }
        gsync();
        B = s_B[grp];
        RK_PROF(4);
        if (B >= 0) {
            kstar = kbase + B;
            break;
        }
        carried = s_tot[grp];
#pragma unroll
        for (int ch = 0; ch < NCH; ch++)
            if (((cand_bits >> ch) & 1u) && (int)((k_bits >> (5 * ch)) & 31u) < np) done_bits |= 1u << ch;
        if (gt < 32) hist[gt] = 0;
        kbase += np;
        if (kbase >= len) {
            kstar = len;
            break;
        }
        np = min(P, len - kbase);
        gsync();
    }

    // outputs of round s for this chain
    for (int k = b + gt; k < kstar; k += GL) A.p_round[off + k] = s;
    if (gt == 0) {
        A.wstat[(size_t)s * C + gc] = (kstar > b) ? 2 : 1;
        if (kstar < len) {   // same value from every writer: plain stores
            A.active[s] = 1;
            if (A.hflag) *A.hflag = s + 1;   // last step of a batch: the host's flag (mapped memory)
        }
        A.Bm[(size_t)(s + 1) * C + gc] = kstar;
    }
    if (kstar < len) {
        const int pk = kstar - kbase;   // inside the staged window
        // S row of the boundary event: the candidates it strongly sees (bit j of word j/64)
        const size_t srow = ((size_t)(s + 1) * C + gc) * A.nw;
#pragma unroll
        for (int ch = 0; ch < NCH; ch++) {   // (seen in an earlier window: seen at B)
            const bool sb = ((cand_bits >> ch) & 1u) &&
                            (((done_bits >> ch) & 1u) || (int)((k_bits >> (5 * ch)) & 31u) <= B);
            const uint64_t bits = __ballot(sb);
            const int wd = ch * CG + cw;
            if (h == 0 && lane == 0 && wd < A.nw) A.Smat[srow + wd] = bits;
        }
        RK_PROF(6);
        // the new candidate's rows for round s+1
        const size_t nrow = ((size_t)(s + 1) * C + gc) * n;
        auto fd_raw = [&](int i) -> CT {
            if constexpr (STG) {
                const int col = (i / CPI) * 65 + (i % CPI) * CW;   // dword offset of column i
                if constexpr (sizeof(CT) == 2) return fdc[2 * col + fsh + pk];
                else return fdc[col + pk];
            } else {
                return ((const CT*)A.FDT)[(size_t)i * A.Pcap + off + kstar];
            }
        };
        int32_t* fdrow = (int32_t*)win;   // not staged: the row's gathered values, read twice below
        for (int i = gt; i < n; i += GL) {
            A.WLA[nrow + i] = la_at(kbase, pk, i);
            const CT f = fd_raw(i);
            if constexpr (!STG) fdrow[i] = (int32_t)f;
            if constexpr (sizeof(CT) == 2) ((uint16_t*)A.WFD)[nrow + i] = f;
            else A.WFD[nrow + i] = f;
        }
        if constexpr (!STG) gsync();
        // rebased FD row (base(s+1) = Index of this round's candidates) for the next step
        uint32_t* nfd = A.FD8;
        bool of = false;
        for (int d = gt; d < NDW; d += GL) {
            uint32_t w = 0;
#pragma unroll
            for (int q = 0; q < 4; q++) {
                const int i = 4 * d + q;
                uint32_t v = 127u;
                if (i < n) {
                    const int32_t f = Coord<CT>::fd(STG ? fd_raw(i) : (CT)fdrow[i]);
                    if (f != kMaxI32) {
                        const int32_t x = f - bm1[i] + 1;
                        if (x > 126) of = true;
                        else v = (uint32_t)x;
                    }
                }
                w |= v << (8 * q);
            }
            nfd[fd8_at(par ^ 1, C, n, NDW, GWD, g, cl, d)] = w;
        }
        if (of) A.ovf[s + 1] = 1;   // same value from every writer
        if (gt == 0) A.wflag[(size_t)(s + 1) * C + gc] = 1;
    } else if (gt == 0) {
        A.wflag[(size_t)(s + 1) * C + gc] = 0;
    }
    RK_PROF(5);
    RK_PROF_END();
}

// round r's candidate rows (round 0: the first event of every chain; r > 0: the restart
// round of an incremental DivideRounds), rebased to base(r) = c_base + Bm[r-1], from the
// row-major WFD rows k_round_gather has just written (raw uint16 or int32 FD)
template <typename CT>
__global__ void k_round_k_gather(RoundArgs A, int ndw, int gwd, int r) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= (int64_t)A.C * ndw) return;
    const int gc = (int)(t / ndw), d = (int)(t % ndw);
    const int n = A.n, C = A.C, g = gc / n;
    uint32_t w = 0;
    bool of = false;
    const bool have = A.wflag[(size_t)r * C + gc] != 0;
    const CT* __restrict__ row = (const CT*)A.WFD + ((size_t)r * C + gc) * n;
    for (int q = 0; q < 4; q++) {
        const int i = 4 * d + q;
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
        w |= v << (8 * q);
    }
    A.FD8[fd8_at(r & 1, C, n, ndw, gwd, g, gc % n, d)] = w;
    if (of) A.ovf[r] = 1;
}

int round_k_ndw(int n) {
    int d = (n + 3) / 4;
    int p = 2;
    while (p < d) p *= 2;
    return p;
}

template <typename CT, int NDW, int CG, int H, int GPB, bool STG, int NCH>
static hipError_t round_k_launch_v(hipStream_t st, const RoundArgs& A, int s) {
    const void* f = (const void*)k_round_k<CT, NDW, CG, H, GPB, STG, NCH>;
    const RoundKLds L = round_k_lds<NDW, CG * H, sizeof(CT) == 2 ? 2 : 4>(STG);
    const size_t lds = (size_t)L.total * GPB;
    {
        const hipError_t e = ensure_lds_limit(f, lds);
        if (e != hipSuccess) return e;
    }
    const unsigned grid = (unsigned)((A.C + GPB - 1) / GPB);
    hipLaunchKernelGGL((k_round_k<CT, NDW, CG, H, GPB, STG, NCH>), dim3(grid), dim3(64 * CG * H * GPB), lds, st, A, s);
    return hipGetLastError();
}

template <typename CT, int NDW, int CG, int H, int GPB, int NCH = 1>
static hipError_t round_k_launch(hipStream_t st, const RoundArgs& A, int s) {
    const RoundKLds L = round_k_lds<NDW, CG * H, sizeof(CT) == 2 ? 2 : 4>(true);
    if ((size_t)L.total * GPB <= 140 * 1024) return round_k_launch_v<CT, NDW, CG, H, GPB, true, NCH>(st, A, s);
    return round_k_launch_v<CT, NDW, CG, H, GPB, false, NCH>(st, A, s);
}

// a wave's share of a candidate row (dwords) in the configuration launch_round_k_t picks
static int round_k_hd(int n, int C) {
    const bool many = C >= 1024;
    switch (round_k_ndw(n)) {
        case 2: return 2;
        case 4: return many ? 4 : 2;
        case 8: return many ? 8 : 2;
        case 16: return many ? 16 : 2;
        case 32: return 8;
        case 64: return 32;
        case 128: return 32;
        case 256: return 32;
        default: return 2;
    }
}

// one wave per chain, four chains per block, when chains are many (batched simulations);
// otherwise one chain per block with its rows split over 8 waves (two per SIMD)
template <typename CT>
static hipError_t launch_round_k_t(hipStream_t st, const RoundArgs& A, int s) {
    const bool many = A.C >= 1024;
    switch (round_k_ndw(A.n)) {
        case 2: return many ? round_k_launch<CT, 2, 1, 1, 4>(st, A, s) : round_k_launch<CT, 2, 1, 1, 1>(st, A, s);
        case 4: return many ? round_k_launch<CT, 4, 1, 1, 4>(st, A, s) : round_k_launch<CT, 4, 1, 2, 1>(st, A, s);
        case 8: return many ? round_k_launch<CT, 8, 1, 1, 4>(st, A, s) : round_k_launch<CT, 8, 1, 4, 1>(st, A, s);
        case 16: return many ? round_k_launch<CT, 16, 1, 1, 4>(st, A, s) : round_k_launch<CT, 16, 1, 8, 1>(st, A, s);
        case 32: return round_k_launch<CT, 32, 2, 4, 1>(st, A, s);
        case 64: return round_k_launch<CT, 64, 4, 2, 1>(st, A, s);
        // n > 256: the candidates in chunks of 128 (4 / 8 chunks), rows split over 4 / 8 waves
        case 128: return round_k_launch<CT, 128, 2, 4, 1, 4>(st, A, s);
        case 256: return round_k_launch<CT, 256, 2, 8, 1, 8>(st, A, s);
        default: return hipErrorInvalidValue;
    }
}

hipError_t launch_round_k(hipStream_t st, const RoundArgs& A, int s) {
    return A.compact ? launch_round_k_t<uint16_t>(st, A, s) : launch_round_k_t<int32_t>(st, A, s);
}

void launch_round_k_gather(hipStream_t st, const RoundArgs& A, int r) {
    const int ndw = round_k_ndw(A.n);
    const int gwd = fd8_gwd(round_k_hd(A.n, A.C));
    const int64_t work = (int64_t)A.C * ndw;
    if (work <= 0) return;
    if (A.compact)
        hipLaunchKernelGGL(k_round_k_gather<uint16_t>, dim3((unsigned)((work + 255) / 256)), dim3(256), 0, st, A, ndw, gwd, r);
    else
        hipLaunchKernelGGL(k_round_k_gather<int32_t>, dim3((unsigned)((work + 255) / 256)), dim3(256), 0, st, A, ndw, gwd, r);
}

}  // namespace hgx
