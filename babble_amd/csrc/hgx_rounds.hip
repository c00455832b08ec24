// Round assignment for n <= 256: one launch per round, kStepBatch launches replayed
// as one hipGraph. Rounds are a sequential recurrence (round r+1's
// candidates are the boundaries found in round r); a dependent kernel boundary costs
// ~1.5 us on MI355X, less than an in-launch grid barrier (MI355X_MICROARCH.md price
// list; a persistent variant measured 53 us/round against 34 for launches), so the
// step is a plain launch and the work is in making its body short.
//
// Round r, chain c, candidates W'_r = first event of every chain with round >= r.
// The chain's boundary Bm[r+1][c] is the first offset k >= Bm[r][c] whose event
// strongly sees >= SM candidates (RoundInc, hashgraph.go:285-305; StronglySee
// hashgraph.go:170-198). The count is monotone in k (lastAncestors only grow along a
// chain), so a group of waves binary-searches k over a window of P probe rows staged
// in LDS: each level tests ONE probe row against all candidates (each wave holds its
// candidates' firstDescendants rows in registers; lane = coordinate, v_cmp -> 64-bit
// ballot -> s_bcnt1), so the tests of a level are independent (ILP), and the group
// sums the per-wave counts. The window's firstDescendants columns (FDT[i][p..p+P),
// one 128-B line per coordinate) are staged beside it, so the new candidate's FD row
// needs no dependent gather. The boundary event's bitmask of strongly-seen candidates
// is DecideFame's S_{r+1} row (hashgraph.go:688-705) for free.
//
// Group = 16 waves (one chain per block) for 64 < n <= 256; one wave per chain for
// n <= 64 (4 chains per 256-thread block); n > 256: k_round_step_big.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <type_traits>
#include <utility>

#include "hgx_device.h"
#include "hgx_kernels.h"

namespace hgx {

// Optional phase timing (build with -DHGX_STEP_PROF, variant "prof"): thread 0 of
// every block adds s_memtime deltas per phase into hgx_step_prof[8].
#ifdef HGX_STEP_PROF
__device__ unsigned long long hgx_step_prof[8];
// deltas accumulate in thread 0's registers and are added to the global counters once,
// at HGX_PROF_END (atomics inside the step would be waited for at every barrier)
#define HGX_PROF_BEGIN() long long _pt = clock64(); unsigned long long _pa[8] = {0, 0, 0, 0, 0, 0, 0, 0}
#define HGX_PROF(i)                            \
    do {                                       \
        if (threadIdx.x == 0) {                \
            const long long _t = clock64();    \
            _pa[i] += (unsigned long long)(_t - _pt); \
            _pt = _t;                          \
        }                                      \
    } while (0)
#define HGX_PROF_COUNT(i) do { if (threadIdx.x == 0) _pa[i] += 1ull; } while (0)
#define HGX_PROF_END()                                                            \
    do {                                                                          \
        if (threadIdx.x == 0)                                                     \
            for (int _i = 0; _i < 8; _i++)                                        \
                if (_pa[_i]) atomicAdd(&hgx_step_prof[_i], _pa[_i]);              \
    } while (0)
#else
#define HGX_PROF_BEGIN() (void)0
#define HGX_PROF(i) (void)0
#define HGX_PROF_COUNT(i) (void)0
#define HGX_PROF_END() (void)0
#endif

// total of candidate O goes to lane O of tv (v_writelane with an immediate lane: a
// select on lane == O would make the compiler hoist OWN 64-bit lane masks and spill them)
// Candidates whose bit is clear in `test` are skipped (wave-uniform branch).
// The CPL compares of one candidate go to distinct SGPR pairs in one asm block, so they
// issue back to back; left to itself the compiler (at this SGPR pressure) funnels every
// compare through one pair and each v_cmp -> s_bcnt1 round trip serialises the tally.
template <int CPL>
__device__ __forceinline__ int count_seen(const int32_t (&la)[CPL], const int32_t (&fd)[CPL]) {
    if constexpr (CPL == 4) {
        uint64_t m0, m1, m2, m3;
        asm volatile(
            "v_cmp_ge_i32_e64 %0, %4, %8\n\t"
            "v_cmp_ge_i32_e64 %1, %5, %9\n\t"
            "v_cmp_ge_i32_e64 %2, %6, %10\n\t"
            "v_cmp_ge_i32_e64 %3, %7, %11"
            : "=s"(m0), "=s"(m1), "=s"(m2), "=s"(m3)
            : "v"(la[0]), "v"(la[1]), "v"(la[2]), "v"(la[3]), "v"(fd[0]), "v"(fd[1]), "v"(fd[2]), "v"(fd[3]));
        return (__popcll(m0) + __popcll(m1)) + (__popcll(m2) + __popcll(m3));
    } else if constexpr (CPL == 2) {
        uint64_t m0, m1;
        asm volatile(
            "v_cmp_ge_i32_e64 %0, %2, %4\n\t"
            "v_cmp_ge_i32_e64 %1, %3, %5"
            : "=s"(m0), "=s"(m1)
            : "v"(la[0]), "v"(la[1]), "v"(fd[0]), "v"(fd[1]));
        return __popcll(m0) + __popcll(m1);
    } else {
        int tot = 0;
#pragma unroll
        for (int q = 0; q < CPL; q++) tot += __popcll(__ballot(la[q] >= fd[q]));
        return tot;
    }
}

// Candidates whose bit is clear in `test` are skipped (wave-uniform branch; a 32-bit mask
// when OWN <= 32, so the skip is one scalar bit test). The popcount of
// each of the CPL compare masks goes to lane O of its own partial register tv[q] and the
// partials are added once per probe in VALU, instead of CPL - 1 scalar adds per candidate
// (the tally is scalar-issue-bound: 4 s_bcnt1 + 3 s_add + skip test per candidate).
template <int OWN>
using TallyMask = typename std::conditional<(OWN <= 32), uint32_t, uint64_t>::type;
template <int O, int CPL, int OWN>
__device__ __forceinline__ void tally_one(const int32_t (&la)[CPL], const int32_t (&fd)[OWN][CPL], int (&tv)[CPL],
                                          TallyMask<OWN> test) {
    if ((test >> O) & 1u) {
        if constexpr (CPL == 4) {
            uint64_t m0, m1, m2, m3;
            asm volatile(
                "v_cmp_ge_i32_e64 %0, %4, %8\n\t"
                "v_cmp_ge_i32_e64 %1, %5, %9\n\t"
                "v_cmp_ge_i32_e64 %2, %6, %10\n\t"
                "v_cmp_ge_i32_e64 %3, %7, %11"
                : "=s"(m0), "=s"(m1), "=s"(m2), "=s"(m3)
                : "v"(la[0]), "v"(la[1]), "v"(la[2]), "v"(la[3]), "v"(fd[O][0]), "v"(fd[O][1]), "v"(fd[O][2]),
                  "v"(fd[O][3]));
            asm volatile("v_writelane_b32 %0, %1, %2" : "+v"(tv[0]) : "s"(__popcll(m0)), "i"(O));
            asm volatile("v_writelane_b32 %0, %1, %2" : "+v"(tv[1]) : "s"(__popcll(m1)), "i"(O));
            asm volatile("v_writelane_b32 %0, %1, %2" : "+v"(tv[2]) : "s"(__popcll(m2)), "i"(O));
            asm volatile("v_writelane_b32 %0, %1, %2" : "+v"(tv[3]) : "s"(__popcll(m3)), "i"(O));
        } else if constexpr (CPL == 2) {
            uint64_t m0, m1;
            asm volatile(
                "v_cmp_ge_i32_e64 %0, %2, %4\n\t"
                "v_cmp_ge_i32_e64 %1, %3, %5"
                : "=s"(m0), "=s"(m1)
                : "v"(la[0]), "v"(la[1]), "v"(fd[O][0]), "v"(fd[O][1]));
            asm volatile("v_writelane_b32 %0, %1, %2" : "+v"(tv[0]) : "s"(__popcll(m0)), "i"(O));
            asm volatile("v_writelane_b32 %0, %1, %2" : "+v"(tv[1]) : "s"(__popcll(m1)), "i"(O));
        } else {
            const int tot = count_seen<CPL>(la, fd[O]);
            asm volatile("v_writelane_b32 %0, %1, %2" : "+v"(tv[0]) : "s"(tot), "i"(O));
        }
    }
}

template <int CPL, int OWN, int... O>
__device__ __forceinline__ int tally(const int32_t (&la)[CPL], const int32_t (&fd)[OWN][CPL], TallyMask<OWN> test,
                                     std::integer_sequence<int, O...>) {
    int tv[CPL];
#pragma unroll
    for (int q = 0; q < CPL; q++) tv[q] = 0;
    (tally_one<O, CPL, OWN>(la, fd, tv, test), ...);
    int t = tv[0];
#pragma unroll
    for (int q = 1; q < CPL; q++) t += tv[q];
    return t;
}

// CPL consecutive coordinates of type CT as one load (VEC: n % CPL == 0, so the
// lane's slice is aligned) or CPL scalar loads
template <typename CT, int CPL, bool VEC>
__device__ __forceinline__ void load_slice(const CT* __restrict__ p, uint32_t (&v)[CPL]) {
    constexpr int B = CPL * (int)sizeof(CT);
    if constexpr (VEC && B > 16 && B % 16 == 0) {   // several 16-byte pieces
        constexpr int PER = 16 / (int)sizeof(CT);   // coordinates per piece
#pragma unroll
        for (int k = 0; k < B / 16; k++) {
            const uint4 x = ((const uint4*)p)[k];
            const uint32_t w[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
            for (int u = 0; u < 4; u++) {
                if constexpr (sizeof(CT) == 4) {
                    v[k * PER + u] = w[u];
                } else {
                    v[k * PER + 2 * u] = w[u] & 0xFFFFu;
                    v[k * PER + 2 * u + 1] = w[u] >> 16;
                }
            }
        }
    } else if constexpr (VEC && B == 16 && sizeof(CT) == 2) {   // 8 x uint16
        const uint4 x = *(const uint4*)p;
        const uint32_t w[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
        for (int u = 0; u < 4; u++) {
            v[2 * u] = w[u] & 0xFFFFu;
            v[2 * u + 1] = w[u] >> 16;
        }
    } else if constexpr (VEC && B == 16) {
        const uint4 x = *(const uint4*)p;
        v[0] = x.x; v[1] = x.y; v[2] = x.z; v[3] = x.w;
    } else if constexpr (VEC && B == 8 && sizeof(CT) == 4) {
        const uint2 x = *(const uint2*)p;
        v[0] = x.x; v[1] = x.y;
    } else if constexpr (VEC && B == 8) {   // 4 x uint16
        const uint2 x = *(const uint2*)p;
        v[0] = x.x & 0xFFFFu; v[1] = x.x >> 16; v[2] = x.y & 0xFFFFu; v[3] = x.y >> 16;
    } else if constexpr (VEC && B == 4 && sizeof(CT) == 2) {   // 2 x uint16
        const uint32_t x = *(const uint32_t*)p;
        v[0] = x & 0xFFFFu; v[1] = x >> 16;
    } else {
#pragma unroll
        for (int q = 0; q < CPL; q++) v[q] = (uint32_t)p[q];
    }
}

// bitmask (bit o = candidate o held by this wave) of the candidates that the probe row
// strongly sees; candidate `excl` (own chain's candidate when the probe is that event)
// never counts. Only the candidates in `test` are tallied; `known` (seen at an earlier
// probe, hence seen here) are added without a tally. Lane l holds coordinates [CPL*l, CPL*l + CPL). Coordinates i >= n read
// past the row (slack / the next row), but their fd is +inf (MaxInt32) and la is
// clamped below it, so they never count.
template <int CPL, int OWN, typename CT, bool VEC>
__device__ __forceinline__ uint64_t seen_mask(const CT* __restrict__ row, const int32_t (&fd)[OWN][CPL],
                                              int lane, int sm, int excl, uint64_t test, uint64_t known) {
    uint32_t raw[CPL];
    load_slice<CT, CPL, VEC>(row + CPL * lane, raw);
    int32_t la[CPL];
    // compact: raw LA (value + 1, none = 0) against fd + 1 (none = 0x10000): raw >= fd + 1
    // iff LA >= FD, without decoding; int32: LA clamped below the none value MaxInt32
#pragma unroll
    for (int q = 0; q < CPL; q++) la[q] = (sizeof(CT) == 2) ? (int32_t)raw[q] : min(Coord<CT>::la(raw[q]), kMaxI32 - 1);
    // the masks are wave-uniform: keep them in SGPRs so the skips are scalar branches
    test = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(test >> 32)) << 32) |
           (uint32_t)__builtin_amdgcn_readfirstlane((int)test);
    const int tv = tally<CPL, OWN>(la, fd, (TallyMask<OWN>)test, std::make_integer_sequence<int, OWN>{});
    return (__ballot(lane < OWN && tv >= sm && lane != excl) & test) | known;
}

// LDS of one group: P LA rows (+ slack) | n FD columns of the window. Compact storage
// stages each FD column as FDW aligned dwords (P + 2 coordinates: the window starts at
// an odd or even position), so the staging stays dword LDS-DMA.
template <int P, typename CT>
struct StepLds {
    static constexpr int FDW = P / 2 + 1;   // dwords per compact FD column
    __host__ __device__ static constexpr size_t la_bytes(int n, int cpl) {
        return ((size_t)(P * n + 64 * cpl) * sizeof(CT) + 15) & ~(size_t)15;
    }
    __host__ __device__ static constexpr size_t fd_bytes(int n) {
        return sizeof(CT) == 4 ? (size_t)n * P * 4 : (((size_t)n * FDW * 4 + 15) & ~(size_t)15);
    }
    __host__ __device__ static constexpr size_t group_bytes(int n, int cpl) { return la_bytes(n, cpl) + fd_bytes(n); }
};

template <int CPL, int NWC, int OWN, int P, int GPB, typename CT, bool VEC>
__global__ void __launch_bounds__(GPB * NWC * 64) k_round_step(RoundArgs A, int kstep) {
    constexpr int NT = NWC * 64;   // threads per group
    typedef __attribute__((address_space(3))) void* lds_ptr_t;
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    __shared__ int32_t s_cnt[2][NWC];
    __shared__ uint32_t s_wbits[NWC];

    const int n = A.n, C = A.C, sm = A.sm;
    const int r = kstep;   // the round (graph node argument, rewritten per batch)
    // readfirstlane: the compiler does not know threadIdx.x >> 6 is wave-uniform, and
    // everything derived from it (chain, window, search bounds) would go to VGPRs
    const int lane = lane_id(), wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int gslot = (NWC == 1) ? wave : 0;              // group within block
    const int wg = (NWC == 1) ? 0 : wave;                 // wave within group
    const int gt = (NWC == 1) ? lane : (int)threadIdx.x;  // thread within group
    const int gc = blockIdx.x * GPB + gslot;
    if (gc >= C) return;   // group-uniform; no block barrier is used when NWC == 1
    typedef StepLds<P, CT> L;
    uint8_t* gl_lds = lds + gslot * L::group_bytes(n, CPL);
    CT* __restrict__ la_s = (CT*)gl_lds;
    CT* __restrict__ fd_s = (CT*)(gl_lds + L::la_bytes(n, CPL));
    int fsh = 0;   // compact: parity of the staged window's first position

    HGX_PROF_BEGIN();
    HGX_PROF_COUNT(0);
    const int g = gc / n, cl = gc % n;
    constexpr int rot = 0;   // slot o of wave wg holds candidate j = wg + NWC*((o + rot) % OWN)
    // candidates of this wave: chains j = wg + NWC*o. Their rows do not depend on this
    // chain's boundary, so they are loaded first (their latency overlaps the boundary
    // load and the window staging); unconditionally (every slot of WFD exists), masked
    // by the candidate flag after the window wait.
    const size_t crow = (size_t)r * C + (size_t)g * n;
    uint32_t fl[CPL];
#pragma unroll
    for (int q = 0; q < CPL; q++) {
        const int j = lane + 64 * q;
        fl[q] = (j < n) ? A.wflag[crow + j] : 0u;
    }
    // WFD rows hold the firstDescendants: raw uint16 for compact coordinates (half the
    // bytes every block loads per round), decoded int32 (MaxInt32 = none) otherwise; lane
    // l loads coordinates [CPL*l, CPL*l + CPL) of each row in one load when VEC
    uint32_t fdr[OWN][CPL];
    const int lc = (CPL * lane < n) ? CPL * lane : 0;
#pragma unroll
    for (int o = 0; o < OWN; o++) {
        const int j = wg + NWC * ((o + rot) % OWN);
        const int jj = j < n ? j : 0;
        if constexpr (sizeof(CT) == 2)
            load_slice<uint16_t, CPL, VEC>((const uint16_t*)A.WFD + (crow + jj) * n + lc, fdr[o]);
        else
            load_slice<int32_t, CPL, VEC>(A.WFD + (crow + jj) * n + lc, fdr[o]);
    }
    const int len = A.c_len[gc], off = A.c_off[gc];
    const int b = A.Bm[(size_t)r * C + gc];
    if (b >= len) {
        if (gt == 0) {
            A.wstat[(size_t)r * C + gc] = 0;
            A.wflag[(size_t)(r + 1) * C + gc] = 0;
            A.Bm[(size_t)(r + 1) * C + gc] = len;
        }
        return;
    }
    // stage the probe window [kbase, kbase+np): LA rows (contiguous) and FD columns
    // fd_s[i*P + p] = FDT[i][off+kbase+p] (one wave instruction = 64/P columns)
    auto stage = [&](int kbase, int np) {
        // LA rows [kbase, kbase+np) are contiguous: nel dwords
        const int nel = (int)((size_t)np * n * sizeof(CT) / 4);
        const uint32_t* __restrict__ src = (const uint32_t*)A.LA + (size_t)(off + kbase) * n * sizeof(CT) / 4;
        uint32_t* la_w = (uint32_t*)la_s;
        if (((n * (int)sizeof(CT)) & 15) == 0) {
            for (int c0 = wg * 256; c0 < nel; c0 += NWC * 256) {
                const int t = c0 + lane * 4;
                if (t < nel)
                    __builtin_amdgcn_global_load_lds((const void*)(src + t), (lds_ptr_t)(la_w + c0), 16, 0, 0);
            }
        } else {
            for (int c0 = wg * 64; c0 < nel; c0 += NWC * 64) {
                const int t = c0 + lane;
                if (t < nel) __builtin_amdgcn_global_load_lds((const void*)(src + t), (lds_ptr_t)(la_w + c0), 4, 0, 0);
            }
        }
        if (sizeof(CT) == 4) {
            constexpr int CPI = 64 / P;
            const int pcol = lane % P, icol = lane / P;
            const CT* __restrict__ fsrc = (const CT*)A.FDT + off + kbase + pcol;
            for (int i0 = wg * CPI; i0 < n; i0 += NWC * CPI) {
                const int i = i0 + icol;
                if (i < n && pcol < np)
                    __builtin_amdgcn_global_load_lds((const void*)(fsrc + (size_t)i * A.Pcap),
                                                     (lds_ptr_t)(fd_s + i0 * P), 4, 0, 0);
            }
        } else {
            // column i: dwords covering positions [p0, p0 + 2*FDW), p0 = even start
            constexpr int FDW = L::FDW, CPI = 64 / FDW;
            const int64_t p0 = (off + kbase) & ~1;
            fsh = (off + kbase) & 1;
            const int pcol = lane % FDW, icol = lane / FDW;
            const uint32_t* __restrict__ fsrc = (const uint32_t*)((const CT*)A.FDT + p0) + pcol;
            uint32_t* fd_w = (uint32_t*)fd_s;
            for (int i0 = wg * CPI; i0 < n; i0 += NWC * CPI) {
                const int i = i0 + icol;
                if (i < n && icol < CPI)
                    __builtin_amdgcn_global_load_lds((const void*)(fsrc + (size_t)i * (A.Pcap / 2)),
                                                     (lds_ptr_t)(fd_w + i0 * FDW), 4, 0, 0);
            }
        }
    };
    HGX_PROF(4);
    stage(b, min(P, len - b));   // in flight while the candidate rows load
    HGX_PROF(5);
    // window landed (and the candidate rows with it): everyone may read the LDS window
    __builtin_amdgcn_s_waitcnt(0);
    if (NWC == 1) wave_lds_fence(); else __syncthreads();
    int32_t fd[OWN][CPL];
    uint64_t cmask = 0;   // this wave's slots that hold a candidate
#pragma unroll
    for (int o = 0; o < OWN; o++) {
        const int j = wg + NWC * ((o + rot) % OWN);
        uint32_t f = 0;
#pragma unroll
        for (int q = 0; q < CPL; q++) {
            const uint32_t v = __shfl(fl[q], j & 63);
            if (q == (j >> 6)) f = v;
        }
        const bool cand = (j < n) && f == 1u;
        cmask |= (uint64_t)cand << o;
#pragma unroll
        for (int q = 0; q < CPL; q++) {
            const int i = CPL * lane + q;
            fd[o][q] = (cand && i < n) ? ((sizeof(CT) == 2) ? (int32_t)fdr[o][q] + 1 : (int32_t)fdr[o][q]) : kMaxI32;
            // opaque from here on: otherwise the compiler keeps (cand && i < n) as a lane
            // mask per candidate and ANDs it into every compare (SGPR pressure, spills)
            asm volatile("" : "+v"(fd[o][q]));
        }
    }
    HGX_PROF(1);
    // own-chain candidate slot (never counts for the probe that is itself)
    const int own_o = (cl >= wg && (cl - wg) % NWC == 0) ? ((cl - wg) / NWC - rot + OWN) % OWN : -1;
    int kbase = b, np = min(P, len - b), lo = 0, kstar = len, lv = 0;
    // this wave's strongly-seen bits at the last probe that reached SM: the search ends on
    // such a probe when the boundary is in the window, so it is the boundary's S row
    uint64_t hit_bits = 0;
    // monotone along the chain: candidates seen at the last probe below the boundary
    // (s_lo) are seen at every later probe; candidates not seen at the first probe
    // that reached SM (s_hi) are not seen below it. Only s_hi & ~s_lo are tallied.
    uint64_t s_lo = 0;
    bool staged = true;
    for (;;) {
        if (!staged) {
            stage(kbase, np);
            __builtin_amdgcn_s_waitcnt(0);
            if (NWC == 1) wave_lds_fence(); else __syncthreads();
        }
        staged = false;
        HGX_PROF(2);
        lo = 0;
        int hi = np;
        uint64_t s_hi = cmask;
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            const int ex = (kbase + mid == b) ? own_o : -1;
#ifdef HGX_STEP_PROF
            if (threadIdx.x == 0) _pa[6] += (unsigned long long)__popcll(s_hi & ~s_lo) * 1000ull + 1ull;
#endif
            const uint64_t bits =
                seen_mask<CPL, OWN, CT, VEC>(la_s + mid * n, fd, lane, sm, ex, s_hi & ~s_lo, s_lo);
            int tot = __popcll(bits);
            if (NWC > 1) {
                if (lane == 0) s_cnt[lv & 1][wave] = tot;
                __syncthreads();
                tot = 0;
#pragma unroll
                for (int w = 0; w < NWC; w++) tot += s_cnt[lv & 1][w];
                lv++;
            }
            if (tot >= sm) { hi = mid; hit_bits = bits; s_hi = bits; } else { lo = mid + 1; s_lo = bits; }
        }
        HGX_PROF(3);
        if (lo < np) { kstar = kbase + lo; break; }
        kbase += np;
        if (kbase >= len) { kstar = len; break; }
        np = min(P, len - kbase);
        // everyone is done with the window before it is restaged
        if (NWC == 1) wave_lds_fence(); else __syncthreads();
    }
    // outputs of round r for this chain
    for (int k = b + gt; k < kstar; k += NT) A.p_round[off + k] = r;
    if (gt == 0) {
        A.wstat[(size_t)r * C + gc] = (kstar > b) ? 2 : 1;
        if (kstar < len) {   // same value from every writer: plain stores
            A.active[r] = 1;
            if (A.hflag) *A.hflag = r + 1;   // last step of a batch: the host's flag
        }
        A.Bm[(size_t)(r + 1) * C + gc] = kstar;
    }
    HGX_PROF(7);
    if (kstar < len) {
        // S row of the boundary event (the candidate of round r+1): W'_r members it
        // strongly sees, bit o of wave wg = candidate j = wg + NWC*((o + rot) % OWN)
        const int pk = kstar - kbase;   // inside the staged window
        const size_t srow = ((size_t)(r + 1) * C + gc) * A.nw;
        if (NWC == 1) {   // j = (o + rot) % OWN: rotate left by rot within OWN bits
            const uint64_t msk = (OWN >= 64) ? ~0ull : ((1ull << OWN) - 1ull);
            const uint64_t hb = hit_bits & msk;
            const uint64_t rb = rot ? (((hb << rot) | (hb >> (OWN - rot))) & msk) : hb;
            if (lane == 0) A.Smat[srow] = rb;
        } else {
            if (lane == 0) s_wbits[wave] = (uint32_t)hit_bits;
            __syncthreads();
            if (wg < A.nw) {   // wave x assembles word x: candidate j = 64x + lane
                const int j = 64 * wg + lane;
                const bool bit = j < n && ((s_wbits[j % NWC] >> ((j / NWC - rot + OWN) % OWN)) & 1u);
                const uint64_t word = __ballot(bit);
                if (lane == 0) A.Smat[srow + wg] = word;
            }
        }
        HGX_PROF(7);
        // coordinate rows of the new candidate, both from the staged window
        const size_t nrow = ((size_t)(r + 1) * C + gc) * n;
        for (int i = gt; i < n; i += NT) {
            A.WLA[nrow + i] = Coord<CT>::la(la_s[pk * n + i]);
            if constexpr (sizeof(CT) == 2) ((uint16_t*)A.WFD)[nrow + i] = fd_s[i * 2 * L::FDW + fsh + pk];
            else A.WFD[nrow + i] = fd_s[i * P + pk];
        }
        if (gt == 0) A.wflag[(size_t)(r + 1) * C + gc] = 1;
    } else if (gt == 0) {
        A.wflag[(size_t)(r + 1) * C + gc] = 0;
    }
    HGX_PROF(7);
    HGX_PROF_END();
}

// n in (256, 1024]: the candidates' firstDescendants rows (up to 4 MB per round) fit
// neither in registers nor in LDS, so the search is per candidate: every wave streams
// the FD rows of its candidates (shared by all chains of the round, so L2-resident).
// A window of P probe rows is staged in LDS; each candidate is first tested against the
// window's last probe (monotone: a candidate not seen there is not seen anywhere in the
// window, and if fewer than SM are seen there the boundary is beyond the window), and
// only the candidates seen there are binary-searched for their first seeing probe.
// The count at probe p is the number of candidates first seen at or before p (an LDS
// histogram). The own-chain candidate never counts at the probe that is itself.
// waves per block: the candidates of a chain are walked per wave, so more waves per block
// wins over more resident blocks (c5 step: 16 waves 470 us, 8 waves 539 us, 4 waves 854 us)
constexpr int kBigWaves = 16;
template <int CPL, int P, typename CT, bool VEC>
__global__ void __launch_bounds__(kBigWaves * 64) k_round_step_big(RoundArgs A, int kstep) {
    constexpr int NWV = kBigWaves;
    typedef __attribute__((address_space(3))) void* lds_ptr_t;
    extern __shared__ __attribute__((aligned(16))) uint8_t big_lds[];
    CT* __restrict__ la_s = (CT*)big_lds;   // [P][n] probe rows (+ slack)
    __shared__ int32_t hist[P + 1];
    __shared__ uint8_t fhit[1024];               // first probe seeing candidate j (255: none / no candidate)
    __shared__ uint8_t s_cand[1024];             // candidate flags of the round (staged once)
    __shared__ unsigned long long s_mask[16];
    __shared__ int32_t s_cnt[NWV];
    __shared__ int32_t s_f;
    const int n = A.n, C = A.C, sm = A.sm;
    const int r = kstep;   // the round (graph node argument, rewritten per batch)
    const int lane = lane_id(), wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int gc = blockIdx.x;
    const int g = gc / n, cl = gc % n;
    const int len = A.c_len[gc], off = A.c_off[gc];
    const int b = A.Bm[(size_t)r * C + gc];
    if (b >= len) {
        if (threadIdx.x == 0) {
            A.wstat[(size_t)r * C + gc] = 0;
            A.wflag[(size_t)(r + 1) * C + gc] = 0;
            A.Bm[(size_t)(r + 1) * C + gc] = len;
        }
        return;
    }
    const size_t crow = (size_t)r * C + (size_t)g * n;
    // coordinates of lane l, slot q: int32 i = l + 64q; compact i = 2l + (q & 1) + 128(q >> 1)
    // (pairs as one dword): coalesced row loads and conflict-free LDS reads
    auto coord = [&](int q) -> int {
        return sizeof(CT) == 4 ? lane + 64 * q : 2 * lane + (q & 1) + 128 * (q >> 1);
    };
    auto load_row = [&](const CT* __restrict__ row, uint32_t (&raw)[CPL], bool clamp) {
        if constexpr (sizeof(CT) == 4) {
#pragma unroll
            for (int q = 0; q < CPL; q++) {
                const int i = lane + 64 * q;
                raw[q] = (uint32_t)row[(clamp && i >= n) ? 0 : i];
            }
        } else {
#pragma unroll
            for (int q2 = 0; q2 < CPL / 2; q2++) {
                const int i = 2 * lane + 128 * q2;
                const uint32_t w = *(const uint32_t*)(row + ((clamp && i >= n) ? 0 : i));
                raw[2 * q2] = w & 0xFFFFu;
                raw[2 * q2 + 1] = w >> 16;
            }
        }
    };
    // compact: raw LA (value + 1, none = 0) against the raw WFD value + 1 (none = 0x10000),
    // no decode; int32: LA clamped below the none value MaxInt32
    auto seen_at = [&](const int32_t (&fd)[CPL], int pp, int j, int kb) -> bool {
        uint32_t raw[CPL];
        load_row(la_s + pp * n, raw, false);
        // per-lane count over the CPL slots in VALU, one DPP wave sum: CPL scalar popcounts
        // and adds per test would make the walk scalar-issue-bound
        uint32_t c = 0;
#pragma unroll
        for (int q = 0; q < CPL; q++) {
            const int32_t la = (sizeof(CT) == 2) ? (int32_t)raw[q] : min(Coord<CT>::la(raw[q]), kMaxI32 - 1);
            c += (la >= fd[q]) ? 1u : 0u;
        }
        const int tot = (int)__builtin_amdgcn_readlane((int)wave_scan_add_u32(c), 63);
        return tot >= sm && !(j == cl && kb + pp == b);
    };
    // WFD row of candidate j in the lane's coordinate order (compact rows are raw uint16,
    // read as coordinate pairs); j >= n loads nothing. Issued one candidate ahead of use.
    auto load_fd = [&](int j, int32_t (&fd)[CPL]) {
        if (j >= n) return;
        if constexpr (sizeof(CT) == 2) {
            const uint16_t* __restrict__ row = (const uint16_t*)A.WFD + (crow + j) * n;
#pragma unroll
            for (int q2 = 0; q2 < CPL / 2; q2++) {
                const int i = 2 * lane + 128 * q2;
                const uint32_t w = (i < n) ? *(const uint32_t*)(row + i) : 0u;
                fd[2 * q2] = (i < n) ? (int32_t)(w & 0xFFFFu) + 1 : kMaxI32;
                fd[2 * q2 + 1] = (i < n) ? (int32_t)(w >> 16) + 1 : kMaxI32;
            }
        } else {
            const int32_t* __restrict__ row = A.WFD + (crow + j) * n;
#pragma unroll
            for (int q = 0; q < CPL; q++) {
                const int i = coord(q);
                fd[q] = (i < n) ? row[i] : kMaxI32;
            }
        }
    };
    for (int t = threadIdx.x; t < n; t += blockDim.x) s_cand[t] = A.wflag[crow + t];   // before the first barrier
    int kbase = b, np = 0, kstar = len, pk = 0;
    for (;;) {
        np = min(P, len - kbase);
        {   // stage the window's LA rows (contiguous, nel dwords)
            const int nel = (int)((size_t)np * n * sizeof(CT) / 4);
            const uint32_t* __restrict__ src = (const uint32_t*)A.LA + (size_t)(off + kbase) * n * sizeof(CT) / 4;
            uint32_t* la_w = (uint32_t*)la_s;
            if (((n * (int)sizeof(CT)) & 15) == 0) {
                for (int c0 = wave * 256; c0 < nel; c0 += NWV * 256) {
                    const int t = c0 + lane * 4;
                    if (t < nel)
                        __builtin_amdgcn_global_load_lds((const void*)(src + t), (lds_ptr_t)(la_w + c0), 16, 0, 0);
                }
            } else {
                for (int c0 = wave * 64; c0 < nel; c0 += NWV * 64) {
                    const int t = c0 + lane;
                    if (t < nel)
                        __builtin_amdgcn_global_load_lds((const void*)(src + t), (lds_ptr_t)(la_w + c0), 4, 0, 0);
                }
            }
        }
        for (int t = threadIdx.x; t <= P; t += blockDim.x) hist[t] = 0;
        __builtin_amdgcn_s_waitcnt(0);
        __syncthreads();
        // pass 1: every candidate against the window's last probe
        int cnt = 0;
        int32_t fdn[CPL];
        load_fd(wave, fdn);
        for (int j = wave; j < n; j += NWV) {
            int32_t fd[CPL];
#pragma unroll
            for (int q = 0; q < CPL; q++) fd[q] = fdn[q];
            load_fd(j + NWV, fdn);   // next candidate's row in flight during this test
            const bool cand = s_cand[j] == 1;
            const bool sl = cand && seen_at(fd, np - 1, j, kbase);
            cnt += sl ? 1 : 0;
            if (lane == 0) fhit[j] = sl ? (uint8_t)(np - 1) : (uint8_t)255;
        }
        if (lane == 0) s_cnt[wave] = cnt;
        __syncthreads();
        int tot = 0;
#pragma unroll
        for (int w = 0; w < NWV; w++) tot += s_cnt[w];
        if (tot >= sm) {
            // pass 2: first seeing probe of the candidates seen at the last probe
            // this wave's candidates seen at the last probe (fhit written by this wave's
            // lane 0, so the walk is wave-uniform), rows loaded one candidate ahead
            auto next_seen = [&](int j) {
                while (j < n && fhit[j] == 255) j += NWV;
                return j;
            };
            int jn = next_seen(wave);
            int32_t fdn2[CPL];
            load_fd(jn, fdn2);
            while (jn < n) {
                const int j = jn;
                int32_t fd[CPL];
#pragma unroll
                for (int q = 0; q < CPL; q++) fd[q] = fdn2[q];
                jn = next_seen(j + NWV);
                load_fd(jn, fdn2);
                int lo = 0, hi = np - 1;
                while (lo < hi) {
                    const int mid = (lo + hi) >> 1;
                    if (seen_at(fd, mid, j, kbase)) hi = mid; else lo = mid + 1;
                }
                if (lane == 0) {
                    fhit[j] = (uint8_t)lo;
                    atomicAdd(&hist[lo], 1);
                }
            }
            __syncthreads();
            if (threadIdx.x == 0) {
                int acc = 0, f = np - 1;
                for (int pp = 0; pp < np; pp++) {
                    acc += hist[pp];
                    if (acc >= sm) { f = pp; break; }
                }
                s_f = f;
            }
            __syncthreads();
            kstar = kbase + s_f;
            pk = s_f;
            break;
        }
        kbase += np;
        if (kbase >= len) { kstar = len; break; }
        __syncthreads();
    }
    for (int k = b + (int)threadIdx.x; k < kstar; k += blockDim.x) A.p_round[off + k] = r;
    if (threadIdx.x == 0) {
        A.wstat[(size_t)r * C + gc] = (kstar > b) ? 2 : 1;
        if (kstar < len) {   // same value from every writer: plain stores
            A.active[r] = 1;
            if (A.hflag) *A.hflag = r + 1;   // last step of a batch: the host's flag
        }
        A.Bm[(size_t)(r + 1) * C + gc] = kstar;
    }
    if (kstar < len) {
        // S row of the boundary event: candidates first seen at or before it
        if (threadIdx.x < 16) s_mask[threadIdx.x] = 0;
        __syncthreads();
        for (int j = threadIdx.x; j < n; j += blockDim.x)
            if (fhit[j] <= pk) atomicOr(&s_mask[j >> 6], 1ull << (j & 63));
        __syncthreads();
        const size_t srow = ((size_t)(r + 1) * C + gc) * A.nw;
        if ((int)threadIdx.x < A.nw) A.Smat[srow + threadIdx.x] = s_mask[threadIdx.x];
        const int p = off + kstar;
        const size_t nrow = ((size_t)(r + 1) * C + gc) * n;
        for (int i = threadIdx.x; i < n; i += blockDim.x) {
            A.WLA[nrow + i] = Coord<CT>::la(la_s[pk * n + i]);
            if constexpr (sizeof(CT) == 2) ((uint16_t*)A.WFD)[nrow + i] = ((const CT*)A.FDT)[(size_t)i * A.Pcap + p];
            else A.WFD[nrow + i] = ((const CT*)A.FDT)[(size_t)i * A.Pcap + p];
        }
        if (threadIdx.x == 0) A.wflag[(size_t)(r + 1) * C + gc] = 1;
    } else if (threadIdx.x == 0) {
        A.wflag[(size_t)(r + 1) * C + gc] = 0;
    }
}

template <int CPL, int P, typename CT, bool VEC>
static hipError_t step_big_launch_v(hipStream_t s, const RoundArgs& A, int kstep) {
    const void* f = (const void*)k_round_step_big<CPL, P, CT, VEC>;
    const size_t lds = (size_t)(P * A.n + 64 * CPL) * sizeof(CT);
    {
        const hipError_t e = ensure_lds_limit(f, 160 * 1024 - 4096);
        if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL((k_round_step_big<CPL, P, CT, VEC>), dim3(A.C), dim3(kBigWaves * 64), lds, s, A, kstep);
    return hipGetLastError();
}

template <int CPL, int P, typename CT>
static hipError_t step_big_launch(hipStream_t s, const RoundArgs& A, int kstep) {
    return step_big_launch_v<CPL, P, CT, false>(s, A, kstep);
}

template <int CPL, int NWC, int OWN, int P, int GPB, typename CT, bool VEC>
static hipError_t step_launch_v(hipStream_t s, const RoundArgs& A, int kstep) {
    const void* f = (const void*)k_round_step<CPL, NWC, OWN, P, GPB, CT, VEC>;
    const size_t lds = (size_t)GPB * StepLds<P, CT>::group_bytes(A.n, CPL);
    {
        const hipError_t e = ensure_lds_limit(f, 160 * 1024 - 2048);
        if (e != hipSuccess) return e;
    }
    const unsigned grid = (unsigned)((A.C + GPB - 1) / GPB);
    hipLaunchKernelGGL((k_round_step<CPL, NWC, OWN, P, GPB, CT, VEC>), dim3(grid), dim3(GPB * NWC * 64), lds, s, A,
                       kstep);
    return hipGetLastError();
}

template <int CPL, int NWC, int OWN, int P, int GPB, typename CT>
static hipError_t step_launch(hipStream_t s, const RoundArgs& A, int kstep) {
    if (CPL == 1 || A.n % CPL == 0) return step_launch_v<CPL, NWC, OWN, P, GPB, CT, true>(s, A, kstep);
    return step_launch_v<CPL, NWC, OWN, P, GPB, CT, false>(s, A, kstep);
}

template <typename CT>
static hipError_t launch_round_step_t(hipStream_t s, const RoundArgs& A, int kstep) {
    const int n = A.n;
    // many chains (batched graphs): one wave per chain; few chains: a 16-wave group per
    // chain, so the candidates' tests of a level are spread over 16 waves
    if (A.C < 1024 && n > 16) {
        if (n <= 32) return step_launch<1, 16, 2, 32, 1, CT>(s, A, kstep);
        if (n <= 64) return step_launch<1, 16, 4, 32, 1, CT>(s, A, kstep);
    }
    if (n <= 16) return step_launch<1, 1, 16, 32, 4, CT>(s, A, kstep);
    if (n <= 32) return step_launch<1, 1, 32, 32, 4, CT>(s, A, kstep);
    if (n <= 64) return step_launch<1, 1, 64, 32, 4, CT>(s, A, kstep);
    if (n <= 128) return step_launch<2, 16, 8, 32, 1, CT>(s, A, kstep);
    if (n <= 256) return step_launch<4, 16, 16, 32, 1, CT>(s, A, kstep);
    if (n <= 512) return step_big_launch<8, 32, CT>(s, A, kstep);
    if (n <= 1024) return step_big_launch<16, 32, CT>(s, A, kstep);
    return hipErrorInvalidValue;
}

hipError_t launch_round_step(hipStream_t s, const RoundArgs& A, int kstep, int block_search) {
    if (!block_search && A.n <= 1024) return launch_round_k(s, A, kstep);
    return A.compact ? launch_round_step_t<uint16_t>(s, A, kstep) : launch_round_step_t<int32_t>(s, A, kstep);
}



// lastRound per graph after the round steps: the largest r in [rs, R) with a witness
// (wstat 2) in any chain of graph g. Grid (G, ceil((R - rs) / 64)).
__global__ void __launch_bounds__(256) k_last_round(int rs, int R, int C, int n, const uint8_t* __restrict__ wstat,
                                                    int32_t* __restrict__ lr) {
    __shared__ int32_t s_max[4];
    const int g = blockIdx.x;
    const int r0 = rs + blockIdx.y * 64;
    const int nr = min(64, R - r0);   // (a resumed call scans a few rounds)
    int m = -1;
    for (int t = threadIdx.x; t < nr * n; t += blockDim.x) {
        const int r = r0 + t / n, i = t - (t / n) * n;
        if (wstat[(size_t)r * C + (size_t)g * n + i] == 2) m = max(m, r);
    }
    for (int o = 32; o >= 1; o >>= 1) m = max(m, __shfl_xor(m, o));
    if ((threadIdx.x & 63) == 0) s_max[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0) {
        m = max(max(s_max[0], s_max[1]), max(s_max[2], s_max[3]));
        if (m >= 0) atomicMax(&lr[g], m);
    }
}

void launch_last_round(hipStream_t s, int rs, int R, int G, int C, int n, const uint8_t* wstat, int32_t* lr) {
    if (R <= rs) return;
    hipLaunchKernelGGL(k_last_round, dim3(G, (R - rs + 63) / 64), dim3(256), 0, s, rs, R, C, n, wstat, lr);
}


#ifdef HGX_STEP_PROF
void step_prof_dump() {
    unsigned long long h[8];
    if (hipMemcpyFromSymbol(h, HIP_SYMBOL(hgx_step_prof), sizeof(h)) != hipSuccess) return;
    fprintf(stderr, "[hgx] round phases (clk sums; 0 = block-rounds, 6 = wave-0 tallies*1000 + levels):");
    for (int i = 0; i < 8; i++) fprintf(stderr, " %d:%llu", i, h[i]);
    fprintf(stderr, "\n");
    round_k_prof_dump();
    round_p_prof_dump();
    round_pb_prof_dump();
    round_g_prof_dump();
}
#else
void step_prof_dump() {}
#endif

}  // namespace hgx
