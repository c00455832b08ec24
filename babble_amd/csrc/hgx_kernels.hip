// HIP kernels of libhgx for gfx950 (CDNA4, wave64). See DESIGN.md for the data
// layout, the reformulation of the reference loops, and the roofline of each kernel.
//
// Layout recap (all int32 unless noted):
//   positions p: events in chain-major order, p = c_off[c] + (Index - c_base[c])
//   LA  [P x n]  lastAncestors  (row-major per position)      hashgraph.go:448-499
//   FDT [n x P]  firstDescendants, column-major (FDT[c][p])     hashgraph.go:502-530
//   per round r and global chain gc: Bm[r][gc] = first chain offset with round >= r,
//   WLA/WFD[r][gc][:] = coordinate rows of that candidate event, wflag 1/2.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <tuple>

#include "hgx_device.h"
#include "hgx_kernels.h"

namespace hgx {


// ---------------------------------------------------------------------------------
// layout: gid order -> chain-major positions. Consecutive gids belong to different
// chains, so a direct per-gid scatter writes every output array 4-8 bytes at a time at
// random positions. A block instead takes kLayoutB consecutive gids, groups them by chain
// in LDS (a chain's events in the block have consecutive indices, hence consecutive
// positions) and writes each chain's run contiguously.
constexpr int kLayoutB = 4096;   // gids per block
constexpr int kLayoutH = 1024;   // chain-id range a block can group (else direct scatter)

// The op parent's (chain, chain offset) come from ONE 8-byte read of g_ck (k_ck_pack) instead of two
// gathers (its creator and its Index) from different arrays: an op parent is an arbitrary earlier event,
// so each gather was a line of its own (c4: 204 bytes fetched per laid-out event)
__global__ void __launch_bounds__(256) k_ck_pack(int64_t E0, int64_t E, const int32_t* __restrict__ g_creator,
                                                 const int32_t* __restrict__ g_index, const int32_t* __restrict__ c_base,
                                                 int64_t* __restrict__ g_ck) {
    const int64_t gid = E0 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (gid >= E) return;
    const int c = g_creator[gid];
    g_ck[gid] = ((int64_t)c << 32) | (uint32_t)(g_index[gid] - c_base[c]);
}

__device__ __forceinline__ void layout_one(int64_t gid, int p, const int32_t* __restrict__ g_creator,
                                           const int64_t* __restrict__ g_ck, const int32_t* __restrict__ g_op,
                                           const int64_t* __restrict__ g_ts, const int32_t* __restrict__ g_rr,
                                           const int64_t* __restrict__ g_cts, const int32_t* __restrict__ c_off,
                                           const int32_t* __restrict__ c_base, int32_t* __restrict__ p_gid,
                                           int32_t* __restrict__ p_chain, int32_t* __restrict__ p_op,
                                           int32_t* __restrict__ p_opu, int32_t* __restrict__ p_opk,
                                           int64_t* __restrict__ p_ts, int32_t* __restrict__ p_rr,
                                           int64_t* __restrict__ p_cts, int C, int n, int seg) {
    const int c = g_creator[gid];
    const int op = g_op[gid];
    int opp = -1, opu = -1, opk = -1;
    if (op >= 0) {
        const int64_t ck = g_ck[op];
        const int oc = (int)(ck >> 32);
        const int ok = (int)(uint32_t)ck;
        opp = c_off[oc] + ok;
        opu = (ok / seg) * C + oc;   // lastAncestors unit of the op row (k_la_sweep)
        // op chain within the graph | op row (k_la_wave; only used when rows < 2^kOpkBits)
        opk = ((oc % n) << kOpkBits) | (ok & ((1 << kOpkBits) - 1));
    }
    p_opk[p] = opk;
    p_gid[p] = (int32_t)gid;
    p_chain[p] = c;
    p_op[p] = opp;
    p_opu[p] = opu;
    p_ts[p] = g_ts[gid];
    p_rr[p] = g_rr[gid];
    p_cts[p] = g_cts[gid];
}

// a few thousand new events (the incremental schedule): one thread per event, direct scatter
// (a 4 096-event block of k_layout would run the whole batch on one CU)
__global__ void __launch_bounds__(256) k_layout_direct(int64_t E0, int64_t E, const int32_t* __restrict__ g_creator,
                                                       const int32_t* __restrict__ g_index, const int64_t* __restrict__ g_ck,
                                                       const int32_t* __restrict__ g_op,
                                                       const int64_t* __restrict__ g_ts, const int32_t* __restrict__ g_rr,
                                                       const int64_t* __restrict__ g_cts, const int32_t* __restrict__ c_off,
                                                       const int32_t* __restrict__ c_base, int32_t* __restrict__ g_pos,
                                                       int32_t* __restrict__ p_gid, int32_t* __restrict__ p_chain,
                                                       int32_t* __restrict__ p_op, int32_t* __restrict__ p_opu,
                                                       int32_t* __restrict__ p_opk, int64_t* __restrict__ p_ts,
                                                       int32_t* __restrict__ p_rr, int64_t* __restrict__ p_cts, int C,
                                                       int n, int seg) {
    const int64_t gid = E0 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (gid >= E) return;
    const int c = g_creator[gid];
    const int p = c_off[c] + g_index[gid] - c_base[c];
    g_pos[gid] = p;
    layout_one(gid, p, g_creator, g_ck, g_op, g_ts, g_rr, g_cts, c_off, c_base, p_gid, p_chain, p_op, p_opu, p_opk,
               p_ts, p_rr, p_cts, C, n, seg);
}


// Round 5: the same grouping, with every input column read in gid order (coalesced) and written out in
// slot order (coalesced) through an LDS stage: the slot-order pass of k_layout read six columns scattered
// over its 4 096 gids while ~190 blocks per XCD were in flight, so most of those reads missed L2 (c4 PMC:
// 3.97 GB fetched per pass, 473 bytes per event against 40 read). A thread's 8 events have all their
// columns loaded at once (one global round trip, then one for the op parents' packed words), then each
// output column goes through the stage in turn.
constexpr int kLayoutB2 = 2048;   // gids per block
__global__ void __launch_bounds__(256) k_layout_staged(int64_t E0, int64_t E, const int32_t* __restrict__ g_creator,
                                                       const int32_t* __restrict__ g_index, const int64_t* __restrict__ g_ck,
                                                       const int32_t* __restrict__ g_op, const int64_t* __restrict__ g_ts,
                                                       const int32_t* __restrict__ g_rr, const int64_t* __restrict__ g_cts,
                                                       const int32_t* __restrict__ c_off, const int32_t* __restrict__ c_base,
                                                       int32_t* __restrict__ g_pos, int32_t* __restrict__ p_gid,
                                                       int32_t* __restrict__ p_chain, int32_t* __restrict__ p_op,
                                                       int32_t* __restrict__ p_opu, int32_t* __restrict__ p_opk,
                                                       int64_t* __restrict__ p_ts, int32_t* __restrict__ p_rr,
                                                       int64_t* __restrict__ p_cts, int C, int n, int seg) {
    constexpr int B = kLayoutB2, PT = B / 256;   // events per thread
    __shared__ int32_t s_cnt[kLayoutH], s_min[kLayoutH];
    __shared__ int32_t s_slot[B];   // slot -> gid offset in the block
    __shared__ int32_t s_cr[B], s_ix[B];
    __shared__ __attribute__((aligned(16))) int64_t s_stg[B];
    __shared__ int32_t s_lo, s_hi;
    const int nbk = (int)gridDim.x, q8 = nbk / 8, r8 = nbk % 8, x8 = (int)blockIdx.x % 8;
    const int lb = x8 * q8 + min(x8, r8) + (int)blockIdx.x / 8;   // XCD-grouped block order (k_layout)
    const int64_t g0 = E0 + (int64_t)lb * B;
    const int nb = (int)min<int64_t>(B, E - g0);
    const int t0 = threadIdx.x;
    // every column of this thread's events at once
    int32_t cr[PT], ix[PT], op[PT], rr[PT];
    int64_t ts[PT], cts[PT], ck[PT];
#pragma unroll
    for (int k = 0; k < PT; k++) {
        const int t = t0 + 256 * k;
        const bool v = t < nb;
        const int64_t gid = g0 + (v ? t : 0);
        cr[k] = g_creator[gid];
        ix[k] = g_index[gid];
        op[k] = g_op[gid];
        rr[k] = g_rr[gid];
        ts[k] = g_ts[gid];
        cts[k] = g_cts[gid];
    }
#pragma unroll
    for (int k = 0; k < PT; k++) ck[k] = op[k] >= 0 ? g_ck[op[k]] : -1ll;   // (op parents: recent events)
    if (t0 == 0) { s_lo = 0x7FFFFFFF; s_hi = -1; }
    for (int h = t0; h < kLayoutH; h += 256) { s_cnt[h] = 0; s_min[h] = 0x7FFFFFFF; }
    int lo = 0x7FFFFFFF, hi = -1;
#pragma unroll
    for (int k = 0; k < PT; k++) {
        const int t = t0 + 256 * k;
        if (t < nb) {
            s_cr[t] = cr[k];
            s_ix[t] = ix[k];
            lo = min(lo, cr[k]);
            hi = max(hi, cr[k]);
        }
    }
    __syncthreads();
    for (int o = 32; o >= 1; o >>= 1) { lo = min(lo, __shfl_xor(lo, o)); hi = max(hi, __shfl_xor(hi, o)); }
    if ((t0 & 63) == 0) { atomicMin(&s_lo, lo); atomicMax(&s_hi, hi); }
    __syncthreads();
    const int clo = s_lo;
    if (s_hi - clo >= kLayoutH) {   // block-uniform: too many chains to group, direct scatter
        for (int t = t0; t < nb; t += 256) {
            const int64_t gid = g0 + t;
            const int c = s_cr[t];
            const int p = c_off[c] + s_ix[t] - c_base[c];
            g_pos[gid] = p;
            layout_one(gid, p, g_creator, g_ck, g_op, g_ts, g_rr, g_cts, c_off, c_base, p_gid, p_chain, p_op,
                       p_opu, p_opk, p_ts, p_rr, p_cts, C, n, seg);
        }
        return;
    }
#pragma unroll
    for (int k = 0; k < PT; k++) {
        const int t = t0 + 256 * k;
        if (t < nb) {
            const int h = cr[k] - clo;
            atomicAdd(&s_cnt[h], 1);
            atomicMin(&s_min[h], ix[k]);
        }
    }
    __syncthreads();
    if (t0 < 64) {   // exclusive scan of the counts (one wave)
        constexpr int PER = kLayoutH / 64;
        int v[PER], sum = 0;
#pragma unroll
        for (int k = 0; k < PER; k++) { v[k] = s_cnt[t0 * PER + k]; sum += v[k]; }
        int incl = sum;
        for (int o = 1; o < 64; o <<= 1) {
            const int y = __shfl_up(incl, o);
            if (t0 >= o) incl += y;
        }
        int run = incl - sum;
#pragma unroll
        for (int k = 0; k < PER; k++) { s_cnt[t0 * PER + k] = run; run += v[k]; }
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < PT; k++) {
        const int t = t0 + 256 * k;
        if (t < nb) {
            const int h = cr[k] - clo;
            s_slot[s_cnt[h] + ix[k] - s_min[h]] = t;
            g_pos[g0 + t] = c_off[cr[k]] + ix[k] - c_base[cr[k]];
        }
        if (t < nb) s_stg[t] = ck[k];
    }
    __syncthreads();
    // slot sl -> (gid offset, position): consecutive slots = consecutive positions of a chain's run
    auto pos_of = [&](int t) { const int c = s_cr[t]; return c_off[c] + s_ix[t] - c_base[c]; };
    for (int sl = t0; sl < nb; sl += 256) {   // the op parent's (chain, offset) -> p_op, p_opu, p_opk
        const int t = s_slot[sl], p = pos_of(t);
        const int64_t cki = s_stg[t];
        int opp = -1, opu = -1, opk = -1;
        if (cki >= 0) {
            const int oc = (int)(cki >> 32), ok = (int)(uint32_t)cki;
            opp = c_off[oc] + ok;
            opu = (ok / seg) * C + oc;
            opk = ((oc % n) << kOpkBits) | (ok & ((1 << kOpkBits) - 1));
        }
        p_op[p] = opp;
        p_opu[p] = opu;
        p_opk[p] = opk;
        p_gid[p] = (int32_t)(g0 + t);
        p_chain[p] = s_cr[t];
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < PT; k++)
        if (t0 + 256 * k < nb) s_stg[t0 + 256 * k] = ts[k];
    __syncthreads();
    for (int sl = t0; sl < nb; sl += 256) {
        const int t = s_slot[sl];
        p_ts[pos_of(t)] = s_stg[t];
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < PT; k++)
        if (t0 + 256 * k < nb) s_stg[t0 + 256 * k] = cts[k];
    __syncthreads();
    for (int sl = t0; sl < nb; sl += 256) {
        const int t = s_slot[sl];
        p_cts[pos_of(t)] = s_stg[t];
    }
    __syncthreads();
    int32_t* s_rr = (int32_t*)s_stg;
#pragma unroll
    for (int k = 0; k < PT; k++)
        if (t0 + 256 * k < nb) s_rr[t0 + 256 * k] = rr[k];
    __syncthreads();
    for (int sl = t0; sl < nb; sl += 256) {
        const int t = s_slot[sl];
        p_rr[pos_of(t)] = s_rr[t];
    }
}

// ---------------------------------------------------------------------------------
// lastAncestors: in-place monotone sweeps (Gauss-Seidel) over units, with dirty tracking.
// LA[x] = max(LA[sp(x)], LA[op(x)]), LA[x][cr(x)] = Index(x)   (hashgraph.go:470-496)
// A unit = (segment s of SEG rows, chain c), enumerated time-major (u = s*C + c) so
// that earlier segments of every chain are usually finished before later ones read
// them. Values only grow and stale reads are lower bounds, so a recomputed row is
// never below its stored value and repeating sweeps until none changes anything
// reaches the fixed point. A unit's rows can only change if one of its
// inputs changed: the previous unit of its chain (the carry) or the unit of one of its
// op rows; sweep t+1 recomputes only those (stamp == t), marking with stamp t+1 the units
// whose values changed. "Changed" is detected without reading the old rows: a unit's
// values only grow, so they are unchanged iff their sum equals the stored sum usum[u].
// Per recomputed row: read the op row, write the row (8n bytes).
// Word view of an LA row: int32 storage = one coordinate per 32-bit word; compact
// (uint16) storage = two coordinates per word, merged with packed 16-bit max
// (v_pk_max_u16 on the value+1 encoding).
template <typename CT>
struct LaWord;
template <>
struct LaWord<int32_t> {
    static constexpr uint32_t kNone = 0xFFFFFFFFu;   // -1
    __device__ __forceinline__ static uint32_t wmax(uint32_t a, uint32_t b) {
        return (uint32_t)max((int32_t)a, (int32_t)b);
    }
    // word i holds coordinate i; the own coordinate cl gets `own`
    __device__ __forceinline__ static uint32_t set_own(uint32_t v, int i, int cl, int32_t own) {
        return i == cl ? (uint32_t)own : v;
    }
    __device__ __forceinline__ static int64_t wsum(uint32_t v) { return (int32_t)v; }
};
template <>
struct LaWord<uint16_t> {
    static constexpr uint32_t kNone = 0u;
    typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
    __device__ __forceinline__ static uint32_t wmax(uint32_t a, uint32_t b) {
        const u16x2 m = __builtin_elementwise_max(__builtin_bit_cast(u16x2, a), __builtin_bit_cast(u16x2, b));
        return __builtin_bit_cast(uint32_t, m);
    }
    __device__ __forceinline__ static uint32_t set_own(uint32_t v, int i, int cl, int32_t own) {
        if (i != (cl >> 1)) return v;
        const uint32_t e = (uint32_t)(own + 1) & 0xFFFFu;
        return (cl & 1) ? ((v & 0xFFFFu) | (e << 16)) : ((v & 0xFFFF0000u) | e);
    }
    __device__ __forceinline__ static int64_t wsum(uint32_t v) { return (int64_t)((v & 0xFFFFu) + (v >> 16)); }
};

// LA rows as 32-bit words: nwd words per row (n for int32, n/2 for compact storage).
// VERIFY (with first): every unit is recomputed from rows that already hold lower bounds
// (k_la_wave's time segments) and marked changed only where a word actually grew; unchanged
// words are not rewritten.
template <int GS, int CPL, typename CT, bool VERIFY>
__global__ void k_la_sweep(uint32_t* __restrict__ LA, const int32_t* __restrict__ p_op,
                           const int32_t* __restrict__ p_opu, const int32_t* __restrict__ c_off,
                           const int32_t* __restrict__ c_len, const int32_t* __restrict__ c_base, int C, int n,
                           int nwd, int nseg, int seg, int first, int32_t* __restrict__ chg, int32_t stamp,
                           int64_t* __restrict__ usum, int32_t* __restrict__ out, int32_t* __restrict__ out_next,
                           const int32_t* __restrict__ c_old, int64_t u0) {
    typedef LaWord<CT> W;
    // the next sweep's counters (its slot is not read before this sweep ends)
    if (blockIdx.x == 0 && threadIdx.x == 0) { out_next[0] = 0; out_next[1] = 0; }
    const int lane = lane_id();
    const int gl = lane % GS;
    int rows = 0, nwr = 0;   // rows recomputed / units changed (counted by group lane 0)
    // grid-stride over units in time-major order (one reduction + atomic per wave)
    const int64_t nunits = (int64_t)nseg * C;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x / GS;
    for (int64_t unit = u0 + ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / GS;
         unit - (lane / GS) < nunits; unit += stride) {
        if (unit >= nunits) continue;
        const int s = (int)(unit / C), c = (int)(unit % C);
        const int len = c_len[c];
        const int k0 = s * seg;
        if (k0 >= len) continue;
        const int off = c_off[c];
        const int k1 = min(len, k0 + seg);
        // incremental DivideRounds: rows of earlier calls are final (their parents are)
        if (c_old && k1 <= c_old[c]) continue;
        if (!first) {
            // dirty iff the carry unit or an op unit of one of its rows changed last sweep
            bool d = (s > 0 && gl == 0) ? chg[unit - C] == stamp - 1 : false;
            for (int k = k0 + gl; k < k1; k += GS) {
                const int u = p_opu[off + k];
                d = d || (u >= 0 && chg[u] == stamp - 1);
            }
            const uint64_t gm = group_mask(GS, lane / GS);
            if ((__ballot(d) & gm) == 0) continue;
        }
        if (gl == 0) rows += k1 - k0;
        const int base = c_base[c], cl = c % n;
        uint32_t carry[CPL];
#pragma unroll
        for (int q = 0; q < CPL; q++) {
            const int i = gl + GS * q;
            carry[q] = (k0 > 0 && i < nwd) ? LA[(size_t)(off + k0 - 1) * nwd + i] : W::kNone;
        }
        int64_t sum = 0;
        // UB rows per batch: all their op-row loads are issued before the first use (one
        // memory round trip per batch; a whole 16-row unit when the rows are narrow)
        constexpr int UB = (CPL <= 2) ? 16 : (CPL <= 4 ? 8 : 4);
        bool grew = false;   // VERIFY: some word of the unit grew
        for (int k = k0; k < k1; k += UB) {
            uint32_t opr[UB][CPL];
            uint32_t cur[VERIFY ? UB : 1][CPL];
            int opp[UB];
#pragma unroll
            for (int u = 0; u < UB; u++) opp[u] = (k + u < k1) ? p_op[off + k + u] : -1;
#pragma unroll
            for (int u = 0; u < UB; u++) {
#pragma unroll
                for (int q = 0; q < CPL; q++) {
                    const int i = gl + GS * q;
                    opr[u][q] = (opp[u] >= 0 && i < nwd) ? LA[(size_t)opp[u] * nwd + i] : W::kNone;
                    if constexpr (VERIFY)
                        cur[u][q] = (k + u < k1 && i < nwd) ? LA[(size_t)(off + k + u) * nwd + i] : W::kNone;
                }
            }
#pragma unroll
            for (int u = 0; u < UB; u++) {
                if (k + u < k1) {
#pragma unroll
                    for (int q = 0; q < CPL; q++) {
                        const int i = gl + GS * q;
                        const uint32_t v = W::set_own(W::wmax(carry[q], opr[u][q]), i, cl, base + k + u);
                        if (i < nwd) {
                            if constexpr (VERIFY) {
                                if (v != cur[u][q]) {
                                    LA[(size_t)(off + k + u) * nwd + i] = v;
                                    grew = true;
                                }
                            } else {
                                LA[(size_t)(off + k + u) * nwd + i] = v;
                            }
                            sum += W::wsum(v);
                        }
                        carry[q] = v;
                    }
                }
            }
        }
        // group sum of the unit's values vs the stored one
        for (int o = 1; o < GS; o <<= 1) sum += __shfl_xor(sum, o);
        if constexpr (VERIFY) grew = (__ballot(grew) & group_mask(GS, lane / GS)) != 0;
        if (gl == 0) {
            if (VERIFY ? grew : (first || usum[unit] != sum)) {
                chg[unit] = stamp;
                nwr++;
            }
            usum[unit] = sum;
        }
    }
    if (GS < 64) {
        for (int o = 32; o >= 1; o >>= 1) {
            rows += __shfl_xor(rows, o);
            nwr += __shfl_xor(nwr, o);
        }
    }
    if (lane == 0) {
        if (rows) atomicAdd(out, rows);
        if (nwr) atomicAdd(out + 1, nwr);
    }
}

// inclusive max-scan over the 64 lanes of non-negative values (DPP row shifts, then row
// broadcasts 15 / 31). Unsigned with 0 as the identity, so every step folds into one
// v_max_u32_dpp (a signed scan with -1 as the identity needed a v_mov of -1 and a separate
// v_mov_dpp per step).
__device__ __forceinline__ uint32_t wave_incl_max_u(uint32_t x) {
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xf, 0xf, false));   // row_shr:1
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xf, 0xf, false));   // row_shr:2
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xf, 0xf, false));   // row_shr:4
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xf, 0xf, false));   // row_shr:8
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xa, 0xf, false));   // row_bcast:15
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xc, 0xf, false));   // row_bcast:31
    return x;
}

// ---------------------------------------------------------------------------------
// firstDescendants: FD[(d,j)][c] = min{k : LA[(c,k)][d] >= j}, written
// column-major FDT[c][pos(d,j)]. Block = (chain c, tile of FT rows, block of DB target chains).
// Each (d, j, c) is written exactly once; j beyond the chain's last LA value gets MaxInt32.
// The tile holds only the block's DB target columns of its rows, so the rows per tile need not
// shrink as n grows (round 6: n = 1 024 held all 1 024 columns of 16-row tiles, each (tile,
// target) pair's fixed cost spread over 16 rows; now 64 rows x 256 targets per block).
template <typename CT, int RPL>
__global__ void k_fd_build(const uint32_t* __restrict__ LA, CT* __restrict__ FDT, const int32_t* __restrict__ c_off,
                           const int32_t* __restrict__ c_len, const int32_t* __restrict__ c_base, int n, int nwd,
                           int FT, int64_t P, const int32_t* __restrict__ c_old, int d_lo, int d_hi, int DB, int zs) {
    typedef Coord<CT> K;
    constexpr int CPW = (int)(4 / sizeof(CT));   // coordinates per LA word
    extern __shared__ __attribute__((aligned(16))) int32_t sm[];
    const int c = blockIdx.x;
    const int len = c_len[c];
    // new positions start as none (k_init_new)
    int k0;
    if (c_old) {
        // incremental: tiles from the chain's first new row itself (not from the 64-aligned tile
        // holding it): an older row already owns every position up to its own value, so only the
        // new rows can own a position whose firstDescendant on c changes (a chunked call then
        // stages its few new rows per chain instead of up to 65)
        if (c_old[c] >= len) return;
        k0 = c_old[c] + (int)blockIdx.y * FT;
        if (k0 >= len) return;
    } else {
        const int ntiles = max(1, (len + FT - 1) / FT);
        if ((int)blockIdx.y >= ntiles) return;
        k0 = (int)blockIdx.y * FT;
    }
    // this block's target chains [db0, db1): column block blockIdx.z / zs; the zs blocks of a column
    // block split its targets (a resumed call with a few new rows per chain)
    const int zb = (int)blockIdx.z, cb = zs == 1 ? zb : zb / zs, sub = zb - cb * zs;
    const int db0 = d_lo + cb * DB, db1 = min(d_hi, db0 + DB);
    if (db0 >= db1) return;
    const int wb0 = db0 / CPW, wdw = (db1 + CPW - 1) / CPW - wb0;   // LA words of a tile row
    const int tb = wb0 * CPW;                                      // first coordinate the tile holds
    const int k1 = min(len, k0 + FT), rows = k1 - k0;
    const int off = c_off[c], base_c = c_base[c];
    const int g = c / n, cl = c % n;
    // per target chain d of the block (index d - db0), then the (FT+1)-row tile (row 0 = row
    // k0-1), rows padded to ldw words against bank conflicts of the per-d searches
    int32_t* m_len = sm;
    int32_t* m_base = m_len + DB;
    int32_t* m_off = m_base + DB;
    uint32_t* tw = (uint32_t*)(m_off + DB);
    const int ldw = wdw + 1;
    const int ld = ldw * CPW;   // in coordinates
    const CT* __restrict__ tile = (const CT*)tw;
    for (int i = threadIdx.x; i < db1 - db0; i += blockDim.x) {
        m_len[i] = c_len[g * n + db0 + i];
        m_base[i] = c_base[g * n + db0 + i];
        m_off[i] = c_off[g * n + db0 + i];
    }
    {   // words [wb0, wb0 + wdw) of rows k0-1 .. k1-1
        const int r0 = (k0 > 0) ? 0 : 1;   // tile row 0 is unused when k0 == 0
        const uint32_t* __restrict__ src = LA + (size_t)(off + k0 - 1) * nwd + wb0;
        if (wdw >= 32) {
            // straight into LDS (global_load_lds): one wave instruction = <= 64 words of one row
            typedef __attribute__((address_space(3))) void* lds_ptr_t;
            const int lane = lane_id(), wave = threadIdx.x >> 6, nwaves = blockDim.x >> 6;
            const int per_row = (wdw + 63) >> 6;
            for (int q = wave + r0 * per_row; q < (rows + 1) * per_row; q += nwaves) {
                const int rr = q / per_row, cc = (q % per_row) << 6;
                if (cc + lane < wdw)
                    __builtin_amdgcn_global_load_lds((const void*)(src + (size_t)rr * nwd + cc + lane),
                                                     (lds_ptr_t)(tw + rr * ldw + cc), 4, 0, 0);
            }
            __builtin_amdgcn_s_waitcnt(0);
        } else {
            const int nel = (rows + 1 - r0) * wdw;
            const uint32_t* __restrict__ s0 = src + (size_t)r0 * nwd;
            for (int t0 = threadIdx.x; t0 < nel; t0 += 4 * blockDim.x) {
                uint32_t v[4];
#pragma unroll
                for (int u = 0; u < 4; u++) {
                    const int tt = t0 + u * blockDim.x;
                    v[u] = (tt < nel) ? s0[(size_t)(tt / wdw) * nwd + tt % wdw] : 0u;
                }
#pragma unroll
                for (int u = 0; u < 4; u++) {
                    const int tt = t0 + u * blockDim.x;
                    if (tt < nel) tw[(tt / wdw + r0) * ldw + (tt % wdw)] = v[u];
                }
            }
        }
    }
    __syncthreads();
    const bool last = (k1 == len);
    // (wave index in an SGPR: the per-target loop bounds below are then scalar, not an exec-masked
    // loop with a VALU division)
    const int lane = lane_id(), wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), nwaves = blockDim.x >> 6;
    // per target chain d: lane k = tile row k owns d's events j in (v[k-1], v[k]]
    // (v = LA[(c, k0+k)][d], monotone in k; FD[(d,j)][c] = row k). The owner of every
    // position is found without per-lane loops: each non-empty range marks its first
    // position in a wave-private LDS slot array, and an inclusive max-scan over the 64
    // positions of a chunk carries the owner forward; then one coalesced store per 64
    // positions. (A per-lane store loop measured 9 stores and ~76 VALU per (tile, d),
    // VALU-issue-bound at 6.2 ms for c3.)
    // Per-d values are wave-uniform (SGPRs, and so is the chunk loop). The per-d scalars of up to 64 of the wave's chains are read in one LDS batch (lane q
    // holds chain d0 + nwaves*q) and taken with readlane, and the next chain's tile column is
    // read while the current one is written: no dependent LDS round trip per chain.
    int32_t* slot = sm + ((3 * DB + (FT + 1) * ldw + 1) & ~1) + 128 * wave;   // 128 positions per chunk, 8-byte aligned
    const int ownv = base_c + k0;
    const int S = __builtin_amdgcn_readfirstlane(nwaves * zs);   // target stride
    for (int d0 = __builtin_amdgcn_readfirstlane(db0 + wave + nwaves * sub); d0 < db1; d0 += S * 64) {
        const int dq = d0 + S * lane;
        int q_len = 0, q_base = 0, q_off = 0, q_lo = 0, q_hv = 0;
        if (dq < db1) {
            q_len = m_len[dq - db0];
            q_base = m_base[dq - db0];
            q_off = m_off[dq - db0];
            q_lo = (k0 > 0) ? K::la(tile[dq - tb]) : q_base - 1;
            if (rows > 0) q_hv = K::la(tile[rows * ld + dq - tb]);
        }
        const int nq = __builtin_amdgcn_readfirstlane(min(64, (db1 - d0 + S - 1) / S));
        // this lane's RPL consecutive tile rows r = RPL lane + u (tile row r + 1: row 0 is k0 - 1)
        int vnext[RPL];
#pragma unroll
        for (int u = 0; u < RPL; u++)
            vnext[u] = (RPL * lane + u < rows) ? K::la(tile[(RPL * lane + u + 1) * ld + d0 - tb]) : 0;
        for (int q = 0; q < nq; q++) {
            int vraw[RPL];
#pragma unroll
            for (int u = 0; u < RPL; u++) vraw[u] = vnext[u];
            if (q + 1 < nq) {
#pragma unroll
                for (int u = 0; u < RPL; u++)
                    if (RPL * lane + u < rows) vnext[u] = K::la(tile[(RPL * lane + u + 1) * ld + d0 + S * (q + 1) - tb]);
            }
            const int len_d = __builtin_amdgcn_readlane(q_len, q);
            if (len_d == 0) continue;
            const int base_d = __builtin_amdgcn_readlane(q_base, q);
            const int off_d = __builtin_amdgcn_readlane(q_off, q);
            int lo = __builtin_amdgcn_readlane(q_lo, q);
            if (lo < base_d - 1) lo = base_d - 1;
            const int vmax = base_d + len_d - 1;
            const int hi_val = (rows > 0) ? __builtin_amdgcn_readlane(q_hv, q) : lo;
            const int hi = last ? vmax : min(hi_val, vmax);
            CT* __restrict__ out = FDT + (size_t)cl * P + off_d - base_d;
            int v[RPL], start[RPL];
            bool own[RPL];
#pragma unroll
            for (int u = 0; u < RPL; u++) v[u] = (RPL * lane + u < rows) ? min(max(vraw[u], lo), vmax) : hi_val;
            // first position of each row's range = the previous row's v + 1 (row 0: lo + 1); the previous
            // row of a lane's first row is the last row of the lane before
            start[0] = __builtin_amdgcn_update_dpp(lo, v[RPL - 1], 0x138, 0xf, 0xf, false) + 1;   // wave_shr:1
#pragma unroll
            for (int u = 1; u < RPL; u++) start[u] = v[u - 1] + 1;
#pragma unroll
            for (int u = 0; u < RPL; u++) own[u] = RPL * lane + u < rows && v[u] >= start[u];
            const int vlast = max(lo, min(hi_val, vmax));   // end of the tile's last range
            // slots hold owner + 1 (0 = no range starts here); a chunk is 128 positions, two per lane
            // (positions j0 + 2 lane and j0 + 2 lane + 1): half the chunk iterations of one per lane
            uint32_t carry = 0;
            for (int j0 = lo + 1; j0 <= hi; j0 += 128) {   // scalar loop
                *(uint2*)(slot + 2 * lane) = make_uint2(0u, 0u);
                wave_lds_fence();
#pragma unroll
                for (int u = 0; u < RPL; u++)
                    if (own[u] && (unsigned)(start[u] - j0) < 128u) slot[start[u] - j0] = RPL * lane + u + 1;
                // past the last row (last tile only): none = MaxInt32, sentinel owner FT
                if (last && lane == 0 && (unsigned)(vlast + 1 - j0) < 128u) slot[vlast + 1 - j0] = 64 * RPL + 1;
                wave_lds_fence();
                const uint2 ab = *(const uint2*)(slot + 2 * lane);
                const uint32_t inc = wave_incl_max_u(max(ab.x, ab.y));
                // the owners before this lane's pair: the inclusive scan one lane back (lane 0: the carry)
                const uint32_t before = max((uint32_t)__builtin_amdgcn_update_dpp(0, (int)inc, 0x138, 0xf, 0xf, false), carry);
                const uint32_t oa = max(before, ab.x), ob = max(oa, ab.y);
                carry = max(carry, (uint32_t)__builtin_amdgcn_readlane((int)inc, 63));
                const int ja = j0 + 2 * lane;
                if (ja <= hi) out[ja] = K::enc_fd((int)oa - 1 < rows ? ownv + (int)oa - 1 : kMaxI32);
                if (ja + 1 <= hi) out[ja + 1] = K::enc_fd((int)ob - 1 < rows ? ownv + (int)ob - 1 : kMaxI32);
            }
        }
    }
}

// ---------------------------------------------------------------------------------
// rounds. Step r: W'_r = {first event of each chain with round >= r}.
// gather: copy the candidates' coordinate rows into compact per-round tables.
// wfd16: the WFD rows are kept as raw uint16 firstDescendants (compact coordinates),
// otherwise as decoded int32.
template <typename CT>
__global__ void k_round_gather(int r, const int32_t* __restrict__ Bm, const int32_t* __restrict__ c_off,
                               const int32_t* __restrict__ c_len, const CT* __restrict__ LA,
                               const CT* __restrict__ FDT, const int32_t* __restrict__ p_gid,
                               const uint8_t* __restrict__ g_coin, int32_t* __restrict__ WLA,
                               int32_t* __restrict__ WFD, uint8_t* __restrict__ wflag, uint8_t* __restrict__ wcoin,
                               int C, int n, int64_t P, int wfd16) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= (int64_t)C * n) return;
    const int gc = (int)(t / n), i = (int)(t % n);
    const int b = Bm[(size_t)r * C + gc];
    const int len = c_len[gc];
    const size_t wrow = ((size_t)r * C + gc) * n + i;
    if (b < len) {
        const int p = c_off[gc] + b;
        WLA[wrow] = Coord<CT>::la(LA[(size_t)p * n + i]);
        if (wfd16) ((uint16_t*)WFD)[wrow] = (uint16_t)FDT[(size_t)i * P + p];
        else WFD[wrow] = Coord<CT>::fd(FDT[(size_t)i * P + p]);
        if (i == 0) {
            wflag[(size_t)r * C + gc] = 1;
            wcoin[(size_t)r * C + gc] = g_coin[p_gid[p]];
        }
    } else if (i == 0) {
        wflag[(size_t)r * C + gc] = 0;
    }
}

// coin bit (middleBit, hashgraph.go:1039-1048: hash[16] != 0) of every round's
// candidate, gathered once after the rounds (kept off the per-round critical path)
__global__ void k_wcoin(int64_t RC, int C, const int32_t* __restrict__ Bm, const int32_t* __restrict__ c_off,
                        const int32_t* __restrict__ c_len, const int32_t* __restrict__ p_gid,
                        const uint8_t* __restrict__ g_coin, uint8_t* __restrict__ wcoin) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= RC) return;
    const int gc = (int)(t % C);
    const int b = Bm[t];
    wcoin[t] = (b < c_len[gc]) ? g_coin[p_gid[c_off[gc] + b]] : 0;
}

// ---------------------------------------------------------------------------------
// fame. S_j[y] = { w in W_{j-1} : StronglySee(y, w) } as bit masks is produced by the
// round step (hgx_rounds.hip) for the boundary event of every chain.
// vote tally and decisions (DecideFame, hashgraph.go:649-730). One block per
// (graph g, round i). Votes V[x] are bit masks over the witnesses of the previous
// round; yays = popcount(S_j[y] & V[x]). Ties vote yes; coin rounds use middleBit.
__global__ void __launch_bounds__(256) k_fame_vote(int R, int r0, int nw, const int32_t* __restrict__ lr,
                            const uint8_t* __restrict__ wstat, const uint8_t* __restrict__ wcoin,
                            const int32_t* __restrict__ Bm, const int32_t* __restrict__ c_base,
                            const int32_t* __restrict__ WLA, const uint64_t* __restrict__ Smat,
                            uint64_t* __restrict__ Vbuf, int8_t* __restrict__ fame, int C, int n, int sm) {
    __shared__ int32_t xs[1024];
    __shared__ int32_t dec[1024];
    __shared__ int32_t s_nx, s_und;
    __shared__ unsigned long long wm[16];   // witnesses of round j-1 (S rows may cover jumped candidates)
    const int RR = R - r0;
    const int g = blockIdx.x / RR, i = r0 + blockIdx.x % RR;
    const int LR = lr[g];
    if (i > LR) return;
    const size_t gi = (size_t)g * n;
    if (threadIdx.x == 0) s_nx = 0;
    __syncthreads();
    for (int c = threadIdx.x; c < n; c += blockDim.x)
        if (wstat[(size_t)i * C + gi + c] == 2) xs[atomicAdd(&s_nx, 1)] = c;
    __syncthreads();
    const int nx = s_nx;
    for (int x = threadIdx.x; x < nx; x += blockDim.x) dec[x] = 0;
    __syncthreads();
    if (i + 2 > LR) {   // no round can decide: fame stays undefined
        for (int x = threadIdx.x; x < nx; x += blockDim.x) fame[(size_t)i * C + gi + xs[x]] = 0;
        return;
    }
    // V buffers for this (g,i): [2][n][nw]
    uint64_t* V0 = Vbuf + (((size_t)i * 2 + 0) * C + gi) * nw;
    uint64_t* V1 = Vbuf + (((size_t)i * 2 + 1) * C + gi) * nw;
    // j = i+1: vote(y, x) = See(y, x) = LA[y][cr(x)] >= Index(x)
    for (int t = threadIdx.x; t < nx * nw; t += blockDim.x) {
        const int x = t / nw, wd = t % nw;
        const int xc = xs[x];
        const int32_t xidx = c_base[gi + xc] + Bm[(size_t)i * C + gi + xc];
        uint64_t bits = 0;
        for (int bb = 0; bb < 64; bb++) {
            const int y = wd * 64 + bb;
            if (y >= n) break;
            if (wstat[(size_t)(i + 1) * C + gi + y] != 2) continue;
            if (WLA[((size_t)(i + 1) * C + gi + y) * n + xc] >= xidx) bits |= 1ull << bb;
        }
        V0[(size_t)x * nw + wd] = bits;
    }
    __syncthreads();
    uint64_t* Vc = V0;
    uint64_t* Vn = V1;
    for (int j = i + 2; j <= LR; j++) {
        const bool normal = ((j - i) % n) != 0;
        const size_t jr = (size_t)j * C + gi;
        for (int k = threadIdx.x; k < nw; k += blockDim.x) wm[k] = 0;
        __syncthreads();
        for (int c = threadIdx.x; c < n; c += blockDim.x)
            if (wstat[(size_t)(j - 1) * C + gi + c] == 2) atomicOr(&wm[c >> 6], 1ull << (c & 63));
        __syncthreads();
        for (int t = threadIdx.x; t < nx * nw; t += blockDim.x) {
            const int x = t / nw, wd = t % nw;
            if (dec[x] != 0) continue;
            uint64_t bits = 0;
            for (int bb = 0; bb < 64; bb++) {
                const int y = wd * 64 + bb;
                if (y >= n) break;
                if (wstat[jr + y] != 2) continue;
                int yays = 0, tot = 0;
                for (int k = 0; k < nw; k++) {
                    const uint64_t s = Smat[(jr + y) * nw + k] & wm[k];
                    tot += __popcll(s);
                    yays += __popcll(s & Vc[(size_t)x * nw + k]);
                }
                const int nays = tot - yays;
                const bool v = yays >= nays;
                const int tt = v ? yays : nays;
                bool bit;
                if (normal) {
                    if (tt >= sm) atomicCAS(&dec[x], 0, v ? 1 : 2);
                    bit = v;
                } else {
                    bit = (tt >= sm) ? v : (wcoin[jr + y] != 0);
                }
                if (bit) bits |= 1ull << bb;
            }
            Vn[(size_t)x * nw + wd] = bits;
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            int u = 0;
            for (int x = 0; x < nx; x++) u += (dec[x] == 0);
            s_und = u;
        }
        __syncthreads();
        if (s_und == 0) break;
        uint64_t* tmp = Vc; Vc = Vn; Vn = tmp;
    }
    for (int x = threadIdx.x; x < nx; x += blockDim.x) fame[(size_t)i * C + gi + xs[x]] = (int8_t)dec[x];
}

// ---------------------------------------------------------------------------------
// fame for n >= 128 (same decisions as k_fame_vote, DecideFame hashgraph.go:649-730).
// The decision of a witness x depends on x's own votes only, so a block takes one
// (graph g, round i, tile of 64 witnesses x of round i) and walks j = i+1.. on its own:
// G*R*ceil(n/64) independent blocks instead of G*R. Per step j the tally
//   yays[y][x] = sum_w S_j[y][w] * wm_{j-1}[w] * V_{j-1}[x][w]      (y voter of round j)
// is a 0/1 matrix product (K = n witnesses of round j-1, bit-packed, 64 per word).
//   kMfma:  v_mfma_i32_16x16x64_i8. A = S rows expanded bit->byte in registers (one
//           64-bit word is one K step: lane group h takes bits [16h, 16h+16)), B = the
//           tile's votes expanded once per step into an int8 LDS image [x][w].
//   !kMfma: AND + popcount, lane = x, S words wave-uniform.
// tot[y] = popcount(S_j[y] & wm); votes of the step are OR-ed into LDS bit rows.
typedef int int4v __attribute__((ext_vector_type(4)));
constexpr int kFameTile = 64;     // witnesses x per block
constexpr int kFameMaxW = 16;     // words per bit row (n <= 1024)
constexpr int kFameSW = 4096;     // S words of a voter round staged in LDS (n <= 512)

// 16 bits -> 16 bytes of 0/1 (bit q of b -> byte q): nibble * 0x00204081 puts bits
// 0..3 at 0, 8, 16, 24 with no overlapping partial products.
__device__ __forceinline__ int4v expand16(uint32_t b) {
    int4v r;
    r[0] = (int)(((b & 0xFu) * 0x00204081u) & 0x01010101u);
    r[1] = (int)((((b >> 4) & 0xFu) * 0x00204081u) & 0x01010101u);
    r[2] = (int)((((b >> 8) & 0xFu) * 0x00204081u) & 0x01010101u);
    r[3] = (int)((((b >> 12) & 0xFu) * 0x00204081u) & 0x01010101u);
    return r;
}

// the block compacts { c < n : st[c] == 2 } into out (ascending; count to *cnt) and/or writes it
// as a bit mask (word k = chains [64k, 64k+64)): wave w takes the words w, w+4, ... (a resumed
// call's DecideFame is a chain of these per voter round: one wave walking every word serially
// was a load latency per word). All threads call it; it synchronizes once inside, the caller
// after. wcnt: LDS scratch of kFameMaxW ints.
__device__ __forceinline__ void compact_witnesses(const uint8_t* __restrict__ st, int n, int32_t* out, int* cnt,
                                                  uint64_t* mask, int* wcnt) {
    const int lane = lane_id(), wave = threadIdx.x >> 6;
    const int nwd = (n + 63) >> 6;
    uint64_t m[kFameMaxW / 4];
#pragma unroll
    for (int q = 0; q < kFameMaxW / 4; q++) {
        const int k = wave + 4 * q;
        m[q] = 0;
        if (k < nwd) {
            const int c = 64 * k + lane;
            m[q] = __ballot(c < n && st[c] == 2);
            if (lane == 0) {
                wcnt[k] = __popcll(m[q]);
                if (mask) mask[k] = m[q];
            }
        }
    }
    __syncthreads();
    int base = 0, tot = 0;
    for (int k = 0; k < nwd; k++) tot += wcnt[k];
#pragma unroll
    for (int q = 0; q < kFameMaxW / 4; q++) {
        const int k = wave + 4 * q;
        if (k < nwd && out) {
            base = 0;
            for (int k2 = 0; k2 < k; k2++) base += wcnt[k2];
            if ((m[q] >> lane) & 1ull) out[base + __popcll(m[q] & ((1ull << lane) - 1ull))] = 64 * k + lane;
        }
    }
    if (cnt && threadIdx.x == 0) *cnt = tot;
}

template <bool kMfma>
__global__ void __launch_bounds__(256) k_fame_tile(int R, int r0, int XT, const int32_t* __restrict__ lr,
                            const uint8_t* __restrict__ wstat, const uint8_t* __restrict__ wcoin,
                            const int32_t* __restrict__ Bm, const int32_t* __restrict__ c_base,
                            const int32_t* __restrict__ WLA, const uint64_t* __restrict__ Smat,
                            int8_t* __restrict__ fame, int C, int n, int nw, int sm, int sw) {
    extern __shared__ __align__(16) unsigned char fsm[];   // kMfma: int8 vote image [64][nw*64+16]
    __shared__ int32_t xs[kFameTile], dec[kFameTile], xidx[kFameTile];
    __shared__ int32_t ys[1024], ytot[1024];
    __shared__ int32_t s_ny, s_und, wcnt[kFameMaxW];
    __shared__ uint64_t wmask[2][kFameMaxW];   // witness masks of rounds j-1 / j (by parity)
    __shared__ uint64_t Vb[2][kFameTile][kFameMaxW];   // vote bit rows V[x][w] (current / next)
    // !kMfma: the dynamic LDS holds S_j[y] & wm of the round's voters (sw words; 0 = none)
    uint64_t* sS = reinterpret_cast<uint64_t*>(fsm);
    const int RR = R - r0;   // rounds [r0, R): the undecided ones and later
    const int xt = blockIdx.x % XT;
    const int i = r0 + (blockIdx.x / XT) % RR;
    const int g = blockIdx.x / (XT * RR);
    const int LR = lr[g];
    if (i > LR) return;
    const size_t gi = (size_t)g * n;
    const int lane = lane_id(), wave = threadIdx.x >> 6;
    // witnesses of round i, this block's slice
    compact_witnesses(wstat + (size_t)i * C + gi, n, ys, &s_ny, nullptr, wcnt);
    __syncthreads();
    const int nxt = min(kFameTile, s_ny - xt * kFameTile);
    if (nxt <= 0) return;
    if (threadIdx.x < kFameTile) {
        xs[threadIdx.x] = threadIdx.x < nxt ? ys[xt * kFameTile + threadIdx.x] : 0;
        dec[threadIdx.x] = 0;
    }
    __syncthreads();
    if (i + 2 > LR) {   // no round can decide: fame stays undefined
        if ((int)threadIdx.x < nxt) fame[(size_t)i * C + gi + xs[threadIdx.x]] = 0;
        return;
    }
    // j = i+1: vote(y, x) = See(y, x) = LA[y][cr(x)] >= Index(x), one (witness y of round i+1,
    // x) pair per lane: independent loads (a lane walking 64 y with a dependent witness test
    // each was most of a resumed call's DecideFame)
    compact_witnesses(wstat + (size_t)(i + 1) * C + gi, n, ys, &s_ny, wmask[(i + 1) & 1], wcnt);
    for (int t = threadIdx.x; t < kFameTile * nw; t += blockDim.x) Vb[0][t / nw][t % nw] = 0;
    if ((int)threadIdx.x < nxt) {
        const int xc = xs[threadIdx.x];
        xidx[threadIdx.x] = c_base[gi + xc] + Bm[(size_t)i * C + gi + xc];
    }
    __syncthreads();
    {
        // lane = x, wave w takes the voters w, w+4, ...: the bits gather in registers, one LDS
        // OR per word at the end
        const size_t jr = (size_t)(i + 1) * C + gi;
        const int ny1 = s_ny;
        const int x = lane;
        const int xc = x < nxt ? xs[x] : 0;
        const int32_t xi = x < nxt ? xidx[x] : 0x7FFFFFFF;
        uint64_t acc[kFameMaxW];
#pragma unroll
        for (int k = 0; k < kFameMaxW; k++) acc[k] = 0;
        for (int yi = wave; yi < ny1; yi += 4) {
            const int y = ys[yi];
            const uint64_t b = WLA[(jr + y) * n + xc] >= xi ? 1ull << (y & 63) : 0ull;
#pragma unroll
            for (int k = 0; k < kFameMaxW; k++)
                if (k == (y >> 6)) acc[k] |= b;
        }
        if (x < nxt)
#pragma unroll
            for (int k = 0; k < kFameMaxW; k++)
                if (k < nw && acc[k]) atomicOr((unsigned long long*)&Vb[0][x][k], acc[k]);
    }
    __syncthreads();
    const int KB = nw * 64 + 16;   // int8 image row stride (16-B pad: 16 lanes of one x-group hit distinct banks)
    int cur = 0;
    for (int j = i + 2; j <= LR; j++) {
        const bool normal = ((j - i) % n) != 0;
        const size_t jr = (size_t)j * C + gi;
        const uint64_t* wm = wmask[(j - 1) & 1];   // witnesses of round j-1 (S rows may cover jumped candidates)
        for (int t = threadIdx.x; t < kFameTile * nw; t += blockDim.x) Vb[cur ^ 1][t / nw][t % nw] = 0;
        compact_witnesses(wstat + jr, n, ys, &s_ny, wmask[j & 1], wcnt);
        __syncthreads();
        const int ny = s_ny;
        // the voters' S rows (masked to the witnesses of j-1) staged in LDS by all lanes at once:
        // the tally then reads them as broadcasts instead of one dependent HBM row per voter
        const bool s_lds = !kMfma && ny * nw <= sw;
        if (s_lds) {
            for (int t = threadIdx.x; t < ny * nw; t += blockDim.x) {
                const int y = t / nw, k = t - y * nw;
                sS[t] = Smat[(jr + ys[y]) * nw + k] & wm[k];
            }
            __syncthreads();
        }
        // tot[y] = #{w witness of j-1 : S_j[y][w]}
        for (int t = threadIdx.x; t < ny; t += blockDim.x) {
            int tot = 0;
            if (s_lds) {
                for (int k = 0; k < nw; k++) tot += __popcll(sS[t * nw + k]);
            } else {
                const uint64_t* srow = Smat + (jr + ys[t]) * nw;
                for (int k = 0; k < nw; k++) tot += __popcll(srow[k] & wm[k]);
            }
            ytot[t] = tot;
        }
        if constexpr (kMfma) {
            // int8 image of the current votes: byte [x][w] = bit w of V[x]
            int* img = reinterpret_cast<int*>(fsm);
            for (int t = threadIdx.x; t < kFameTile * nw * 16; t += blockDim.x) {
                const int x = t / (nw * 16), q = t % (nw * 16);   // q: 4-byte group of the row
                const uint32_t nib = (uint32_t)(Vb[cur][x][q >> 4] >> ((q & 15) * 4)) & 0xFu;
                img[(x * KB >> 2) + q] = (int)((nib * 0x00204081u) & 0x01010101u);
            }
        }
        __syncthreads();
        auto vote = [&](int yi, int x, int yays) {
            const int y = ys[yi];
            const int nays = ytot[yi] - yays;
            const bool v = yays >= nays;
            const int tt = v ? yays : nays;
            bool bit;
            if (normal) {
                if (tt >= sm) atomicCAS(&dec[x], 0, v ? 1 : 2);
                bit = v;
            } else {
                bit = (tt >= sm) ? v : (wcoin[jr + y] != 0);
            }
            if (bit) atomicOr((unsigned long long*)&Vb[cur ^ 1][x][y >> 6], 1ull << (y & 63));
        };
        if constexpr (kMfma) {
            // wave: 32 voter rows (2 row tiles) x 64 witnesses (4 column tiles) per pass
            const int h = lane >> 4, r16 = lane & 15;
            const signed char* img = reinterpret_cast<const signed char*>(fsm);
            for (int rp = wave; rp * 32 < ny; rp += 4) {
                int4v acc[2][4];
#pragma unroll
                for (int a = 0; a < 2; a++)
#pragma unroll
                    for (int b = 0; b < 4; b++) acc[a][b] = int4v{0, 0, 0, 0};
                const int yi0 = rp * 32 + r16, yi1 = yi0 + 16;
                const uint64_t* s0 = yi0 < ny ? Smat + (jr + ys[yi0]) * nw : nullptr;
                const uint64_t* s1 = yi1 < ny ? Smat + (jr + ys[yi1]) * nw : nullptr;
                for (int k = 0; k < nw; k++) {
                    const uint64_t w0 = s0 ? (s0[k] & wm[k]) : 0ull;
                    const uint64_t w1 = s1 ? (s1[k] & wm[k]) : 0ull;
                    const int4v a0 = expand16((uint32_t)(w0 >> (16 * h)) & 0xFFFFu);
                    const int4v a1 = expand16((uint32_t)(w1 >> (16 * h)) & 0xFFFFu);
#pragma unroll
                    for (int b = 0; b < 4; b++) {
                        const int4v bf = *reinterpret_cast<const int4v*>(img + (b * 16 + r16) * KB + k * 64 + 16 * h);
                        acc[0][b] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a0, bf, acc[0][b], 0, 0, 0);
                        acc[1][b] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a1, bf, acc[1][b], 0, 0, 0);
                    }
                }
                // C/D: column x = 16b + (lane & 15), row = 4 (lane >> 4) + q
#pragma unroll
                for (int a = 0; a < 2; a++)
#pragma unroll
                    for (int b = 0; b < 4; b++)
#pragma unroll
                        for (int q = 0; q < 4; q++) {
                            const int yi = rp * 32 + a * 16 + 4 * h + q, x = b * 16 + r16;
                            if (yi < ny && x < nxt) vote(yi, x, acc[a][b][q]);
                        }
            }
        } else {
            // lane = witness x; S words are wave-uniform
            const int x = lane;
            uint64_t vx[kFameMaxW];
#pragma unroll
            for (int k = 0; k < kFameMaxW; k++) vx[k] = k < nw ? Vb[cur][x][k] : 0ull;
            for (int yi = wave; yi < ny; yi += 4) {
                int yays = 0;
                if (s_lds) {
                    const uint64_t* srow = sS + yi * nw;
#pragma unroll
                    for (int k = 0; k < kFameMaxW; k++)
                        if (k < nw) yays += __popcll(srow[k] & vx[k]);
                } else {
                    const uint64_t* srow = Smat + (jr + ys[yi]) * nw;
#pragma unroll
                    for (int k = 0; k < kFameMaxW; k++)
                        if (k < nw) yays += __popcll(srow[k] & wm[k] & vx[k]);
                }
                if (x < nxt) vote(yi, x, yays);
            }
        }
        __syncthreads();
        if (threadIdx.x < 64) {
            const bool u = (int)threadIdx.x < nxt && dec[threadIdx.x] == 0;
            const uint64_t m = __ballot(u);
            if (threadIdx.x == 0) s_und = __popcll(m);
        }
        __syncthreads();
        if (s_und == 0) break;
        cur ^= 1;
    }
    if ((int)threadIdx.x < nxt) fame[(size_t)i * C + gi + xs[threadIdx.x]] = (int8_t)dec[threadIdx.x];
}

// ---------------------------------------------------------------------------------
// WLAT[i][g][d][c] = WLA[i][g][c][d]: per round, the lastAncestors of the candidates
// transposed so that "which witnesses of round i see chain d up to index j" is one
// contiguous row (k_threshold, k_cts_*). 64 x 64 tiles through LDS; eligible rounds only.
// The famous flag is folded in: the row of a witness that is not famous (or no witness) holds
// kWlatNotFamous, below every Index and every lastAncestors value (-1 = sees none of d).
__global__ void __launch_bounds__(256) k_wla_transpose(int R, int r0, int G, int C, int n,
                                                       const uint8_t* __restrict__ elig, const uint8_t* __restrict__ fw,
                                                       const int32_t* __restrict__ WLA, int32_t* __restrict__ WLAT) {
    __shared__ int32_t t[64][65];
    const int ig = blockIdx.y, i = r0 + ig / G, g = ig % G;
    if (!elig[(size_t)g * R + i]) return;
    const int nt = (n + 63) / 64, tc = blockIdx.x % nt, td = blockIdx.x / nt;
    const size_t base = ((size_t)i * C + (size_t)g * n) * n;
    if ((n & 63) == 0) {   // whole 64 x 64 tiles: 16-byte loads and stores (thread = 4 coordinates x 4 rows)
        const uint8_t* __restrict__ fwr = fw + (size_t)i * C + (size_t)g * n + tc * 64;
        const int c4 = (threadIdx.x & 15) * 4, r4 = threadIdx.x >> 4;   // 16 threads per 256-byte row
#pragma unroll
        for (int h = 0; h < 4; h++) {
            const int r = r4 + 16 * h;   // candidate tc * 64 + r, coordinates td * 64 + c4 ..
            const int4 v = *(const int4*)(WLA + base + (size_t)(tc * 64 + r) * n + td * 64 + c4);
            const bool f = fwr[r] != 0;
            t[r][c4] = f ? v.x : kWlatNotFamous;
            t[r][c4 + 1] = f ? v.y : kWlatNotFamous;
            t[r][c4 + 2] = f ? v.z : kWlatNotFamous;
            t[r][c4 + 3] = f ? v.w : kWlatNotFamous;
        }
        __syncthreads();
#pragma unroll
        for (int h = 0; h < 4; h++) {
            const int d = r4 + 16 * h;   // coordinate td * 64 + d, candidates tc * 64 + c4 ..
            *(int4*)(WLAT + base + (size_t)(td * 64 + d) * n + tc * 64 + c4) =
                make_int4(t[c4][d], t[c4 + 1][d], t[c4 + 2][d], t[c4 + 3][d]);
        }
        return;
    }
    for (int k = threadIdx.x; k < 64 * 64; k += 256) {
        const int r = k >> 6, col = k & 63, c = tc * 64 + r, d = td * 64 + col;
        t[r][col] = (c < n && d < n) ? (fw[(size_t)i * C + (size_t)g * n + c] ? WLA[base + (size_t)c * n + d]
                                                                               : kWlatNotFamous) : 0;
    }
    __syncthreads();
    for (int k = threadIdx.x; k < 64 * 64; k += 256) {
        const int r = k >> 6, col = k & 63, d = td * 64 + r, c = tc * 64 + col;
        if (c < n && d < n) WLAT[base + (size_t)d * n + c] = t[col][r];
    }
}

// round received: T[i][d] = (m/2+1)-th largest LA[w][d] over famous witnesses w of
// round i (DecideRoundReceived hashgraph.go:767-775). One wave per (i, d),
// reading the contiguous WLAT row.
template <int CPL>
__global__ void __launch_bounds__(256) k_threshold(int R, int r0, const uint8_t* __restrict__ elig,
                            const uint8_t* __restrict__ fw,
                            const int32_t* __restrict__ WLAT, int32_t* __restrict__ T, int C, int n) {
    const int64_t item = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    if (item >= (int64_t)(R - r0) * C) return;
    const int i = r0 + (int)(item / C), gd = (int)(item % C);
    const int g = gd / n;
    if (!elig[(size_t)g * R + i]) return;
    const int lane = lane_id();
    const size_t row = ((size_t)i * C + gd) * n;
    uint32_t v[CPL];   // int32 order as u32: sign bit flipped
    bool ok[CPL];
    int m = 0;
#pragma unroll
    for (int q = 0; q < CPL; q++) {
        const int c = lane + 64 * q;
        const int32_t x = c < n ? WLAT[row + c] : kWlatNotFamous;
        ok[q] = x != kWlatNotFamous;
        v[q] = (uint32_t)x ^ 0x80000000u;
        m += __popcll(__ballot(ok[q]));
    }
    int32_t res = -1;
    if (m > 0) {   // (m/2)-th largest = (m-1-m/2)-th smallest
        const uint32_t u = wave_select_kth32_bisect<CPL>(v, ok, m - 1 - m / 2);
        res = (int32_t)(u ^ 0x80000000u);
    }
    if (lane == 0) T[(size_t)i * C + gd] = res;
}

// rr(x) = first eligible i > round(x) with Index(x) <= T[i][cr(x)]; compacts the
// newly received positions (block-aggregated append). Block = (tile of 256, chain c) over
// the chain's events not received by an earlier call, [fu[c], len[c]). The received events
// of a chain are always a prefix of it: a famous witness that sees x sees x's self-parent,
// so rr(self-parent) <= rr(x) under the same eligible rounds (hashgraph.go:753-799). So the
// newly received events of chain c are [fu[c], fu[c] + rcnt[c]).
// A block takes kRrPer x 256 consecutive positions of one chain (thread t: t, t + 256, ...); the received
// lanes of each batch get their slots from the waves' ballots (no LDS atomics), and the block appends
// once to the global list (one global atomic per kRrPer x 256 events: at c3 39 k blocks with one
// returning atomic each on the same word were the kernel's tail).
constexpr int kRrPer = 4;
__global__ void __launch_bounds__(256) k_round_received(int R, const int32_t* __restrict__ c_off,
                                 const int32_t* __restrict__ c_len, const int32_t* __restrict__ c_base,
                                 const int32_t* __restrict__ fu, const int32_t* __restrict__ p_round,
                                 const int32_t* __restrict__ lr, const uint8_t* __restrict__ elig,
                                 const uint8_t* __restrict__ ur_empty, const int32_t* __restrict__ T,
                                 int32_t* __restrict__ p_rr, int32_t* __restrict__ rcnt, int32_t* __restrict__ recv_list,
                                 int32_t* __restrict__ counters, int C, int n) {
    __shared__ int32_t s_wcnt[kRrPer][4], s_base;
    const int gc = blockIdx.y;
    const int f = fu[gc];
    const int len = c_len[gc];
    const int k0 = f + blockIdx.x * (256 * kRrPer);
    if (k0 >= len) return;   // block-uniform
    const int g = gc / n;
    const int LR = lr[g];
    const int64_t co = c_off[gc];
    const int jb = c_base[gc];
    const int w = threadIdx.x >> 6;
    const uint8_t* el = elig + (size_t)g * R;
    bool got[kRrPer];
    uint32_t below[kRrPer];   // received lanes of this wave below this lane, per batch
#pragma unroll
    for (int q = 0; q < kRrPer; q++) {
        const int k = k0 + q * 256 + (int)threadIdx.x;
        got[q] = false;
        if (k < len) {
            const int64_t p = co + k;
            const int j = jb + k;
            const int r = p_round[p];
            if (r + 1 <= LR && ur_empty[g]) atomicOr(&counters[1], 1);   // Go panics on UndecidedRounds[0]
            for (int i = r + 1; i <= LR; i++) {
                if (el[i] && j <= T[(size_t)i * C + gc]) {
                    p_rr[p] = i;
                    got[q] = true;
                    break;
                }
            }
        }
        const uint64_t b = __ballot(got[q]);
        below[q] = (uint32_t)__builtin_amdgcn_mbcnt_hi((uint32_t)(b >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)b, 0u));
        if (lane_id() == 0) s_wcnt[q][w] = __popcll(b);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        int tot = 0;
        for (int q = 0; q < kRrPer; q++)
            for (int v = 0; v < 4; v++) { const int c = s_wcnt[q][v]; s_wcnt[q][v] = tot; tot += c; }   // exclusive
        s_base = tot ? atomicAdd(&counters[0], tot) : 0;
        if (tot) atomicAdd(&rcnt[gc], tot);
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < kRrPer; q++)
        if (got[q]) recv_list[s_base + s_wcnt[q][w] + (int)below[q]] = (int32_t)(co + k0 + q * 256 + (int)threadIdx.x);
}

// fu[c] += rcnt[c] after the order of a FindOrder is written
__global__ void k_fu_advance(int C, int32_t* __restrict__ fu, const int32_t* __restrict__ rcnt) {
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c < C) fu[c] += rcnt[c];
}

// fu[c] = events of chain c already received (a prefix, see k_round_received): after a
// rebuild of the layout, from the gid-order roundReceived
__global__ void k_fu_count(int64_t E, const int32_t* __restrict__ g_creator, const int32_t* __restrict__ g_rr,
                           int32_t* __restrict__ fu) {
    const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (gid < E && g_rr[gid] >= 0) atomicAdd(&fu[g_creator[gid]], 1);
}

// new rows of an incremental DivideRounds start as none: LA rows (read before they are
// computed by the sweeps) and FD entries (no chain has seen the new events yet)
template <typename CT>
__global__ void __launch_bounds__(256) k_init_new(int64_t E0, int64_t m, const int32_t* __restrict__ g_pos,
                                                  CT* __restrict__ LA, CT* __restrict__ FDT, int n, int64_t P) {
    // a tile of 16 new events x 64 observers per workgroup: the lastAncestors rows with the
    // observer fastest, the firstDescendants entries with the event fastest (a chain's new
    // positions are adjacent)
    __shared__ int32_t s_pos[16];
    const int64_t k0 = (int64_t)blockIdx.x * 16;
    const int kn = (int)min<int64_t>(16, m - k0);
    const int i0 = blockIdx.y * 64;
    if ((int)threadIdx.x < kn) s_pos[threadIdx.x] = g_pos[E0 + k0 + threadIdx.x];
    __syncthreads();
    for (int t = threadIdx.x; t < 16 * 64; t += blockDim.x) {
        const int k = t >> 6, i = i0 + (t & 63);
        if (k < kn && i < n) LA[(size_t)s_pos[k] * n + i] = Coord<CT>::enc_la(-1);
        const int k2 = t & 15, i2 = i0 + (t >> 4);
        if (k2 < kn && i2 < n) FDT[(size_t)i2 * P + s_pos[k2]] = Coord<CT>::enc_fd(kMaxI32);
    }
}

// consensus timestamp: upper median (ByTimestamp, index floor(|s|/2), event.go:227-237)
// of the timestamps of OldestSelfAncestorToSee(a, x) = FD[x][cr(a)] over the famous
// witnesses a of round rr(x) that see x (hashgraph.go:141-167, 780-787, 860-868).
// "a sees x" is WLAT[rr][cr(x)][cr(a)] >= Index(x); the value is the timestamp of
// event (cr(a), FD[x][cr(a)]). The median VALUE does not depend on how ties are ordered.

// n <= 32: one lane per event; FDT[c][p] over consecutive p is coalesced, the
// selection is a rank count over <= 32 values in registers.
template <int NP, typename CT>
__global__ void __launch_bounds__(256) k_cts_small(const int32_t* __restrict__ fu, const int32_t* __restrict__ rcnt,
                                                   const int32_t* __restrict__ p_rr,
                                                   const int32_t* __restrict__ c_off, const int32_t* __restrict__ c_base,
                                                   const uint8_t* __restrict__ fw, const int32_t* __restrict__ WLAT,
                                                   const CT* __restrict__ FDT, const int64_t* __restrict__ p_ts,
                                                   int64_t* __restrict__ p_cts, int C, int n, int64_t Pcap, int c_lo) {
    const int gc = c_lo + blockIdx.y;
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= rcnt[gc]) return;
    const int g = gc / n;
    const int64_t p = (int64_t)c_off[gc] + fu[gc] + e;
    const int j = c_base[gc] + fu[gc] + e;
    const int i = p_rr[p];
    const size_t row = ((size_t)i * C + gc) * n;
    int64_t v[NP];
    uint32_t ok = 0;
#pragma unroll
    for (int c = 0; c < NP; c++) {
        v[c] = 0;
        if (c < n && WLAT[row + c] >= j) {
            const int ch = g * n + c;
            v[c] = p_ts[c_off[ch] - c_base[ch] + Coord<CT>::fd(FDT[(size_t)c * Pcap + p])];
            ok |= 1u << c;
        }
    }
    const int K = __popc(ok) / 2;
    int64_t res = 0;
#pragma unroll
    for (int a = 0; a < NP; a++) {
        int rank = 0;
#pragma unroll
        for (int b = 0; b < NP; b++)
            rank += (((ok >> b) & 1u) && (v[b] < v[a] || (v[b] == v[a] && b < a))) ? 1 : 0;
        if (((ok >> a) & 1u) && rank == K) res = v[a];
    }
    p_cts[p] = res;
}

// n > 32: a block owns T = kCtsTile consecutive positions of one chain (mostly one round
// received). Phase 1, lanes = events: for each witness chain c the T FD values
// FDT[c][p0..p0+T) are one segment, and since firstDescendants are monotone along
// a chain the T timestamp gathers p_ts[pos(c, FD)] hit one or two lines. The kernel is
// bound by the dependent FD -> timestamp latency per tile, not by bytes: smaller tiles
// keep more blocks (and tiles) in flight per CU. Values are
// kept in LDS as 32-bit offsets from the event's own timestamp (an event whose offsets
// do not fit is flagged and redone from global memory in 64 bits). Phase 2, one wave
// per event: radix select of element floor(m/2) in registers.
constexpr int kCtsTile = 8;   // c3: 10.77 ms at 32 positions, 10.35 at 16, 10.05 at 8 (round 2); 4: 13.4 vs 8.2 (round 3);
                              // round 4 (two levels, runs): 8 -> 7.2 ms, 16 -> 7.6, 4 -> 13.6
template <int NPAD, typename CT>
__global__ void __launch_bounds__(256) k_cts_tile(const int32_t* __restrict__ fu, const int32_t* __restrict__ rcnt,
                                                  const int32_t* __restrict__ p_rr,
                                                  const int32_t* __restrict__ c_off, const int32_t* __restrict__ c_base,
                                                  const uint8_t* __restrict__ fw, const int32_t* __restrict__ WLAT,
                                                  const CT* __restrict__ FDT, const int64_t* __restrict__ p_ts,
                                                  int64_t* __restrict__ p_cts, int C, int n, int64_t Pcap, int c_lo,
                                                  int c_cnt) {
    constexpr int T = kCtsTile;
    constexpr int LD = T + 1;                     // row stride of vals (bank spread)
    constexpr int CPL = NPAD / 64;
    extern __shared__ __attribute__((aligned(16))) uint32_t vals[];   // [NPAD][LD] offsets + 2^31
    __shared__ uint32_t mem[T][NPAD / 32];         // membership bits per event
    __shared__ int32_t e_row[T];
    __shared__ int64_t e_ts[T];
    __shared__ int32_t e_ovf[T];
    __shared__ __attribute__((aligned(16))) uint32_t whist[4][256];
    // time-major tiles over the newly received events [fu, fu + rcnt) of each chain, so the blocks
    // in flight cover every chain at about the same time and their timestamp gathers (events of
    // other chains at that time) share lines in L2.
    // XCD-grouped: blocks b and b + 8 share an XCD (MI355X_MICROARCH.md), so XCD x = b % 8 takes the
    // chains = x (mod 8) and runs the 8 tiles of one chain that share its FD lines (8 x 8 positions
    // = 128 bytes of a column) as 8 consecutive blocks of its own: a line is fetched into that
    // XCD's L2 once instead of once per tile (the 256 lines of a tile across all chains exceed an
    // L2 before the chain's next tile comes round in a plain time-major order: c3 7.29 -> 7.14 ms,
    // c5 3.29 -> 3.07)
    const unsigned bx = blockIdx.x, x8 = bx & 7u, k8 = bx >> 3, r8 = k8 & 7u, k64 = k8 >> 3;
    const unsigned cpx = ((unsigned)c_cnt + 7u) >> 3;
    const int cl = (int)((k64 % cpx) * 8u + x8);
    if (cl >= c_cnt) return;
    const int tc = c_lo + cl, tt = (int)((k64 / cpx) * 8u + r8);
    const int64_t q0 = (int64_t)c_off[tc] + fu[tc];
    const int64_t p0 = q0 + (int64_t)tt * T, pend = q0 + rcnt[tc];
    if (p0 >= pend) return;   // (block-uniform) no event in this tile
    // phase 1: lane = event e (32 per half-wave), 8 chain groups over the block. Two dependent
    // global levels per tile: (1) the event's round received and timestamp, the FD values of its
    // chains and the chains' position bases; (2) the famous witnesses' lastAncestors (WLAT row of
    // the round received) beside the timestamp gathers, whose positions need only the FD values
    // (an FD of a chain that turns out not to be a member gathers a valid timestamp, masked
    // after). Round 3 read rr / ts in a first level and WLAT and FD in a second, so the gathers
    // were a third level.
    constexpr int NG = 256 / T;                                  // chain groups
    const int e = threadIdx.x & (T - 1), cg = threadIdx.x / T;   // cg in [0, NG)
    const int64_t p = p0 + e;
    const bool ev = p < pend;
    const int64_t pl = ev ? p : p0;   // a valid position for the loads of a missing event
    const int i = p_rr[pl];
    const int64_t base = p_ts[pl];
    const int g = tc / n;
    const int j = c_base[tc] + (int)(pl - c_off[tc]);
    // runs of U consecutive chains per thread, every load of a level issued before anything waits
    // for it (branch-free: non-members load valid dummy addresses and are masked). The kernel is
    // bound by its vector-memory instruction count (the no-gather / no-select builds: 8.6 ms with
    // everything, 8.1 without the selects, 4.9 without the gathers too), so the per-chain terms a
    // thread needs for a run (its chains' position bases c_off - c_base and the WLAT row) are
    // 16-byte loads, and a run's membership bits are one LDS atomic. The FD values, the chain
    // bases and the gathered timestamps of a run are live at once: runs of at most 8 chains (16 at
    // n = 1 024: 227 VGPRs, 2 waves per SIMD, c5 4.2 against 3.7 ms).
    constexpr int U = (NPAD / NG < 8) ? NPAD / NG : 8;
    constexpr int NB = NPAD / (NG * U);   // runs per thread (n <= NPAD)
    constexpr int NBP = NB < 16 / U ? NB : (16 / U > 0 ? 16 / U : 1);   // runs loaded in level 1
    static_assert(U == 2 || U % 4 == 0, "k_cts_tile: runs of 2 or of a multiple of 4 chains");
    const bool vec = (n & (U == 2 ? 1 : 3)) == 0;   // rows and runs 8- / 16-byte aligned
    // o[u] = src[c0 + u] for the run's chains below n (src[0] past n)
    auto ld_run = [&](const int32_t* __restrict__ src, int c0, int32_t (&o)[U]) {
        if (vec && c0 + U <= n) {
            if constexpr (U == 2) {
                const int2 v = *(const int2*)(src + c0);
                o[0] = v.x; o[1] = v.y;
            } else {
#pragma unroll
                for (int k = 0; k < U / 4; k++) {
                    const int4 v = ((const int4*)(src + c0))[k];
                    o[4 * k] = v.x; o[4 * k + 1] = v.y; o[4 * k + 2] = v.z; o[4 * k + 3] = v.w;
                }
            }
        } else {
#pragma unroll
            for (int u = 0; u < U; u++) o[u] = src[c0 + u < n ? c0 + u : 0];
        }
    };
    int32_t fdv[U][NBP], kdv[U][NBP];
    auto load_fd = [&](int bq, int32_t (&f)[U], int32_t (&kd)[U]) {
        const int c0 = (bq * NG + cg) * U;
#pragma unroll
        for (int u = 0; u < U; u++) {
            const int cc = c0 + u < n ? c0 + u : 0;
            f[u] = Coord<CT>::fd(FDT[(size_t)cc * Pcap + pl]);
        }
        int32_t co[U], cb[U];
        ld_run(c_off + g * n, c0, co);
        ld_run(c_base + g * n, c0, cb);
#pragma unroll
        for (int u = 0; u < U; u++) kd[u] = co[u] - cb[u];
    };
#pragma unroll
    for (int bq = 0; bq < NBP; bq++) {
        int32_t f[U], kd[U];
        load_fd(bq, f, kd);
#pragma unroll
        for (int u = 0; u < U; u++) { fdv[u][bq] = f[u]; kdv[u][bq] = kd[u]; }
    }
    // the membership words start empty; e_ovf too (after this barrier every wave may set them).
    // An LDS-only barrier: the loads above stay in flight across it.
    for (int k = threadIdx.x; k < T * (NPAD / 32); k += 256) mem[k / (NPAD / 32)][k % (NPAD / 32)] = 0;
    if (threadIdx.x < T) {
        e_row[e] = (ev && i >= 0) ? i : -1;
        e_ts[e] = base;
        e_ovf[e] = 0;
    }
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    {
        const bool evi = ev && i >= 0;
        const int32_t* __restrict__ wrow = WLAT + ((size_t)(evi ? i : 0) * C + tc) * n;   // WLAT row (i, chain of the event)
        bool ovf = false;
#pragma unroll
        for (int bq = 0; bq < NB; bq++) {
            const int c0 = (bq * NG + cg) * U;
            int32_t w[U];
            int64_t x[U];
            ld_run(wrow, c0, w);
            int32_t f[U], kd[U];
            if (bq < NBP) {
#pragma unroll
                for (int u = 0; u < U; u++) { f[u] = fdv[u][bq < NBP ? bq : 0]; kd[u] = kdv[u][bq < NBP ? bq : 0]; }
            } else {
                load_fd(bq, f, kd);   // (n > 512: a third level for the later runs)
            }
#pragma unroll
            for (int u = 0; u < U; u++) x[u] = p_ts[f[u] != kMaxI32 ? kd[u] + f[u] : 0];
            uint32_t bits = 0;   // the run's membership bits (a run of <= 8 chains lies in one 32-bit word)
#pragma unroll
            for (int u = 0; u < U; u++) {
                const int c = c0 + u;
                // a member's FD exists: its famous witness descends from the event
                const bool ok = evi && c < n && w[u] >= j;
                const int64_t dlt = x[u] - base;
                ovf |= ok && (dlt < INT32_MIN || dlt > INT32_MAX);
                if (c < n) vals[c * LD + e] = (uint32_t)(int32_t)dlt ^ 0x80000000u;
                bits |= (ok ? 1u : 0u) << u;
            }
            if (bits) atomicOr(&mem[e][c0 >> 5], bits << (c0 & 31));
        }
        if (ovf) e_ovf[e] = 1;
    }
    __syncthreads();
    // phase 2: one wave per event
    const int lane = lane_id(), wave = threadIdx.x >> 6;
    for (int e = wave; e < T; e += 4) {
        if (e_row[e] < 0) continue;   // wave-uniform
        bool ok[CPL];
        int m = 0;
#pragma unroll
        for (int q = 0; q < CPL; q++) {
            const int c = lane + 64 * q;
            ok[q] = c < n && ((mem[e][c >> 5] >> (c & 31)) & 1u);
            m += __popcll(__ballot(ok[q]));
        }
        int64_t res;
        if (!e_ovf[e]) {
            uint32_t v[CPL];
#pragma unroll
            for (int q = 0; q < CPL; q++) v[q] = vals[(lane + 64 * q) * LD + e];
            const uint32_t u = wave_select_kth32<CPL>(v, ok, m / 2, whist[wave]);
            res = e_ts[e] + (int64_t)(int32_t)(u ^ 0x80000000u);
        } else {   // rare: offsets beyond 32 bits -> regather and select in 64 bits
            const int64_t p = p0 + e;
            const int g = tc / n;
            uint64_t v[CPL];
#pragma unroll
            for (int q = 0; q < CPL; q++) {
                const int c = lane + 64 * q;
                int64_t x = 0;
                if (ok[q]) {
                    const int ch = g * n + c;
                    x = p_ts[c_off[ch] - c_base[ch] + Coord<CT>::fd(FDT[(size_t)c * Pcap + p])];
                }
                v[q] = (uint64_t)x ^ 0x8000000000000000ull;
            }
            res = (int64_t)(wave_select_kth<CPL>(v, ok, m / 2, whist[wave]) ^ 0x8000000000000000ull);
        }
        if (lane == 0) p_cts[p0 + e] = res;
    }
}

// ---------------------------------------------------------------------------------
// order: LSD radix sort (8-bit digits) of (u64 key, u32 value), stable.
constexpr int kSortThreads = 256;
constexpr int kSortItems = 8;
constexpr int kSortTile = kSortThreads * kSortItems;

__global__ void __launch_bounds__(kSortThreads) k_radix_hist(const uint64_t* __restrict__ keys, int32_t m, int shift,
                                                             uint32_t* __restrict__ hist, int nblocks) {
    __shared__ uint32_t h[256];
    h[threadIdx.x] = 0;
    __syncthreads();
    for (int s = 0; s < kSortItems; s++) {
        const int idx = blockIdx.x * kSortTile + s * kSortThreads + threadIdx.x;
        if (idx < m) atomicAdd(&h[(keys[idx] >> shift) & 255], 1u);
    }
    __syncthreads();
    hist[(size_t)threadIdx.x * nblocks + blockIdx.x] = h[threadIdx.x];
}

// exclusive scan of `total` u32 in place: per-2048 chunk sums, scan of the sums in
// one block, then per-chunk rescan with the chunk offset.
constexpr int kScanChunk = 2048;

__device__ __forceinline__ uint32_t block_excl_scan256(uint32_t v, uint32_t* sh, uint32_t* total) {
    // 256 threads: wave-level inclusive scan by shuffles, then wave totals
    const int lane = lane_id(), wave = threadIdx.x >> 6;
    uint32_t x = v;
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(x, o);
        if (lane >= o) x += y;
    }
    if (lane == 63) sh[wave] = x;
    __syncthreads();
    uint32_t wbase = 0;
    for (int w = 0; w < wave; w++) wbase += sh[w];
    *total = sh[0] + sh[1] + sh[2] + sh[3];
    __syncthreads();
    return wbase + x - v;
}

__global__ void __launch_bounds__(256) k_scan_reduce(const uint32_t* __restrict__ a, int64_t total,
                                                     uint32_t* __restrict__ part) {
    __shared__ uint32_t sh[4];
    const int64_t base = (int64_t)blockIdx.x * kScanChunk;
    uint32_t s = 0;
    for (int k = threadIdx.x; k < kScanChunk; k += 256)
        if (base + k < total) s += a[base + k];
    for (int o = 32; o >= 1; o >>= 1) s += __shfl_xor(s, o);
    if (lane_id() == 0) sh[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) part[blockIdx.x] = sh[0] + sh[1] + sh[2] + sh[3];
}

__global__ void __launch_bounds__(256) k_scan_top(uint32_t* __restrict__ part, int nparts) {
    __shared__ uint32_t sh[4];
    uint32_t carry = 0;
    for (int b0 = 0; b0 < nparts; b0 += 256) {
        const int k = b0 + threadIdx.x;
        const uint32_t v = (k < nparts) ? part[k] : 0u;
        uint32_t tot;
        const uint32_t ex = block_excl_scan256(v, sh, &tot);
        if (k < nparts) part[k] = carry + ex;
        carry += tot;
    }
}

__global__ void __launch_bounds__(256) k_scan_down(uint32_t* __restrict__ a, int64_t total,
                                                   const uint32_t* __restrict__ part) {
    __shared__ uint32_t sh[4];
    constexpr int IT = kScanChunk / 256;
    const int64_t base = (int64_t)blockIdx.x * kScanChunk + (int64_t)threadIdx.x * IT;
    uint32_t v[IT];
    uint32_t s = 0;
#pragma unroll
    for (int k = 0; k < IT; k++) {
        v[k] = (base + k < total) ? a[base + k] : 0u;
        s += v[k];
    }
    uint32_t tot;
    uint32_t run = part[blockIdx.x] + block_excl_scan256(s, sh, &tot);
#pragma unroll
    for (int k = 0; k < IT; k++) {
        if (base + k < total) a[base + k] = run;
        run += v[k];
    }
}

__global__ void __launch_bounds__(kSortThreads) k_radix_scatter(const uint64_t* __restrict__ kin, const uint32_t* __restrict__ vin,
                                                                int32_t m, int shift, const uint32_t* __restrict__ hist,
                                                                int nblocks, uint64_t* __restrict__ kout,
                                                                uint32_t* __restrict__ vout) {
    __shared__ uint32_t run[256];
    __shared__ uint32_t wcnt[kSortThreads / 64][256];
    __shared__ uint32_t woff[kSortThreads / 64][256];
    const int lane = lane_id(), wave = threadIdx.x >> 6;
    run[threadIdx.x] = 0;
    const uint64_t lt = (1ull << lane) - 1ull;
    for (int s = 0; s < kSortItems; s++) {
        for (int w = 0; w < kSortThreads / 64; w++) wcnt[w][threadIdx.x] = 0;
        __syncthreads();
        const int idx = blockIdx.x * kSortTile + s * kSortThreads + threadIdx.x;
        const bool valid = idx < m;
        const uint64_t key = valid ? kin[idx] : 0;
        const uint32_t val = valid ? vin[idx] : 0;
        const int d = (int)((key >> shift) & 255);
        uint64_t peers = __ballot(valid);
#pragma unroll
        for (int bit = 0; bit < 8; bit++) {
            const uint64_t bb = __ballot(valid && ((d >> bit) & 1));
            peers &= ((d >> bit) & 1) ? bb : ~bb;
        }
        const int rk = __popcll(peers & lt);
        if (valid && rk == 0) wcnt[wave][d] = (uint32_t)__popcll(peers);
        __syncthreads();
        {
            uint32_t rr = run[threadIdx.x];
            for (int w = 0; w < kSortThreads / 64; w++) {
                woff[w][threadIdx.x] = rr;
                rr += wcnt[w][threadIdx.x];
            }
            run[threadIdx.x] = rr;
        }
        __syncthreads();
        if (valid) {
            const uint32_t o = hist[(size_t)d * nblocks + blockIdx.x] + woff[wave][d] + (uint32_t)rk;
            kout[o] = key;
            vout[o] = val;
        }
        __syncthreads();
    }
}

__global__ void k_keys_cts(int32_t m, const int32_t* __restrict__ list, const int64_t* __restrict__ p_cts,
                           int64_t cmin, uint64_t* __restrict__ keys, uint32_t* __restrict__ vals) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= m) return;
    const int p = list[i];
    keys[i] = (uint64_t)(p_cts[p] - cmin);
    vals[i] = (uint32_t)p;
}

// one key (graph, rr, cts - min) when it fits in 64 bits: a single LSD sort over it
__global__ void k_keys_comb(int32_t m, const int32_t* __restrict__ list, const int64_t* __restrict__ p_cts,
                            const int32_t* __restrict__ p_chain, const int32_t* __restrict__ p_rr, int64_t cmin,
                            int cts_bits, int R, int n, uint64_t* __restrict__ keys, uint32_t* __restrict__ vals) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= m) return;
    const int p = list[i];
    const uint64_t seg = (uint64_t)(p_chain[p] / n) * (uint64_t)R + (uint64_t)p_rr[p];
    keys[i] = (seg << cts_bits) | (uint64_t)(p_cts[p] - cmin);
    vals[i] = (uint32_t)p;
}

__global__ void k_keys_seg(int32_t m, const uint32_t* __restrict__ vals, const int32_t* __restrict__ p_chain,
                           const int32_t* __restrict__ p_rr, int R, int n, uint64_t* __restrict__ keys) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= m) return;
    const int p = (int)vals[i];
    keys[i] = (uint64_t)(p_chain[p] / n) * (uint64_t)R + (uint64_t)p_rr[p];
}

// ---------------------------------------------------------------------------------
// order, segmented (round 5): the received events bucketed by (graph, rr) -- one counting pass and
// one scatter -- and every bucket then sorted by its combined key in one workgroup's LDS (bitonic),
// instead of 5-6 LSD radix passes over the whole list (c4: 4.8 GB of sort traffic per pass, 6.6x the
// one-pass bytes). A bucket holds the events received in one round (c3 ~3 500, c4 ~120); a list with a
// bucket over kSegSortCap takes the radix sort (consensus_sorter.go:5-52, hashgraph.go:822-823).
constexpr int kSegSortCap = 8192;

// runs of equal segments among a wave's lanes [0, nvalid) (the list is chain-major with rr
// non-decreasing along a chain, so a wave holds a few runs): the run head's lane, the run length
__device__ __forceinline__ void wave_seg_runs(bool valid, int seg, bool& head, int& head_lane, int& run_len) {
    const int lane = lane_id();
    const int prev = __shfl_up(seg, 1);
    head = valid && (lane == 0 || prev != seg);
    const uint64_t hm = __ballot(head), vm = __ballot(valid);
    const int nv = __popcll(vm);   // (valid lanes are a prefix)
    const uint64_t upto = lane == 63 ? ~0ull : ((2ull << lane) - 1ull);
    const uint64_t above = hm & ~upto;
    run_len = (above ? (int)__builtin_ctzll(above) : nv) - lane;
    const uint64_t below = hm & upto;
    head_lane = below ? 63 - (int)__builtin_clzll(below) : 0;
}

// the bucket counts and the timestamp range in one pass over the received list (the range read back
// decides the key width; grid-stride, one atomic pair per block for the range)
__global__ void __launch_bounds__(256) k_seg_count_mm(int32_t m, const int32_t* __restrict__ list,
                                                      const int64_t* __restrict__ p_cts,
                                                      const int32_t* __restrict__ p_chain, const int32_t* __restrict__ p_rr,
                                                      int R, int n, uint32_t* __restrict__ segc,
                                                      unsigned long long* __restrict__ mm) {
    __shared__ unsigned long long slo[4], shi[4];
    unsigned long long lo = ~0ull, hi = 0ull;
    const int stride = gridDim.x * blockDim.x;
    for (int i0 = blockIdx.x * blockDim.x; i0 < m; i0 += stride) {   // (wave-uniform trip count)
        const int i = i0 + (int)threadIdx.x;
        const bool v = i < m;
        int seg = -1;
        if (v) {
            const int p = list[i];
            seg = (p_chain[p] / n) * R + p_rr[p];
            const unsigned long long u = (unsigned long long)p_cts[p] ^ 0x8000000000000000ull;
            lo = min(lo, u);
            hi = max(hi, u);
        }
        bool head;
        int hl, len;
        wave_seg_runs(v, seg, head, hl, len);
        if (head) atomicAdd(&segc[seg], (uint32_t)len);
    }
    for (int o = 32; o >= 1; o >>= 1) {
        lo = min(lo, (unsigned long long)__shfl_xor(lo, o));
        hi = max(hi, (unsigned long long)__shfl_xor(hi, o));
    }
    if (lane_id() == 0) { slo[threadIdx.x >> 6] = lo; shi[threadIdx.x >> 6] = hi; }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int w = 0; w < 4; w++) { lo = min(lo, slo[w]); hi = max(hi, shi[w]); }
        atomicMin(&mm[0], lo);
        atomicMax(&mm[1], hi);
    }
}

// the combined key of every received event straight into its bucket (k_keys_comb + k_seg_scatter)
__global__ void __launch_bounds__(256) k_seg_keys_scatter(int32_t m, const int32_t* __restrict__ list,
                                                          const int64_t* __restrict__ p_cts,
                                                          const int32_t* __restrict__ p_chain,
                                                          const int32_t* __restrict__ p_rr, int64_t cmin, int cts_bits,
                                                          int R, int n, const uint32_t* __restrict__ segoff,
                                                          uint32_t* __restrict__ segcur, uint64_t* __restrict__ kout,
                                                          uint32_t* __restrict__ vout) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    const bool v = i < m;
    int seg = -1, p = 0;
    uint64_t key = 0;
    if (v) {
        p = list[i];
        seg = (p_chain[p] / n) * R + p_rr[p];
        key = ((uint64_t)seg << cts_bits) | (uint64_t)(p_cts[p] - cmin);
    }
    bool head;
    int hl, len;
    wave_seg_runs(v, seg, head, hl, len);
    uint32_t base = 0;
    if (head) base = atomicAdd(&segcur[seg], (uint32_t)len);
    base = (uint32_t)__shfl((int)base, hl);
    if (v) {
        const uint32_t slot = segoff[seg] + base + (uint32_t)(lane_id() - hl);
        kout[slot] = key;
        vout[slot] = (uint32_t)p;
    }
}

__global__ void __launch_bounds__(256) k_seg_max(int nseg, const uint32_t* __restrict__ segc,
                                                 unsigned long long* __restrict__ out) {
    uint32_t mx = 0;
    for (int s = blockIdx.x * blockDim.x + threadIdx.x; s < nseg; s += gridDim.x * blockDim.x) mx = max(mx, segc[s]);
    for (int o = 32; o >= 1; o >>= 1) mx = max(mx, (uint32_t)__shfl_xor(mx, o));
    if (lane_id() == 0 && mx) atomicMax(out, (unsigned long long)mx);
}

// equal (graph, rr, cts) runs are ordered by S (big-endian 256-bit; consensus_sorter.go:37-42)
__device__ __forceinline__ int cmp_s(const uint8_t* a, const uint8_t* b) {
    for (int k = 0; k < 32; k++)
        if (a[k] != b[k]) return a[k] < b[k] ? -1 : 1;
    return 0;
}

// What k_finish_order does for an element of the order, done by the sort that places it (the bucket
// sort's buckets are the blocks: bucket = graph * R + rr): the order's gid (written straight into the
// pinned host arena when order_gid points there, so the host-link writes overlap the other buckets'
// sorting), rr and the timestamp back in gid order, and the block's count, transactions, loaded events
// and nil-ness (its first event's) written by the bucket's own group, no atomics.
struct SortFinish {
    const int32_t* p_rr;
    const int64_t* p_cts;
    const int32_t* g_ntx;
    const uint8_t* g_loaded;
    const uint8_t* g_txnil;
    int32_t* order_gid;
    int32_t* g_rr;
    int64_t* g_cts;
    int32_t* blk_cnt;
    int64_t* blk_ntx;
    int32_t* blk_loaded;
    uint8_t* blk_nil;
};

// One bucket per group of GS threads (a workgroup of 1 024 threads, or a wave, GS = 64, four buckets
// per workgroup when every bucket holds <= 512 events: 256 threads per bucket at c3 left the LDS latency
// of the compare-exchange stages exposed, 1.14 ms per pass): bitonic sort of its (key, value) pairs in LDS
// (cap = the largest bucket rounded up to a power of two), then the runs of equal keys (same graph,
// rr and timestamp) ordered by S in the same kernel: a run's members get the first 8 bytes of their S
// (big-endian) in place of the key they share, and each member's place in its run is its rank by
// (S prefix, full S on equal prefixes, index) -- the radix path's k_tie_prefix / k_tiefix_rank, with
// the run in LDS (consensus_sorter.go:36-51). Writes the final values and finishes them (SortFinish).
template <int GS, int TB>
__global__ void __launch_bounds__(TB) k_seg_sort(int nseg, int seg0, int seg1, int32_t m, const uint32_t* __restrict__ segoff,
                                                  const uint64_t* __restrict__ kin, const uint32_t* __restrict__ vin,
                                                  const int32_t* __restrict__ p_gid, const uint8_t* __restrict__ g_S,
                                                  uint32_t* __restrict__ vout, int cap, SortFinish F) {
    extern __shared__ __attribute__((aligned(16))) uint64_t smem[];
    __shared__ int64_t red_ntx[TB / 64];
    __shared__ int32_t red_ld[TB / 64];
    constexpr int NG = TB / GS;   // groups (buckets) per workgroup
    const int grp = (int)threadIdx.x / GS, t = (int)threadIdx.x % GS;
    uint64_t* sk = smem + (size_t)grp * cap;                               // [cap] keys, then S prefixes
    uint32_t* sv = (uint32_t*)(smem + (size_t)NG * cap) + (size_t)grp * cap;   // [cap] values
    uint16_t* rs = (uint16_t*)((uint32_t*)(smem + (size_t)NG * cap) + (size_t)NG * cap) + (size_t)grp * 2 * cap;   // [2][cap]
    auto sync = [&]() {
        if constexpr (GS == 64) wave_lds_fence(); else __syncthreads();
    };
    const int sgi = seg0 + (int)blockIdx.x * NG + grp;   // buckets [seg0, seg1) of nseg
    int o = 0, len = 0;
    if (sgi < seg1) {
        o = (int)segoff[sgi];
        len = (sgi + 1 < nseg ? (int)segoff[sgi + 1] : m) - o;
    }
    // element o + i of the order is position p
    int64_t ntx = 0;
    int ld = 0;
    auto emit = [&](int i, uint32_t p) {
        vout[o + i] = p;
        const int gid = p_gid[p];
        F.order_gid[o + i] = gid;
        F.g_rr[gid] = F.p_rr[p];
        F.g_cts[gid] = F.p_cts[p];
        ntx += F.g_ntx[gid];
        ld += F.g_loaded[gid] ? 1 : 0;
        if (i == 0) F.blk_nil[sgi] = F.g_txnil[gid];   // NewBlock(rr, first.Transactions()), hashgraph.go:838-845
    };
    // the block's totals (group-uniform: every way out of the kernel goes through here)
    auto block_totals = [&]() {
        for (int w = 32; w >= 1; w >>= 1) {
            ntx += __shfl_xor(ntx, w);
            ld += __shfl_xor(ld, w);
        }
        if constexpr (GS > 64) {
            if (lane_id() == 0) { red_ntx[threadIdx.x >> 6] = ntx; red_ld[threadIdx.x >> 6] = ld; }
            __syncthreads();
            if (threadIdx.x == 0)
                for (int w = 1; w < TB / 64; w++) { ntx += red_ntx[w]; ld += red_ld[w]; }
        }
        if (t == 0 && len > 0) {
            F.blk_cnt[sgi] = len;
            F.blk_ntx[sgi] = ntx;
            F.blk_loaded[sgi] = ld;
        }
    };
    if (len <= 1) {   // (group-uniform)
        if (len == 1 && t == 0) emit(0, vin[o]);
        block_totals();
        return;
    }
    int P = 2;
    while (P < len) P <<= 1;
    for (int i = t; i < P; i += GS) {
        sk[i] = i < len ? kin[o + i] : ~0ull;
        sv[i] = i < len ? vin[o + i] : 0u;
    }
    sync();
    for (int k = 2; k <= P; k <<= 1) {
        for (int j = k >> 1; j > 0; j >>= 1) {
            for (int q = t; q < (P >> 1); q += GS) {
                const int lo = 2 * j * (q / j) + (q & (j - 1)), hi = lo + j;
                const bool asc = (lo & k) == 0;
                const uint64_t a = sk[lo], b = sk[hi];
                if ((a > b) == asc) {
                    sk[lo] = b;
                    sk[hi] = a;
                    const uint32_t x = sv[lo];
                    sv[lo] = sv[hi];
                    sv[hi] = x;
                }
            }
            sync();
        }
    }
    // run starts: inclusive max-scan of (head ? i : 0) over [0, len), ping-pong between rs[0] and rs[1]
    bool tie_any = false;
    for (int i = t; i < len; i += GS) {
        const bool head = i == 0 || sk[i - 1] != sk[i];
        rs[i] = (uint16_t)(head ? i : 0);
        tie_any |= !head;
    }
    if constexpr (GS == 64) tie_any = __any(tie_any); else tie_any = __syncthreads_or(tie_any);
    if (!tie_any) {   // (group-uniform) every key distinct: the values are final
        for (int i = t; i < len; i += GS) emit(i, sv[i]);
        block_totals();
        return;
    }
    sync();
    int cur = 0;
    for (int d = 1; d < len; d <<= 1) {
        const uint16_t* src = rs + cur * cap;
        uint16_t* dst = rs + (cur ^ 1) * cap;
        for (int i = t; i < len; i += GS) dst[i] = i >= d ? max(src[i], src[i - d]) : src[i];
        sync();
        cur ^= 1;
    }
    const uint16_t* st = rs + cur * cap;
    // run members: the S prefix in place of the shared key (a member is not its run's only element)
    for (int i = t; i < len; i += GS) {
        const int s0 = st[i];
        const bool member = s0 != i || (i + 1 < len && st[i + 1] == i);
        if (member) {
            // (S rows are 32-byte aligned: the big-endian prefix is one 8-byte load, byte-swapped)
            sk[i] = __builtin_bswap64(*(const uint64_t*)(g_S + (size_t)p_gid[sv[i]] * 32));
        }
    }
    sync();
    for (int i = t; i < len; i += GS) {
        const int s0 = st[i];
        const bool member = s0 != i || (i + 1 < len && st[i + 1] == i);
        if (!member) {
            emit(i, sv[i]);
            continue;
        }
        const uint64_t my = sk[i];
        const uint32_t vi = sv[i];
        const uint8_t* si = g_S + (size_t)p_gid[vi] * 32;
        int rank = 0;
        for (int jx = s0; jx < len && st[jx] == s0; jx++) {
            const uint64_t pj = sk[jx];
            const int c = pj != my ? (pj < my ? -1 : 1) : (jx == i ? 0 : cmp_s(g_S + (size_t)p_gid[sv[jx]] * 32, si));
            rank += c < 0 || (c == 0 && jx < i);   // equal S (never in a valid trace): stable
        }
        emit(s0 + rank, vi);
    }
    block_totals();
}

// grid-stride min/max of the received events' timestamps (biased to unsigned order);
// one atomic pair per block
__global__ void __launch_bounds__(256) k_minmax_cts(int32_t m, const int32_t* __restrict__ list,
                                                    const int64_t* __restrict__ p_cts,
                                                    unsigned long long* __restrict__ mm) {
    __shared__ unsigned long long slo[4], shi[4];
    unsigned long long lo = ~0ull, hi = 0ull;
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < m; i += gridDim.x * blockDim.x) {
        const unsigned long long u = (unsigned long long)p_cts[list[i]] ^ 0x8000000000000000ull;
        lo = min(lo, u);
        hi = max(hi, u);
    }
    for (int o = 32; o >= 1; o >>= 1) {
        lo = min(lo, (unsigned long long)__shfl_xor(lo, o));
        hi = max(hi, (unsigned long long)__shfl_xor(hi, o));
    }
    if (lane_id() == 0) { slo[threadIdx.x >> 6] = lo; shi[threadIdx.x >> 6] = hi; }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int w = 1; w < 4; w++) { lo = min(lo, slo[w]); hi = max(hi, shi[w]); }
        lo = min(lo, slo[0]);
        hi = max(hi, shi[0]);
        atomicMin(&mm[0], lo);
        atomicMax(&mm[1], hi);
    }
}


// runs of equal combined keys (same graph, rr and timestamp) ordered by S (256-bit
// big-endian, consensus_sorter.go:36-51 with the zero whitening).
// k_tie_prefix: pre[i] = S's first 8 bytes as a big-endian u64, for members of runs.
// k_tiefix_rank: element i of a run [s, e) goes to s + #{j in run : S_j < S_i} (prefix
// compare, full compare on equal prefixes), so each run is placed in parallel; runs longer
// than kTieRankMax are insertion-sorted by their first thread (degenerate traces only).
constexpr int kTieRankMax = 8192;

__global__ void k_tie_prefix(int32_t m, const uint32_t* __restrict__ vals, const uint64_t* __restrict__ keys,
                             const int32_t* __restrict__ p_gid, const uint8_t* __restrict__ g_S,
                             uint64_t* __restrict__ pre) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= m) return;
    const uint64_t k = keys[i];
    const bool tie = (i > 0 && keys[i - 1] == k) || (i + 1 < m && keys[i + 1] == k);
    if (!tie) return;
    pre[i] = __builtin_bswap64(*(const uint64_t*)(g_S + (size_t)p_gid[vals[i]] * 32));   // (big-endian prefix)
}

__global__ void k_tiefix_rank(int32_t m, const uint32_t* __restrict__ vals, uint32_t* __restrict__ out,
                              const uint64_t* __restrict__ keys, const uint64_t* __restrict__ pre,
                              const int32_t* __restrict__ p_gid, const uint8_t* __restrict__ g_S) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= m) return;
    const uint64_t k = keys[i];
    const uint32_t vi = vals[i];
    if (!((i > 0 && keys[i - 1] == k) || (i + 1 < m && keys[i + 1] == k))) {
        out[i] = vi;
        return;
    }
    int s = i, e = i + 1;
    while (s > 0 && keys[s - 1] == k && i - s <= kTieRankMax) s--;
    while (e < m && keys[e] == k && e - s <= kTieRankMax) e++;
    if (e - s > kTieRankMax) {   // long run: first element's thread insertion-sorts it
        if (i > 0 && keys[i - 1] == k) return;
        e = i + 1;
        while (e < m && keys[e] == k) e++;
        for (int a = i; a < e; a++) out[a] = vals[a];
        for (int a = i + 1; a < e; a++) {
            const uint32_t va = out[a];
            const uint8_t* sa = g_S + (size_t)p_gid[va] * 32;
            int b = a - 1;
            while (b >= i && cmp_s(g_S + (size_t)p_gid[out[b]] * 32, sa) > 0) {
                out[b + 1] = out[b];
                b--;
            }
            out[b + 1] = va;
        }
        return;
    }
    const uint64_t my = pre[i];
    const uint8_t* si = g_S + (size_t)p_gid[vi] * 32;
    int rank = 0;
    for (int j = s; j < e; j++) {
        const uint64_t pj = pre[j];
        const int c = (pj != my) ? (pj < my ? -1 : 1) : (j == i ? 0 : cmp_s(g_S + (size_t)p_gid[vals[j]] * 32, si));
        rank += c < 0 || (c == 0 && j < i);   // equal S (never in a valid trace): stable
    }
    out[s + rank] = vi;
}

__global__ void k_tiefix(int32_t m, uint32_t* __restrict__ vals, const uint64_t* __restrict__ segk,
                         const int64_t* __restrict__ p_cts, const int32_t* __restrict__ p_gid,
                         const uint8_t* __restrict__ g_S) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= m) return;
    const int p = (int)vals[i];
    if (i > 0) {
        const int pp = (int)vals[i - 1];
        if (segk[i - 1] == segk[i] && p_cts[pp] == p_cts[p]) return;   // not a run start
    }
    int e = i + 1;
    while (e < m && segk[e] == segk[i] && p_cts[vals[e]] == p_cts[p]) e++;
    if (e - i < 2) return;
    for (int a = i + 1; a < e; a++) {   // insertion sort by S (run owned by this thread)
        const uint32_t va = vals[a];
        const uint8_t* sa = g_S + (size_t)p_gid[va] * 32;
        int b = a - 1;
        while (b >= i && cmp_s(g_S + (size_t)p_gid[vals[b]] * 32, sa) > 0) {
            vals[b + 1] = vals[b];
            b--;
        }
        vals[b + 1] = va;
    }
}

// final: order gids, block stats per (graph, rr), persist rr/cts to gid order
__global__ void k_finish_order(int32_t m, const uint32_t* __restrict__ vals, const int32_t* __restrict__ p_gid,
                               const int32_t* __restrict__ p_chain, const int32_t* __restrict__ p_rr,
                               const int64_t* __restrict__ p_cts, const int32_t* __restrict__ g_ntx,
                               const uint8_t* __restrict__ g_loaded, const uint8_t* __restrict__ g_txnil, int R, int n,
                               int32_t* __restrict__ order_gid, int32_t* __restrict__ g_rr, int64_t* __restrict__ g_cts,
                               int32_t* __restrict__ blk_cnt, int64_t* __restrict__ blk_ntx,
                               int32_t* __restrict__ blk_loaded, uint8_t* __restrict__ blk_nil) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    const bool ok = i < m;
    int64_t b = -1;
    int cnt = 0, ntx = 0, ld = 0;
    if (ok) {
        const int p = (int)vals[i];
        const int gid = p_gid[p];
        order_gid[i] = gid;
        g_rr[gid] = p_rr[p];
        g_cts[gid] = p_cts[p];
        b = (int64_t)(p_chain[p] / n) * R + p_rr[p];
        cnt = 1;
        ntx = g_ntx[gid];
        ld = g_loaded[gid] ? 1 : 0;
        // NewBlock(rr, first.Transactions()) (hashgraph.go:838-845): the block's nil-ness
        // starts from its first event's slice
        const int pp = i > 0 ? (int)vals[i - 1] : -1;
        if (pp < 0 || (int64_t)(p_chain[pp] / n) * R + p_rr[pp] != b) blk_nil[b] = g_txnil[gid];
    }
    // the order is sorted by (graph, rr): most waves hit one block -> one atomic per wave
    const int64_t b0 = __shfl(b, 0);
    if (__all(!ok || b == b0)) {
        for (int o = 32; o >= 1; o >>= 1) {
            cnt += __shfl_xor(cnt, o);
            ntx += __shfl_xor(ntx, o);
            ld += __shfl_xor(ld, o);
        }
        if (lane_id() == 0 && b0 >= 0) {
            atomicAdd(&blk_cnt[b0], cnt);
            if (ntx) atomicAdd((unsigned long long*)&blk_ntx[b0], (unsigned long long)ntx);
            if (ld) atomicAdd(&blk_loaded[b0], ld);
        }
    } else if (ok) {
        atomicAdd(&blk_cnt[b], 1);
        if (ntx) atomicAdd((unsigned long long*)&blk_ntx[b], (unsigned long long)ntx);
        if (ld) atomicAdd(&blk_loaded[b], 1);
    }
}

__global__ void k_gather_i32(int64_t E, const int32_t* __restrict__ src, const int32_t* __restrict__ g_pos,
                             int32_t* __restrict__ dst) {
    const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (gid < E) dst[gid] = src[g_pos[gid]];
}

// ---------------------------------------------------------------------------------
// root floors after a Reset (hashgraph.go:202-262 with Roots): an event that sees the first
// event of chain i (Root.Round(i) + 1 by RoundInc's isRoot rule) has round >= Root.Round(i) + 1,
// so R_{r+1} = {W'_r test} u {G >= r+1}, G(x) = max over those chains
template <typename CT>
__global__ void k_root_floor(const int32_t* __restrict__ c_off, const int32_t* __restrict__ c_len,
                             const int32_t* __restrict__ c_base, const int32_t* __restrict__ root_round,
                             const CT* __restrict__ LA, int32_t* __restrict__ gfl, int C, int n, int max_len) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= (int64_t)C * max_len) return;
    const int c = (int)(t % C), k = (int)(t / C);
    if (k >= c_len[c]) return;
    const int g = c / n;
    const int64_t p = (int64_t)c_off[c] + k;
    int G = 0;
    for (int i = 0; i < n; i++) {
        const int gi = g * n + i;
        const int32_t la = Coord<CT>::la(LA[(size_t)p * n + i]);
        if (c_len[gi] > 0 && la >= c_base[gi]) G = max(G, root_round[gi] + 1);
    }
    gfl[p] = G;
}

__global__ void k_root_bound_init(int32_t* __restrict__ gB, const int32_t* __restrict__ c_len, int C, int gmax) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= (int64_t)(gmax + 1) * C) return;
    gB[t] = c_len[t % C];
}

__global__ void k_root_bound(const int32_t* __restrict__ c_off, const int32_t* __restrict__ c_len,
                             const int32_t* __restrict__ gfl, int32_t* __restrict__ gB, int C, int gmax,
                             int max_len) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= (int64_t)C * max_len) return;
    const int c = (int)(t % C), k = (int)(t / C);
    if (k >= c_len[c]) return;
    const int64_t p = (int64_t)c_off[c] + k;
    const int gp = k > 0 ? gfl[p - 1] : -1;
    const int G = min(gfl[p], gmax);
    for (int r = gp + 1; r <= G; r++) gB[(size_t)r * C + c] = k;   // G is monotone along the chain
}

// ---------------------------------------------------------------------------------
// order of a small received set (m <= kSortSmallMax, the incremental schedule's usual
// case) by ranks: an event's place is the number of events before it in (graph, rr, cts, S)
// order (consensus_sorter.go:36-51), S compared from HBM only when the first 8 bytes tie.
// A (256 events) x (64 events) tile per workgroup, the column tile's keys broadcast from LDS,
// partial counts added to rank[]; then one scatter. One workgroup's 78 bitonic stages were
// LDS-bandwidth bound (145 us per call); 256 x 256 tiles with a branchy compare loop took 46 us at
// m ~ 3 500 (the chunked schedule's FindOrder at c3: 196 workgroups, under one wave per SIMD, each
// thread 256 dependent LDS round trips). 64-key tiles put ~12 waves on every CU and the compare is
// branch-free (the full-S tie path only on 24 equal key bytes).
constexpr int kSortSmallMax = 4096;
constexpr int kRankTile = 256;
constexpr int kRankJT = 64;

struct SortKey {
    uint64_t hi, lo, s8;   // (graph << 32 | rr), cts with the sign flipped, S's first 8 bytes
    int32_t p;             // position
};

__device__ __forceinline__ SortKey sort_key(int p, const int64_t* __restrict__ p_cts, const int32_t* __restrict__ p_chain,
                                            const int32_t* __restrict__ p_rr, const int32_t* __restrict__ p_gid,
                                            const uint8_t* __restrict__ g_S, int n) {
    SortKey k;
    k.hi = ((uint64_t)(uint32_t)(p_chain[p] / n) << 32) | (uint64_t)(uint32_t)p_rr[p];
    k.lo = (uint64_t)p_cts[p] ^ 0x8000000000000000ull;
    const uint2 w = *(const uint2*)(g_S + (size_t)p_gid[p] * 32);
    k.s8 = ((uint64_t)__builtin_bswap32(w.x) << 32) | (uint64_t)__builtin_bswap32(w.y);
    k.p = p;
    return k;
}

__global__ void __launch_bounds__(256) k_sort_rank(int32_t m, const int32_t* __restrict__ list,
                                                    const int64_t* __restrict__ p_cts,
                                                    const int32_t* __restrict__ p_chain,
                                                    const int32_t* __restrict__ p_rr, const int32_t* __restrict__ p_gid,
                                                    const uint8_t* __restrict__ g_S, int n,
                                                    uint32_t* __restrict__ rank) {
    __shared__ uint64_t jhi[kRankJT], jlo[kRankJT], js8[kRankJT];
    __shared__ int32_t jp[kRankJT];
    const int i = blockIdx.x * kRankTile + threadIdx.x;
    const int j0 = blockIdx.y * kRankJT;
    const int jn = min(kRankJT, m - j0);
    if ((int)threadIdx.x < jn) {
        const SortKey k = sort_key(list[j0 + threadIdx.x], p_cts, p_chain, p_rr, p_gid, g_S, n);
        jhi[threadIdx.x] = k.hi;
        jlo[threadIdx.x] = k.lo;
        js8[threadIdx.x] = k.s8;
        jp[threadIdx.x] = k.p;
    }
    const bool ok = i < m;
    SortKey me{};
    if (ok) me = sort_key(list[i], p_cts, p_chain, p_rr, p_gid, g_S, n);
    __syncthreads();
    if (!ok) return;
    uint32_t cnt = 0;
    bool tie = false;   // some key of the tile equals this one in all 24 compared bytes (not itself)
#pragma unroll 8
    for (int jj = 0; jj < kRankJT; jj++) {
        if (jj < jn) {
            const uint64_t h = jhi[jj], l = jlo[jj], q = js8[jj];
            const bool eh = h == me.hi, el = l == me.lo;
            const bool before = h < me.hi || (eh && (l < me.lo || (el && q < me.s8)));
            cnt += before ? 1u : 0u;
            tie |= eh && el && q == me.s8 && j0 + jj != i;
        }
    }
    if (tie) {   // 8 equal bytes of S: the whole S, then the list order
        const uint8_t* si = g_S + (size_t)p_gid[me.p] * 32;
        for (int jj = 0; jj < jn; jj++) {
            if (jhi[jj] != me.hi || jlo[jj] != me.lo || js8[jj] != me.s8 || j0 + jj == i) continue;
            const int c = cmp_s(g_S + (size_t)p_gid[jp[jj]] * 32, si);
            cnt += (c < 0 || (c == 0 && j0 + jj < i)) ? 1u : 0u;
        }
    }
    if (cnt) atomicAdd(&rank[i], cnt);
}

__global__ void __launch_bounds__(256) k_sort_place(int32_t m, const int32_t* __restrict__ list,
                                                     const uint32_t* __restrict__ rank, uint32_t* __restrict__ out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < m) out[rank[i]] = (uint32_t)list[i];
}

// ---------------------------------------------------------------------------------
// host-side launchers (template dispatch on n)
#define HGX_DISPATCH_N(n, MACRO)                      \
    do {                                              \
        if ((n) <= 4) { MACRO(4, 1, 1); }             \
        else if ((n) <= 8) { MACRO(8, 1, 1); }        \
        else if ((n) <= 16) { MACRO(16, 1, 1); }      \
        else if ((n) <= 32) { MACRO(32, 1, 1); }      \
        else if ((n) <= 64) { MACRO(64, 1, 1); }      \
        else if ((n) <= 128) { MACRO(64, 2, 2); }     \
        else if ((n) <= 256) { MACRO(64, 4, 4); }     \
        else if ((n) <= 512) { MACRO(64, 8, 8); }     \
        else { MACRO(64, 16, 16); }                   \
    } while (0)

static inline unsigned nblk(int64_t work, int bs) { return (unsigned)((work + bs - 1) / bs); }

struct FillArgs {
    FillRange r[kFillMax];
    int count;
};
__global__ void __launch_bounds__(256) k_fill_many(FillArgs f) {
    const FillRange r = f.r[blockIdx.y];
    const uint32_t v4 = 0x01010101u * r.value;
    uint32_t* p = (uint32_t*)r.p;
    const uint32_t nw = r.bytes / 4;
    for (uint32_t t = blockIdx.x * blockDim.x + threadIdx.x; t < nw; t += gridDim.x * blockDim.x) p[t] = v4;
    if (blockIdx.x == 0 && threadIdx.x < (r.bytes & 3u)) ((uint8_t*)r.p)[nw * 4 + threadIdx.x] = r.value;
}

namespace {
std::mutex g_attr_mu;
std::map<std::pair<int, const void*>, size_t> g_lds_set;
std::map<std::tuple<int, const void*, int, size_t>, int> g_occ;
}  // namespace

hipError_t ensure_lds_limit(const void* f, size_t bytes) {
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    std::lock_guard<std::mutex> lk(g_attr_mu);
    size_t& cur = g_lds_set[{dev, f}];
    if (bytes <= cur) return hipSuccess;
    e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
    if (e == hipSuccess) cur = bytes;
    return e;
}

hipError_t blocks_per_cu(const void* f, int T, size_t lds, int* out) {
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    std::lock_guard<std::mutex> lk(g_attr_mu);
    const auto key = std::make_tuple(dev, f, T, lds);
    auto it = g_occ.find(key);
    if (it != g_occ.end()) {
        *out = it->second;
        return hipSuccess;
    }
    int v = 0;
    e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&v, f, T, lds);
    if (e == hipSuccess) g_occ[key] = *out = v;
    return e;
}

void launch_fill_many(hipStream_t s, const FillRange* r, int count) {
    if (count <= 0) return;
    FillArgs f{};
    uint32_t mx = 0;
    for (int i = 0; i < count && i < kFillMax; i++) {
        f.r[i] = r[i];
        mx = std::max(mx, r[i].bytes);
    }
    f.count = std::min(count, kFillMax);
    const unsigned bx = std::max(1u, std::min(256u, (mx / 4 + 255) / 256));
    hipLaunchKernelGGL(k_fill_many, dim3(bx, f.count), dim3(256), 0, s, f);
}

struct CopyArgs {
    CopyRange r[kCopyMax];
};
__global__ void __launch_bounds__(256) k_copy_many(CopyArgs f) {
    const CopyRange r = f.r[blockIdx.y];
    const uint32_t t0 = blockIdx.x * blockDim.x + threadIdx.x, st = gridDim.x * blockDim.x;
    const uintptr_t al = (uintptr_t)r.src | (uintptr_t)r.dst;
    uint32_t done = 0;
    const bool rs = r.reset >= 0;
    const uint32_t f4 = 0x01010101u * (uint32_t)(r.reset & 0xFF);
    if ((al & 15u) == 0) {
        uint4* s4 = (uint4*)r.src;
        uint4* d4 = (uint4*)r.dst;
        const uint32_t nq = r.bytes / 16;
        for (uint32_t t = t0; t < nq; t += st) {
            d4[t] = s4[t];
            if (rs) s4[t] = make_uint4(f4, f4, f4, f4);
        }
        done = nq * 16;
    } else if ((al & 3u) == 0) {
        uint32_t* s1 = (uint32_t*)r.src;
        uint32_t* d1 = (uint32_t*)r.dst;
        const uint32_t nw = r.bytes / 4;
        for (uint32_t t = t0; t < nw; t += st) {
            d1[t] = s1[t];
            if (rs) s1[t] = f4;
        }
        done = nw * 4;
    }
    uint8_t* sb = (uint8_t*)r.src;
    uint8_t* db = (uint8_t*)r.dst;
    for (uint32_t t = done + t0; t < r.bytes; t += st) {
        db[t] = sb[t];
        if (rs) sb[t] = (uint8_t)r.reset;
    }
}

void launch_copy_many(hipStream_t s, const CopyRange* r, int count) {
    if (count <= 0) return;
    CopyArgs f{};
    uint32_t mx = 0;
    for (int i = 0; i < count && i < kCopyMax; i++) {
        f.r[i] = r[i];
        mx = std::max(mx, r[i].bytes);
    }
    const unsigned bx = std::max(1u, std::min(64u, (mx / 16 + 255) / 256));
    hipLaunchKernelGGL(k_copy_many, dim3(bx, std::min(count, kCopyMax)), dim3(256), 0, s, f);
}

void launch_layout(hipStream_t s, int64_t E0, int64_t E, const DevArrays& a, int C, int n, int seg) {
    if (E <= E0) return;
    hipLaunchKernelGGL(k_ck_pack, dim3(nblk(E - E0, 256)), dim3(256), 0, s, E0, E, a.g_creator, a.g_index, a.c_base,
                       a.g_ck);
    if (E - E0 <= 8 * kLayoutB) {
        hipLaunchKernelGGL(k_layout_direct, dim3(nblk(E - E0, 256)), dim3(256), 0, s, E0, E, a.g_creator, a.g_index,
                           a.g_ck, a.g_op, a.g_ts, a.g_rr, a.g_cts, a.c_off, a.c_base, a.g_pos, a.p_gid, a.p_chain, a.p_op,
                           a.p_opu, a.p_opk, a.p_ts, a.p_rr, a.p_cts, C, n, seg);
        return;
    }
    hipLaunchKernelGGL(k_layout_staged, dim3(nblk(E - E0, kLayoutB2)), dim3(256), 0, s, E0, E, a.g_creator, a.g_index,
                       a.g_ck, a.g_op, a.g_ts, a.g_rr, a.g_cts, a.c_off, a.c_base, a.g_pos, a.p_gid, a.p_chain, a.p_op,
                       a.p_opu, a.p_opk, a.p_ts, a.p_rr, a.p_cts, C, n, seg);
}

void launch_la_sweep(hipStream_t s, const DevArrays& a, int C, int n, int max_len, int seg, int first, int32_t* chg,
                     int32_t stamp, int64_t* usum, int32_t* out, int32_t* out_next, const int32_t* c_old, int64_t u0) {
    const int nseg = (max_len + seg - 1) / seg;
    if ((int64_t)nseg * C <= u0) return;
    const int nwd = a.compact ? n / 2 : n;
#define LA_LAUNCH_V(GS, CPL, CT, V)                                                                           \
    {                                                                                                         \
        const int64_t threads = ((int64_t)nseg * C - u0) * GS;                                                \
        hipLaunchKernelGGL((k_la_sweep<GS, CPL, CT, V>), dim3(std::min(nblk(threads, 256), 2048u)), dim3(256), 0, \
                           s, (uint32_t*)a.LA, a.p_op, a.p_opu, a.c_off, a.c_len, a.c_base, C, n, nwd, nseg, seg, \
                           first ? 1 : 0, chg, stamp, usum, out, out_next, c_old, u0);                        \
    }
#define LA_LAUNCH_T(GS, CPL, CT)                                   \
    {                                                              \
        if (first == 2) LA_LAUNCH_V(GS, CPL, CT, true) else LA_LAUNCH_V(GS, CPL, CT, false) \
    }
#define LA_LAUNCH(GS, CPL, NW)                                        \
    {                                                                 \
        if (a.compact) LA_LAUNCH_T(GS, CPL, uint16_t) else LA_LAUNCH_T(GS, CPL, int32_t) \
    }
    HGX_DISPATCH_N(nwd, LA_LAUNCH);
#undef LA_LAUNCH
#undef LA_LAUNCH_T
#undef LA_LAUNCH_V
}

int fd_tile_rows(int n, int compact) {
    // one 64-row tile per block up to round 5 (measured at c3, all 256 columns in LDS: 16 rows 17.2 ms,
    // 32 rows 10.0, 64 rows 6.8; 128 rows as two 64-row chunks 8.9, 256 rows 14.9 -- fewer resident
    // blocks). Round 6: the tile holds fd_cols target columns (~38 KB of LDS at any n, 4 blocks per CU)
    // and each lane owns 2 consecutive tile rows (4 at n <= 32), so a (tile, target) pair's fixed cost
    // -- the scalars, the first chunk -- is spread over 128 (256) rows: k_fd_build at c3 5.2 -> 4.35 ms,
    // c5 2.05 -> 1.75, c4 0.68 -> 0.42 -> 0.33 ms
    (void)compact;
    return n <= 32 ? 256 : 128;
}

int fd_cols(int compact, int ft) { return (compact ? 256 : 128) * 64 / ft; }   // target columns per block

void launch_fd_build(hipStream_t s, const DevArrays& a, int C, int n, int max_len, int64_t P, const int32_t* c_old,
                     int max_new, int d_lo, int d_hi) {
    if (d_hi < 0) d_hi = n;
    if (d_hi <= d_lo) return;
    const int ft = fd_tile_rows(n, a.compact);
    // incremental (c_old): tiles from each chain's first new row; max_new = the most new rows of a chain
    const int tiles = c_old ? max(1, (max_new + ft - 1) / ft) : max(1, (max_len + ft - 1) / ft);
    const int nwd = a.compact ? n / 2 : n;
    const int DB = std::min(fd_cols(a.compact, ft), d_hi - d_lo);
    const int ncb = (d_hi - d_lo + DB - 1) / DB;
    const int wdw = DB / (a.compact ? 2 : 1) + 1;   // words of a tile row, the worst alignment
    // tile + per-target scalars + 8 waves x 64 owner slots
    const size_t lds = ((size_t)(ft + 1) * (wdw + 1) + 1 + 3 * (size_t)DB + 8 * 128) * sizeof(int32_t);
    // a resumed call with a few new rows per chain: a column block's targets split over up to 8 blocks
    const int zs = (c_old && max_new <= ft) ? max(1, min(8, DB / 64)) : 1;
    const dim3 grid(C, tiles, ncb * zs);
#define FD_LAUNCH(CT_, RPL_)                                                                                    \
    hipLaunchKernelGGL((k_fd_build<CT_, RPL_>), grid, dim3(512), lds, s, (const uint32_t*)a.LA, (CT_*)a.FDT, a.c_off, \
                       a.c_len, a.c_base, n, nwd, ft, P, c_old, d_lo, d_hi, DB, zs)
    if (a.compact) {
        if (ft == 256) FD_LAUNCH(uint16_t, 4);
        else if (ft == 128) FD_LAUNCH(uint16_t, 2);
        else FD_LAUNCH(uint16_t, 1);
    } else {
        if (ft == 256) FD_LAUNCH(int32_t, 4);
        else if (ft == 128) FD_LAUNCH(int32_t, 2);
        else FD_LAUNCH(int32_t, 1);
    }
#undef FD_LAUNCH
}

void launch_round_gather(hipStream_t s, const DevArrays& a, int r, int C, int n, int64_t P) {
    if (a.compact)
        hipLaunchKernelGGL(k_round_gather<uint16_t>, dim3(nblk((int64_t)C * n, 256)), dim3(256), 0, s, r, a.Bm,
                           a.c_off, a.c_len, (const uint16_t*)a.LA, (const uint16_t*)a.FDT, a.p_gid, a.g_coin, a.WLA,
                           a.WFD, a.wflag, a.wcoin, C, n, P, 1);
    else
        hipLaunchKernelGGL(k_round_gather<int32_t>, dim3(nblk((int64_t)C * n, 256)), dim3(256), 0, s, r, a.Bm,
                           a.c_off, a.c_len, (const int32_t*)a.LA, (const int32_t*)a.FDT, a.p_gid, a.g_coin, a.WLA,
                           a.WFD, a.wflag, a.wcoin, C, n, P, 0);
}

void launch_wcoin(hipStream_t s, const DevArrays& a, int r0, int R, int C) {
    const int64_t RC = (int64_t)(R - r0) * C;
    if (RC <= 0) return;
    const size_t o = (size_t)r0 * C;
    hipLaunchKernelGGL(k_wcoin, dim3(nblk(RC, 256)), dim3(256), 0, s, RC, C, a.Bm + o, a.c_off, a.c_len, a.p_gid,
                       a.g_coin, a.wcoin + o);
}

// fame kernel choice (hgx_set_fame_tally): the witness-tiled kernel with the popcount tally
// by default (measured faster than the int8 MFMA tally at every n); the
// per-round popcount kernel and the MFMA tally stay selectable for measurement.
void launch_fame(hipStream_t s, const DevArrays& a, int r0, int R, int C, int n, int nw, int sm, int G, int tally) {
    if (R <= r0) return;
    const int mode = tally == 1 ? 0 : tally == 2 ? 2 : 1;
    if (mode != 0 && n <= kFameMaxW * 64) {
        const int XT = (n + kFameTile - 1) / kFameTile;
        const dim3 grid((unsigned)((int64_t)G * (R - r0) * XT));
        if (mode == 2) {
            const int shm = kFameTile * (nw * 64 + 16);
            (void)ensure_lds_limit((const void*)k_fame_tile<true>, kFameTile * (kFameMaxW * 64 + 16));
            hipLaunchKernelGGL(k_fame_tile<true>, grid, dim3(256), shm, s, R, r0, XT, a.lr, a.wstat, a.wcoin, a.Bm,
                               a.c_base, a.WLA, a.Smat, a.fame, C, n, nw, sm, 0);
        } else {
            // the voters' S rows in LDS up to 512 chains (n x nw words <= 32 KB)
            const int sw = (size_t)n * nw * 8 <= kFameSW * 8 ? n * nw : 0;
            hipLaunchKernelGGL(k_fame_tile<false>, grid, dim3(256), (size_t)sw * 8, s, R, r0, XT, a.lr, a.wstat, a.wcoin,
                               a.Bm, a.c_base, a.WLA, a.Smat, a.fame, C, n, nw, sm, sw);
        }
        return;
    }
    hipLaunchKernelGGL(k_fame_vote, dim3((unsigned)G * (R - r0)), dim3(256), 0, s, R, r0, nw, a.lr, a.wstat, a.wcoin, a.Bm,
                       a.c_base, a.WLA, a.Smat, a.Vbuf, a.fame, C, n, sm);
}

void launch_wla_transpose(hipStream_t s, const DevArrays& a, int r0, int R, int G, int C, int n) {
    if (R <= r0) return;
    const int nt = (n + 63) / 64;
    hipLaunchKernelGGL(k_wla_transpose, dim3(nt * nt, (R - r0) * G), dim3(256), 0, s, R, r0, G, C, n, a.elig, a.fw, a.WLA,
                       a.WLAT);
}

void launch_threshold(hipStream_t s, const DevArrays& a, int r0, int R, int C, int n) {
    if (R <= r0) return;
#define TH_LAUNCH(GS, CPL, NW)                                                                                \
    {                                                                                                         \
        const int64_t threads = (int64_t)(R - r0) * C * 64;                                                   \
        hipLaunchKernelGGL((k_threshold<CPL>), dim3(nblk(threads, 256)), dim3(256), 0, s, R, r0, a.elig, a.fw, \
                           a.WLAT, a.T, C, n);                                                                \
    }
    HGX_DISPATCH_N(n, TH_LAUNCH);
#undef TH_LAUNCH
}

void launch_round_received(hipStream_t s, const DevArrays& a, int R, int C, int n, int max_unrecv) {
    if (max_unrecv <= 0) return;
    hipLaunchKernelGGL(k_round_received, dim3(nblk(max_unrecv, 256 * kRrPer), C), dim3(256), 0, s, R, a.c_off, a.c_len,
                       a.c_base, a.fu, a.p_round, a.lr, a.elig, a.ur_empty, a.T, a.p_rr, a.rcnt, a.recv_list,
                       a.counters, C, n);
}

void launch_fu_advance(hipStream_t s, const DevArrays& a, int C) {
    hipLaunchKernelGGL(k_fu_advance, dim3(nblk(C, 256)), dim3(256), 0, s, C, a.fu, a.rcnt);
}

void launch_fu_count(hipStream_t s, const DevArrays& a, int64_t E) {
    if (E > 0) hipLaunchKernelGGL(k_fu_count, dim3(nblk(E, 256)), dim3(256), 0, s, E, a.g_creator, a.g_rr, a.fu);
}

void launch_init_new(hipStream_t s, const DevArrays& a, int64_t E0, int64_t m, int n, int64_t P) {
    if (m <= 0) return;
    if (a.compact)
        hipLaunchKernelGGL(k_init_new<uint16_t>, dim3(nblk(m, 16), (n + 63) / 64), dim3(256), 0, s, E0, m, a.g_pos,
                           (uint16_t*)a.LA, (uint16_t*)a.FDT, n, P);
    else
        hipLaunchKernelGGL(k_init_new<int32_t>, dim3(nblk(m, 16), (n + 63) / 64), dim3(256), 0, s, E0, m, a.g_pos,
                           (int32_t*)a.LA, (int32_t*)a.FDT, n, P);
}

template <int NP, typename CT>
static void cts_small_launch(hipStream_t s, const DevArrays& a, int c_lo, int c_cnt, int C, int n, int64_t P,
                             int max_cnt) {
    hipLaunchKernelGGL((k_cts_small<NP, CT>), dim3(nblk(max_cnt, 256), c_cnt), dim3(256), 0, s, a.fu, a.rcnt, a.p_rr,
                       a.c_off, a.c_base, a.fw, a.WLAT, (const CT*)a.FDT, a.p_ts, a.p_cts, C, n, P, c_lo);
}

template <int NPAD, typename CT>
static void cts_tile_launch(hipStream_t s, const DevArrays& a, int c_lo, int c_cnt, int C, int n, int64_t P,
                            int max_cnt) {
    const size_t lds = (size_t)NPAD * (kCtsTile + 1) * sizeof(uint32_t);
    (void)ensure_lds_limit((const void*)k_cts_tile<NPAD, CT>, lds);
    const int64_t ntiles = (max_cnt + kCtsTile - 1) / kCtsTile;
    const int64_t g64 = (int64_t)64 * ((c_cnt + 7) / 8) * ((ntiles + 7) / 8);   // (the XCD-grouped order)
    if (g64 == 0) return;
    hipLaunchKernelGGL((k_cts_tile<NPAD, CT>), dim3((unsigned)g64), dim3(256), lds, s, a.fu, a.rcnt, a.p_rr,
                       a.c_off, a.c_base, a.fw, a.WLAT, (const CT*)a.FDT, a.p_ts, a.p_cts, C, n, P, c_lo, c_cnt);
}

template <typename CT>
static void launch_cts_t(hipStream_t s, const DevArrays& a, int c_lo, int c_cnt, int C, int n, int64_t P,
                         int max_cnt) {
    if (n <= 4) cts_small_launch<4, CT>(s, a, c_lo, c_cnt, C, n, P, max_cnt);
    else if (n <= 8) cts_small_launch<8, CT>(s, a, c_lo, c_cnt, C, n, P, max_cnt);
    else if (n <= 16) cts_small_launch<16, CT>(s, a, c_lo, c_cnt, C, n, P, max_cnt);
    else if (n <= 32) cts_small_launch<32, CT>(s, a, c_lo, c_cnt, C, n, P, max_cnt);
    else if (n <= 64) cts_tile_launch<64, CT>(s, a, c_lo, c_cnt, C, n, P, max_cnt);
    else if (n <= 128) cts_tile_launch<128, CT>(s, a, c_lo, c_cnt, C, n, P, max_cnt);
    else if (n <= 256) cts_tile_launch<256, CT>(s, a, c_lo, c_cnt, C, n, P, max_cnt);
    else if (n <= 512) cts_tile_launch<512, CT>(s, a, c_lo, c_cnt, C, n, P, max_cnt);
    else cts_tile_launch<1024, CT>(s, a, c_lo, c_cnt, C, n, P, max_cnt);
}

void launch_cts(hipStream_t s, const DevArrays& a, int c_lo, int c_cnt, int C, int n, int64_t P, int max_cnt) {
    if (max_cnt <= 0 || c_cnt <= 0) return;
    if (a.compact) launch_cts_t<uint16_t>(s, a, c_lo, c_cnt, C, n, P, max_cnt);
    else launch_cts_t<int32_t>(s, a, c_lo, c_cnt, C, n, P, max_cnt);
}

// consensus timestamps of the newly received events of chains [lo, hi), chain-major at
// offs[c] (to_buf: p_cts -> buf, else buf -> p_cts): the shard exchange of a row-sharded graph
__global__ void k_cts_shard_copy(int lo, const int32_t* __restrict__ c_off, const int32_t* __restrict__ fu,
                                 const int32_t* __restrict__ rcnt, const int32_t* __restrict__ offs,
                                 int64_t* __restrict__ p_cts, int64_t* __restrict__ buf, int to_buf) {
    const int gc = lo + blockIdx.x;
    const int cnt = rcnt[gc];
    const int64_t p0 = (int64_t)c_off[gc] + fu[gc];
    const int o = offs[gc];
    for (int k = threadIdx.x; k < cnt; k += blockDim.x) {
        if (to_buf) buf[o + k] = p_cts[p0 + k];
        else p_cts[p0 + k] = buf[o + k];
    }
}

void launch_cts_shard_copy(hipStream_t s, const DevArrays& a, int lo, int hi, const int32_t* offs, int64_t* buf,
                           int to_buf) {
    if (hi <= lo) return;
    hipLaunchKernelGGL(k_cts_shard_copy, dim3(hi - lo), dim3(256), 0, s, lo, a.c_off, a.fu, a.rcnt, offs, a.p_cts,
                       buf, to_buf);
}

void launch_minmax(hipStream_t s, const DevArrays& a, int32_t m) {
    hipLaunchKernelGGL(k_minmax_cts, dim3(std::min(1024u, nblk(m, 256))), dim3(256), 0, s, m, a.recv_list, a.p_cts,
                       (unsigned long long*)a.minmax);
}

static void scan_u32(hipStream_t s, const DevArrays& a, uint32_t* buf, int64_t total) {
    const int nparts = (int)((total + kScanChunk - 1) / kScanChunk);
    hipLaunchKernelGGL(k_scan_reduce, dim3(nparts), dim3(256), 0, s, buf, total, a.scan_part);
    hipLaunchKernelGGL(k_scan_top, dim3(1), dim3(256), 0, s, a.scan_part, nparts);
    hipLaunchKernelGGL(k_scan_down, dim3(nparts), dim3(256), 0, s, buf, total, a.scan_part);
}

static void radix_pass(hipStream_t s, const DevArrays& a, int32_t m, int shift, const uint64_t* kin,
                       const uint32_t* vin, uint64_t* kout, uint32_t* vout) {
    const int nb = (m + kSortTile - 1) / kSortTile;
    hipLaunchKernelGGL(k_radix_hist, dim3(nb), dim3(kSortThreads), 0, s, kin, m, shift, a.hist, nb);
    scan_u32(s, a, a.hist, (int64_t)256 * nb);
    hipLaunchKernelGGL(k_radix_scatter, dim3(nb), dim3(kSortThreads), 0, s, kin, vin, m, shift, a.hist, nb, kout,
                       vout);
}

// sorts the received list by (graph, rr, cts, S); result values (positions) are
// returned in *final_vals (one of the two ping-pong buffers).
void launch_sort(hipStream_t s, const DevArrays& a, int32_t m, int64_t cmin, int cts_bits, int R, int n,
                 int seg_bits, uint32_t** final_vals, uint64_t** final_keys) {
    uint64_t *ka = a.key_a, *kb = a.key_b;
    uint32_t *va = a.val_a, *vb = a.val_b;
    if (cts_bits + seg_bits <= 64) {   // one key, one sort, ties found on the keys
        hipLaunchKernelGGL(k_keys_comb, dim3(nblk(m, 256)), dim3(256), 0, s, m, a.recv_list, a.p_cts, a.p_chain,
                           a.p_rr, cmin, cts_bits, R, n, ka, va);
        for (int sh = 0; sh < cts_bits + seg_bits; sh += 8) {
            radix_pass(s, a, m, sh, ka, va, kb, vb);
            uint64_t* tk = ka; ka = kb; kb = tk;
            uint32_t* tv = va; va = vb; vb = tv;
        }
        // kb / vb are free after the passes: prefixes and the placed values
        hipLaunchKernelGGL(k_tie_prefix, dim3(nblk(m, 256)), dim3(256), 0, s, m, va, ka, a.p_gid, a.g_S, kb);
        hipLaunchKernelGGL(k_tiefix_rank, dim3(nblk(m, 256)), dim3(256), 0, s, m, va, vb, ka, kb, a.p_gid, a.g_S);
        va = vb;
        *final_vals = va;
        *final_keys = ka;
        return;
    }
    hipLaunchKernelGGL(k_keys_cts, dim3(nblk(m, 256)), dim3(256), 0, s, m, a.recv_list, a.p_cts, cmin, ka, va);
    for (int sh = 0; sh < cts_bits; sh += 8) {
        radix_pass(s, a, m, sh, ka, va, kb, vb);
        uint64_t* tk = ka; ka = kb; kb = tk;
        uint32_t* tv = va; va = vb; vb = tv;
    }
    hipLaunchKernelGGL(k_keys_seg, dim3(nblk(m, 256)), dim3(256), 0, s, m, va, a.p_chain, a.p_rr, R, n, ka);
    for (int sh = 0; sh < seg_bits; sh += 8) {
        radix_pass(s, a, m, sh, ka, va, kb, vb);
        uint64_t* tk = ka; ka = kb; kb = tk;
        uint32_t* tv = va; va = vb; vb = tv;
    }
    hipLaunchKernelGGL(k_tiefix, dim3(nblk(m, 256)), dim3(256), 0, s, m, va, ka, a.p_cts, a.p_gid, a.g_S);
    *final_vals = va;
    *final_keys = ka;
}

int seg_sort_cap() { return kSegSortCap; }

void launch_seg_count(hipStream_t s, const DevArrays& a, int32_t m, int R, int n, int nseg, uint32_t* segc,
                      unsigned long long* max_out) {
    // (with the timestamp range: minmax[0..1], as launch_minmax)
    hipLaunchKernelGGL(k_seg_count_mm, dim3(std::min(2048u, nblk(m, 256))), dim3(256), 0, s, m, a.recv_list, a.p_cts,
                       a.p_chain, a.p_rr, R, n, segc, (unsigned long long*)a.minmax);
    hipLaunchKernelGGL(k_seg_max, dim3(std::max(1, std::min(256, (nseg + 255) / 256))), dim3(256), 0, s, nseg, segc,
                       max_out);
}

hipError_t launch_sort_seg(hipStream_t s, const DevArrays& a, int32_t m, int64_t cmin, int cts_bits, int R, int n,
                           int nseg, uint32_t* segoff, uint32_t* segcur, int max_seg, uint32_t** final_vals,
                           uint64_t** final_keys, const std::vector<int>* cuts,
                           const std::function<hipError_t(int)>& after_part) {
    uint64_t* kb = a.key_b;
    uint32_t *va = a.val_a, *vb = a.val_b;
    int cap = 2;
    while (cap < max_seg) cap <<= 1;
    if (cap > 512) {   // (before anything is launched: the caller takes the radix passes on a refusal)
        const hipError_t e = ensure_lds_limit((const void*)k_seg_sort<1024, 1024>, (size_t)cap * 16);
        if (e != hipSuccess) return e;
    }
    scan_u32(s, a, segoff, nseg);   // bucket counts -> bucket starts
    (void)hipMemsetAsync(segcur, 0, (size_t)nseg * 4, s);
    hipLaunchKernelGGL(k_seg_keys_scatter, dim3(nblk(m, 256)), dim3(256), 0, s, m, a.recv_list, a.p_cts, a.p_chain,
                       a.p_rr, cmin, cts_bits, R, n, segoff, segcur, kb, vb);
    // (the runs of equal keys are ordered by S inside k_seg_sort: the final values land in va)
    const SortFinish F{a.p_rr, a.p_cts, a.g_ntx, a.g_loaded, a.g_txnil, a.order_gid, a.g_rr, a.g_cts,
                       a.blk_cnt, a.blk_ntx, a.blk_loaded, a.blk_nil};
    // the buckets in parts [cuts[k], cuts[k + 1]) (one part without cuts), after_part(k) behind each part's
    // launch (the caller's D2H of that part's order, overlapping the next part's sort)
    const int np = cuts ? (int)cuts->size() - 1 : 1;
    for (int k = 0; k < np; k++) {
        const int s0 = cuts ? (*cuts)[k] : 0, s1 = cuts ? (*cuts)[k + 1] : nseg;
        if (s1 > s0) {
            if (cap <= 512) {   // a wave per bucket, four per workgroup
                const size_t lds = (size_t)4 * cap * 16;
                hipLaunchKernelGGL((k_seg_sort<64, 256>), dim3((s1 - s0 + 3) / 4), dim3(256), lds, s, nseg, s0, s1, m,
                                   segoff, kb, vb, a.p_gid, a.g_S, va, cap, F);
            } else {
                const size_t lds = (size_t)cap * 16;
                hipLaunchKernelGGL((k_seg_sort<1024, 1024>), dim3(s1 - s0), dim3(1024), lds, s, nseg, s0, s1, m, segoff,
                                   kb, vb, a.p_gid, a.g_S, va, cap, F);
            }
        }
        if (after_part) {
            const hipError_t e = after_part(k);
            if (e != hipSuccess) return e;
        }
    }
    *final_vals = va;
    *final_keys = kb;
    return hipGetLastError();
}

void launch_root_floor(hipStream_t s, const DevArrays& a, const int32_t* root_round, int32_t* gfl, int32_t* gB,
                       int gmax, int C, int n, int max_len) {
    const int64_t work = (int64_t)C * max_len;
    if (work <= 0 || gmax < 0) return;
    if (a.compact)
        hipLaunchKernelGGL(k_root_floor<uint16_t>, dim3(nblk(work, 256)), dim3(256), 0, s, a.c_off, a.c_len, a.c_base,
                           root_round, (const uint16_t*)a.LA, gfl, C, n, max_len);
    else
        hipLaunchKernelGGL(k_root_floor<int32_t>, dim3(nblk(work, 256)), dim3(256), 0, s, a.c_off, a.c_len, a.c_base,
                           root_round, (const int32_t*)a.LA, gfl, C, n, max_len);
    hipLaunchKernelGGL(k_root_bound_init, dim3(nblk((int64_t)(gmax + 1) * C, 256)), dim3(256), 0, s, gB, a.c_len, C,
                       gmax);
    hipLaunchKernelGGL(k_root_bound, dim3(nblk(work, 256)), dim3(256), 0, s, a.c_off, a.c_len, gfl, gB, C, gmax,
                       max_len);
}

// UndecidedRounds order of rounds first seen after a Reset: first[r - r0] = the smallest gid
// of a witness of round r (the first event of its chain in the round has the chain's smallest
// gid there)
__global__ void k_round_first_gid(int r0, int R, int C, const int32_t* __restrict__ Bm, const uint8_t* __restrict__ wstat,
                                  const int32_t* __restrict__ c_off, const int32_t* __restrict__ p_gid,
                                  int32_t* __restrict__ first) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= (int64_t)(R - r0) * C) return;
    const int r = r0 + (int)(t / C), c = (int)(t % C);
    if (wstat[(size_t)r * C + c] != 2) return;
    atomicMin(&first[r - r0], p_gid[c_off[c] + Bm[(size_t)r * C + c]]);
}

void launch_round_first_gid(hipStream_t s, const DevArrays& a, int r0, int R, int C, int32_t* first) {
    if (R <= r0) return;
    hipLaunchKernelGGL(k_round_first_gid, dim3(nblk((int64_t)(R - r0) * C, 256)), dim3(256), 0, s, r0, R, C, a.Bm,
                       a.wstat, a.c_off, a.p_gid, first);
}

bool sort_small_ok(int32_t m) { return m <= kSortSmallMax; }

void launch_sort_small(hipStream_t s, const DevArrays& a, int32_t m, int n, uint32_t** final_vals) {
    // (rank[] = val_b[0, m) zeroed by the caller)
    const unsigned t = (unsigned)((m + kRankTile - 1) / kRankTile), tj = (unsigned)((m + kRankJT - 1) / kRankJT);
    hipLaunchKernelGGL(k_sort_rank, dim3(t, tj), dim3(kRankTile), 0, s, m, a.recv_list, a.p_cts, a.p_chain, a.p_rr,
                       a.p_gid, a.g_S, n, a.val_b);
    hipLaunchKernelGGL(k_sort_place, dim3(nblk(m, 256)), dim3(256), 0, s, m, a.recv_list, a.val_b, a.val_a);
    *final_vals = a.val_a;
}

void launch_finish_order(hipStream_t s, const DevArrays& a, int32_t m, const uint32_t* vals, int R, int n) {
    hipLaunchKernelGGL(k_finish_order, dim3(nblk(m, 256)), dim3(256), 0, s, m, vals, a.p_gid, a.p_chain, a.p_rr,
                       a.p_cts, a.g_ntx, a.g_loaded, a.g_txnil, R, n, a.order_gid, a.g_rr, a.g_cts, a.blk_cnt,
                       a.blk_ntx, a.blk_loaded, a.blk_nil);
}

void launch_gather_i32(hipStream_t s, int64_t E, const int32_t* src, const int32_t* g_pos, int32_t* dst) {
    if (E <= 0) return;
    hipLaunchKernelGGL(k_gather_i32, dim3(nblk(E, 256)), dim3(256), 0, s, E, src, g_pos, dst);
}

}  // namespace hgx
