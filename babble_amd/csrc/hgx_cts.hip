// Consensus timestamps, software-pipelined (DecideRoundReceived's median, hashgraph.go:780-787,
// MedianTimestamp :860-868, OldestSelfAncestorToSee :141-167). DESIGN.md §3.5.
//
// Same math as k_cts_tile (hgx_kernels.hip): for a newly received event x at position p of
// chain tc, round received i = rr(x), and every witness chain c of its graph, c contributes
// ts(c, FD[x][c]) when the round-i witness of c is famous and sees x (WLAT[i][tc][c] >= j);
// the consensus timestamp is element floor(m/2) of the m contributions (upper median).
//
// What changes is the schedule. k_cts_tile handles one tile of 8 positions per block and walks
// three dependent global levels per tile (the tile's rr/ts -> the famous flag, WLAT and FD
// of every witness chain -> the FD event's timestamp) with only one tile's loads in flight.
// Here a block is resident (grid = what fits the device) and loops over its tiles with the
// three levels of three consecutive tiles in flight at once, behind the selects of a fourth:
//    gathers of tile k+1 | WLAT/FD loads of tile k+2 | rr/ts of tile k+3 | selects of tile k
// so one tile costs about one global latency or one tile's selects, whichever is longer.
// The per-chain terms that k_cts_tile loaded per lane (c_off - c_base of every chain, the
// tile geometry fu / rcnt / c_off of the launched chains) are read once per block into LDS.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <climits>
#include <cstdint>

#include "hgx_device.h"
#include "hgx_kernels.h"

namespace hgx {

constexpr int kCpT = 8;        // positions per tile (one chain, consecutive)
constexpr int kCpRing = 4;     // tile-info ring slots (a slot is rewritten 4 tiles later)
constexpr int kCpMaxC = 4096;  // chains whose per-chain terms fit the LDS tables
constexpr int64_t kCtsRedo = (int64_t)0x8000000000000000ull;   // p_cts marker: select again in 64 bits

struct CtsTileInfo {
    int32_t row[kCpT];   // round received of the event, -1 = no event at this position
    int64_t ts[kCpT];    // the event's own timestamp (base of the 32-bit offsets)
    int32_t tc, p0;      // chain (global id) and first position of the tile
};

__device__ __forceinline__ void cp_lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }
__device__ __forceinline__ void cp_order() { asm volatile("" ::: "memory"); }

template <int NPAD, typename CT>
__global__ void __launch_bounds__(256) k_cts_pipe(const int32_t* __restrict__ fu, const int32_t* __restrict__ rcnt,
                                                  const int32_t* __restrict__ p_rr, const int32_t* __restrict__ c_off,
                                                  const int32_t* __restrict__ c_base, const int32_t* __restrict__ WLAT, const CT* __restrict__ FDT,
                                                  const int64_t* __restrict__ p_ts, int64_t* __restrict__ p_cts, int C,
                                                  int n, int64_t Pcap, int c_lo, int c_cnt, int ntt) {
    constexpr int T = kCpT, LD = T + 1, NG = 256 / T, U = NPAD / NG, CPL = NPAD / 64;
    extern __shared__ __attribute__((aligned(16))) uint8_t dyn[];
    // dynamic LDS: kd[C] | tp0[c_cnt] | trc[c_cnt] | vals[2][NPAD * LD] | memb[2][NPAD * LD]
    int32_t* kd = (int32_t*)dyn;
    int32_t* tp0 = kd + C;
    int32_t* trc = tp0 + c_cnt;
    uint32_t* vals = (uint32_t*)(dyn + ((4 * (C + 2 * c_cnt) + 15) & ~15));   // (offsets from dyn keep LDS addressing)
    uint8_t* memb = (uint8_t*)(vals + 2 * NPAD * LD);
    __shared__ CtsTileInfo ring[kCpRing];
    __shared__ __attribute__((aligned(16))) uint32_t whist[4][256];

    const int t = threadIdx.x;
    for (int c = t; c < C; c += 256) kd[c] = c_off[c] - c_base[c];
    for (int c = t; c < c_cnt; c += 256) {
        tp0[c] = c_off[c_lo + c] + fu[c_lo + c];
        trc[c] = rcnt[c_lo + c];
    }
    __syncthreads();
    const int total = c_cnt * ntt;
    const int gstep = (int)gridDim.x;
    // the block's tiles: u = blockIdx.x + k * gridDim.x, time-major (u = tt * c_cnt + chain), so
    // the blocks in flight cover every chain at about the same time (their timestamp gathers
    // share L2 lines); empty tiles (past a chain's received events) are skipped
    auto next_tile = [&](int u) -> int {
        for (; u < total; u += gstep) {
            const int ci = u % c_cnt, tt = u / c_cnt;
            if (tt * T < trc[ci]) break;
        }
        return __builtin_amdgcn_readfirstlane(min(u, total));
    };
    // Every global load below is issued unconditionally (a missing event or tile reads a valid
    // dummy address and is masked afterwards): loads under a branch make the compiler's
    // vmcnt accounting at the join conservative, and it would then wait for the gathers of the
    // tile before the loads of the next tiles are even issued.
    // level 1 of tile u: rr and own timestamp of its positions (lane t: position t % T); a tile
    // u >= total gets a dummy entry (no events) so that its level 2 reads valid addresses
    const int e = t & (T - 1), cg = t / T;
    int32_t l1_rr = -1;
    int64_t l1_ts = 0;
    bool l1_in = false;
    auto l1_issue = [&](int u) {
        const bool vu = u < total;
        const int ci = vu ? u % c_cnt : 0, tt = vu ? u / c_cnt : 0;
        l1_in = vu && tt * T + e < trc[ci];
        const int p = l1_in ? tp0[ci] + tt * T + e : 0;
        l1_rr = p_rr[p];
        l1_ts = p_ts[p];
    };
    auto l1_store = [&](int u, int slot) {
        const bool vu = u < total;
        const int ci = vu ? u % c_cnt : 0, tt = vu ? u / c_cnt : 0;
        int32_t rr_v = l1_in ? l1_rr : -1;
        int64_t ts_v = l1_ts;
        asm volatile("" : "+v"(rr_v), "+v"(ts_v));   // the loads are consumed here, outside the branch
        if (t < T) {
            ring[slot].row[t] = rr_v;
            ring[slot].ts[t] = ts_v;
            if (t == 0) {
                ring[slot].tc = c_lo + ci;
                ring[slot].p0 = tp0[ci] + tt * T;
            }
        }
    };
    // level 2 of the tile in `slot`: lane (e, cg) loads WLAT (famous flag folded in) and FD of
    // chains cg + NG*u; idx = position of the FD event's timestamp, -1 = not a member
    int32_t l2_w[U];
    CT l2_fd[U];
    auto l2_issue = [&](int slot) {
        const int i = ring[slot].row[e];
        const int tc = ring[slot].tc, g = tc / n;
        const int p = ring[slot].p0 + e;
        const size_t fb = (size_t)max(i, 0) * C + (size_t)g * n;
        const size_t wrow = (fb + (tc - g * n)) * n;
#pragma unroll
        for (int u = 0; u < U; u++) {
            const int c = cg + NG * u;
            const bool in = i >= 0 && c < n;
            const int cc = in ? c : 0;
            l2_w[u] = WLAT[wrow + cc];
            l2_fd[u] = FDT[(size_t)cc * Pcap + (in ? p : 0)];
        }
    };
    int32_t idx[U];
    auto l2_finish = [&](int slot) {
        const int i = ring[slot].row[e];
        const int tc = ring[slot].tc, g = tc / n;
        const int j = ring[slot].p0 + e - kd[tc];   // Index of the event
#pragma unroll
        for (int u = 0; u < U; u++) {
            const int c = cg + NG * u;
            const bool in = i >= 0 && c < n;
            const int cc = in ? c : 0;
            const int32_t k = kd[g * n + cc] + Coord<CT>::fd(l2_fd[u]);
            idx[u] = (in & (l2_w[u] >= j)) ? k : -1;
        }
    };

    // prologue: tiles 0 and 1's level 1, tile 0's level 2, then tile 0's gathers, tile 1's level
    // 2 and tile 2's level 1 go out
    int u0 = next_tile(blockIdx.x);
    if (u0 >= total) return;
    int u1 = next_tile(u0 + gstep);
    int u2 = next_tile(u1 + gstep);
    l1_issue(u0);
    l1_store(u0, 0);
    l1_issue(u1);
    l1_store(u1, 1);
    __syncthreads();
    l2_issue(0);
    l2_finish(0);
    const int lane = lane_id(), wave = t >> 6;
    int64_t x[U];
#pragma unroll
    for (int u = 0; u < U; u++) x[u] = p_ts[max(idx[u], 0)];
    cp_order();
    l2_issue(1);
    cp_order();
    l1_issue(u2);
    cp_order();

    // iteration k: (A) tile k's gathers land -> offsets and membership into LDS buffer k & 1;
    // (B) tile k+1's gather indices, tile k+2's level 1 into the ring; barrier; (C) tile k+1's
    // gathers, tile k+2's level 2 and tile k+3's level 1 go out; (D) tile k's selects run while
    // they are in flight
    for (int k = 0; u0 < total; k++) {
        const int s0 = k & (kCpRing - 1), s1 = (k + 1) & (kCpRing - 1), s2 = (k + 2) & (kCpRing - 1);
        {   // (A)
            uint32_t* v = vals + (k & 1) * NPAD * LD;
            uint8_t* mb = memb + (k & 1) * NPAD * LD;
            const int64_t base = ring[s0].ts[e];
#pragma unroll
            for (int u = 0; u < U; u++) {
                const int c = cg + NG * u;
                const bool ok = idx[u] >= 0;
                const int64_t dlt = x[u] - base;
                const bool ov = ok && (dlt < INT32_MIN || dlt > INT32_MAX);
                v[c * LD + e] = (uint32_t)(int32_t)dlt ^ 0x80000000u;   // (c >= n: not a member)
                mb[c * LD + e] = (uint8_t)((ok ? 1 : 0) | (ov ? 2 : 0));
            }
        }
        // (B)
        l2_finish(s1);
        l1_store(u2, s2);
        cp_lds_barrier();
        // (C)
        const int u3 = next_tile(u2 + gstep);
#pragma unroll
        for (int u = 0; u < U; u++) x[u] = p_ts[max(idx[u], 0)];
        cp_order();
        l2_issue(s2);
        cp_order();
        l1_issue(u3);
        cp_order();
        // (D) one wave per event: radix select of element floor(m/2)
        {
            const uint32_t* v = vals + (k & 1) * NPAD * LD;
            const uint8_t* mb = memb + (k & 1) * NPAD * LD;
            for (int ev = wave; ev < T; ev += 4) {
                if (ring[s0].row[ev] < 0) continue;   // wave-uniform
                bool ok[CPL];
                uint32_t vv[CPL];
                int m = 0;
                bool any_ov = false;
#pragma unroll
                for (int q = 0; q < CPL; q++) {
                    const int c = lane + 64 * q;
                    const uint8_t b = mb[c * LD + ev];
                    ok[q] = (b & 1) != 0;
                    vv[q] = v[c * LD + ev];
                    m += __popcll(__ballot(ok[q]));
                    any_ov |= __ballot((b & 2) != 0) != 0;
                }
                // rare: an offset beyond 32 bits -> kCtsRedo, k_cts_redo selects in 64 bits
                int64_t res = kCtsRedo;
                if (!any_ov) {
                    const uint32_t sel = wave_select_kth32<CPL>(vv, ok, m / 2, whist[wave]);
                    res = ring[s0].ts[ev] + (int64_t)(int32_t)(sel ^ 0x80000000u);
                }
                if (lane == 0) p_cts[ring[s0].p0 + ev] = res;
            }
        }
        u0 = u1;
        u1 = u2;
        u2 = u3;
    }
}

// the events k_cts_pipe left at kCtsRedo (a timestamp offset beyond 32 bits): one wave per
// event regathers the contributions and selects in 64 bits. A true median equal to kCtsRedo
// is recomputed to the same value, so the marker needs no separate flag.
template <int NPAD, typename CT>
__global__ void __launch_bounds__(256) k_cts_redo(const int32_t* __restrict__ fu, const int32_t* __restrict__ rcnt,
                                                  const int32_t* __restrict__ p_rr, const int32_t* __restrict__ c_off,
                                                  const int32_t* __restrict__ c_base, const int32_t* __restrict__ WLAT,
                                                  const CT* __restrict__ FDT, const int64_t* __restrict__ p_ts,
                                                  int64_t* __restrict__ p_cts, int C, int n, int64_t Pcap, int c_lo) {
    constexpr int CPL = NPAD / 64;
    __shared__ int32_t list[256];
    __shared__ int32_t cnt;
    __shared__ __attribute__((aligned(16))) uint32_t whist[4][256];
    const int gc = c_lo + blockIdx.y, g = gc / n;
    const int k = (int)blockIdx.x * 256 + threadIdx.x;
    if (threadIdx.x == 0) cnt = 0;
    __syncthreads();
    const int64_t p0 = (int64_t)c_off[gc] + fu[gc];
    if (k < rcnt[gc] && p_cts[p0 + k] == kCtsRedo) list[atomicAdd(&cnt, 1)] = k;
    __syncthreads();
    const int lane = lane_id(), wave = threadIdx.x >> 6;
    for (int q0 = wave; q0 < cnt; q0 += 4) {
        const int64_t p = p0 + list[q0];
        const int i = p_rr[p];
        const int j = c_base[gc] + (int)(p - c_off[gc]);
        const size_t row = ((size_t)i * C + gc) * n;
        uint64_t v[CPL];
        bool ok[CPL];
        int m = 0;
#pragma unroll
        for (int q = 0; q < CPL; q++) {
            const int c = lane + 64 * q;
            ok[q] = c < n && WLAT[row + c] >= j;
            int64_t x = 0;
            if (ok[q]) {
                const int ch = g * n + c;
                x = p_ts[c_off[ch] - c_base[ch] + Coord<CT>::fd(FDT[(size_t)c * Pcap + p])];
            }
            v[q] = (uint64_t)x ^ 0x8000000000000000ull;
            m += __popcll(__ballot(ok[q]));
        }
        const int64_t res = (int64_t)(wave_select_kth<CPL>(v, ok, m / 2, whist[wave]) ^ 0x8000000000000000ull);
        if (lane == 0) p_cts[p] = res;
    }
}

template <int NPAD, typename CT>
static bool cts_pipe_launch(hipStream_t s, const DevArrays& a, int c_lo, int c_cnt, int C, int n, int64_t P,
                            int max_cnt) {
    constexpr int LD = kCpT + 1;
    const size_t lds = (((size_t)4 * C + (size_t)8 * c_cnt + 15) & ~(size_t)15) + (size_t)2 * NPAD * LD * 5;
    const void* f = (const void*)k_cts_pipe<NPAD, CT>;
    static int dev_cus[64] = {0};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return false;
    if (ensure_lds_limit(f, lds) != hipSuccess) return false;
    if (dev_cus[dev] == 0) {
        int cus = 0;
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
            return false;
        dev_cus[dev] = cus;
    }
    int per_cu = 0;
    if (blocks_per_cu(f, 256, lds, &per_cu) != hipSuccess || per_cu < 1) return false;
    const int ntt = (max_cnt + kCpT - 1) / kCpT;
    const int64_t tiles = (int64_t)c_cnt * ntt;
    if (tiles <= 0) return true;
    if (tiles > 0x7FFFFFFF - (int64_t)dev_cus[dev] * per_cu) return false;
    const unsigned grid = (unsigned)std::min<int64_t>(tiles, (int64_t)dev_cus[dev] * per_cu);
    hipLaunchKernelGGL((k_cts_pipe<NPAD, CT>), dim3(grid), dim3(256), lds, s, a.fu, a.rcnt, a.p_rr, a.c_off, a.c_base,
                       a.WLAT, (const CT*)a.FDT, a.p_ts, a.p_cts, C, n, P, c_lo, c_cnt, ntt);
    hipLaunchKernelGGL((k_cts_redo<NPAD, CT>), dim3((max_cnt + 255) / 256, c_cnt), dim3(256), 0, s, a.fu, a.rcnt, a.p_rr,
                       a.c_off, a.c_base, a.WLAT, (const CT*)a.FDT, a.p_ts, a.p_cts, C, n, P, c_lo);
    return true;
}

template <typename CT>
static bool launch_cts_pipe_t(hipStream_t s, const DevArrays& a, int c_lo, int c_cnt, int C, int n, int64_t P,
                              int max_cnt) {
    if (n <= 64) return cts_pipe_launch<64, CT>(s, a, c_lo, c_cnt, C, n, P, max_cnt);
    if (n <= 128) return cts_pipe_launch<128, CT>(s, a, c_lo, c_cnt, C, n, P, max_cnt);
    if (n <= 256) return cts_pipe_launch<256, CT>(s, a, c_lo, c_cnt, C, n, P, max_cnt);
    return cts_pipe_launch<512, CT>(s, a, c_lo, c_cnt, C, n, P, max_cnt);
}

bool cts_pipe_ok(int n, int C) { return n > 32 && n <= 512 && C <= kCpMaxC; }

bool launch_cts_pipe(hipStream_t s, const DevArrays& a, int c_lo, int c_cnt, int C, int n, int64_t P, int max_cnt) {
    if (max_cnt <= 0 || c_cnt <= 0) return true;
    if (!cts_pipe_ok(n, C)) return false;
    return a.compact ? launch_cts_pipe_t<uint16_t>(s, a, c_lo, c_cnt, C, n, P, max_cnt)
                     : launch_cts_pipe_t<int32_t>(s, a, c_lo, c_cnt, C, n, P, max_cnt);
}

}  // namespace hgx
