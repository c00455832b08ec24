// lastAncestors in one pass: a dataflow wavefront per (graph, column block).
//
// LA[x] = max(LA[sp(x)], LA[op(x)]), LA[x][cr(x)] = Index(x)  (hashgraph.go:470-496). Every
// column j of a row depends only on column j of its two parents, so the columns split into
// independent 16-byte blocks (8 compact / 4 int32 coordinates; 4 bytes for n > 256). One
// workgroup owns one block of one graph and every chain of that graph: lane i walks chain i
// in order, carrying the self-parent row in registers, and takes the op row's block from an
// LDS ring where the op chain's lane published it. A row therefore costs one LDS round
// trip plus a 16-byte store, instead of the ~12 recomputations per row of the Gauss-Seidel
// sweeps (k_la_sweep, hgx_kernels.hip), whose within-window staleness propagates along every
// chain. The price is latency: a chain waits for its op rows, so the pass follows the DAG's
// op depth (about 2.3 x the chain length on gossip traces) at one LDS hop per level.
//
// LDS per workgroup (n chains, ring of R rows per chain, queue of Q op descriptors):
//   ring_d [R][NP][DW] op-row blocks, slot = row % R (NP = n rounded up to a power of two)
//   ring_t [R][NP]     slot tags: the row held, -1 empty, -2 being rewritten (seqlock)
//   q      [Q][NP]     packed op descriptors (p_opk) of the rows ahead of each lane
//   lqv [n], prog [n], s_old [n], s_off [n], s_len [n]
// One extra wave streams the op descriptors from HBM into q (the compute lanes never wait
// on a global load in the steady state). A row whose op row already left the ring is read
// from HBM: its producer drained its stores (vmcnt) before reusing that ring slot.
// All waits are bounded; a lane that gives up sets *err and the host falls back to the
// sweeps.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>

#include "hgx_device.h"
#include "hgx_kernels.h"

namespace hgx {

namespace {

template <typename CT>
struct LaW;
template <>
struct LaW<int32_t> {
    static constexpr uint32_t kNone = 0xFFFFFFFFu;
    __device__ __forceinline__ static uint32_t wmax(uint32_t a, uint32_t b) {
        return (uint32_t)max((int32_t)a, (int32_t)b);
    }
    static constexpr int kPerWord = 1;
    // the own coordinate of chain cl: word cl, all 32 bits
    __device__ __forceinline__ static uint32_t own_mask(int) { return 0xFFFFFFFFu; }
    __device__ __forceinline__ static uint32_t own_bits(int, int32_t own) { return (uint32_t)own; }
};
template <>
struct LaW<uint16_t> {
    static constexpr uint32_t kNone = 0u;
    typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
    __device__ __forceinline__ static uint32_t wmax(uint32_t a, uint32_t b) {
        const u16x2 m = __builtin_elementwise_max(__builtin_bit_cast(u16x2, a), __builtin_bit_cast(u16x2, b));
        return __builtin_bit_cast(uint32_t, m);
    }
    static constexpr int kPerWord = 2;
    // the own coordinate of chain cl: half (cl & 1) of word cl / 2, stored as value + 1
    __device__ __forceinline__ static uint32_t own_mask(int cl) { return 0xFFFFu << ((cl & 1) * 16); }
    __device__ __forceinline__ static uint32_t own_bits(int cl, int32_t own) {
        return ((uint32_t)(own + 1) & 0xFFFFu) << ((cl & 1) * 16);
    }
};

// LDS accesses in program order: a wave's LDS operations execute in issue order, and the
// empty asm (a compiler-only memory barrier) keeps the compiler from reordering, merging or
// hoisting them. Not `volatile`: the backend follows every volatile access with a wait for
// ALL outstanding memory operations (s_waitcnt vmcnt(0)), which would stall each row on the
// previous rows' HBM stores.
#define HGX_CB() asm volatile("" ::: "memory")
__device__ __forceinline__ int32_t lds_ld(const int32_t* p) {
    HGX_CB();
    const int32_t v = *p;
    HGX_CB();
    return v;
}
__device__ __forceinline__ void lds_st(int32_t* p, int32_t v) {
    HGX_CB();
    *p = v;
    HGX_CB();
}

// Uses the loaded registers inside the (rare) branch that loaded them from HBM, so the
// compiler's wait for those loads lands there; otherwise the hot path after the join would
// wait for every outstanding store (s_waitcnt vmcnt(0)) on every row.
template <int DW>
__device__ __forceinline__ void settle(uint32_t (&v)[DW]) {
#pragma unroll
    for (int w = 0; w < DW; w++) asm volatile("" : "+v"(v[w]));
}

// a block of DW words: one LDS / HBM access (DW * 4 bytes, naturally aligned)
template <int DW>
__device__ __forceinline__ void ring_load(const uint32_t* p, uint32_t (&v)[DW]) {
    HGX_CB();
    if constexpr (DW % 8 == 0) {   // 8 or 16 words: 16-byte accesses
#pragma unroll
        for (int k = 0; k < DW / 4; k++) {
            const uint4 x = ((const uint4*)p)[k];
            v[4 * k] = x.x; v[4 * k + 1] = x.y; v[4 * k + 2] = x.z; v[4 * k + 3] = x.w;
        }
    } else if constexpr (DW == 4) {
        const uint4 x = *(const uint4*)p;
        v[0] = x.x; v[1] = x.y; v[2] = x.z; v[3] = x.w;
    } else if constexpr (DW == 2) {
        const uint2 x = *(const uint2*)p;
        v[0] = x.x; v[1] = x.y;
    } else {
        v[0] = *p;
    }
    HGX_CB();
}
template <int DW>
__device__ __forceinline__ void ring_store(uint32_t* p, const uint32_t (&v)[DW]) {
    HGX_CB();
    if constexpr (DW % 8 == 0) {
#pragma unroll
        for (int k = 0; k < DW / 4; k++) ((uint4*)p)[k] = make_uint4(v[4 * k], v[4 * k + 1], v[4 * k + 2], v[4 * k + 3]);
    } else if constexpr (DW == 4) *(uint4*)p = make_uint4(v[0], v[1], v[2], v[3]);
    else if constexpr (DW == 2) *(uint2*)p = make_uint2(v[0], v[1]);
    else *p = v[0];
    HGX_CB();
}
template <int DW>
__device__ __forceinline__ void row_store(uint32_t* p, const uint32_t (&v)[DW]) {
    if constexpr (DW % 8 == 0) {
#pragma unroll
        for (int k = 0; k < DW / 4; k++) ((uint4*)p)[k] = make_uint4(v[4 * k], v[4 * k + 1], v[4 * k + 2], v[4 * k + 3]);
    } else if constexpr (DW == 4) *(uint4*)p = make_uint4(v[0], v[1], v[2], v[3]);
    else if constexpr (DW == 2) *(uint2*)p = make_uint2(v[0], v[1]);
    else *p = v[0];
}

constexpr int kTagEmpty = -1, kTagBusy = -2;
constexpr int kNoDesc = -2147483647 - 1;
constexpr uint32_t kSpinCap = 1u << 24;   // consecutive idle iterations before a lane gives up

}  // namespace

// lower_bound of gid `x` in the chain's (increasing) gids p_gid[off, off + len)
__device__ __forceinline__ int chain_lower_bound(const int32_t* __restrict__ p_gid, int off, int len, int64_t x) {
    int lo = 0, hi = len;
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if ((int64_t)p_gid[off + mid] < x) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

// DW words per block, R ring rows, Q queued descriptors, NLW loader waves, J chains per
// loader lane (n <= 64 NLW J), CH descriptors per refill. MODE 0: all rows, exact;
// 1 (incremental): rows from c_old, the rows below are final; 2 (time segments, one graph):
// workgroup (segment ts, block) builds the rows with gids in [E ts / nts, E (ts + 1) / nts),
// taking every row before its segment as none, so its rows are lower bounds (it reads from
// LA only its own rows whose ring slot moved on, so LA needs no reset); 3
// (segment heads, after 2):
// the first `head` rows of every chain in each segment again, now that the earlier
// segments' tails hold their final values (a segment's lower bounds are wrong only near its
// start: the missing knowledge is soon superseded by newer events). k_la_sweep's verify
// sweep then confirms (or completes) the result.
template <typename CT, int DW, int R, int Q, int NLW, int J, int CH, int MODE>
__global__ void __launch_bounds__(1024) k_la_wave(uint32_t* __restrict__ LA, const int32_t* __restrict__ p_opk,
                                                  const int32_t* __restrict__ c_off, const int32_t* __restrict__ c_len,
                                                  const int32_t* __restrict__ c_base,
                                                  const int32_t* __restrict__ c_old,
                                                  const int32_t* __restrict__ p_gid, int64_t E, int nts, int head,
                                                  int n, int lgnp, int nwd, int nblk, int32_t* __restrict__ err,
                                                  const int32_t* __restrict__ lmap, int na) {
    typedef LaW<CT> W;
    extern __shared__ uint32_t smem[];
    // slot-major arrays with a power-of-two chain stride NP = 2^lgnp >= n (index = shifts)
    const int NP = 1 << lgnp;
    uint32_t* ring_d = smem;                                      // [R][NP][DW]
    int32_t* ring_t = (int32_t*)(ring_d + (size_t)R * NP * DW);   // [R][NP]
    int32_t* q = ring_t + R * NP;                                 // [Q][NP]
    int32_t* lqv = q + Q * NP;
    int32_t* prog = lqv + n;
    int32_t* s_old = prog + n;
    int32_t* s_off = s_old + n;
    int32_t* s_len = s_off + n;
    int32_t* s_abort = s_len + n;
    const int b = blockIdx.x % nblk, ts = (blockIdx.x / nblk) % nts, g = blockIdx.x / nblk / nts;
    const int c0 = g * n;
    const int wb = b * DW;   // first word of the block
    const int tid = threadIdx.x;
    for (int t = tid; t < R * NP; t += blockDim.x) ring_t[t] = kTagEmpty;
    for (int t = tid; t < n; t += blockDim.x) {
        const int off = c_off[c0 + t], len = c_len[c0 + t];
        int o = 0, e = len;
        if constexpr (MODE == 1) o = c_old[c0 + t];
        if constexpr (MODE >= 2) {
            o = ts == 0 ? 0 : chain_lower_bound(p_gid, off, len, E * ts / nts);
            e = ts == nts - 1 ? len : chain_lower_bound(p_gid, off, len, E * (ts + 1) / nts);
            if constexpr (MODE == 3) e = ts == 0 ? o : min(e, o + head);
        }
        lqv[t] = o;
        prog[t] = o;
        s_old[t] = o;   // rows below: from HBM (final, or lower bounds in MODE 2)
        s_off[t] = off;
        s_len[t] = e;   // rows from here: later segments (MODE 3: not rebuilt, from HBM)
    }
    if (tid == 0) *s_abort = 0;
    __syncthreads();
    // compute lanes (whole waves): one per chain, or per chain with events (lmap); the last NLW
    // waves load (they walk every chain: those without events have nothing to load)
    const int nl = lmap ? na : n;
    const int ncw = (nl + 63) & ~63;
    if (tid >= ncw) {
        // ---- loader wave: op descriptors of rows [lqv, lqv + CH) of each owned chain -> q
        // (its per-chain state lives in LDS: lqv is written by this wave only)
        const int l = tid - ncw;
        uint32_t idle = 0;
        for (;;) {
            bool left = false, need[J];
            int lq[J];
#pragma unroll
            for (int j = 0; j < J; j++) {
                const int i = l + 64 * NLW * j;
                need[j] = false;
                lq[j] = 0;
                if (i < n) {
                    lq[j] = lds_ld(&lqv[i]);
                    if (lq[j] < s_len[i]) {
                        left = true;
                        need[j] = lq[j] + CH <= lds_ld(&prog[i]) + Q;
                    }
                }
            }
            if (!left) break;
            int32_t v[J][CH];
#pragma unroll
            for (int j = 0; j < J; j++)
                if (need[j]) {
                    const int i = l + 64 * NLW * j;
                    const int o = s_off[i] + lq[j], m = s_len[i] - lq[j];
#pragma unroll
                    for (int t = 0; t < CH; t++) v[j][t] = (t < m) ? p_opk[o + t] : -1;
                }
            bool any = false;
#pragma unroll
            for (int j = 0; j < J; j++)
                if (need[j]) {
                    const int i = l + 64 * NLW * j;
#pragma unroll
                    for (int t = 0; t < CH; t++) lds_st(&q[(((unsigned)(lq[j] + t) % Q) << lgnp) + i], v[j][t]);
                    HGX_CB();
                    lds_st(&lqv[i], min(lq[j] + CH, s_len[i]));
                    any = true;
                }
            if (any) {
                idle = 0;
            } else {
                if (lds_ld(s_abort) || ++idle > kSpinCap) break;
                __builtin_amdgcn_s_sleep(1);
            }
        }
        return;
    }
    // ---- compute lane: chain c0 + i, rows [s_old[i], len)
    if (tid >= nl) return;
    const int i = lmap ? lmap[tid] : tid;
    const int len = s_len[i];
    const int off = s_off[i];
    int own0 = c_base[c0 + i];   // Index of the chain's row 0
    asm volatile("" : "+v"(own0));   // wait for this load here, not inside the loop (settle)
    const int ow = i / W::kPerWord - wb;   // the block word holding the own coordinate (if in [0, DW))
    const uint32_t omask = W::own_mask(i);
    int k = s_old[i];
    uint32_t carry[DW];
#pragma unroll
    for (int w = 0; w < DW; w++)
        carry[w] = (k > 0 && MODE != 2) ? LA[(size_t)(off + k - 1) * nwd + wb + w] : W::kNone;
    settle(carry);
    uint32_t* dst = LA + (size_t)(off + k) * nwd + wb;   // row k's block (advanced per row)
    // descriptor of row k: p_opk, or kNoDesc while the loader has not queued it
    int opv = kNoDesc;
    uint32_t idle = 0;
    while (k < len) {
        // one LDS round trip: the queue (rows k, k + 1) and the op row's ring slot
        const int lv = lds_ld(&lqv[i]);
        const int q0 = lds_ld(&q[(((unsigned)k % Q) << lgnp) + i]);
        const int q1 = lds_ld(&q[(((unsigned)(k + 1) % Q) << lgnp) + i]);
        const bool has_op = opv >= 0;
        const int opc = has_op ? (opv >> kOpkBits) : 0;
        const int opk = has_op ? (opv & ((1 << kOpkBits) - 1)) : 0;
        const int sl = (((unsigned)opk % R) << lgnp) + opc;
        int old = 0;
        int end = 0x7FFFFFFF;
        if constexpr (MODE != 0) old = lds_ld(&s_old[opc]);
        if constexpr (MODE == 3) end = lds_ld(&s_len[opc]);
        const int t1 = lds_ld(&ring_t[sl]);
        uint32_t od[DW];
        ring_load<DW>(ring_d + (size_t)sl * DW, od);
        const int t2 = lds_ld(&ring_t[sl]);
        bool ready = opv == -1 || (has_op && t1 == opk && t2 == opk);
        if (opv == -1) {
#pragma unroll
            for (int w = 0; w < DW; w++) od[w] = W::kNone;
        }
        // rare: the op row is in HBM (a row of an earlier call, or its ring slot moved on;
        // its producer drained that store before reusing the slot, and the load bypasses L1)
        const bool from_old = MODE != 0 && has_op && (opk < old || opk >= end);
        if (from_old || (has_op && !ready && t1 > opk)) {
            if (MODE == 2 && from_old) {
                // an earlier segment's row: LA may still hold an earlier DivideRounds's row there;
                // none is a lower bound (the head pass and the verify sweep complete it)
#pragma unroll
                for (int w = 0; w < DW; w++) od[w] = W::kNone;
            } else {
                uint32_t* src = LA + (size_t)(s_off[opc] + opk) * nwd + wb;
#pragma unroll
                for (int w = 0; w < DW; w++)
                    od[w] = __hip_atomic_load(src + w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                settle(od);
            }
            ready = true;
        }
        const bool wave_idle = __ballot(ready) == 0;
        if (!ready) {
            if (opv == kNoDesc && lv > k) opv = q0;
            if (wave_idle) __builtin_amdgcn_s_sleep(1);   // leave the SIMD to the other waves
            if (((++idle) & 4095) == 0 && (idle > kSpinCap || lds_ld(s_abort))) {
                lds_st(s_abort, 1);
                atomicOr(err, 1);
                break;
            }
            continue;
        }
        idle = 0;
        uint32_t v[DW];
#pragma unroll
        for (int w = 0; w < DW; w++) {
            v[w] = W::wmax(carry[w], od[w]);
            v[w] = w == ow ? ((v[w] & ~omask) | W::own_bits(i, own0 + k)) : v[w];
        }
        // the store of row k - R (this slot's previous row) must be complete before the
        // slot is reused: at least R - 1 later stores of this lane were issued since
        // (64-byte blocks: four stores per row, so 23 outstanding = at most rows k - 1 .. k - 6)
        if constexpr (DW == 16 && R == 8) asm volatile("s_waitcnt vmcnt(23)" ::: "memory");
        else if constexpr (R >= 16) asm volatile("s_waitcnt vmcnt(15)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(7)" ::: "memory");
        const int ws = (((unsigned)k % R) << lgnp) + i;
        lds_st(&ring_t[ws], kTagBusy);
        ring_store<DW>(ring_d + (size_t)ws * DW, v);
        lds_st(&ring_t[ws], k);
        row_store<DW>(dst, v);
        dst += nwd;
        lds_st(&prog[i], k + 1);
#pragma unroll
        for (int w = 0; w < DW; w++) carry[w] = v[w];
        k++;
        opv = lv > k ? q1 : kNoDesc;
    }
}

namespace {
template <typename CT, int DW, int R, int Q, int NLW, int J, int CH, int MODE>
hipError_t la_wave_launch1(hipStream_t s, const DevArrays& a, int G, int n, const int32_t* c_old, int64_t E, int nts,
                           int head, int32_t* err, const int32_t* lmap, int na) {
    const int nwd = a.compact ? n / 2 : n;
    const int nblk = nwd / DW;
    int lgnp = 0;
    while ((1 << lgnp) < n) lgnp++;
    const size_t np2 = (size_t)1 << lgnp;
    const size_t words = np2 * (R * DW + R + Q) + 5 * (size_t)n + 1;
    auto kern = k_la_wave<CT, DW, R, Q, NLW, J, CH, MODE>;
    {
        const hipError_t e = ensure_lds_limit((const void*)kern, 160 * 1024);
        if (e != hipSuccess) return e;
    }
    const int threads = (((lmap ? na : n) + 63) & ~63) + 64 * NLW;
    if (threads > 1024 || (lmap && G != 1)) return hipErrorInvalidValue;
    hipLaunchKernelGGL(kern, dim3(G * nts * nblk), dim3(threads), words * 4, s, (uint32_t*)a.LA, a.p_opk, a.c_off,
                       a.c_len, a.c_base, c_old, a.p_gid, E, nts, head, n, lgnp, nwd, nblk, err, lmap, na);
    return hipGetLastError();
}
template <typename CT, int DW, int R, int Q, int NLW, int J, int CH>
hipError_t la_wave_launch(hipStream_t s, const DevArrays& a, int G, int n, const int32_t* c_old, int64_t E,
                          int32_t* err, const int32_t* lmap, int na) {
    if (c_old) return la_wave_launch1<CT, DW, R, Q, NLW, J, CH, 1>(s, a, G, n, c_old, E, 1, 0, err, lmap, na);
    return la_wave_launch1<CT, DW, R, Q, NLW, J, CH, 0>(s, a, G, n, nullptr, E, 1, 0, err, lmap, na);
}
// block width and ring sizes of the time-segment passes: one workgroup per CU (the passes
// are issue-bound, so wider blocks share the per-row overhead over more coordinates)
struct SegCfg {
    int dw, r, q;
};
inline SegCfg seg_cfg(int n, int nwd) {
    // n in (128, 256]: 64-byte blocks (half the column blocks, so twice the time segments fill the CUs: a
    // segment's pass walks half the DAG depth), the descriptor queue at 16 to keep one workgroup's LDS
    // under 160 KB
    if (n > 128 && n <= 256 && nwd % 16 == 0) return {16, 8, 16};
    if (n <= 256) return {nwd % 8 == 0 ? 8 : (nwd % 4 == 0 ? 4 : 1), 8, 32};
    if (n <= 512) return {nwd % 4 == 0 ? 4 : 1, 8, 16};
    return {nwd % 2 == 0 ? 2 : 1, 8, 8};
}
// LDS: NP * (R * DW + R + Q) + 5 n words <= 160 KB (NP = n rounded up to a power of two); DW divides the row's words
template <typename CT>
hipError_t la_wave_dispatch(hipStream_t s, const DevArrays& a, int G, int n, const int32_t* c_old, int64_t E, int nts,
                            int head, int32_t* err, const int32_t* lmap, int na, bool narrow) {
    const int nwd = a.compact ? n / 2 : n;
    if (nts > 1) {   // time segments: wider blocks, smaller rings (seg_cfg)
        const SegCfg g = seg_cfg(n, nwd);
#define SEG(DW_, R_, Q_, NLW_, J_, CH_)                                                                                \
    return head > 0 ? la_wave_launch1<CT, DW_, R_, Q_, NLW_, J_, CH_, 3>(s, a, G, n, nullptr, E, nts, head, err, lmap, \
                                                                          na)                                          \
                    : la_wave_launch1<CT, DW_, R_, Q_, NLW_, J_, CH_, 2>(s, a, G, n, nullptr, E, nts, 0, err, lmap, na)
        if (n <= 256) {
            if (g.dw == 16) SEG(16, 8, 16, 1, 4, 8);
            if (g.dw == 8) SEG(8, 8, 32, 1, 4, 8);
            if (g.dw == 4) SEG(4, 8, 32, 1, 4, 8);
            SEG(1, 8, 32, 1, 4, 8);
        }
        if (n <= 512) {
            if (g.dw == 4) SEG(4, 8, 16, 1, 8, 4);
            SEG(1, 8, 16, 1, 8, 4);
        }
        if (g.dw == 2) SEG(2, 8, 8, 2, 8, 2);
        SEG(1, 8, 8, 2, 8, 2);
#undef SEG
    }
    if (n <= 128) {
        if (nwd % 4 == 0 && !(narrow && c_old)) return la_wave_launch<CT, 4, 32, 64, 1, 2, 16>(s, a, G, n, c_old, E, err, lmap, na);
        return la_wave_launch<CT, 1, 32, 64, 1, 2, 16>(s, a, G, n, c_old, E, err, lmap, na);
    }
    if (n <= 256) {
        if (nwd % 4 == 0 && !(narrow && c_old))
            return la_wave_launch<CT, 4, 16, 64, 1, 4, 16>(s, a, G, n, c_old, E, err, lmap, na);
        return la_wave_launch<CT, 1, 16, 64, 1, 4, 16>(s, a, G, n, c_old, E, err, lmap, na);
    }
    if (n <= 512) return la_wave_launch<CT, 1, 16, 32, 1, 8, 8>(s, a, G, n, c_old, E, err, lmap, na);
    // n > 512: 8-byte blocks and an 8-row ring (one workgroup per CU: half the workgroups of
    // 4-byte blocks, which ran in two generations)
    if (nwd % 2 == 0) return la_wave_launch<CT, 2, 8, 8, 2, 8, 2>(s, a, G, n, c_old, E, err, lmap, na);
    return la_wave_launch<CT, 1, 8, 16, 2, 8, 4>(s, a, G, n, c_old, E, err, lmap, na);
}
}  // namespace

// ---- small graphs: the whole graph in one workgroup's LDS ----------------------------------
// Every row (n <= 32 coordinates: nwd <= 16 words, padded to NW) and every op descriptor of the graph
// sit in LDS, packed chain after chain; one wave walks the chains (lane c = chain c, the self-parent
// row carried in registers) and polls the op chain's progress counter in LDS: a lane takes its next
// row as soon as prog[op chain] > op row. A row costs ONE LDS round trip: its descriptor (op row's
// packed index, op chain, op row) was prefetched with the previous row's reads, and the op row, the
// progress word and the next descriptor are read together. No ring, tags or loader wave. The new
// rows go to HBM coalesced at the end; rows below c_old (incremental) are read from HBM first.
template <int NW>
__global__ void __launch_bounds__(256) k_la_small(uint32_t* __restrict__ LA, const int32_t* __restrict__ p_opk,
                                                  const int32_t* __restrict__ c_off, const int32_t* __restrict__ c_len,
                                                  const int32_t* __restrict__ c_base, const int32_t* __restrict__ c_old,
                                                  int n, int nwd, int compact, int32_t* __restrict__ err) {
    extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
    const int g = blockIdx.x, c0 = g * n, tid = threadIdx.x, nt = blockDim.x;
    __shared__ int32_t s_P;
    int32_t* prog = (int32_t*)smem;   // [64] rows done per chain
    int32_t* cpos = prog + 64;        // [64] chain start in the packed rows
    if (tid == 0) {
        int acc = 0;
        for (int c = 0; c < n; c++) {
            cpos[c] = acc;
            acc += c_len[c0 + c];
        }
        s_P = acc;
    }
    for (int c = tid; c < n; c += nt) prog[c] = c_old ? c_old[c0 + c] : 0;
    __syncthreads();
    const int P = s_P;
    int2* desc = (int2*)(cpos + 64);                       // [P + 1, even] {op row's packed index, p_opk}
    uint32_t* rows = (uint32_t*)(desc + ((P + 2) & ~1));   // [P][NW], 16-byte aligned
    for (int c = 0; c < n; c++) {
        const int o = cpos[c], len = c_len[c0 + c], off = c_off[c0 + c];
        for (int x = tid; x < len; x += nt) {
            const int v = p_opk[off + x];
            desc[o + x] = make_int2(v >= 0 ? cpos[v >> kOpkBits] + (v & ((1 << kOpkBits) - 1)) : -1, v);
        }
        if (c_old) {   // final rows of earlier calls
            const int m = c_old[c0 + c];
            for (int x = tid; x < m * nwd; x += nt) rows[(size_t)(o + x / nwd) * NW + x % nwd] = LA[(size_t)off * nwd + x];
        }
    }
    if (tid == 0) desc[P] = make_int2(-1, -1);   // (the prefetch past the last row)
    __syncthreads();
    if (tid < 64) {
        const int c = tid;
        const bool live = c < n;
        const int len = live ? c_len[c0 + c] : 0, base = live ? cpos[c] : 0;
        int k = live ? prog[c] : 0;
        const int own0 = live ? c_base[c0 + c] : 0;
        // own coordinate: word c / 2 (compact, value + 1 in half c % 2) or word c
        const int ow = compact ? c >> 1 : c;
        const uint32_t omask = compact ? (0xFFFFu << ((c & 1) * 16)) : 0xFFFFFFFFu;
        const uint32_t none = compact ? 0u : 0xFFFFFFFFu;
        uint32_t carry[NW];
#pragma unroll
        for (int w = 0; w < NW; w++) carry[w] = (k > 0) ? rows[(size_t)(base + k - 1) * NW + w] : none;
        int2 d = k < len ? desc[base + k] : make_int2(-1, -1);
        uint32_t guard = 0;
        while (__any(k < len)) {
            if (k < len) {
                const int opc = d.y >= 0 ? d.y >> kOpkBits : 0, opk = d.y & ((1 << kOpkBits) - 1);
                // one batch: progress word, op row, next descriptor
                const int pr = prog[opc];
                uint32_t od[NW];
                const uint32_t* src = rows + (size_t)(d.x >= 0 ? d.x : 0) * NW;
                if constexpr (NW % 4 == 0) {
#pragma unroll
                    for (int q = 0; q < NW / 4; q++) {
                        const uint4 x4 = ((const uint4*)src)[q];
                        od[4 * q] = x4.x; od[4 * q + 1] = x4.y; od[4 * q + 2] = x4.z; od[4 * q + 3] = x4.w;
                    }
                } else if constexpr (NW == 2) {
                    const uint2 x2 = *(const uint2*)src;
                    od[0] = x2.x; od[1] = x2.y;
                } else {
                    od[0] = src[0];
                }
                const int2 dn = desc[base + k + 1];
                if (d.y < 0 || pr > opk) {
                    uint32_t* dst = rows + (size_t)(base + k) * NW;
#pragma unroll
                    for (int w = 0; w < NW; w++) {
                        const uint32_t o = d.y >= 0 ? od[w] : none;
                        uint32_t v;
                        if (compact) {
                            typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
                            v = __builtin_bit_cast(uint32_t, __builtin_elementwise_max(__builtin_bit_cast(u16x2, carry[w]),
                                                                                       __builtin_bit_cast(u16x2, o)));
                            if (w == ow) v = (v & ~omask) | ((((uint32_t)(own0 + k + 1)) & 0xFFFFu) << ((c & 1) * 16));
                        } else {
                            v = (uint32_t)max((int32_t)carry[w], (int32_t)o);
                            if (w == ow) v = (uint32_t)(own0 + k);
                        }
                        carry[w] = v;
                    }
                    if constexpr (NW % 4 == 0) {
#pragma unroll
                        for (int q = 0; q < NW / 4; q++)
                            ((uint4*)dst)[q] = make_uint4(carry[4 * q], carry[4 * q + 1], carry[4 * q + 2], carry[4 * q + 3]);
                    } else if constexpr (NW == 2) {
                        *(uint2*)dst = make_uint2(carry[0], carry[1]);
                    } else {
                        dst[0] = carry[0];
                    }
                    k++;
                    prog[c] = k;   // (after the row: a wave's LDS writes land in order)
                    d = dn;
                }
            }
            if (++guard > (1u << 26)) {   // (a cycle cannot happen on a validated DAG)
                if (c == 0) atomicOr(err, 1);
                break;
            }
        }
    }
    __syncthreads();
    for (int c = 0; c < n; c++) {   // the new rows to HBM
        const int o = cpos[c], k0 = c_old ? c_old[c0 + c] : 0, len = c_len[c0 + c], off = c_off[c0 + c];
        for (int x = k0 * nwd + tid; x < len * nwd; x += nt)
            LA[(size_t)off * nwd + x] = rows[(size_t)(o + x / nwd) * NW + x % nwd];
    }
}

static int la_small_nw(int nwd) {
    int nw = 1;
    while (nw < nwd) nw <<= 1;
    return nw;
}

// LDS bytes k_la_small needs for a graph of P events (0: not applicable)
size_t la_small_bytes(int n, int compact, int64_t P) {
    const int nwd = compact ? n / 2 : n;
    if (n > 64 || nwd > 16) return 0;
    const size_t b = 128 * 4 + (((size_t)P + 2) & ~(size_t)1) * 8 + (size_t)P * la_small_nw(nwd) * 4;
    return b <= 150 * 1024 ? b : 0;
}

template <int NW>
static hipError_t la_small_launch(hipStream_t s, const DevArrays& a, int G, int n, const int32_t* c_old, size_t lds,
                                  int32_t* err) {
    const hipError_t e = ensure_lds_limit((const void*)k_la_small<NW>, lds);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_la_small<NW>, dim3(G), dim3(256), lds, s, (uint32_t*)a.LA, a.p_opk, a.c_off, a.c_len,
                       a.c_base, c_old, n, a.compact ? n / 2 : n, a.compact, err);
    return hipGetLastError();
}

hipError_t launch_la_small(hipStream_t s, const DevArrays& a, int G, int n, const int32_t* c_old, size_t lds,
                           int32_t* err) {
    switch (la_small_nw(a.compact ? n / 2 : n)) {
        case 1: return la_small_launch<1>(s, a, G, n, c_old, lds, err);
        case 2: return la_small_launch<2>(s, a, G, n, c_old, lds, err);
        case 4: return la_small_launch<4>(s, a, G, n, c_old, lds, err);
        case 8: return la_small_launch<8>(s, a, G, n, c_old, lds, err);
        case 16: return la_small_launch<16>(s, a, G, n, c_old, lds, err);
        default: return hipErrorInvalidValue;
    }
}

int la_wave_blocks(int n, int compact) {
    const int nwd = compact ? n / 2 : n;
    return nwd / seg_cfg(n, nwd).dw;
}

int la_wave_segments(int n, int compact, int num_cus, int max_segs) {
    // workgroups of the segment configuration per CU (LDS bound), times CUs, per column block
    const int nwd = compact ? n / 2 : n;
    const SegCfg g = seg_cfg(n, nwd);
    int np2 = 1;
    while (np2 < n) np2 <<= 1;
    const size_t bytes = ((size_t)np2 * (g.r * g.dw + g.r + g.q) + 5 * (size_t)n + 1) * 4;
    const int per_cu = std::max(1, std::min(4, (int)((160 * 1024) / bytes)));
    return std::max(1, std::min(max_segs, per_cu * num_cus / la_wave_blocks(n, compact)));
}

// ---- exactness check of the time-segmented pass (one graph; replaces the verify sweep when it holds)
// The segment pass (MODE 2) gives row x of segment t the max over x's ancestors y IN segment t
// (every path from such a y to x stays in the segment: parents have smaller gids), per chain c':
// L'[x][c'] = max index of an ancestor of x on c' with gid >= the segment start. Indices and gids
// both grow along a chain, so whenever x has ANY ancestor on c' inside the segment, the largest one
// is inside too and L'[x][c'] is exact; only a coordinate left "none" can be wrong, and only if c'
// has events before the segment. Rows grow along a chain, so if the first row after the head rows
// (the rows MODE 3 rebuilds) has no such coordinate, every later row of the chain in the segment is
// exact. The head rows are rebuilt from exact parents if every parent they read from memory is a
// non-head row (exact by the above) or a segment-0 row, i.e. never another segment's head row,
// which the same launch rebuilds concurrently. Both conditions hold -> every row is exact and the
// verify sweep is skipped; either fails -> *flag = 1 and the sweep runs.
__global__ void __launch_bounds__(256) k_la_seg_bounds(const int32_t* __restrict__ p_gid, const int32_t* __restrict__ c_off,
                                                       const int32_t* __restrict__ c_len, int64_t E, int nts, int n,
                                                       int32_t* __restrict__ tbl) {
    const int t = blockIdx.x;   // [0, nts]: first row of each chain in segment t (nts: the chain's length)
    for (int c = threadIdx.x; c < n; c += blockDim.x) {
        const int len = c_len[c];
        tbl[(size_t)t * n + c] = t == 0 ? 0 : t == nts ? len : chain_lower_bound(p_gid, c_off[c], len, E * t / nts);
    }
}

template <typename CT>
__global__ void __launch_bounds__(256) k_la_seg_check(const CT* __restrict__ LA, const int32_t* __restrict__ p_gid,
                                                      const int32_t* __restrict__ p_op, const int32_t* __restrict__ p_chain,
                                                      const int32_t* __restrict__ c_off, const int32_t* __restrict__ tbl,
                                                      int64_t E, int nts, int n, int head, int32_t* __restrict__ flag) {
    const int t = 1 + (int)blockIdx.x / n, c = (int)blockIdx.x % n;   // segment t >= 1, chain c
    const int o = tbl[(size_t)t * n + c], e = tbl[(size_t)(t + 1) * n + c], off = c_off[c];
    bool bad = false;
    // (a) the first row after the head rows: no "none" coordinate of a chain with events before t
    if (e - o > head) {
        const CT* __restrict__ row = LA + (size_t)(off + o + head) * n;
        for (int i = threadIdx.x; i < n; i += blockDim.x)
            if (Coord<CT>::la(row[i]) < 0 && tbl[(size_t)t * n + i] > 0) bad = true;
    }
    // (b) every head row's parent outside the rebuilt region is not another segment's head row
    const int kh = min(e, o + head);
    for (int k = o + (int)threadIdx.x; k < kh; k += blockDim.x) {
        if (k == o && k > 0) {   // the self-parent: the chain's last row before segment t
            int tz = t - 1;
            while (tz > 0 && tbl[(size_t)tz * n + c] > k - 1) tz--;
            if (tz >= 1 && k - 1 < tbl[(size_t)tz * n + c] + head) bad = true;
        }
        const int opp = p_op[off + k];
        if (opp >= 0) {
            const int d = p_chain[opp], r = opp - c_off[d];
            const int64_t gz = p_gid[opp];
            int tz = (int)min<int64_t>(nts - 1, gz * nts / E);   // the segment holding gid gz
            while (tz > 0 && E * tz / nts > gz) tz--;
            while (tz + 1 < nts && E * (tz + 1) / nts <= gz) tz++;
            if (tz >= 1 && tz < t && r < tbl[(size_t)tz * n + d] + head) bad = true;
        }
    }
    if (bad) atomicOr(flag, 1);
}

hipError_t launch_la_seg_check(hipStream_t s, const DevArrays& a, int n, int64_t E, int nts, int head, int32_t* tbl,
                               int32_t* flag) {
    if (nts < 2) return hipSuccess;
    hipLaunchKernelGGL(k_la_seg_bounds, dim3(nts + 1), dim3(256), 0, s, a.p_gid, a.c_off, a.c_len, E, nts, n, tbl);
    if (a.compact)
        hipLaunchKernelGGL(k_la_seg_check<uint16_t>, dim3((nts - 1) * n), dim3(256), 0, s, (const uint16_t*)a.LA,
                           a.p_gid, a.p_op, a.p_chain, a.c_off, tbl, E, nts, n, head, flag);
    else
        hipLaunchKernelGGL(k_la_seg_check<int32_t>, dim3((nts - 1) * n), dim3(256), 0, s, (const int32_t*)a.LA,
                           a.p_gid, a.p_op, a.p_chain, a.c_off, tbl, E, nts, n, head, flag);
    return hipGetLastError();
}

// one workgroup holds every chain of a graph plus the loader waves (<= 1024 threads)
bool la_wave_ok(int n, int max_len, int n_active) {
    return n >= 1 && n <= 1024 && n_active <= 896 && max_len < (1 << kOpkBits);
}

hipError_t launch_la_wave(hipStream_t s, const DevArrays& a, int G, int n, const int32_t* c_old, int64_t E, int nts,
                          int head, int32_t* err, const int32_t* lmap, int na, bool narrow) {
    if (nts > 1 && (G != 1 || c_old)) return hipErrorInvalidValue;
    return a.compact ? la_wave_dispatch<uint16_t>(s, a, G, n, c_old, E, nts, head, err, lmap, na, narrow)
                     : la_wave_dispatch<int32_t>(s, a, G, n, c_old, E, nts, head, err, lmap, na, narrow);
}

}  // namespace hgx
