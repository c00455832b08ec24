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
    if constexpr (DW == 8) {
        const uint4 x = *(const uint4*)p, y = *(const uint4*)(p + 4);
        v[0] = x.x; v[1] = x.y; v[2] = x.z; v[3] = x.w;
        v[4] = y.x; v[5] = y.y; v[6] = y.z; v[7] = y.w;
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
    if constexpr (DW == 8) {
        *(uint4*)p = make_uint4(v[0], v[1], v[2], v[3]);
        *(uint4*)(p + 4) = make_uint4(v[4], v[5], v[6], v[7]);
    } else if constexpr (DW == 4) *(uint4*)p = make_uint4(v[0], v[1], v[2], v[3]);
    else if constexpr (DW == 2) *(uint2*)p = make_uint2(v[0], v[1]);
    else *p = v[0];
    HGX_CB();
}
template <int DW>
__device__ __forceinline__ void row_store(uint32_t* p, const uint32_t (&v)[DW]) {
    if constexpr (DW == 8) {
        *(uint4*)p = make_uint4(v[0], v[1], v[2], v[3]);
        *(uint4*)(p + 4) = make_uint4(v[4], v[5], v[6], v[7]);
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
        if constexpr (R >= 16) asm volatile("s_waitcnt vmcnt(15)" ::: "memory");
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
