// InsertEvent (hashgraph/hashgraph.go:356-401) for a whole batch, on the device.
//
// The reference inserts one event at a time: CheckSelfParent (:404-420; the self-parent
// must be Store.LastFrom(creator), inmem_store.go:85-102), CheckOtherParent (:423-445;
// the other-parent must be known), then Store.SetEvent -> RollingIndex.Add
// (common/rolling_index.go:54-68; PassedIndex / SkippedIndex), and it stops at the first
// event that fails (Core.Sync, node/core.go:199-211). A batch of m events is checked here
// in parallel with the first-failure rule made data-parallel:
//
//   Event k's checks are evaluated as if every earlier event of the batch was accepted.
//   For k below the first true failure k* that assumption holds, so the first k whose
//   check fails is exactly k*; events >= k* are discarded.
//
// "As if accepted" makes the self-parent rule local: the events of creator c accepted
// before k form a chain linked by self-parents, so k's self-parent sp is the last of
// them iff sp is an event of c earlier than k that no earlier event names as its
// self-parent. Claims record, per event, the smallest gid naming it as self-parent
// (succ) and per creator the smallest gid with self-parent "" (first_none); event k
// passes iff its own claim is the smallest. Claims of discarded events are withdrawn.
// The index rule then compares Index with the self-parent's Index (its creator's last).
#include <hip/hip_runtime.h>

#include <cstdint>

#include "hgx_device.h"
#include "hgx_kernels.h"

namespace hgx {

constexpr uint32_t kNone32 = 0xFFFFFFFFu;

__device__ __forceinline__ void ins_claim(int64_t k, int64_t E0, int64_t cap, int C, const InsertIn& in,
                                          const InsertState& st) {
    const int64_t gid = E0 + k;
    const int cr = in.creator[k];
    const int64_t sp = in.sp_at(k);
    if (sp == -1) {
        if (cr >= 0 && cr < C) atomicMin(&st.first_none[cr], (uint32_t)gid);
    } else if (sp >= 0 && sp < gid && sp < cap) {
        atomicMin(&st.succ[sp], (uint32_t)gid);
    }
}

__global__ void __launch_bounds__(256) k_insert_claim(int64_t m, int64_t E0, int64_t cap, int C, InsertIn in,
                                                      InsertState st) {
    const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k < m) ins_claim(k, E0, cap, C, in, st);
}

__device__ __forceinline__ int creator_of(int64_t x, int64_t E0, const InsertIn& in, const InsertState& st) {
    return x < E0 ? st.g_creator[x] : in.creator[x - E0];
}

__device__ __forceinline__ int64_t index_of(int64_t x, int64_t E0, const InsertIn& in, const InsertState& st) {
    return x < E0 ? (int64_t)st.g_index[x] : in.idx_at(x - E0);
}

// Checks in the reference's order: creator known (LastFrom -> KeyNotFound), self-parent,
// Root.Others has an entry for the event with id h (the keys are sorted 32-byte strings)
__device__ bool others_has(const InsertState& st, const uint8_t* h) {
    uint64_t q[4];
#pragma unroll
    for (int w = 0; w < 4; w++) {
        uint64_t x = 0;
        for (int b = 0; b < 8; b++) x = (x << 8) | h[8 * w + b];
        q[w] = x;
    }
    int64_t lo = 0, hi = st.n_others;
    while (lo < hi) {   // first key >= q
        const int64_t mid = (lo + hi) >> 1;
        const uint64_t* kk = st.others + 4 * mid;
        int cmp = 0;
        for (int w = 0; w < 4 && cmp == 0; w++) cmp = kk[w] < q[w] ? -1 : kk[w] > q[w] ? 1 : 0;
        if (cmp < 0) lo = mid + 1; else hi = mid;
    }
    if (lo >= st.n_others) return false;
    const uint64_t* kk = st.others + 4 * lo;
    return kk[0] == q[0] && kk[1] == q[1] && kk[2] == q[2] && kk[3] == q[3];
}

// other-parent (genesis Root only: "" or a known event of the same graph), capacity,
// then the RollingIndex rules of SetEvent.
__device__ __forceinline__ void ins_check(int64_t k, int64_t E0, int64_t cap, int C, int n, const InsertIn& in,
                                          const InsertState& st) {
    const int64_t gid = E0 + k;
    const int cr = in.creator[k];
    const int64_t sp = in.sp_at(k), op = in.op_at(k), idx = in.idx_at(k);
    int code = INS_OK;
    if (cr < 0 || cr >= C) {
        code = INS_KEY_NOT_FOUND;
    } else if (sp == -1) {
        if (!(st.last_gid[cr] == -1 && st.first_none[cr] == (uint32_t)gid)) code = INS_SELF_PARENT;
    } else {
        const bool ok = sp >= 0 && sp < gid && sp < cap && creator_of(sp, E0, in, st) == cr &&
                        st.succ[sp] == (uint32_t)gid && (sp >= E0 || sp == (int64_t)st.last_gid[cr]);
        if (!ok) code = INS_SELF_PARENT;
    }
    if (code == INS_OK && op != -1) {
        bool ok = op >= 0 && op < gid && op < cap;
        if (ok) {
            const int oc = creator_of(op, E0, in, st);
            ok = oc >= 0 && oc < C && oc / n == cr / n;
        } else {
            // unknown other-parents only through the creator's Root (hashgraph.go:430-440):
            // Root.X == SelfParent && Root.Y == OtherParent, or Root.Others[event] == OtherParent
            ok = (op == kRootY && sp == -1 && st.root_y_ext[cr]) ||
                 (op == kRootOther && st.rooted && (st.others_trust || others_has(st, in.hash + 32 * k)));
        }
        if (!ok) code = INS_OTHER_PARENT;
    }
    if (code == INS_OK && gid >= cap) code = INS_CAPACITY;
    if (code == INS_OK) {
        const int64_t li = sp < 0 ? -1 : index_of(sp, E0, in, st);
        if (idx <= li) code = INS_PASSED_INDEX;
        else if (li >= 0 && idx > li + 1) code = INS_SKIPPED_INDEX;
        else if (idx > 2147483646) code = INS_INDEX_RANGE;
    }
    if (code != INS_OK) atomicMin(st.fail, ((unsigned long long)k << 8) | (unsigned long long)code);
}

__global__ void __launch_bounds__(256) k_insert_check(int64_t m, int64_t E0, int64_t cap, int C, int n, InsertIn in,
                                                      InsertState st) {
    const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k < m) ins_check(k, E0, cap, C, n, in, st);
}

// the accepted prefix of a batch of m from the first-failure words (no host round trip between
// the checks and the commit): Verify comes first in InsertEvent, so at the same event the
// signature's failure wins; fail == nullptr: all m
__device__ __forceinline__ int64_t accepted_prefix(int64_t m, const unsigned long long* fail,
                                                   const unsigned long long* fail_sig) {
    if (!fail) return m;
    unsigned long long f = *fail;
    if (fail_sig) {
        const unsigned long long s = *fail_sig;
        if (s != ~0ull && (s >> 8) <= (f >> 8)) f = s;
    }
    return f == ~0ull ? m : (int64_t)(f >> 8);
}

// Append the accepted events [0, m_ok) to the context's arrays (gid order) and move the
// per-creator state (last event, last Index, first Index) forward.
// grid-stride: the loaded-event count of each graph is kept per wave while the wave's events
// share a graph and added once when it changes (one word per graph: an atomic per wave of
// events saturated it, 1.9 ms for 10 M events of one graph)
// mode: kCommitAll, or the split of hgx_insert_and_run: kCommitStructure (the columns validation
// and DivideRounds read) now, kCommitPayload (timestamps, S, coin, transactions, IsLoaded and the
// graphs' loaded counts) once the payload columns have landed
__device__ __forceinline__ void ins_commit(int64_t m, const unsigned long long* fail, const unsigned long long* fail_sig,
                                           int64_t E0, int n, const InsertIn& in, const InsertState& st, int mode,
                                           int64_t first, int64_t stride) {
    const int64_t m_ok = accepted_prefix(m, fail, fail_sig);
    int acc_g = -1;                 // wave-uniform: the graph whose loaded count is pending
    unsigned long long acc = 0;
    for (int64_t k0 = first; k0 < m_ok; k0 += stride) {
        const int64_t k = k0 + threadIdx.x;
        bool ld = false;
        int g = -1;
        if (k < m_ok) {
            const int64_t gid = E0 + k;
            const int cr = in.creator[k];
            const int64_t idx = in.idx_at(k);
            if (mode != kCommitPayload) {
                const int64_t sp = in.sp_at(k);
                st.g_creator[gid] = cr;
                st.g_index[gid] = (int32_t)idx;
                st.g_sp[gid] = (int32_t)sp;
                st.g_op[gid] = (int32_t)in.op_at(k);
                st.g_rr[gid] = -1;                   // roundReceived = nil
                st.g_cts[gid] = 0;
                if (sp == -1) st.chain_base[cr] = (int32_t)idx;
                if (st.succ[gid] >= (uint32_t)(E0 + m_ok)) {   // no accepted event follows it on its chain
                    st.last_gid[cr] = (int32_t)gid;
                    st.last_index[cr] = (int32_t)idx;
                }
            }
            if (mode != kCommitStructure) {
                const int nt = in.ntx_at(k);
                const int nil = in.nil_at(k);
                st.g_ts[gid] = in.ts[k];
                if (in.S) {   // (the split compact payload copies S straight into g_S)
                    const uint4* s4 = (const uint4*)(in.S + 32 * k);
                    uint4* d4 = (uint4*)(st.g_S + 32 * gid);
                    d4[0] = s4[0];
                    d4[1] = s4[1];
                }
                st.g_coin[gid] = (uint8_t)in.coin_at(k);   // middleBit (hashgraph.go:1039-1048)
                if (in.hash) {   // the event id, for a checkpoint (a compact insert brings only the coin)
                    const uint4* h4 = (const uint4*)(in.hash + 32 * k);
                    uint4* i4 = (uint4*)(st.g_id + 32 * gid);
                    i4[0] = h4[0];
                    i4[1] = h4[1];
                }
                st.g_ntx[gid] = nt;
                st.g_txnil[gid] = (uint8_t)nil;
                ld = idx == 0 || (!nil && nt > 0);   // IsLoaded (event.go:119-126)
                st.g_loaded[gid] = ld ? 1 : 0;
                g = cr / n;
            }
        }
        const int g0 = __builtin_amdgcn_readfirstlane(g);
        const uint64_t lm = __ballot(ld);
        if (__all(g == g0 || g < 0)) {   // one graph (or none) in this wave's events
            if (g0 >= 0) {
                if (g0 != acc_g) {
                    if (acc_g >= 0 && acc && lane_id() == 0) atomicAdd(&st.graph_loaded[acc_g], acc);
                    acc_g = g0;
                    acc = 0;
                }
                acc += (unsigned long long)__popcll(lm);
            }
        } else if (ld) {
            atomicAdd(&st.graph_loaded[g], 1ull);
        }
    }
    if (acc_g >= 0 && acc && lane_id() == 0) atomicAdd(&st.graph_loaded[acc_g], acc);
}

__global__ void __launch_bounds__(256) k_insert_commit(int64_t m, const unsigned long long* fail,
                                                       const unsigned long long* fail_sig, int64_t E0, int n,
                                                       InsertIn in, InsertState st, int mode) {
    ins_commit(m, fail, fail_sig, E0, n, in, st, mode, (int64_t)blockIdx.x * blockDim.x, (int64_t)gridDim.x * blockDim.x);
}

// p_ts of the events [E0, E0 + m) from their gid-order timestamps (the layout copied them
// before the payload of hgx_insert_and_run had landed)
__global__ void k_ts_to_pos(int64_t E0, int64_t m, const int32_t* __restrict__ g_pos, const int64_t* __restrict__ g_ts,
                            int64_t* __restrict__ p_ts) {
    const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k < m) p_ts[g_pos[E0 + k]] = g_ts[E0 + k];
}

void launch_ts_to_pos(hipStream_t s, int64_t E0, int64_t m, const int32_t* g_pos, const int64_t* g_ts, int64_t* p_ts) {
    if (m > 0) hipLaunchKernelGGL(k_ts_to_pos, dim3((unsigned)((m + 255) / 256)), dim3(256), 0, s, E0, m, g_pos, g_ts, p_ts);
}

// withdraw the claims of the discarded events [m_ok, m)
__device__ __forceinline__ void ins_unclaim(int64_t k, int64_t E0, int64_t cap, int C, const InsertIn& in,
                                            const InsertState& st) {
    const int64_t gid = E0 + k;
    const int cr = in.creator[k];
    const int64_t sp = in.sp_at(k);
    if (sp == -1) {
        if (cr >= 0 && cr < C && st.first_none[cr] == (uint32_t)gid) st.first_none[cr] = kNone32;
    } else if (sp >= 0 && sp < gid && sp < cap) {
        if (st.succ[sp] == (uint32_t)gid) st.succ[sp] = kNone32;
    }
}

__global__ void __launch_bounds__(256) k_insert_unclaim(int64_t m, const unsigned long long* fail,
                                                        const unsigned long long* fail_sig, int64_t E0, int64_t cap,
                                                        int C, InsertIn in, InsertState st) {
    const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k < m && k >= accepted_prefix(m, fail, fail_sig)) ins_unclaim(k, E0, cap, C, in, st);
}

// A batch of at most 1 024 events (the chunked schedule's SyncLimit-sized inserts): the four phases
// above in ONE workgroup, a barrier between them instead of a kernel boundary (three launches fewer
// per call).
constexpr int kInsertFusedMax = 1024;
__global__ void __launch_bounds__(kInsertFusedMax) k_insert_fused(int64_t m, const unsigned long long* fail_sig,
                                                                  int64_t E0, int64_t cap, int C, int n, InsertIn in,
                                                                  InsertState st, int mode) {
    const int64_t k = threadIdx.x;
    // (each phase's atomics complete at L2 before the barrier: the next phase's loads miss the L1,
    // which holds no line of succ / first_none / fail before they are read)
    if (k < m) ins_claim(k, E0, cap, C, in, st);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (k < m) ins_check(k, E0, cap, C, n, in, st);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    ins_commit(m, st.fail, fail_sig, E0, n, in, st, mode, 0, blockDim.x);
    __syncthreads();
    if (k < m && k >= accepted_prefix(m, st.fail, fail_sig)) ins_unclaim(k, E0, cap, C, in, st);
}

bool launch_insert_fused(hipStream_t s, int64_t m, const unsigned long long* fail_sig, int64_t E0, int64_t cap, int C,
                         int n, const InsertIn& in, const InsertState& st, int mode) {
    if (m <= 0 || m > kInsertFusedMax) return false;
    const unsigned thr = (unsigned)((m + 63) / 64 * 64);
    hipLaunchKernelGGL(k_insert_fused, dim3(1), dim3(thr), 0, s, m, fail_sig, E0, cap, C, n, in, st, mode);
    return true;
}

static inline unsigned nblocks(int64_t work) { return (unsigned)((work + 255) / 256); }

void launch_insert_claim(hipStream_t s, int64_t m, int64_t E0, int64_t cap, int C, const InsertIn& in,
                         const InsertState& st) {
    if (m > 0) hipLaunchKernelGGL(k_insert_claim, dim3(nblocks(m)), dim3(256), 0, s, m, E0, cap, C, in, st);
}

void launch_insert_check(hipStream_t s, int64_t m, int64_t E0, int64_t cap, int C, int n, const InsertIn& in,
                         const InsertState& st) {
    if (m > 0) hipLaunchKernelGGL(k_insert_check, dim3(nblocks(m)), dim3(256), 0, s, m, E0, cap, C, n, in, st);
}

void launch_insert_commit(hipStream_t s, int64_t m, const unsigned long long* fail, const unsigned long long* fail_sig,
                          int64_t E0, int n, const InsertIn& in, const InsertState& st, int mode) {
    const unsigned grid = nblocks(m) < 4096u ? nblocks(m) : 4096u;   // grid-stride beyond 1 M events
    if (m > 0)
        hipLaunchKernelGGL(k_insert_commit, dim3(grid), dim3(256), 0, s, m, fail, fail_sig, E0, n, in, st, mode);
}

// Event.Verify's place in InsertEvent (hashgraph.go:356-363): the smallest event of the batch
// whose signature failed (k << 8 | code, like the parent checks' first-failure word). A creator
// id outside the participants has no key here; the reference verifies it with the key it
// carries and then fails CheckSelfParent, which k_insert_check reports.
__global__ void __launch_bounds__(256) k_insert_sig_first(int64_t m, int C, const int32_t* __restrict__ creator,
                                                          const uint8_t* __restrict__ vout,
                                                          unsigned long long* __restrict__ fail) {
    const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    unsigned long long w = ~0ull;
    if (k < m) {
        const int cr = creator[k];
        const uint8_t v = vout[k];
        if (cr >= 0 && cr < C && v != 1) w = ((unsigned long long)k << 8) | (v == 2 ? INS_BAD_KEY : INS_BAD_SIG);
    }
    w = wave_min_u64(w);
    if (lane_id() == 0 && w != ~0ull) atomicMin(fail, w);
}

void launch_insert_sig_first(hipStream_t s, int64_t m, int C, const int32_t* creator, const uint8_t* vout,
                             unsigned long long* fail) {
    if (m > 0) hipLaunchKernelGGL(k_insert_sig_first, dim3(nblocks(m)), dim3(256), 0, s, m, C, creator, vout, fail);
}

void launch_insert_unclaim(hipStream_t s, int64_t m, const unsigned long long* fail, const unsigned long long* fail_sig,
                           int64_t E0, int64_t cap, int C, const InsertIn& in, const InsertState& st) {
    if (m > 0)
        hipLaunchKernelGGL(k_insert_unclaim, dim3(nblocks(m)), dim3(256), 0, s, m, fail, fail_sig, E0, cap, C, in, st);
}

// hgx_events_packed's structure columns decoded into the hgx_events32 form (include/hgx.h): a parent
// d back from the event's gid E0 + k, 0 = "", kEscape = its exception entry (k_unpack_exc, launched
// after this on the same stream; without one it reads as HGX_UNKNOWN_PARENT). Two events per thread:
// 4-byte loads of the u16 columns, 8-byte stores.
constexpr int kEscape = 0xFFFF;
constexpr int kUnknownParent = -2;

// A distance that reaches back before gid 0 names no event: HGX_UNKNOWN_PARENT, as an unknown id
// would be (a malformed batch must not decode to gid -1, the empty parent).
__device__ __forceinline__ int32_t unpack_parent(uint32_t d, int64_t gid) {
    return d == 0 ? -1
         : (d == (uint32_t)kEscape || (int64_t)d > gid) ? kUnknownParent
         : (int32_t)(gid - (int64_t)d);
}

__global__ void __launch_bounds__(256) k_unpack_packed(int64_t m, int64_t E0, const uint16_t* __restrict__ c16,
                                                       const uint16_t* __restrict__ spb,
                                                       const uint16_t* __restrict__ opb, int32_t* __restrict__ cr,
                                                       int32_t* __restrict__ sp, int32_t* __restrict__ op) {
    const int64_t pairs = (m + 1) / 2;
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < pairs; t += (int64_t)gridDim.x * blockDim.x) {
        const int64_t k = 2 * t;
        if (k + 1 < m) {   // (the staging buffers are 256-byte aligned: k even keeps both loads aligned)
            const uint32_t c = *(const uint32_t*)(c16 + k), s = *(const uint32_t*)(spb + k),
                           o = *(const uint32_t*)(opb + k);
            const int64_t g = E0 + k;
            *(int2*)(cr + k) = make_int2((int)(c & 0xFFFF), (int)(c >> 16));
            *(int2*)(sp + k) = make_int2(unpack_parent(s & 0xFFFF, g), unpack_parent(s >> 16, g + 1));
            *(int2*)(op + k) = make_int2(unpack_parent(o & 0xFFFF, g), unpack_parent(o >> 16, g + 1));
        } else {
            cr[k] = c16[k];
            sp[k] = unpack_parent(spb[k], E0 + k);
            op[k] = unpack_parent(opb[k], E0 + k);
        }
    }
}

__global__ void __launch_bounds__(256) k_unpack_exc(int64_t n_exc, const int64_t* __restrict__ pos,
                                                    const int32_t* __restrict__ esp, const int32_t* __restrict__ eop,
                                                    int32_t* __restrict__ sp, int32_t* __restrict__ op) {
    const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j < n_exc) {   // (positions checked on the host: in the batch and distinct)
        sp[pos[j]] = esp[j];
        op[pos[j]] = eop[j];
    }
}

void launch_unpack_packed(hipStream_t s, int64_t m, int64_t E0, const uint16_t* c16, const uint16_t* spb,
                          const uint16_t* opb, int64_t n_exc, const int64_t* exc_pos, const int32_t* exc_sp,
                          const int32_t* exc_op, int32_t* cr, int32_t* sp, int32_t* op) {
    if (m <= 0) return;
    const int64_t pairs = (m + 1) / 2;
    const unsigned grid = nblocks(pairs) < 8192u ? nblocks(pairs) : 8192u;
    hipLaunchKernelGGL(k_unpack_packed, dim3(grid), dim3(256), 0, s, m, E0, c16, spb, opb, cr, sp, op);
    if (n_exc > 0)
        hipLaunchKernelGGL(k_unpack_exc, dim3(nblocks(n_exc)), dim3(256), 0, s, n_exc, exc_pos, exc_sp, exc_op, sp, op);
}

}  // namespace hgx
