// Launchers for the HIP kernels in hgx_kernels.hip (all asynchronous on `s`).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <functional>
#include <vector>

namespace hgx {

constexpr int32_t kMaxI32 = 2147483647;
constexpr int32_t kWlatNotFamous = -2147483647 - 1;   // WLAT row of a witness that is not famous
constexpr int kOpkBits = 21;   // p_opk: op row bits (chains of up to 2^21 rows use k_la_wave)

// Raw device pointers of one context (see hgx_engine.h for meaning/sizes).
struct DevArrays {
    // gid order
    const int32_t *g_creator, *g_index, *g_op, *g_ntx;
    const int64_t* g_ts;
    const uint8_t *g_S, *g_coin, *g_loaded, *g_txnil;
    int32_t *g_rr, *g_pos;
    int64_t* g_ck;   // [E] (creator << 32) | (Index - chain base) of every event: the layout's op lookups
    int64_t* g_cts;
    // chains
    const int32_t *c_off, *c_len, *c_base;
    // positions
    int32_t *p_gid, *p_chain, *p_op, *p_opu, *p_round, *p_rr;
    int32_t* p_opk;   // (op chain within the graph << kOpkBits) | op row, -1 none (k_la_wave)
    int64_t *p_ts, *p_cts;
    // coordinates: int32_t, or uint16_t when `compact` (Coord<CT> in hgx_device.h)
    void *LA, *FDT;
    int compact;
    // rounds
    int32_t* Bm;
    uint8_t *wflag, *wstat, *wcoin;   // wflag: candidate of round r exists; wstat: 2 witness, 1 jumped, 0 none
    int32_t *WLA, *WFD, *WLAT;
    int32_t *active, *lr;
    // fame
    uint64_t *Smat, *Vbuf;
    int8_t* fame;
    // round received
    uint8_t *elig, *fw, *ur_empty;
    int32_t* T;
    int32_t* recv_list;
    int32_t *fu, *rcnt;   // [C] per chain: events received by earlier calls (a prefix) / by this call
    uint32_t* scan_part;  // scan partials
    int32_t* counters;   // [0] received count, [1] panic flag, [2] LA changed
    // order
    uint64_t *key_a, *key_b;
    uint32_t *val_a, *val_b;
    uint32_t* hist;
    int64_t* minmax;
    int32_t* order_gid;
    int32_t *blk_cnt, *blk_loaded;
    int64_t* blk_ntx;
    uint8_t* blk_nil;   // [G x R] Transactions of the block's first event are nil
};

// One batch of events to insert, device pointers (the hgx_events columns, include/hgx.h), or
// the compact columns of hgx_events32: Index and parents as int32, the coin byte instead of the
// 32-byte id, len(Transactions) with -1 for nil (then nil == nullptr)
struct InsertIn {
    const int32_t* creator;
    const int64_t *index, *sp, *op, *ts;
    const uint8_t *hash, *S;
    const int32_t *ntx, *nil;
    const int32_t *index32 = nullptr, *sp32 = nullptr, *op32 = nullptr;
    const uint8_t* coin = nullptr;
    __host__ __device__ int64_t idx_at(int64_t k) const { return index32 ? (int64_t)index32[k] : index[k]; }
    __host__ __device__ int64_t sp_at(int64_t k) const { return sp32 ? (int64_t)sp32[k] : sp[k]; }
    __host__ __device__ int64_t op_at(int64_t k) const { return op32 ? (int64_t)op32[k] : op[k]; }
    // middleBit (hashgraph.go:1039-1048): byte 16 of the event id is not 0
    __host__ __device__ int coin_at(int64_t k) const { return coin ? (coin[k] != 0) : (hash[32 * k + 16] != 0); }
    __host__ __device__ int ntx_at(int64_t k) const { return nil ? ntx[k] : (ntx[k] < 0 ? 0 : ntx[k]); }
    __host__ __device__ int nil_at(int64_t k) const { return nil ? (nil[k] ? 1 : 0) : (ntx[k] < 0 ? 1 : 0); }
};

// Device state the insert path reads and writes (hgx_engine.h owns the buffers)
struct InsertState {
    int32_t *g_creator, *g_index, *g_sp, *g_op, *g_ntx, *g_rr;
    int64_t *g_ts, *g_cts;
    uint8_t *g_S, *g_coin, *g_loaded, *g_txnil;
    uint8_t* g_id;          // [cap][32] event ids (Event.Hash) of events inserted with them (checkpoints)
    uint32_t* succ;         // [cap] smallest gid whose self-parent is this event (UINT32_MAX none)
    uint32_t* first_none;   // [C] smallest gid of the chain with self-parent "" (UINT32_MAX none)
    int32_t *last_gid, *last_index, *chain_base;   // [C] per-chain state before / after the batch
    unsigned long long* fail;           // min over failing events of (k << 8 | code)
    unsigned long long* graph_loaded;   // [G] loaded events inserted (IsLoaded, event.go:119-126)
    const uint8_t* root_y_ext;          // [C] Root.Y names an event outside the store (after hgx_reset)
    int rooted;                         // a Reset installed roots
    const uint64_t* others;             // [n_others][4] Root.Others keys (event ids as 4 big-endian words, sorted)
    int64_t n_others;
    int others_trust;                   // accept every Root.Others code (checkpoint replay)
};

// other-parent codes for parents outside the store after a Reset (include/hgx.h)
constexpr int64_t kRootY = -3, kRootOther = -4;

// first-failure codes of the insert check (hgx_insert_events, hashgraph.go:356-401)
enum InsertCode {
    INS_OK = 0, INS_KEY_NOT_FOUND = 1, INS_SELF_PARENT = 2, INS_OTHER_PARENT = 3, INS_CAPACITY = 4,
    INS_PASSED_INDEX = 5, INS_SKIPPED_INDEX = 6, INS_INDEX_RANGE = 7,
    INS_BAD_SIG = 8, INS_BAD_KEY = 9   // Event.Verify: invalid signature / creator key not a P-256 point
};

// arguments of the round step (hgx_rounds.hip)
struct RoundArgs {
    int n, C, sm, nw;
    int64_t Pcap;
    const int32_t *c_len, *c_off, *c_base, *p_gid;
    uint32_t* FD8;    // [2][C][ndw] candidate firstDescendants rebased to 8 bits (k_round_k, by round parity)
    int32_t* ovf;     // [rounds + 2] round r's candidate rows do not fit 8 bits: exact compares
    const void *LA, *FDT;   // int32_t or uint16_t (compact)
    int compact;
    const uint8_t* g_coin;
    int32_t *Bm, *WLA, *WFD, *p_round, *active, *lr;
    uint8_t *wflag, *wstat, *wcoin;
    uint64_t* Smat;
    // Roots (after hgx_reset): gB[r][c] = first offset of chain c whose root floor reaches r
    // (the event sees the first event of a chain whose Root.Round + 1 >= r), rounds r <= gmax;
    // gmax = -1 without roots
    const int32_t* gB;
    int gmax;
    // last step node of a replayed batch only: host-mapped word set to round + 1 when a chain
    // still has events beyond its boundary (the host polls it instead of a D2H copy)
    int32_t* hflag;
};

// A kernel's dynamic-LDS limit raised to at least `bytes` on the current device, once per
// (device, kernel, size); thread-safe (hipFuncSetAttribute applies per device).
hipError_t ensure_lds_limit(const void* f, size_t bytes);
// blocks of T threads with `lds` bytes that fit one compute unit, cached per (device, kernel)
hipError_t blocks_per_cu(const void* f, int T, size_t lds, int* out);

// several small device ranges set to a byte value in one launch (instead of one memset each)
struct FillRange {
    void* p;          // 4-byte aligned
    uint32_t bytes;
    uint8_t value;
};
constexpr int kFillMax = 8;
void launch_fill_many(hipStream_t s, const FillRange* r, int count);
// several small copies between HBM and pinned host memory (device-visible pointers) in one
// launch: the small read-backs and uploads of a call cost one kernel instead of a blit each
struct CopyRange {
    const void* src;
    void* dst;
    uint32_t bytes;
    int reset = -1;   // >= 0: the source bytes are set to this value once copied (a flag re-armed)
};
constexpr int kCopyMax = 8;
void launch_copy_many(hipStream_t s, const CopyRange* r, int count);

int fd_tile_rows(int n, int compact);
// gid order -> chain-major positions; p_opu = lastAncestors unit of the op row (SEG rows),
// p_opk = packed op chain and row (gids [E0, E))
void launch_layout(hipStream_t s, int64_t E0, int64_t E, const DevArrays& a, int C, int n, int seg);
// lastAncestors of the new rows (from c_old[c], all rows when c_old is null) in ONE pass:
// per (graph, 16-byte column block) a workgroup whose lanes own the chains and wait for
// their op rows in an LDS ring. Needs n <= 896 and chains < 2^kOpkBits
// rows. *err != 0 afterwards: a lane gave up waiting (bounded spins); LA is then incomplete.
// nts > 1 (one graph, all rows): the rows split into nts gid segments built concurrently as
// lower bounds (rows outside a segment count as none); then (head > 0) the first `head` rows of each
// chain in every segment but the first are rebuilt from the now final earlier segments, and
// a verify sweep confirms or completes the rows.
// lmap (one graph, n > 896): the chains that have events, one compute lane each (na of them);
// null: lane i = chain i of every graph
// narrow (a resumed call with a few new rows per chain): one-dword column blocks, 4x the workgroups
bool la_wave_ok(int n, int max_len, int n_active);
// small graphs (n <= 32 compact / 16 int32, a graph's rows and descriptors within 150 KB of LDS):
// one workgroup per graph, the whole graph in LDS (hgx_la_wave.hip); la_small_bytes = its LDS
// bytes for P events per graph, 0 when it does not apply
size_t la_small_bytes(int n, int compact, int64_t P);
hipError_t launch_la_small(hipStream_t s, const DevArrays& a, int G, int n, const int32_t* c_old, size_t lds,
                           int32_t* err);
int la_wave_blocks(int n, int compact);   // column blocks of the time-segment passes (workgroups per segment)
int la_wave_segments(int n, int compact, int num_cus, int max_segs);   // time segments that fill the device
// exactness check of a time-segmented lastAncestors pass plus its head pass (one graph): *flag
// |= 1 unless every row is provably exact (then no verify sweep is needed); tbl: (nts + 1) x n ints
hipError_t launch_la_seg_check(hipStream_t s, const DevArrays& a, int n, int64_t E, int nts, int head, int32_t* tbl,
                               int32_t* flag);
hipError_t launch_la_wave(hipStream_t s, const DevArrays& a, int G, int n, const int32_t* c_old, int64_t E, int nts,
                          int head, int32_t* err, const int32_t* lmap = nullptr, int na = 0,
                          bool narrow = false);
// one Gauss-Seidel sweep over the dirty units (all when `first`) from unit u0: a unit is dirty
// when its carry unit or an op unit has chg == stamp - 1, and gets chg = stamp when its values
// change (usum = per-unit sums); out[0] += rows recomputed, out[1] += units changed; out_next
// (the next sweep's counters) is zeroed. c_old (incremental, else null): rows below c_old[c]
// are final and skipped. first == 2: verify sweep over rows holding lower bounds (every unit;
// changed = some word grew).
void launch_la_sweep(hipStream_t s, const DevArrays& a, int C, int n, int max_len, int seg, int first, int32_t* chg,
                     int32_t stamp, int64_t* usum, int32_t* out, int32_t* out_next, const int32_t* c_old, int64_t u0);
// c_old (incremental, else null): only tiles from each chain's first new row; max_new = the
// most new rows of one chain
// d_lo / d_hi: the rows of the events of chains [d_lo, d_hi) of every graph only (default all)
void launch_fd_build(hipStream_t s, const DevArrays& a, int C, int n, int max_len, int64_t P, const int32_t* c_old,
                     int max_new, int d_lo = 0, int d_hi = -1);
// LA rows and FD entries of the new events gids [E0, E0 + m) set to none
void launch_init_new(hipStream_t s, const DevArrays& a, int64_t E0, int64_t m, int n, int64_t P);
void launch_round_gather(hipStream_t s, const DevArrays& a, int r, int C, int n, int64_t P);
void launch_wcoin(hipStream_t s, const DevArrays& a, int r0, int R, int C);
// one round step of round r: the per-candidate kernel (hgx_round_k.hip, n <= 256) unless
// `block_search` or n > 256 (hgx_rounds.hip)
hipError_t launch_round_step(hipStream_t s, const RoundArgs& A, int r, int block_search);
hipError_t launch_round_k(hipStream_t s, const RoundArgs& A, int r);
void launch_round_k_gather(hipStream_t s, const RoundArgs& A, int r);   // round r's rebased rows + ovf[r]
int round_k_ndw(int n);
// persistent round recurrence (hgx_round_p.hip): one resident workgroup per chain runs rounds
// [r0, r_end) in one launch (init: W'_{r0}'s rebased rows and hand-off granules first, from
// the WFD rows of launch_round_gather). status[0] != 0: a workgroup gave up waiting (bounded
// spins), the rounds must be redone per launch; status[1] = the largest round a graph stopped
// at; status[2] = graphs that found W'_s empty in this launch (fin[g] = that s; fin preset to
// -1 per DivideRounds, a finished graph's workgroups leave at once in a later launch).
// launch_round_p_tail writes the empty rows of rounds (fin[g], r_last] of every graph.
bool round_p_ok(int n, int C, int num_cus);
// whole-graph recurrence (hgx_round_g.hip): one workgroup per graph of n <= 16 chains, rounds
// [r0, r_end) in one launch; status / fin as launch_round_p's
bool round_g_ok(int n, int nw);
hipError_t launch_round_g(hipStream_t s, const RoundArgs& A, int32_t* status, int32_t* fin, int r0, int r_end);
constexpr int kRoundPBufs = 4;   // candidate-row buffers of the persistent recurrence (round s: s % 4)
constexpr int kRoundPShift = 2;  // validity bit of round s's rows: (s >> kRoundPShift) & 1
constexpr int kMaxShards = 8;    // shards of a chain-sharded recurrence (hgx_create_sharded)
// The hand-off windows of a chain-sharded recurrence: every shard's candidate rows,
// granules and abort word, each written by every shard (write-through; system scope into a window
// on another device, through the peer mapping), and every shard's firstDescendants (valid for the
// positions of its own chains [c_split[w], c_split[w + 1])). nwin = 0: one launch over every chain,
// its own buffers only.
struct RoundPWindows {
    int nwin = 0;
    uint32_t remote = 0;   // bit w: window w lies on another device
    uint32_t* FD8p[kMaxShards] = {};
    uint64_t* gran[kMaxShards] = {};
    int32_t* st[kMaxShards] = {};
    const void* FDT[kMaxShards] = {};
    int32_t c_split[kMaxShards + 1] = {};
};
// chains [c_lo, c_hi) only (c_hi < 0: all): shard k of a chain-sharded recurrence launches its chain
// block with its nwin = W windows (win_dev: a RoundPWindows in device memory; the W shards' launches
// run concurrently, on W devices or W streams of one); init 2 = the initial rows and granules only
// (of the launch's chains, into every window)
// the recurrence's exchange floor (k_xchg_floor, hgx_round_p.hip): C resident workgroups publish and poll
// one n-coordinate row each per round, `rounds` rounds; rows [4][C n/4] u32, gran [4][C], st[0] = give-up
hipError_t launch_xchg_floor(hipStream_t s, int C, int n, int rounds, uint32_t* rows, uint64_t* gran, int32_t* st);
hipError_t launch_round_p(hipStream_t s, const RoundArgs& A, uint32_t* FD8p, uint64_t* gran, int32_t* status,
                          int32_t* fin, int r0, int r_end, int init, int num_cus, int c_lo = 0, int c_hi = -1,
                          const RoundPWindows* win_dev = nullptr, int nwin = 1);
void launch_round_p_tail(hipStream_t s, const RoundArgs& A, const int32_t* fin, int r_last);
// after the persistent launches: rounds of the events, wstat / wflag / active and the candidates'
// WLA rows of rounds [r_lo, r_hi], from Bm (the persistent loop writes only Bm and the S rows)
void launch_round_p_post(hipStream_t s, const RoundArgs& A, int r_lo, int r_hi);
// persistent recurrence for 256 < n <= 1024, one graph (hgx_round_pb.hip): one resident workgroup
// per chain WITH events (amap: their indices, na of them), rows / granules / status / fin as
// launch_round_p's (init: W'_{r0}'s rows first, compressed to the chains with events);
// hipErrorCooperativeLaunchTooLarge when the na
// workgroups cannot all be resident. launch_round_pb_silent then writes the silent chains' Bm rows
// of rounds [r_lo, r_hi + 1] (0), before launch_round_p_post.
bool round_pb_ok(int n, int G);
hipError_t launch_round_pb(hipStream_t s, const RoundArgs& A, uint32_t* FD8p, uint64_t* gran, int32_t* status,
                           int32_t* fin, const int32_t* amap, int na, int r0, int r_end, int num_cus, bool init);
void launch_round_pb_silent(hipStream_t s, const RoundArgs& A, int r_lo, int r_hi);
// root floors (hgx_reset): per position G = max over chains i whose first event it sees of
// Root.Round(i) + 1, then gB[r][c] = first offset of chain c with G >= r, r in [0, gmax]
void launch_root_floor(hipStream_t s, const DevArrays& a, const int32_t* root_round, int32_t* gfl, int32_t* gB,
                       int gmax, int C, int n, int max_len);
void launch_round_first_gid(hipStream_t s, const DevArrays& a, int r0, int R, int C, int32_t* first);
// lr[g] = max round with a witness in graph g over the first R round steps (lr preset to -1)
void launch_last_round(hipStream_t s, int rs, int R, int G, int C, int n, const uint8_t* wstat, int32_t* lr);
void step_prof_dump();     // -DHGX_STEP_PROF builds only
void round_k_prof_dump();  // -DHGX_STEP_PROF builds only
void round_p_prof_dump();  // -DHGX_STEP_PROF builds only
void round_pb_prof_dump(); // -DHGX_STEP_PROF builds only
void round_g_prof_dump();  // -DHGX_STEP_PROF builds only
// tally: 0 = witness-tiled popcount (default), 1 = per-round popcount kernel, 2 = witness-tiled int8 MFMA
// rounds [r0, R) (r0 = the first undecided round)
void launch_fame(hipStream_t s, const DevArrays& a, int r0, int R, int C, int n, int nw, int sm, int G, int tally);
// rounds [r0, R) (r0 = 1 + the lowest round of an event not yet received)
void launch_wla_transpose(hipStream_t s, const DevArrays& a, int r0, int R, int G, int C, int n);
void launch_threshold(hipStream_t s, const DevArrays& a, int r0, int R, int C, int n);
// chains' unreceived events [fu, len) (max_unrecv = the most of one chain); rcnt += received
void launch_round_received(hipStream_t s, const DevArrays& a, int R, int C, int n, int max_unrecv);
void launch_fu_advance(hipStream_t s, const DevArrays& a, int C);           // fu += rcnt
void launch_fu_count(hipStream_t s, const DevArrays& a, int64_t E);         // fu += received events (fu preset 0)
// the newly received events [fu, fu + rcnt) of chains [c_lo, c_lo + c_cnt) (max_cnt = the
// largest rcnt among them)
void launch_cts(hipStream_t s, const DevArrays& a, int c_lo, int c_cnt, int C, int n, int64_t P, int max_cnt);
// the same, pipelined (hgx_cts.hip): resident blocks, three tiles' loads in flight; false when
// it does not apply (cts_pipe_ok) and nothing was launched
bool cts_pipe_ok(int n, int C);
bool launch_cts_pipe(hipStream_t s, const DevArrays& a, int c_lo, int c_cnt, int C, int n, int64_t P, int max_cnt);
// shard exchange: consensus timestamps of the newly received events of chains [lo, hi) to /
// from a chain-major buffer (offs[c] = start of chain c)
void launch_cts_shard_copy(hipStream_t s, const DevArrays& a, int lo, int hi, const int32_t* offs, int64_t* buf,
                           int to_buf);
void launch_minmax(hipStream_t s, const DevArrays& a, int32_t m);
void launch_sort(hipStream_t s, const DevArrays& a, int32_t m, int64_t cmin, int cts_bits, int R, int n,
                 int seg_bits, uint32_t** final_vals, uint64_t** final_keys);
// the segmented sort (round 5): launch_seg_count counts the received events per (graph, rr) bucket
// into segc[G R] (zeroed by the caller) and their largest bucket into *max_out (atomicMax); if that
// is <= seg_sort_cap() and the combined key fits 64 bits, launch_sort_seg buckets the list and sorts
// every bucket in LDS (segoff = the counts, scanned in place; segcur = [nseg] scratch)
int seg_sort_cap();
void launch_seg_count(hipStream_t s, const DevArrays& a, int32_t m, int R, int n, int nseg, uint32_t* segc,
                      unsigned long long* max_out);
// (cuts: optional bucket boundaries 0 = c_0 < ... < c_K = nseg; the parts are launched in order and
// after_part(k) runs on the host behind part k's launch)
hipError_t launch_sort_seg(hipStream_t s, const DevArrays& a, int32_t m, int64_t cmin, int cts_bits, int R, int n, int nseg,
                     uint32_t* segoff, uint32_t* segcur, int max_seg, uint32_t** final_vals, uint64_t** final_keys,
                     const std::vector<int>* cuts = nullptr,
                     const std::function<hipError_t(int)>& after_part = nullptr);
// m <= 4096: one block sorts (graph, rr, cts, S) (no cts range needed)
bool sort_small_ok(int32_t m);
void launch_sort_small(hipStream_t s, const DevArrays& a, int32_t m, int n, uint32_t** final_vals);
void launch_finish_order(hipStream_t s, const DevArrays& a, int32_t m, const uint32_t* vals, int R, int n);
void launch_gather_i32(hipStream_t s, int64_t E, const int32_t* src, const int32_t* g_pos, int32_t* dst);

// ECDSA P-256 verify (hgx_p256.hip): per-key window tables (+ the base point as key nk),
// then one lane per signature
size_t p256_table_bytes(int nk);
void launch_p256_tables(hipStream_t s, int nk, const uint8_t* keys65, uint32_t* tab, uint8_t* valid);
void launch_p256_verify(hipStream_t s, int64_t count, int nk, const int32_t* key_idx, const uint8_t* dig,
                        const uint8_t* r, const uint8_t* sg, const uint32_t* tab, const uint8_t* valid, uint8_t* out);

// insert path (hgx_insert.hip): events k in [0, m) get gid E0 + k
void launch_insert_claim(hipStream_t s, int64_t m, int64_t E0, int64_t cap, int C, const InsertIn& in,
                         const InsertState& st);
void launch_insert_check(hipStream_t s, int64_t m, int64_t E0, int64_t cap, int C, int n, const InsertIn& in,
                         const InsertState& st);
constexpr int kCommitAll = 0, kCommitStructure = 1, kCommitPayload = 2;
// m_ok = the accepted prefix of m from the first-failure words (all m when fail is null)
void launch_insert_commit(hipStream_t s, int64_t m, const unsigned long long* fail, const unsigned long long* fail_sig,
                          int64_t E0, int n, const InsertIn& in, const InsertState& st, int mode);
void launch_ts_to_pos(hipStream_t s, int64_t E0, int64_t m, const int32_t* g_pos, const int64_t* g_ts, int64_t* p_ts);
void launch_insert_unclaim(hipStream_t s, int64_t m, const unsigned long long* fail, const unsigned long long* fail_sig,
                           int64_t E0, int64_t cap, int C, const InsertIn& in, const InsertState& st);
// claim + check + commit + unclaim of a batch of at most 1 024 events in one workgroup (false: larger)
bool launch_insert_fused(hipStream_t s, int64_t m, const unsigned long long* fail_sig, int64_t E0, int64_t cap, int C,
                         int n, const InsertIn& in, const InsertState& st, int mode);
// verify results vout[k] (1 valid, 0 invalid, 2 key not a point) -> *fail = min (k << 8 | code)
void launch_insert_sig_first(hipStream_t s, int64_t m, int C, const int32_t* creator, const uint8_t* vout,
                             unsigned long long* fail);
// hgx_events_packed -> the hgx_events32 creator / parent columns (cr, sp, op: m entries each)
void launch_unpack_packed(hipStream_t s, int64_t m, int64_t E0, const uint16_t* c16, const uint16_t* spb,
                          const uint16_t* opb, int64_t n_exc, const int64_t* exc_pos, const int32_t* exc_sp,
                          const int32_t* exc_op, int32_t* cr, int32_t* sp, int32_t* op);

}  // namespace hgx
