// Device engine of libhgx: HBM-resident event DAG + the consensus kernels
// (hgx_kernels.hip). One Engine per context, one HIP stream. See DESIGN.md.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>
#include <atomic>
#include <condition_variable>
#include <mutex>
#include <thread>
#include <vector>

#include "hgx_kernels.h"

namespace hgx {


constexpr int kStepBatch = 16;        // round steps per hipGraph replay (a full DivideRounds)
constexpr int kStepBatchSmall = 2;    // ... when resuming at the lowest changed round

// kStepBatch round steps captured as one hipGraph, replayed with rewritten round arguments
struct StepGraph {
    hipGraph_t graph = nullptr;
    hipGraphExec_t exec = nullptr;
    std::vector<hipGraphNode_t> nodes;   // the step nodes, in order
    std::vector<hipKernelNodeParams> params;
    RoundArgs args{};
    RoundArgs args_last[2]{};   // the last step node's arguments: args + the host flag of a batch slot
    int kernel = -1, compact = -1, nb = 0;   // what the graph was captured for
    int32_t round[64] = {};
    void drop();
};

enum KernelId {
    K_LAYOUT = 0, K_LA_SWEEP, K_FD_BUILD, K_ROUND_GATHER, K_ROUND_SEARCH, K_FAME, K_THRESHOLD,
    K_ROUND_RECEIVED, K_CTS, K_SORT, K_NUM
};

struct KernelStat {
    double ms = 0;        // summed device time (HIP events around the timed launches)
    int64_t launches = 0;
    int64_t timed = 0;    // launches inside HIP-event windows (the round steps time a sample of replays)
    double bytes = 0;     // algorithmic bytes summed over launches
};

template <typename T>
struct DBuf {
    T* p = nullptr;
    size_t n = 0;
    bool own = true;   // false: a view into another buffer (never freed here)
    hipError_t alloc(size_t count);
    hipError_t grow_copy(size_t count, size_t keep, hipStream_t s);
    void release();
    void view(T* q, size_t count) {   // point into a block owned elsewhere
        release();
        p = q;
        n = count;
        own = false;
    }
    ~DBuf() { release(); }
};

// What the host bookkeeping needs after DivideRounds
struct RoundsHost {
    int32_t R = 0;                    // rounds materialised: max over graphs of LastRound + 1
    int32_t r_lo = 0;                 // rows below r_lo are unchanged by the last DivideRounds
    std::vector<int32_t> last_round;  // [G], -1 = no events
    std::vector<int32_t> bm;          // [(R+1) x C] first chain offset with round >= r
    std::vector<uint8_t> wflag;       // [R x C] 0 none, 1 candidate with higher round, 2 witness
};

struct OrderHost {
    int32_t m = 0;                    // newly received events
    std::vector<int32_t> order_gid;   // [m] graph-major (rr, cts, S) order
    std::vector<int32_t> blk_cnt;     // [G x R]
    std::vector<int64_t> blk_ntx;     // [G x R]
    std::vector<int32_t> blk_loaded;  // [G x R]
    std::vector<uint8_t> blk_nil;     // [G x R] the block's first event has nil Transactions
    bool panic = false;
};

// Outcome of one insert batch (Engine::insert)
struct InsertOut {
    int64_t accepted = 0;          // events appended (the prefix before the first failure)
    int code = 0;                  // InsertCode of the first failing event (0: none)
    int32_t fail_creator = 0;      // its creator and Index (error messages)
    int64_t fail_index = 0;
    // per-creator state after the batch ([C]) and loaded events per graph ([G], cumulative)
    std::vector<int32_t> last_gid, last_index, chain_base;
    std::vector<unsigned long long> graph_loaded;
};

class Engine;

// A chain-sharded group (hgx_create_sharded / hgx_set_round_shards): W engines in one
// process, shard k's on device dev[k] (devices may repeat), each holding the whole DAG. Shard k
// builds the firstDescendants of its chains' events [c_split[k], c_split[k+1]), runs the persistent
// recurrence for those chains and their consensus timestamps, and hands its candidate rows and
// granules to every shard through that shard's window (peer-mapped device memory, write-through);
// the round outputs of its chains are copied to every shard after each launch. The W engines' host
// threads meet at the group's barriers.
struct ShardGroup {
    int W = 1;
    int dev[kMaxShards] = {};
    int32_t c_split[kMaxShards + 1] = {};
    Engine* eng[kMaxShards] = {};
    int32_t st[kMaxShards][4] = {};   // every shard's status words after its last persistent launch
    // hgx_set_shard_remote (test switch): every other shard's window is written as if it were on
    // another device (system-scope stores), so one GPU runs the instructions an 8-GPU node runs
    bool force_remote = false;
    bool wait();                      // false: a shard failed (or 120 s passed): leave with an error
    void fail();
    void rearm();                     // before a group call (no thread inside the group)
   private:
    std::mutex m;
    std::condition_variable cv;
    int count = 0;
    uint64_t gen = 0;
    bool broken = false;
};

class Engine {
   public:
    ~Engine();
    hipError_t init(int device, int n_graphs, int n_part, int64_t cap_events, std::string& why);

    // InsertEvent for `count` events whose columns are device pointers (hgx_insert_events_device)
    // or host pointers staged to HBM first (hgx_insert_events); validation and append on the GPU.
    hipError_t insert(const InsertIn& in, int64_t count, InsertOut& out);
    // the same with Event.Verify first (hashgraph.go:356-363): digest (EventBody.Hash) and R per
    // event, S = in.S, key = the creator's (set_keys); device pointers
    hipError_t insert_verified(const InsertIn& in, const uint8_t* digest, const uint8_t* r, int64_t count,
                               InsertOut& out);
    hipError_t stage_sig(const uint8_t* digest, const uint8_t* r, int64_t count, const uint8_t** d_digest,
                         const uint8_t** d_r);
    // participants' public keys (65 bytes each, C of them): device window tables built once
    hipError_t set_keys(const uint8_t* keys65);
    bool keys_set = false;
    hipError_t stage_host(const int32_t* creator, const int64_t* index, const int64_t* sp, const int64_t* op,
                          const int64_t* ts, const uint8_t* hash, const uint8_t* S, const int32_t* ntx,
                          const int32_t* nil, int64_t count, InsertIn& in);
    // hgx_insert_and_run's split insert of host columns: the structure columns (creator, index,
    // parents) are staged, validated and committed now (out.graph_loaded is not final); a worker
    // thread copies the payload columns (timestamps, hash, S, transactions) of the accepted
    // prefix on a second stream while the caller runs DivideRounds; payload_end joins it, commits
    // the payload, rewrites the layout's timestamps and the candidates' coins, and returns the
    // graphs' loaded counts. Not for rooted contexts (Root.Others needs the hash at validation).
    hipError_t insert_split_begin(const int32_t* creator, const int64_t* index, const int64_t* sp, const int64_t* op,
                                  int64_t count, InsertOut& out);
    hipError_t payload_begin(const int64_t* ts, const uint8_t* hash, const uint8_t* S, const int32_t* ntx,
                             const int32_t* nil, int64_t m_ok);
    hipError_t payload_end(int64_t E0, int64_t m_ok, bool laid_out_new, int32_t wcoin_r0, std::vector<uint64_t>& loaded);
    // the compact payload's S column (copied last, straight into g_S): wait for it (the sort's
    // tie-break, a read-back, a clear) and for the caller's buffer to be read completely
    hipError_t payload_wait_S();
    // the same three for the compact columns of hgx_events32 (int32 Index and parents, the coin
    // byte instead of the event id, len(Transactions) with -1 for nil): 61 instead of 108 bytes
    // per event cross PCIe
    hipError_t stage_host32(const int32_t* creator, const int32_t* index, const int32_t* sp, const int32_t* op,
                            const int64_t* ts, const uint8_t* coin, const uint8_t* S, const int32_t* ntx, int64_t count,
                            InsertIn& in);
    hipError_t insert_split_begin32(const int32_t* creator, const int32_t* index, const int32_t* sp, const int32_t* op,
                                    int64_t count, InsertOut& out);
    hipError_t payload_begin32(const int64_t* ts, const uint8_t* coin, const uint8_t* S, const int32_t* ntx, int64_t m_ok);
    // hgx_events_packed's structure columns (10 bytes per event) copied to HBM and decoded into
    // the hgx_events32 staging columns (launch_unpack_packed); exceptions already checked
    struct Packed {
        const uint16_t* creator;
        const int32_t* index;
        const uint16_t* spb;
        const uint16_t* opb;
        int64_t n_exc;
        const int64_t* exc_pos;
        const int32_t* exc_sp;
        const int32_t* exc_op;
    };
    // (with the payload columns when ts is not null: hgx_insert_events_packed)
    hipError_t stage_packed(const Packed& pk, int64_t count, InsertIn& in, const int64_t* ts = nullptr,
                            const uint8_t* coin = nullptr, const uint8_t* S = nullptr, const int32_t* ntx = nullptr);
    hipError_t insert_split_begin_packed(const Packed& pk, int64_t count, InsertOut& out);
    // forget every event (a fresh NewHashgraph); allocations are kept
    hipError_t clear();
    // per-event columns (gid order) for the host-side getters
    hipError_t get_events(std::vector<int32_t>& creator, std::vector<int32_t>& index, std::vector<int32_t>& sp,
                          std::vector<int32_t>& op);
    hipError_t get_event_fields(int64_t gid, int64_t* ts, int32_t* ntx, int32_t* tx_nil);
    // event ids (Event.Hash) of events [first, first + count): only when every inserted event
    // brought its id (hgx_events; an hgx_events32 insert brings the coin byte alone)
    bool ids_known = true;
    hipError_t get_ids(int64_t first, int64_t count, uint8_t* out32);
    hipError_t get_keys(uint8_t* out65);   // the participants' keys (hgx_set_participant_keys)
    // every column of the inserted events (gid order) for a checkpoint (hgx_save)
    hipError_t get_columns(std::vector<int32_t>& creator, std::vector<int32_t>& index, std::vector<int32_t>& sp,
                           std::vector<int32_t>& op, std::vector<int64_t>& ts, std::vector<uint8_t>& S,
                           std::vector<uint8_t>& coin, std::vector<int32_t>& ntx, std::vector<uint8_t>& txnil);
    hipError_t divide_rounds(int64_t E, const std::vector<int32_t>& chain_len,
                             const std::vector<int32_t>& chain_base, RoundsHost& out);
    // fame of the witnesses of rounds >= r0 (the first undecided round); rows below stay 0
    hipError_t decide_fame(int32_t r0, std::vector<int8_t>& fame_out);
    // round received etc. for the events not yet received; r0 / max_unrecv from recv_round_lo
    hipError_t find_order(const std::vector<uint8_t>& elig, const std::vector<uint8_t>& famous,
                          const std::vector<uint8_t>& ur_empty, int32_t r0, int max_unrecv, OrderHost& out);
    int32_t recv_round_lo(const RoundsHost& rh, int& max_unrecv) const;
    // the same in two halves around the shard exchange of a row-sharded graph:
    // begin = threshold, roundReceived, consensus timestamps of chains [shard_lo, shard_hi);
    // end = sort and blocks
    hipError_t find_order_begin(const std::vector<uint8_t>& elig, const std::vector<uint8_t>& famous,
                                const std::vector<uint8_t>& ur_empty, int32_t r0, int max_unrecv, OrderHost& out);
    hipError_t find_order_end(OrderHost& out, int32_t* order_dst = nullptr);
    int64_t shard_values(int lo, int hi) const;   // newly received events of chains [lo, hi)
    // their consensus timestamps to (to_buf) or from buf, a device or host pointer
    hipError_t shard_copy(int lo, int hi, void* buf, bool on_device, bool to_buf);
    int shard_lo = 0, shard_hi = 0;               // chains whose consensus timestamps this context computes
    // Roots (hgx_reset): per chain Root.Round and whether Root.Y is an event outside the store;
    // genesis roots (Round -1, Y "") when not rooted
    hipError_t set_roots(const std::vector<int32_t>& round, const std::vector<uint8_t>& y_ext);
    hipError_t set_root_others(const uint8_t* keys32, int64_t count);   // Root.Others keys (event ids)
    bool others_trust = false;   // checkpoint replay: Root.Others codes accepted without a key
    bool rooted = false;
    int root_gmax = -1;   // max Root.Round + 1 (rounds that root floors can force), -1 unrooted
    // smallest gid of a witness of each round in [r0, R) (UndecidedRounds order after a Reset)
    hipError_t round_first_gids(int32_t r0, std::vector<int32_t>& out);
    // D2H of order[first, first+count) of the last find_order (async; then sync())
    hipError_t copy_order(int32_t* dst, int64_t first, int64_t count);
    hipError_t sync() { return hipStreamSynchronize(stream); }

    hipError_t reset_received();
    // per-round tables reserved for `rounds` rounds (testing: a small value forces the growth path)
    hipError_t reserve_rounds(int32_t rounds);
    hipError_t get_rounds(std::vector<int32_t>& round_by_gid);
    hipError_t get_received(std::vector<int32_t>& rr, std::vector<int64_t>& cts);
    hipError_t get_coords(int64_t gid, int32_t* la, int32_t* fd);

    int n = 0, G = 0, C = 0, sm = 0, nw = 1;
    int64_t cap = 0, E = 0, E_div = 0;   // E_div: events laid out by the last divide_rounds
    int64_t Ppos = 0;                    // chain-major positions (events + per-chain slack)
    bool incremental = true;             // hgx_set_incremental(0): every DivideRounds rebuilds
    bool last_rebuild = false;           // the last divide_rounds rebuilt the layout
    int32_t R = 0;
    int la_sweeps = 0;
    int la_kernel = 0;            // 0 dataflow wavefront (k_la_wave) where it applies, 1 sweeps (hgx_set_la_kernel)
    bool la_wave_used = false;    // the last DivideRounds built lastAncestors with k_la_wave
    int la_wave_segs = 1;         // ... on this many time segments
    int la_segs_override = 0;     // > 0: time segments of a rebuild (hgx_set_la_kernel mode >= 2, measurement)
    int num_cus = 256;            // compute units of the device
    static constexpr int kLaMaxSegs = 16;
    static constexpr int kLaHeadRows = 64;   // rows per chain rebuilt at the start of each time segment
    static constexpr int kLaSegMinRows = 512;   // time segments only when the graph has >= this many rows per chain
    int64_t la_wave_fallbacks = 0;   // k_la_wave gave up and the sweeps redid the pass
    bool la_verified = false;        // the last time-segmented pass ran the verify sweep (its exactness check failed)
    bool la_verify_always = false;   // hgx_set_la_kernel(1026): the verify sweep after every segmented pass (tests)
    int compact = 0;             // coordinates of the last DivideRounds stored as uint16
    bool force_coord32 = false;  // hgx_set_coord_storage(1)
    int64_t la_rows = 0;   // rows recomputed over all sweeps of the last divide_rounds
    static constexpr int kLaSeg = 16;   // rows per lastAncestors unit
    hipStream_t stream = nullptr;
    double phase_ms[4] = {0, 0, 0, 0};   // coordinates, rounds, fame, order (last calls)
    KernelStat kstat[K_NUM];
    uint32_t time_mask = 0;   // kernels (bit = KernelId) timed with HIP events
    int fame_tally = 0;       // launch_fame tally (hgx_set_fame_tally)
    int round_kernel = 0;     // hgx_set_round_kernel: 0 persistent recurrence on rebuilds where it applies (3: every call),
                              // else per-launch per-candidate steps; 1 block-search steps; 2 per-candidate steps
    int cts_kernel = 1;       // hgx_set_cts_kernel: 1 per-tile blocks (default: measured faster), 2 pipelined (hgx_cts.hip)
    int64_t round_g_runs = 0;   // whole-graph recurrence launches (n <= 16)
    // shard `shard` of a chain-sharded group (nullptr: not sharded)
    ShardGroup* grp = nullptr;
    int shard = 0;
    // the round outputs of this shard's chains (Bm rows [r_a, r_b], S rows / witness flags [r_a,
    // min(r_b, capacity - 1)]) copied into every other shard's tables (after its launches)
    hipError_t share_round_rows(int32_t r_a, int32_t r_b);
    hipError_t capture_steps(StepGraph& sgr, const RoundArgs& args, int kern, int nb);
    bool la_small_used = false;   // the last DivideRounds built lastAncestors with k_la_small
    int la_small_override = -1;   // 0: never k_la_small (hgx_set_la_kernel 2), else where it applies
    bool sort_seg_enabled = true;      // FindOrder's bucketed sort (hgx_set_sort_kernel)
    int64_t sort_seg_runs = 0;         // FindOrders sorted by buckets
    bool round_pb_enabled = true;   // n > 256: k_round_pb (hgx_set_round_kernel 5 turns it off)
    int64_t round_p_runs = 0, round_p_fallbacks = 0;   // persistent launches / calls redone per launch
    int64_t round_p_ovf = 0;
    int32_t round_p_fail_round = -1, round_p_fail_chain = -1;   // the last give-up: round and chain   // candidate rows the persistent launches counted exactly (over 8 bits)
    int dev = 0;

   private:
    hipError_t ensure_round_cap(int32_t need);
    hipError_t insert_impl(const InsertIn& in, int64_t count, InsertOut& out, const unsigned long long* fail_sig,
                           int commit_mode = kCommitAll);
    hipStream_t stream2 = nullptr;   // payload copies of insert_split (created on first use)
    bool pay32 = false;              // the payload in flight is hgx_events32's (coin byte, ntx -1 = nil)
    bool split32 = false;            // the structure columns staged by insert_split_begin32
    hipEvent_t ev_pay = nullptr;
    // the S column is copied last, straight into g_S: only FindOrder's sort reads it, so DecideFame
    // and the first FindOrder kernels run while it crosses PCIe (payload_wait_S before the sort)
    hipEvent_t ev_pay_S = nullptr;
    std::atomic<int> pay_stage{0};   // 1: ts / coin / ntx (/ hash / nil) issued and ev_pay recorded
    bool pay_S_pending = false;
    std::thread pay_thread;
    hipError_t pay_err = hipSuccess;
    hipError_t pay_err_a = hipSuccess;   // the compact payload's first stage (before pay_stage = 1)
    InsertState insert_state();
    void kbeg(int k, bool sample = true, int64_t count = 1);
    void kend(int k, double bytes);
    void kadd_bytes(int k, double bytes);
    hipError_t collect_kernel_times();
    DevArrays arrays();

    int max_len = 0;
    bool laid_out = false;
    std::vector<int32_t> h_off;        // [C+1] chain slots (positions), fixed until a rebuild
    std::vector<int32_t> h_len_div;    // [C] chain lengths at the last divide_rounds
    std::vector<int32_t> h_fu;         // [C] events of each chain received so far (a prefix)
    int32_t fo_m = 0;                  // events received by the FindOrder in progress
    std::vector<int32_t> fo_cnt;       // [C] ... per chain
    DBuf<int32_t> root_round_d, gfl, gB, rfirst;   // roots: [C], per position floor, [(gmax+1) x C], [R]
    DBuf<uint8_t> root_y_ext_d;
    DBuf<uint64_t> others_d;   // [n_others][4] sorted Root.Others keys
    int64_t n_others = 0;
    DBuf<int32_t> sh_off;              // shard exchange: chain offsets
    DBuf<int64_t> sh_buf;              // ... and staging of host buffers
    // gid order
    DBuf<int32_t> g_creator, g_index, g_sp, g_op, g_ntx, g_rr, g_pos;
    DBuf<int64_t> g_ts, g_cts, g_ck;   // g_ck: (creator << 32) | chain offset (k_ck_pack, the layout's op lookups)
    DBuf<uint8_t> g_S, g_coin, g_loaded, g_txnil, g_id;
    // insert state (hgx_insert.hip)
    DBuf<uint32_t> succ, first_none;
    // small per-call tables in one block each, so that one copy moves them (views below):
    // [last_gid | last_index | chain_base | graph_loaded (8-byte)] read back after every insert
    // batch, [c_len | c_base | c_old] written before every DivideRounds
    DBuf<int32_t> ins_blk, cpar_blk;
    int32_t* h_ins = nullptr;    // pinned staging of ins_blk
    int32_t* h_cpar = nullptr;   // pinned staging of cpar_blk
    size_t ins_gl_off = 0;       // graph_loaded's offset in ins_blk (int32 units, even)
    DBuf<int32_t> last_gid_d, last_index_d, chain_base_d;
    DBuf<unsigned long long> ins_fail, graph_loaded_d;
    // host-batch staging (hgx_insert_events)
    DBuf<int32_t> st_creator, st_ntx, st_nil;
    DBuf<int64_t> st_index, st_sp, st_op, st_ts;
    DBuf<uint8_t> st_hash, st_S, st_dig, st_r;
    DBuf<int32_t> st_index32, st_sp32, st_op32;   // hgx_events32 columns
    DBuf<uint16_t> st_c16, st_spb, st_opb;        // hgx_events_packed columns
    DBuf<int64_t> st_exc_pos;
    DBuf<int32_t> st_exc_sp, st_exc_op;
    DBuf<uint8_t> st_coin;
    // batches of at most kPackEvents from host memory: the columns packed in one pinned buffer,
    // one H2D copy into st_pack
    static constexpr int64_t kPackEvents = 65536;
    hipError_t stage_pinned(int k, const void* const* src, const size_t* bytes, size_t* off);
    DBuf<uint8_t> st_pack;
    uint8_t* h_pack = nullptr;
    size_t h_pack_cap = 0;
    // signatures (Event.Verify): keys, window tables, per-event results, first failure
    DBuf<uint8_t> pk_keys, pk_valid, pk_out;
    DBuf<uint32_t> pk_tab;
    DBuf<unsigned long long> ins_fail_sig;
    // chains
    DBuf<int32_t> c_off, c_len, c_base, c_old, fu, rcnt;
    // positions
    DBuf<int32_t> p_gid, p_chain, p_op, p_opu, p_opk, p_round, p_rr;
    DBuf<int32_t> la_chg;   // [units] change stamps of the lastAncestors sweeps (sweep number)
    int32_t la_stamp = 1;   // stamp of the last sweep launched (monotone over calls)
    DBuf<int64_t> la_usum;  // [units] sum of each unit's values (change detection)
    DBuf<int64_t> p_ts, p_cts;
    // coordinates
    DBuf<int32_t> LA, FDT;   // int32 storage; uint16 views when `compact`
    int64_t fd_ld = 0;       // FDT row stride (coordinates): cap rounded up to even
    // per round
    int32_t r_cap = 0;
    DBuf<int32_t> Bm, WLA, WFD, WLAT, Tthr, active, lr;
    hipEvent_t flag_ev[2] = {nullptr, nullptr};
    static constexpr int kLaRing = 8, kLaAhead = 3;   // lastAncestors sweeps queued ahead of the check
    hipEvent_t la_ev[kLaRing] = {};
    StepGraph step_g[3];   // [0] full DivideRounds, [1] / [2] resumed (incremental) calls of 2 / 4 steps
    void drop_step_graph();
    DBuf<uint8_t> wflag, wstat, wcoin, elig, fw, ur_empty;
    DBuf<uint64_t> Smat, Vbuf;
    DBuf<uint32_t> FD8;   // [2][C][ndw] rebased candidate rows (k_round_k)
    DBuf<uint32_t> FD8p;  // [kRoundPBufs][C][ndw] the same, row-major, self-validating (k_round_p)
    DBuf<uint64_t> rp_gran;   // [4][C] k_round_p hand-off granules
    DBuf<int32_t> rp_st;      // k_round_p status: abort, rounds done, finished
    DBuf<uint32_t> seg_off, seg_cur;   // the segmented order sort's bucket starts / cursors
    DBuf<int32_t> rp_amap;    // k_round_pb: the chains with events
    std::vector<int32_t> h_amap;
    DBuf<uint8_t> rp_win;     // a chain-sharded group's RoundPWindows (device copy read by k_round_p)
    DBuf<int32_t> la_lmap;          // k_la_wave lanes -> chains with events (one graph, n > 896)
    DBuf<int32_t> la_chk;           // k_la_seg_check: [0] flag, then the segments' first rows [(nts + 1) x n]
    std::vector<int32_t> h_lmap;
    DBuf<int32_t> ovf;    // [r_cap + 2]
    DBuf<int8_t> fame;
    // order
    DBuf<int32_t> recv_list, counters, order_gid, blk_cnt, blk_loaded;
    DBuf<uint8_t> blk_nil;
    DBuf<uint32_t> scan_part;
    DBuf<uint64_t> key_a, key_b;
    DBuf<uint32_t> val_a, val_b, hist;
    DBuf<int64_t> minmax, blk_ntx;
    int32_t* h_small = nullptr;   // pinned scratch (flags)
    // pinned staging of the per-call host tables (instead of pageable copies): a cursor per
    // phase; D2H copies land here and are handed out by stage_flush() after the phase's sync.
    // The copies are queued and stage_issue() sends them: up to kCopyMax small ones (together
    // at most kCopyKernelMax bytes) as ONE k_copy_many launch, otherwise one DMA copy each
    uint8_t* h_stage = nullptr;
    uint8_t* d_stage = nullptr;   // its device address
    size_t stage_cap = 0, stage_used = 0;
    struct StagedD2H { void* dst; size_t off, bytes; };
    std::vector<StagedD2H> stage_out;
    // kind 0: stage -> dev (H2D), 1: dev -> stage (D2H), 2: dev -> pinned host (host_dst, its
    // device address dev_dst), 3: pinned host (host_src, its device address dev_src) -> dev
    struct PendCopy {
        int kind;
        size_t off;
        const void* dev;
        void* host_dst;
        void* dev_dst;
        size_t bytes;
        const void* host_src = nullptr;
        const void* dev_src = nullptr;
        int reset = -1;   // kind 2: the device bytes are set to this value once copied
    };
    std::vector<PendCopy> pend;
    static constexpr size_t kCopyKernelMax = 256 << 10;
    hipError_t stage_reserve(size_t bytes);
    hipError_t stage_h2d(void* dev, const void* host, size_t bytes);
    hipError_t stage_d2h(void* host, const void* dev, size_t bytes);
    hipError_t copy_to_pinned(void* pinned_dst, const void* dev, size_t bytes, int reset = -1);   // queued like the stagings
    hipError_t copy_from_pinned(void* dev, const void* pinned_src, size_t bytes);
    hipError_t stage_issue();
    void stage_flush();   // after the stream synchronized: copy the D2H tables out, reset the cursor
    // the bucket sort's parts (find_order_end): bucket counts read back with the timestamp range, the
    // order's D2H copies on their own stream behind each part
    static constexpr int kOrderParts = 4;
    static constexpr size_t kOrderPipeMin = 16u << 20;   // order bytes from which the parts pay
    uint32_t* h_segc = nullptr;
    size_t h_segc_n = 0;
    hipStream_t stream_o = nullptr;
    hipEvent_t ev_o[kOrderParts + 1] = {};
    int32_t* h_flag = nullptr;    // host-mapped, coherent: the round-step batches' "candidates left" flags
    int32_t* d_flag = nullptr;    // its device address
    // timing
    hipEvent_t ph0 = nullptr, ph1 = nullptr, ph2 = nullptr;
    std::vector<int32_t> h_lr;   // DivideRounds: every graph's last round (staged copy)
    std::vector<hipEvent_t> kev;
    struct Open { int k; size_t e0; double bytes; int64_t count; };
    std::vector<Open> kopen;
    size_t kev_used = 0;
};

}  // namespace hgx
