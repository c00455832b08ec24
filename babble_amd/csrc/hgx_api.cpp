// C ABI of libhgx (include/hgx.h) and the host-side mirror of the reference's
// Hashgraph bookkeeping. The device engine computes every DAG-pure quantity
// (coordinates, rounds, witnesses, fame decisions, round-received, consensus
// timestamps, order); this file keeps exactly the schedule-dependent state the Go
// code keeps (hashgraph/hashgraph.go:15-37): UndecidedRounds with its duplicate-0
// quirk, per-witness fame frozen once decided, LastConsensusRound /
// LastCommitedRoundEvents, received events, blocks, counters.
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <tuple>
#include <set>
#include <new>
#include <cstdlib>
#include <string>
#include <thread>
#include <vector>

#include "hgx.h"
#include "hgx_engine.h"

namespace {

struct Block {
    int32_t rr;
    int64_t first;     // position in the graph's consensus order
    int32_t nev;
    int64_t ntx;
    int32_t tx_nil;
    int32_t committed;
};

// growable pinned host array: the consensus order is copied D2H straight into it
// Pinned host arena holding the consensus orders of all graphs: every FindOrder appends
// the device order (graph-major) with ONE copy, and each graph's order is the list of
// its segments in the arena (one per FindOrder call that ordered events of the graph).
struct OrderArena {
    int32_t* p = nullptr;
    size_t used = 0, cap = 0;
    OrderArena() = default;
    OrderArena(const OrderArena&) = delete;
    OrderArena& operator=(const OrderArena&) = delete;
    ~OrderArena() { if (p) (void)hipHostFree(p); }
    bool reserve(size_t want) {
        if (want <= cap) return true;
        size_t nc = std::max<size_t>(want, cap * 2 + 1024);
        int32_t* q = nullptr;
        if (hipHostMalloc((void**)&q, nc * sizeof(int32_t), hipHostMallocDefault) != hipSuccess) return false;
        if (used) std::memcpy(q, p, used * sizeof(int32_t));
        if (p) (void)hipHostFree(p);
        p = q;
        cap = nc;
        return true;
    }
};

struct GraphOrder {
    struct Seg { size_t off, len; };
    std::vector<Seg> segs;
    size_t n = 0;
    size_t size() const { return n; }
};

struct GraphState {
    std::vector<int32_t> undecided{0};     // Hashgraph.UndecidedRounds, init []int{0} (hashgraph.go:64)
    int32_t queued_upto = -1;              // rounds <= this have RoundInfo.queued
    std::vector<uint8_t> queued;           // [r] RoundInfo.queued after a Reset (rounds may appear out of order)
    bool has_lcr = false;
    int32_t lcr = 0;
    int32_t lcre = 0;
    int64_t consensus_tx = 0, pending_loaded = 0, undetermined = 0;
    int32_t last_round = -1;
    std::vector<int8_t> fame;              // [(last_round+1) x n] RoundEvent.Famous (host state)
    std::vector<int32_t> round_events;     // [last_round+1]
    std::vector<Block> blocks;
    void reset() {   // a fresh NewHashgraph's consensus state (keeps allocations)
        undecided.assign(1, 0);
        queued_upto = -1;
        has_lcr = false;
        lcr = lcre = 0;
        consensus_tx = pending_loaded = undetermined = 0;
        last_round = -1;
        fame.clear();
        round_events.clear();
        blocks.clear();
        queued.clear();
    }
};

}  // namespace

struct hgx_ctx {
    hgx::Engine eng;
    int G = 1, n = 0, C = 0, sm = 0;
    int64_t cap = 0;
    // per-creator state after the last insert ([C], copied back from the device)
    std::vector<int32_t> chain_len, chain_base, last_gid, last_index;
    int64_t E = 0, E_div = 0;
    bool divided = false;
    hgx::RoundsHost rh;
    std::vector<int8_t> fame_dev;                  // DecideFame's device fame rows (rows from the first undecided)
    // the first undecided round of every graph at the last FindOrder that ran on the device:
    // while it stays the same the eligible rounds only shrink (see hgx_find_order_begin)
    std::vector<int32_t> fo_prev_u0;
    bool fo_prev_valid = false;
    std::vector<int32_t> fo_pend_u0;   // set by hgx_find_order_begin, committed by _end
    bool fo_pend_valid = false;
    std::vector<uint8_t> fo_elig, fo_fw;           // FindOrder's eligible rounds / famous witnesses
    std::vector<GraphState> gs;
    OrderArena arena;                        // consensus orders (gids) of all graphs
    std::vector<GraphOrder> order;           // [G] segments of each graph's order in the arena
    std::vector<int64_t> g_events, g_loaded;  // [G] inserted events / loaded events per graph
    // per-event columns (gid order), mirrored from the device when a getter needs them
    bool mirror_ok = false;
    std::vector<int32_t> creator, index32, sp, op;
    bool chains_ok = false;
    std::vector<std::vector<int32_t>> chain_gids;   // [C] gids of each creator's events in Index order
    // getter caches
    bool rounds_cached = false;
    std::vector<int32_t> round_cache;
    bool recv_cached = false;
    std::vector<int32_t> rr_cache;
    std::vector<int64_t> cts_cache;
    // FindOrder in progress (between hgx_find_order_begin and _end) and the row shard
    bool fo_open = false;
    hgx::OrderHost fo;
    int32_t shard_rank = 0, shard_world = 1;
    // Roots (root.go:62-67) after hgx_reset: Index, Round, Root.Y is an event outside the store
    std::vector<int32_t> root_index, root_round;
    std::vector<uint8_t> root_y_ext;
    bool rooted = false;
    // what Reset kept (LastConsensusRound, LastCommitedRoundEvents, ConsensusTransactions, the
    // blocks), as it was when the roots were installed: a rooted checkpoint carries it
    struct Kept {
        bool has_lcr = false;
        int32_t lcr = 0, lcre = 0;
        int64_t consensus_tx = 0;
        std::vector<Block> blocks;
    };
    std::vector<Kept> reset_kept;
    std::vector<uint8_t> others_keys;            // Root.Others keys (hgx_set_root_others), 32 bytes each
    std::vector<int64_t> pl_off;                 // per-event payloads restored by hgx_bootstrap ([E0, E0 + m))
    std::vector<uint8_t> pl_blob;
    // commitCh (hashgraph.go:848-854): called for every new block with transactions
    hgx_commit_fn commit_fn = nullptr;
    void* commit_user = nullptr;
    // a chain-sharded group (hgx_create_sharded / hgx_set_round_shards): this context
    // is shard 0 and owns the other shards' contexts (each a whole context on its device, driven
    // with the same calls) and the group; empty / null otherwise
    std::vector<hgx_ctx*> peers;
    hgx::ShardGroup* grp = nullptr;
    void* gx_out = nullptr;   // FindOrder's timestamp exchange: this shard's values (device memory)
    void* gx_in = nullptr;    // ... another shard's, copied here before the import
    size_t gx_out_cap = 0, gx_in_cap = 0;
};

static void set_err(hgx_error* err, int32_t code, const std::string& msg) {
    if (!err) return;
    err->code = code;
    std::snprintf(err->msg, sizeof(err->msg), "%s", msg.c_str());
}

static int32_t ok(hgx_error* err) {
    if (err) set_err(err, HGX_OK, "");
    return HGX_OK;
}

static int32_t dev_err(hgx_error* err, hipError_t e, const char* where) {
    set_err(err, HGX_ERR_DEVICE, std::string(where) + ": " + hipGetErrorString(e));
    return HGX_ERR_DEVICE;
}

// Go's string(int): UTF-8 of the rune (common/rolling_index.go passes string(index))
static std::string go_rune(int64_t v) {
    uint32_t r = (v < 0 || v > 0x10FFFF || (v >= 0xD800 && v <= 0xDFFF)) ? 0xFFFD : (uint32_t)v;
    std::string s;
    if (r < 0x80) s += (char)r;
    else if (r < 0x800) { s += (char)(0xC0 | (r >> 6)); s += (char)(0x80 | (r & 63)); }
    else if (r < 0x10000) { s += (char)(0xE0 | (r >> 12)); s += (char)(0x80 | ((r >> 6) & 63)); s += (char)(0x80 | (r & 63)); }
    else { s += (char)(0xF0 | (r >> 18)); s += (char)(0x80 | ((r >> 12) & 63)); s += (char)(0x80 | ((r >> 6) & 63)); s += (char)(0x80 | (r & 63)); }
    return s;
}

// Every entry point that touches the engine runs on the context's device and restores the
// caller's current device on return (cgo moves goroutines between OS threads; a thread
// starts on device 0).
struct DeviceGuard {
    int prev = -1, want = 0;
    explicit DeviceGuard(const hgx_ctx* c) : want(c ? c->eng.dev : 0) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        if (c && prev != want) (void)hipSetDevice(want);
    }
    ~DeviceGuard() {
        if (prev >= 0 && prev != want) (void)hipSetDevice(prev);
    }
};

// ---- chain-sharded group helpers ----------------------------------------
// f(context, err) on shard 0 (this thread) and on every other shard (a thread each), concurrently:
// the engines meet at the group's barriers inside DivideRounds. A shard whose call fails breaks the
// barriers (the others leave with an error too). Shard 0's outcome first, then the first other one.
template <typename F>
static int32_t on_shards(hgx_ctx* c, hgx_error* err, F&& f) {
    hgx::ShardGroup* g = c->grp;
    g->rearm();
    const size_t np = c->peers.size();
    std::vector<int32_t> rc(np, HGX_OK);
    std::vector<hgx_error> errs(np);
    std::vector<std::thread> th;
    th.reserve(np);
    for (size_t k = 0; k < np; k++)
        th.emplace_back([&, k] {
            rc[k] = f(c->peers[k], &errs[k]);
            if (rc[k]) g->fail();
        });
    const int32_t r0 = f(c, err);
    if (r0) g->fail();
    for (auto& t : th) t.join();
    if (r0) return r0;
    for (size_t k = 0; k < np; k++)
        if (rc[k]) {
            if (err) *err = errs[k];
            return rc[k];
        }
    return r0;
}

template <typename F>
static void each_shard(hgx_ctx* c, F&& f) {
    f(c);
    for (hgx_ctx* q : c->peers) f(q);
}

static int32_t group_only_one(hgx_ctx* c, hgx_error* err, const char* who) {
    if (c && c->grp) {
        set_err(err, HGX_ERR_INVALID, std::string(who) + ": not available on a chain-sharded context");
        return HGX_ERR_INVALID;
    }
    return HGX_OK;
}

static int32_t ensure_mirror(hgx_ctx* c) {
    if (c->mirror_ok) return HGX_OK;
    if (c->eng.get_events(c->creator, c->index32, c->sp, c->op) != hipSuccess) return HGX_ERR_DEVICE;
    c->mirror_ok = true;
    return HGX_OK;
}

static int32_t ensure_chains(hgx_ctx* c) {
    if (c->chains_ok) return HGX_OK;
    if (ensure_mirror(c)) return HGX_ERR_DEVICE;
    for (auto& v : c->chain_gids) v.clear();
    for (int64_t g = 0; g < c->E; g++) c->chain_gids[(size_t)c->creator[(size_t)g]].push_back((int32_t)g);
    c->chains_ok = true;
    return HGX_OK;
}

static int graph_of(const hgx_ctx* c, int64_t x) { return c->creator[(size_t)x] / c->n; }

// walk the graph's order segments over positions [first, first + count)
template <typename F>
static void walk_order(hgx_ctx* c, int32_t g, int64_t first, int64_t count, F&& f) {
    int64_t pos = 0, k = 0;
    for (const GraphOrder::Seg& sg : c->order[g].segs) {
        const int64_t a = std::max<int64_t>(first, pos), b = std::min<int64_t>(first + count, pos + (int64_t)sg.len);
        for (int64_t i = a; i < b; i++) f(k++, (int64_t)c->arena.p[sg.off + (size_t)(i - pos)]);
        pos += (int64_t)sg.len;
        if (pos >= first + count) break;
    }
}


extern "C" {

int32_t hgx_abi_version(void) { return HGX_ABI_VERSION; }

static hgx_ctx* create_batch_impl(int32_t n_graphs, int32_t n_participants, int64_t capacity_events, int32_t device,
                                  hgx_error* err) {
    if (n_graphs <= 0 || n_participants <= 0 || n_participants > 1024 || capacity_events < 0 ||
        (int64_t)n_graphs * n_participants > (1 << 24) || capacity_events >= (1LL << 31)) {
        set_err(err, HGX_ERR_INVALID, "hgx_create: invalid sizes (1 <= n <= 1024, capacity < 2^31)");
        return nullptr;
    }
    hgx_ctx* c = new (std::nothrow) hgx_ctx();
    if (!c) { set_err(err, HGX_ERR_CAPACITY, "hgx_create: out of host memory"); return nullptr; }
    c->G = n_graphs;
    c->n = n_participants;
    c->C = n_graphs * n_participants;
    c->sm = 2 * n_participants / 3 + 1;
    c->cap = capacity_events;
    int prev = -1;
    (void)hipGetDevice(&prev);
    std::string why;
    hipError_t e = c->eng.init(device, n_graphs, n_participants, capacity_events, why);
    if (prev >= 0 && prev != device) (void)hipSetDevice(prev);
    if (e != hipSuccess) {
        set_err(err, HGX_ERR_DEVICE, "hgx_create: " + (why.empty() ? std::string(hipGetErrorString(e)) : why));
        delete c;
        return nullptr;
    }
    c->chain_len.assign(c->C, 0);
    c->chain_base.assign(c->C, 0);
    c->last_gid.assign(c->C, -1);
    c->last_index.assign(c->C, -1);
    c->chain_gids.assign(c->C, {});
    c->root_index.assign(c->C, -1);   // NewBaseRoot (root.go:69-76)
    c->root_round.assign(c->C, -1);
    c->root_y_ext.assign(c->C, 0);
    c->gs.assign(n_graphs, GraphState());
    c->order = std::vector<GraphOrder>(n_graphs);
    c->g_events.assign(n_graphs, 0);
    c->g_loaded.assign(n_graphs, 0);
    // the order arena sized for the capacity up front (at most 64 MB pinned): growing it copies
    // the whole order so far, a multi-millisecond outlier inside one FindOrder of the chunked schedule
    (void)c->arena.reserve((size_t)std::min<int64_t>(capacity_events, (int64_t)1 << 24));
    ok(err);
    return c;
}

// The kernels' first launches in a process (code objects loaded per kernel, LDS limits and occupancy
// queries, the step graphs' instantiation) cost ~20 ms, which used to land in the first call of the
// first context (a chunked node's first Core.Sync: 23.5 ms against 0.3 ms later). The first context of
// each (device, graphs, participants) runs a small synthetic DAG of that size through
// hgx_insert_and_run32 on a scratch context inside hgx_create instead (HGX_NO_WARMUP=1 skips it).
static void warm_up(int32_t device, int32_t G, int32_t n) {
    static std::mutex mu;
    static std::set<std::tuple<int32_t, int32_t, int32_t>> done;
    {
        std::lock_guard<std::mutex> lk(mu);
        if (!done.insert(std::make_tuple(device, G, n)).second) return;
    }
    if (const char* e = getenv("HGX_NO_WARMUP"))
        if (e[0] == '1') return;
    const int64_t per = 4 * (int64_t)n + 8, E = per * G;   // round-robin gossip: a few rounds per graph
    hgx_error err{};
    hgx_ctx* w = create_batch_impl(G, n, E, device, &err);
    if (!w) return;
    std::vector<int32_t> cr(E), ix(E), sp(E), op(E), ntx(E, 0);
    std::vector<int64_t> ts(E);
    std::vector<uint8_t> coin(E), sig((size_t)E * 32);
    for (int64_t g = 0, gid = 0; g < G; g++)
        for (int64_t k = 0; k < per; k++, gid++) {
            cr[gid] = (int32_t)(g * n + k % n);
            ix[gid] = (int32_t)(k / n);
            sp[gid] = k >= n ? (int32_t)(gid - n) : -1;
            op[gid] = (k >= 1 && n > 1) ? (int32_t)(gid - 1) : -1;
            ts[gid] = 1600000000000000000LL + 1000 * k;
            coin[gid] = (uint8_t)(k & 1);
            for (int b = 0; b < 32; b++) sig[(size_t)gid * 32 + b] = (uint8_t)((gid * 131 + b * 17) & 0xFF);
        }
    hgx_events32 ev{cr.data(), ix.data(), sp.data(), op.data(), ts.data(), coin.data(), sig.data(), ntx.data()};
    int64_t ins = 0;
    (void)hgx_insert_and_run32(w, &ev, E, &ins, &err);
    hgx_destroy(w);
}

hgx_ctx* hgx_create_batch(int32_t n_graphs, int32_t n_participants, int64_t capacity_events, int32_t device,
                          hgx_error* err) {
    hgx_ctx* c = create_batch_impl(n_graphs, n_participants, capacity_events, device, err);
    if (c) {
        warm_up(device, n_graphs, n_participants);
        ok(err);
    }
    return c;
}

hgx_ctx* hgx_create(int32_t n_participants, int64_t capacity_events, int32_t device, hgx_error* err) {
    return hgx_create_batch(1, n_participants, capacity_events, device, err);
}

static void free_gx(hgx_ctx* x) {
    DeviceGuard dg(x);
    if (x->gx_out) (void)hipFree(x->gx_out);
    if (x->gx_in) (void)hipFree(x->gx_in);
    x->gx_out = x->gx_in = nullptr;
    x->gx_out_cap = x->gx_in_cap = 0;
}

// back to one context: the other shards' contexts and the group go
static void drop_group(hgx_ctx* c) {
    for (hgx_ctx* q : c->peers) {
        free_gx(q);
        DeviceGuard dg(q);
        delete q;
    }
    c->peers.clear();
    free_gx(c);
    delete c->grp;
    c->grp = nullptr;
    c->eng.grp = nullptr;
    c->eng.shard = 0;
    c->shard_rank = 0;
    c->shard_world = 1;
    c->eng.shard_lo = 0;
    c->eng.shard_hi = c->C;
}

void hgx_destroy(hgx_ctx* ctx) {
    if (!ctx) return;
    drop_group(ctx);
    DeviceGuard dg(ctx);
    delete ctx;
}

// ---- InsertEvent (hashgraph.go:356-401) ------------------------------------------
// Both entry points validate and append on the device (hgx_insert.hip), then mirror the
// per-creator state and the Hashgraph counters (UndeterminedEvents, PendingLoadedEvents).
static int32_t finish_insert(hgx_ctx* c, const hgx::InsertOut& out, int64_t* n_inserted, hgx_error* err) {
    for (int cl = 0; cl < c->C; cl++) {
        const int32_t nl = out.last_gid[cl] >= 0 ? out.last_index[cl] - out.chain_base[cl] + 1 : 0;
        const int32_t d = nl - c->chain_len[cl];
        if (d) {
            c->g_events[cl / c->n] += d;
            c->gs[cl / c->n].undetermined += d;
        }
        c->chain_len[cl] = nl;
    }
    c->last_gid = out.last_gid;
    c->last_index = out.last_index;
    c->chain_base = out.chain_base;
    for (int g = 0; g < c->G; g++) {
        const int64_t l = (int64_t)out.graph_loaded[g];
        c->gs[g].pending_loaded += l - c->g_loaded[g];
        c->g_loaded[g] = l;
    }
    c->E = c->eng.E;
    if (out.accepted > 0) {
        c->mirror_ok = c->chains_ok = false;
        c->rounds_cached = c->recv_cached = false;
    }
    if (n_inserted) *n_inserted = out.accepted;
    std::string msg;
    int32_t rc = HGX_OK;
    switch (out.code) {
        case hgx::INS_OK: return ok(err);
        case hgx::INS_KEY_NOT_FOUND:   // Store.LastFrom of an unknown creator (inmem_store.go:85-90)
            rc = HGX_ERR_KEY_NOT_FOUND;
            msg = "CheckSelfParent: " + std::to_string(out.fail_creator) + ", Not Found";
            break;
        case hgx::INS_SELF_PARENT:
            rc = HGX_ERR_SELF_PARENT;
            msg = "CheckSelfParent: Self-parent not last known event by creator";
            break;
        case hgx::INS_OTHER_PARENT:
            rc = HGX_ERR_OTHER_PARENT;
            msg = "CheckOtherParent: Other-parent not known";
            break;
        case hgx::INS_CAPACITY:
            rc = HGX_ERR_CAPACITY;
            msg = "hgx_insert_events: context capacity exceeded";
            break;
        case hgx::INS_PASSED_INDEX:
            rc = HGX_ERR_PASSED_INDEX;
            msg = "SetEvent: " + go_rune(out.fail_index) + ", Passed Index";
            break;
        case hgx::INS_SKIPPED_INDEX:
            rc = HGX_ERR_SKIPPED_INDEX;
            msg = "SetEvent: " + go_rune(out.fail_index) + ", Skipped Index";
            break;
        case hgx::INS_BAD_SIG:
            rc = HGX_ERR_SIGNATURE;
            msg = "Invalid signature";
            break;
        case hgx::INS_BAD_KEY:   // elliptic.Unmarshal returned nil; ecdsa.Verify dereferences it
            rc = HGX_ERR_PANIC;
            msg = "runtime error: invalid memory address or nil pointer dereference";
            break;
        default:
            rc = HGX_ERR_INVALID;
            msg = "hgx_insert_events: index out of int32 range";
    }
    set_err(err, rc, msg);
    return rc;
}

static int32_t insert_events_one(hgx_ctx* c, const hgx_events* ev, int64_t count, int64_t* n_inserted, hgx_error* err) {
    if (n_inserted) *n_inserted = 0;
    if (!c || !ev || count < 0 ||
        (count > 0 && (!ev->creator || !ev->index || !ev->self_parent || !ev->other_parent || !ev->timestamp_ns ||
                       !ev->hash || !ev->sig_s || !ev->ntx || !ev->tx_nil))) {
        set_err(err, HGX_ERR_INVALID, "hgx_insert_events: bad arguments");
        return HGX_ERR_INVALID;
    }
    DeviceGuard dg(c);
    hgx::InsertIn in{};
    if (count > 0) {
        hipError_t e = c->eng.stage_host(ev->creator, ev->index, ev->self_parent, ev->other_parent, ev->timestamp_ns,
                                         ev->hash, ev->sig_s, ev->ntx, ev->tx_nil, count, in);
        if (e != hipSuccess) return dev_err(err, e, "hgx_insert_events");
    }
    hgx::InsertOut out;
    hipError_t e = c->eng.insert(in, count, out);
    if (e != hipSuccess) return dev_err(err, e, "hgx_insert_events");
    return finish_insert(c, out, n_inserted, err);
}

// a chain-sharded context: every shard inserts the batch (each holds the whole DAG)
int32_t hgx_insert_events(hgx_ctx* c, const hgx_events* ev, int64_t count, int64_t* n_inserted, hgx_error* err) {
    if (c && c->grp)
        return on_shards(c, err, [&](hgx_ctx* x, hgx_error* e) {
            return insert_events_one(x, ev, count, x == c ? n_inserted : nullptr, e);
        });
    return insert_events_one(c, ev, count, n_inserted, err);
}

// Bootstrap / Core.Sync + RunConsensus in one call (hashgraph.go:1008-1037, node/core.go:190-303):
// InsertEvent for the batch, then DivideRounds, DecideFame and FindOrder. The insert is split
// (Engine::insert_split_begin): the structure columns are validated and committed first, and
// the payload columns (timestamps, hash, S, transactions: 80 of the 108 bytes per event) are
// copied to HBM while DivideRounds runs, committed before DecideFame reads the coins.
int32_t hgx_insert_and_run(hgx_ctx* c, const hgx_events* ev, int64_t count, int64_t* n_inserted, hgx_error* err) {
    if (n_inserted) *n_inserted = 0;
    if (!c || !ev || count < 0 ||
        (count > 0 && (!ev->creator || !ev->index || !ev->self_parent || !ev->other_parent || !ev->timestamp_ns ||
                       !ev->hash || !ev->sig_s || !ev->ntx || !ev->tx_nil))) {
        set_err(err, HGX_ERR_INVALID, "hgx_insert_and_run: bad arguments");
        return HGX_ERR_INVALID;
    }
    if (count < 65536 || c->rooted || c->shard_world > 1) {   // small batches gain nothing from the overlap
        int32_t rc = hgx_insert_events(c, ev, count, n_inserted, err);
        if (rc) return rc;
        return hgx_run_consensus(c, err);
    }
    DeviceGuard dg(c);
    const int64_t E0 = c->eng.E;
    hgx::InsertOut out;
    hipError_t e = c->eng.insert_split_begin(ev->creator, ev->index, ev->self_parent, ev->other_parent, count, out);
    if (e != hipSuccess) return dev_err(err, e, "hgx_insert_and_run");
    e = c->eng.payload_begin(ev->timestamp_ns, ev->hash, ev->sig_s, ev->ntx, ev->tx_nil, out.accepted);
    if (e != hipSuccess) return dev_err(err, e, "hgx_insert_and_run");
    // the per-creator mirrors and UndeterminedEvents now; PendingLoadedEvents once the payload
    // (IsLoaded) is committed
    hgx::InsertOut head = out;
    head.graph_loaded.assign(c->g_loaded.begin(), c->g_loaded.end());
    hgx_error ins_err{};
    const int32_t ins_rc = finish_insert(c, head, n_inserted, &ins_err);
    int32_t rc = ins_rc ? ins_rc : hgx_divide_rounds(c, err);
    const bool laid_out = ins_rc == 0 && rc == 0;
    std::vector<uint64_t> loaded;
    e = c->eng.payload_end(E0, out.accepted, laid_out, c->rh.r_lo, loaded);
    if (e != hipSuccess) return dev_err(err, e, "hgx_insert_and_run");
    for (int g = 0; g < c->G; g++) {
        const int64_t l = (int64_t)loaded[g];
        c->gs[g].pending_loaded += l - c->g_loaded[g];
        c->g_loaded[g] = l;
    }
    c->mirror_ok = false;
    if (ins_rc) {   // the accepted prefix is inserted; consensus does not run (as hgx_bootstrap)
        if (err) *err = ins_err;
        return ins_rc;
    }
    if (rc) return rc;
    rc = hgx_decide_fame(c, err);
    if (rc) return rc;
    return hgx_find_order(c, err);
}

static bool bad_events32(const hgx_events32* ev, int64_t count) {
    return !ev || count < 0 ||
           (count > 0 && (!ev->creator || !ev->index || !ev->self_parent || !ev->other_parent || !ev->timestamp_ns ||
                          !ev->coin || !ev->sig_s || !ev->ntx));
}

static int32_t insert_events32_one(hgx_ctx* c, const hgx_events32* ev, int64_t count, int64_t* n_inserted, hgx_error* err) {
    if (n_inserted) *n_inserted = 0;
    if (!c || bad_events32(ev, count)) {
        set_err(err, HGX_ERR_INVALID, "hgx_insert_events32: bad arguments");
        return HGX_ERR_INVALID;
    }
    if (c->rooted) {
        set_err(err, HGX_ERR_INVALID, "hgx_insert_events32: a reset context checks Root.Others by event id: use hgx_insert_events");
        return HGX_ERR_INVALID;
    }
    DeviceGuard dg(c);
    hgx::InsertIn in{};
    if (count > 0) {
        hipError_t e = c->eng.stage_host32(ev->creator, ev->index, ev->self_parent, ev->other_parent, ev->timestamp_ns,
                                           ev->coin, ev->sig_s, ev->ntx, count, in);
        if (e != hipSuccess) return dev_err(err, e, "hgx_insert_events32");
    }
    hgx::InsertOut out;
    hipError_t e = c->eng.insert(in, count, out);
    if (e != hipSuccess) return dev_err(err, e, "hgx_insert_events32");
    return finish_insert(c, out, n_inserted, err);
}

int32_t hgx_insert_events32(hgx_ctx* c, const hgx_events32* ev, int64_t count, int64_t* n_inserted, hgx_error* err) {
    if (c && c->grp)
        return on_shards(c, err, [&](hgx_ctx* x, hgx_error* e) {
            return insert_events32_one(x, ev, count, x == c ? n_inserted : nullptr, e);
        });
    return insert_events32_one(c, ev, count, n_inserted, err);
}

// the rest of a compact-payload insert_and_run once the structure is committed and the payload copy
// started (hgx_insert_and_run32 / _packed): DivideRounds beside the copy, then DecideFame, FindOrder
static int32_t run_after_split32(hgx_ctx* c, int64_t E0, hgx::InsertOut& out, int64_t* n_inserted, hgx_error* err,
                                 const char* who) {
    hipError_t e;
    // S lands last (FindOrder's sort waits for it); on every way out the caller's S buffer has been
    // read completely
    struct WaitS {
        hgx::Engine& eng;
        ~WaitS() { (void)eng.payload_wait_S(); }
    } wait_s{c->eng};
    hgx::InsertOut head = out;
    head.graph_loaded.assign(c->g_loaded.begin(), c->g_loaded.end());
    hgx_error ins_err{};
    const int32_t ins_rc = finish_insert(c, head, n_inserted, &ins_err);
    int32_t rc = ins_rc ? ins_rc : hgx_divide_rounds(c, err);
    const bool laid_out = ins_rc == 0 && rc == 0;
    std::vector<uint64_t> loaded;
    e = c->eng.payload_end(E0, out.accepted, laid_out, c->rh.r_lo, loaded);
    if (e != hipSuccess) return dev_err(err, e, who);
    for (int g = 0; g < c->G; g++) {
        const int64_t l = (int64_t)loaded[g];
        c->gs[g].pending_loaded += l - c->g_loaded[g];
        c->g_loaded[g] = l;
    }
    c->mirror_ok = false;
    if (ins_rc) {
        if (err) *err = ins_err;
        return ins_rc;
    }
    if (rc) return rc;
    rc = hgx_decide_fame(c, err);
    if (rc) return rc;
    rc = hgx_find_order(c, err);
    if (rc) return rc;
    // the S copy's outcome is reported here (FindOrder waits for it only when it sorts; a skipped
    // FindOrder would leave a failed copy unnoticed and g_S stale for a later tie-break); the
    // guard's wait stays for the early ways out
    e = c->eng.payload_wait_S();
    if (e != hipSuccess) return dev_err(err, e, who);
    return ok(err);
}

// hgx_insert_and_run with the compact columns: the structure columns (16 bytes per event) are
// validated and committed first, the payload (45 bytes) copied beside DivideRounds
int32_t hgx_insert_and_run32(hgx_ctx* c, const hgx_events32* ev, int64_t count, int64_t* n_inserted, hgx_error* err) {
    if (n_inserted) *n_inserted = 0;
    if (!c || bad_events32(ev, count)) {
        set_err(err, HGX_ERR_INVALID, "hgx_insert_and_run32: bad arguments");
        return HGX_ERR_INVALID;
    }
    if (count < 65536 || c->rooted || c->shard_world > 1) {
        int32_t rc = hgx_insert_events32(c, ev, count, n_inserted, err);
        if (rc) return rc;
        return hgx_run_consensus(c, err);
    }
    DeviceGuard dg(c);
    const int64_t E0 = c->eng.E;
    hgx::InsertOut out;
    hipError_t e = c->eng.insert_split_begin32(ev->creator, ev->index, ev->self_parent, ev->other_parent, count, out);
    if (e != hipSuccess) return dev_err(err, e, "hgx_insert_and_run32");
    e = c->eng.payload_begin32(ev->timestamp_ns, ev->coin, ev->sig_s, ev->ntx, out.accepted);
    if (e != hipSuccess) return dev_err(err, e, "hgx_insert_and_run32");
    return run_after_split32(c, E0, out, n_inserted, err, "hgx_insert_and_run32");
}

// ---- hgx_events_packed (include/hgx.h): 10-byte structure columns, decoded on the device ----
static bool bad_packed(const hgx_events_packed* ev, int64_t count) {
    if (!ev || count < 0) return true;
    if (count == 0) return false;
    if (!ev->creator || !ev->index || !ev->self_parent_back || !ev->other_parent_back || !ev->timestamp_ns ||
        !ev->coin || !ev->sig_s || !ev->ntx || ev->n_exc < 0 || ev->n_exc > count)
        return true;
    if (ev->n_exc == 0) return false;
    if (!ev->exc_pos || !ev->exc_self_parent || !ev->exc_other_parent) return true;
    // the device scatters the exceptions unchecked: positions in the batch and distinct
    std::vector<int64_t> p(ev->exc_pos, ev->exc_pos + ev->n_exc);
    std::sort(p.begin(), p.end());
    return p.front() < 0 || p.back() >= count || std::adjacent_find(p.begin(), p.end()) != p.end();
}

static hgx::Engine::Packed packed_of(const hgx_events_packed* ev) {
    return hgx::Engine::Packed{ev->creator, ev->index, ev->self_parent_back, ev->other_parent_back,
                               ev->n_exc, ev->exc_pos, ev->exc_self_parent, ev->exc_other_parent};
}

static int32_t insert_events_packed_one(hgx_ctx* c, const hgx_events_packed* ev, int64_t count, int64_t* n_inserted,
                                        hgx_error* err) {
    if (n_inserted) *n_inserted = 0;
    if (c->rooted) {
        set_err(err, HGX_ERR_INVALID, "hgx_insert_events_packed: a reset context checks Root.Others by event id: use hgx_insert_events");
        return HGX_ERR_INVALID;
    }
    DeviceGuard dg(c);
    hgx::InsertIn in{};
    if (count > 0) {
        hipError_t e = c->eng.stage_packed(packed_of(ev), count, in, ev->timestamp_ns, ev->coin, ev->sig_s, ev->ntx);
        if (e != hipSuccess) return dev_err(err, e, "hgx_insert_events_packed");
    }
    hgx::InsertOut out;
    hipError_t e = c->eng.insert(in, count, out);
    if (e != hipSuccess) return dev_err(err, e, "hgx_insert_events_packed");
    return finish_insert(c, out, n_inserted, err);
}

int32_t hgx_insert_events_packed(hgx_ctx* c, const hgx_events_packed* ev, int64_t count, int64_t* n_inserted,
                                 hgx_error* err) {
    if (n_inserted) *n_inserted = 0;
    if (!c || bad_packed(ev, count)) {
        set_err(err, HGX_ERR_INVALID, "hgx_insert_events_packed: bad arguments");
        return HGX_ERR_INVALID;
    }
    if (c->grp)
        return on_shards(c, err, [&](hgx_ctx* x, hgx_error* e) {
            return insert_events_packed_one(x, ev, count, x == c ? n_inserted : nullptr, e);
        });
    return insert_events_packed_one(c, ev, count, n_inserted, err);
}

// hgx_insert_and_run32 with the packed structure columns: 10 bytes per event staged, decoded and
// validated before DivideRounds, the payload (45 bytes) copied beside it as in hgx_insert_and_run32
int32_t hgx_insert_and_run_packed(hgx_ctx* c, const hgx_events_packed* ev, int64_t count, int64_t* n_inserted,
                                  hgx_error* err) {
    if (n_inserted) *n_inserted = 0;
    if (!c || bad_packed(ev, count)) {
        set_err(err, HGX_ERR_INVALID, "hgx_insert_and_run_packed: bad arguments");
        return HGX_ERR_INVALID;
    }
    if (count < 65536 || c->rooted || c->shard_world > 1) {
        int32_t rc = hgx_insert_events_packed(c, ev, count, n_inserted, err);
        if (rc) return rc;
        return hgx_run_consensus(c, err);
    }
    DeviceGuard dg(c);
    const int64_t E0 = c->eng.E;
    hgx::InsertOut out;
    hipError_t e = c->eng.insert_split_begin_packed(packed_of(ev), count, out);
    if (e != hipSuccess) return dev_err(err, e, "hgx_insert_and_run_packed");
    e = c->eng.payload_begin32(ev->timestamp_ns, ev->coin, ev->sig_s, ev->ntx, out.accepted);
    if (e != hipSuccess) return dev_err(err, e, "hgx_insert_and_run_packed");
    return run_after_split32(c, E0, out, n_inserted, err, "hgx_insert_and_run_packed");
}

int32_t hgx_pack_events32(const hgx_events32* ev, int64_t count, int64_t base, uint16_t* creator16, uint16_t* sp_back,
                          uint16_t* op_back, int64_t* exc_pos, int32_t* exc_sp, int32_t* exc_op, int64_t exc_cap,
                          int64_t* n_exc, hgx_error* err) {
    if (n_exc) *n_exc = 0;
    if (bad_events32(ev, count) || base < 0 || exc_cap < 0 || !n_exc ||
        (count > 0 && (!creator16 || !sp_back || !op_back)) || (exc_cap > 0 && (!exc_pos || !exc_sp || !exc_op))) {
        set_err(err, HGX_ERR_INVALID, "hgx_pack_events32: bad arguments");
        return HGX_ERR_INVALID;
    }
    // a parent's distance back from gid g, or the escape (a parent the form cannot hold: later than
    // g, more than 65 534 back, or a negative value other than "")
    auto back = [](int64_t p, int64_t g) -> uint32_t {
        if (p == -1) return 0;
        return p >= 0 && p < g && g - p < HGX_PARENT_ESCAPE ? (uint32_t)(g - p) : (uint32_t)HGX_PARENT_ESCAPE;
    };
    int64_t x = 0;
    for (int64_t k = 0; k < count; k++) {
        const int32_t cr = ev->creator[k];
        if (cr < 0 || cr > 0xFFFF) {
            set_err(err, HGX_ERR_INVALID, "hgx_pack_events32: creator outside 0..65535");
            return HGX_ERR_INVALID;
        }
        const int64_t g = base + k;
        const uint32_t s = back(ev->self_parent[k], g), o = back(ev->other_parent[k], g);
        creator16[k] = (uint16_t)cr;
        sp_back[k] = (uint16_t)s;
        op_back[k] = (uint16_t)o;
        if (s == HGX_PARENT_ESCAPE || o == HGX_PARENT_ESCAPE) {
            if (x < exc_cap) {
                exc_pos[x] = k;
                exc_sp[x] = ev->self_parent[k];
                exc_op[x] = ev->other_parent[k];
            }
            x++;
        }
    }
    *n_exc = x;
    if (x > exc_cap) {
        set_err(err, HGX_ERR_INVALID, "hgx_pack_events32: exception list full");
        return HGX_ERR_INVALID;
    }
    return ok(err);
}

// page-locked, portable (any device's context may copy from it), not mapped: the column copies are
// plain DMA transfers from it
void* hgx_host_alloc(int64_t bytes) {
    if (bytes <= 0) return nullptr;
    void* p = nullptr;
    if (hipHostMalloc(&p, (size_t)bytes, hipHostMallocPortable) != hipSuccess) return nullptr;
    return p;
}

void hgx_host_free(void* p) {
    if (p) (void)hipHostFree(p);
}

int32_t hgx_set_participant_keys(hgx_ctx* c, const uint8_t* keys65, hgx_error* err) {
    if (!c || !keys65) {
        set_err(err, HGX_ERR_INVALID, "hgx_set_participant_keys: bad arguments");
        return HGX_ERR_INVALID;
    }
    DeviceGuard dg(c);
    const hipError_t e = c->eng.set_keys(keys65);
    if (e != hipSuccess) return dev_err(err, e, "hgx_set_participant_keys");
    return ok(err);
}

static int32_t insert_verified(hgx_ctx* c, const hgx_events* ev, const uint8_t* digest32, const uint8_t* sig_r32,
                               int64_t count, int64_t* n_inserted, hgx_error* err, bool on_device) {
    const char* who = on_device ? "hgx_insert_events_verified_device" : "hgx_insert_events_verified";
    if (n_inserted) *n_inserted = 0;
    if (!c || !ev || count < 0 ||
        (count > 0 && (!ev->creator || !ev->index || !ev->self_parent || !ev->other_parent || !ev->timestamp_ns ||
                       !ev->hash || !ev->sig_s || !ev->ntx || !ev->tx_nil || !digest32 || !sig_r32)) ||
        (on_device && (((uintptr_t)ev->sig_s & 15) || ((uintptr_t)ev->hash & 15)))) {
        set_err(err, HGX_ERR_INVALID, std::string(who) + ": bad arguments");
        return HGX_ERR_INVALID;
    }
    if (group_only_one(c, err, who)) return HGX_ERR_INVALID;
    DeviceGuard dg(c);
    if (!c->eng.keys_set) {
        set_err(err, HGX_ERR_INVALID, std::string(who) + ": participant keys not set");
        return HGX_ERR_INVALID;
    }
    hgx::InsertIn in{};
    const uint8_t *dd = digest32, *dr = sig_r32;
    if (on_device) {
        in.creator = ev->creator; in.index = ev->index; in.sp = ev->self_parent; in.op = ev->other_parent;
        in.ts = ev->timestamp_ns; in.hash = ev->hash; in.S = ev->sig_s; in.ntx = ev->ntx; in.nil = ev->tx_nil;
    } else if (count > 0) {
        hipError_t e = c->eng.stage_host(ev->creator, ev->index, ev->self_parent, ev->other_parent, ev->timestamp_ns,
                                         ev->hash, ev->sig_s, ev->ntx, ev->tx_nil, count, in);
        if (e == hipSuccess) e = c->eng.stage_sig(digest32, sig_r32, count, &dd, &dr);
        if (e != hipSuccess) return dev_err(err, e, who);
    }
    hgx::InsertOut out;
    const hipError_t e = c->eng.insert_verified(in, dd, dr, count, out);
    if (e != hipSuccess) return dev_err(err, e, who);
    return finish_insert(c, out, n_inserted, err);
}

int32_t hgx_insert_events_verified(hgx_ctx* c, const hgx_events* ev, const uint8_t* digest32, const uint8_t* sig_r32,
                                   int64_t count, int64_t* n_inserted, hgx_error* err) {
    return insert_verified(c, ev, digest32, sig_r32, count, n_inserted, err, false);
}

int32_t hgx_insert_events_verified_device(hgx_ctx* c, const hgx_events* ev, const uint8_t* digest32,
                                          const uint8_t* sig_r32, int64_t count, int64_t* n_inserted, hgx_error* err) {
    return insert_verified(c, ev, digest32, sig_r32, count, n_inserted, err, true);
}

// Core.Sync's loop (node/core.go:199-211) over a SyncResponse's WireEvents: ReadWireInfo
// (hashgraph.go:569-614, parents through Store.ParticipantEvent, which sees the events of the
// batch inserted before) then InsertEvent(ev, false), stopping at the first error. Parents are
// resolved on the host against the participants' RollingIndexes plus the batch so far ("as if
// every earlier event was accepted", like the device insert); the prefix before the first
// resolution error goes through the batched device insert, whose first failure comes first.
int32_t hgx_insert_wire_events(hgx_ctx* c, const hgx_wire_events* w, int64_t count, int64_t* n_inserted,
                               hgx_error* err) {
    if (n_inserted) *n_inserted = 0;
    if (!c || !w || count < 0 ||
        (count > 0 && (!w->creator_id || !w->index || !w->self_parent_index || !w->other_parent_creator ||
                       !w->other_parent_index || !w->timestamp_ns || !w->hash || !w->sig_s || !w->ntx || !w->tx_nil))) {
        set_err(err, HGX_ERR_INVALID, "hgx_insert_wire_events: bad arguments");
        return HGX_ERR_INVALID;
    }
    if (group_only_one(c, err, "hgx_insert_wire_events")) return HGX_ERR_INVALID;
    DeviceGuard dg(c);
    if (ensure_chains(c)) return dev_err(err, hipErrorUnknown, "hgx_insert_wire_events");
    const int64_t E0 = c->E;
    std::vector<std::vector<std::pair<int64_t, int64_t>>> pend((size_t)c->C);   // (index, gid) of the batch
    // RollingIndex.GetItem over the participant's events plus the batch's (common/rolling_index.go:40-50)
    auto participant_event = [&](int32_t p, int64_t idx, int64_t* gid, std::string& msg) -> int32_t {
        if (p < 0 || p >= c->C) {   // ReverseParticipants miss: participantEvents[""] is nil
            msg = "runtime error: invalid memory address or nil pointer dereference";
            return HGX_ERR_PANIC;
        }
        const auto& pb = pend[(size_t)p];
        const int64_t items = c->chain_len[(size_t)p] + (int64_t)pb.size();
        const int64_t last = pb.empty() ? c->last_index[(size_t)p] : pb.back().first;
        const int64_t oldest = last - items + 1;
        if (idx < oldest) { msg = go_rune(idx) + ", Too Late"; return HGX_ERR_TOO_LATE; }
        const int64_t f = idx - oldest;
        if (f >= items) { msg = go_rune(idx) + ", Not Found"; return HGX_ERR_KEY_NOT_FOUND; }
        const int64_t cl = c->chain_len[(size_t)p];
        *gid = f < cl ? c->chain_gids[(size_t)p][(size_t)f] : pb[(size_t)(f - cl)].second;
        return HGX_OK;
    };
    std::vector<int32_t> creator((size_t)count);
    std::vector<int64_t> sp((size_t)count), op((size_t)count);
    int64_t m = count;
    int32_t rrc = HGX_OK;
    std::string rmsg;
    for (int64_t k = 0; k < count; k++) {
        const int32_t cr = w->creator_id[k];
        if (cr < 0 || cr >= c->C) {   // creator[2:] of "" (hashgraph.go:578-582)
            m = k;
            rrc = HGX_ERR_PANIC;
            rmsg = "runtime error: slice bounds out of range [2:0]";
            break;
        }
        int64_t s = -1, o = -1;
        int32_t rc = HGX_OK;
        if (w->self_parent_index[k] >= 0) rc = participant_event(cr, w->self_parent_index[k], &s, rmsg);
        if (rc == HGX_OK && w->other_parent_index[k] >= 0)
            rc = participant_event(w->other_parent_creator[k], w->other_parent_index[k], &o, rmsg);
        if (rc != HGX_OK) {
            m = k;
            rrc = rc;
            break;
        }
        creator[(size_t)k] = cr;
        sp[(size_t)k] = s;
        op[(size_t)k] = o;
        pend[(size_t)cr].push_back({w->index[k], E0 + k});
    }
    const hgx_events ev{creator.data(), w->index, sp.data(), op.data(), w->timestamp_ns, w->hash, w->sig_s, w->ntx,
                        w->tx_nil};
    int64_t ins = 0;
    const int32_t rc = m > 0 ? hgx_insert_events(c, &ev, m, &ins, err) : ok(err);
    if (n_inserted) *n_inserted = ins;
    if (ins > 0) {   // the host mirrors stay valid: append the accepted events (no O(E) rebuild per sync)
        for (int64_t k = 0; k < ins; k++) {
            c->creator.push_back(creator[(size_t)k]);
            c->index32.push_back((int32_t)w->index[k]);
            c->sp.push_back((int32_t)sp[(size_t)k]);
            c->op.push_back((int32_t)op[(size_t)k]);
            c->chain_gids[(size_t)creator[(size_t)k]].push_back((int32_t)(E0 + k));
        }
        c->mirror_ok = c->chains_ok = true;
    }
    if (rc != HGX_OK) return rc;
    if (rrc != HGX_OK) {
        set_err(err, rrc, rmsg);
        return rrc;
    }
    return HGX_OK;
}

static int32_t insert_events_device_one(hgx_ctx* c, const hgx_events* ev, int64_t count, int64_t* n_inserted,
                                        hgx_error* err) {
    if (n_inserted) *n_inserted = 0;
    if (!c || !ev || count < 0 ||
        (count > 0 && (!ev->creator || !ev->index || !ev->self_parent || !ev->other_parent || !ev->timestamp_ns ||
                       !ev->hash || !ev->sig_s || !ev->ntx || !ev->tx_nil)) ||
        ((uintptr_t)ev->sig_s & 15) || ((uintptr_t)ev->hash & 15)) {
        set_err(err, HGX_ERR_INVALID, "hgx_insert_events_device: bad arguments (hash / sig_s must be 16-byte aligned)");
        return HGX_ERR_INVALID;
    }
    DeviceGuard dg(c);
    hgx::InsertIn in{ev->creator, ev->index, ev->self_parent, ev->other_parent, ev->timestamp_ns,
                     ev->hash, ev->sig_s, ev->ntx, ev->tx_nil};
    hgx::InsertOut out;
    hipError_t e = c->eng.insert(in, count, out);
    if (e != hipSuccess) return dev_err(err, e, "hgx_insert_events_device");
    return finish_insert(c, out, n_inserted, err);
}

// a chain-sharded context: the columns are device pointers of shard 0's device; the other shards'
// kernels read them through the peer mapping
int32_t hgx_insert_events_device(hgx_ctx* c, const hgx_events* ev, int64_t count, int64_t* n_inserted,
                                 hgx_error* err) {
    if (c && c->grp)
        return on_shards(c, err, [&](hgx_ctx* x, hgx_error* e) {
            return insert_events_device_one(x, ev, count, x == c ? n_inserted : nullptr, e);
        });
    return insert_events_device_one(c, ev, count, n_inserted, err);
}

static int32_t clear_one(hgx_ctx* c) {
    if (!c) return HGX_ERR_INVALID;
    DeviceGuard dg(c);
    if (c->eng.clear() != hipSuccess) return HGX_ERR_DEVICE;
    std::fill(c->chain_len.begin(), c->chain_len.end(), 0);
    std::fill(c->chain_base.begin(), c->chain_base.end(), 0);
    std::fill(c->last_gid.begin(), c->last_gid.end(), -1);
    std::fill(c->last_index.begin(), c->last_index.end(), -1);
    for (int g = 0; g < c->G; g++) {
        c->gs[g].reset();
        c->order[g] = GraphOrder();
    }
    std::fill(c->g_events.begin(), c->g_events.end(), 0);
    std::fill(c->g_loaded.begin(), c->g_loaded.end(), 0);
    c->arena.used = 0;
    c->E = c->E_div = 0;
    c->divided = false;
    c->fo_prev_valid = false;
    c->mirror_ok = c->chains_ok = false;
    c->rounds_cached = c->recv_cached = false;
    c->pl_off.clear();
    c->pl_blob.clear();
    c->reset_kept.clear();
    c->others_keys.clear();
    if (c->rooted) {   // a fresh NewHashgraph has genesis roots
        std::fill(c->root_index.begin(), c->root_index.end(), -1);
        std::fill(c->root_round.begin(), c->root_round.end(), -1);
        std::fill(c->root_y_ext.begin(), c->root_y_ext.end(), 0);
        c->rooted = false;
        if (c->eng.set_roots(c->root_round, c->root_y_ext) != hipSuccess) return HGX_ERR_DEVICE;
    }
    return HGX_OK;
}

int32_t hgx_clear(hgx_ctx* c) {
    if (c && c->grp) return on_shards(c, nullptr, [](hgx_ctx* x, hgx_error*) { return clear_one(x); });
    return clear_one(c);
}

// ---- checkpoint file + Bootstrap (hashgraph.go:1008-1037, badger_store.go:345-386) ----------
// Format: include/hgx.h. The file is the replay log Bootstrap needs: the events in topological
// (gid) order with the columns consensus reads, plus the roots of a context after a Reset.
static const char kCkptMagic[8] = {'H', 'G', 'X', 'C', 'K', 'P', 'T', '1'};

static uint64_t fnv1a(uint64_t h, const void* p, size_t n) {
    const uint8_t* b = (const uint8_t*)p;
    for (size_t i = 0; i < n; i++) {
        h ^= b[i];
        h *= 1099511628211ull;
    }
    return h;
}

uint64_t hgx_checksum(const void* data, int64_t bytes) {
    return fnv1a(14695981039346656037ull, data, bytes > 0 && data ? (size_t)bytes : 0);
}

namespace {
struct CkptWriter {
    FILE* f;
    uint64_t h = 14695981039346656037ull;
    bool ok = true;
    void put(const void* p, size_t n) {
        if (!ok || n == 0) return;
        h = fnv1a(h, p, n);
        ok = std::fwrite(p, 1, n, f) == n;
    }
};
struct CkptReader {
    std::vector<uint8_t> buf;
    size_t pos = 0;
    bool get(void* p, size_t n) {
        if (buf.size() - pos < n) return false;
        if (n) std::memcpy(p, buf.data() + pos, n);
        pos += n;
        return true;
    }
};
}  // namespace

enum : int32_t { kCkRooted = 1, kCkIds = 2, kCkKeys = 4, kCkPayloads = 8 };

int32_t hgx_save_ex(hgx_ctx* c, const char* path, const int64_t* payload_off, const uint8_t* payload, hgx_error* err) {
    if (!c || !path || (payload_off && !payload && c->E > 0)) {
        set_err(err, HGX_ERR_INVALID, "hgx_save: bad arguments");
        return HGX_ERR_INVALID;
    }
    DeviceGuard dg(c);
    std::vector<int32_t> creator, index, sp, op, ntx;
    std::vector<int64_t> ts;
    std::vector<uint8_t> S, coin, nil, ids, keys;
    hipError_t e = c->eng.get_columns(creator, index, sp, op, ts, S, coin, ntx, nil);
    if (e != hipSuccess) return dev_err(err, e, "hgx_save");
    const int64_t E = (int64_t)creator.size();
    const bool have_ids = c->eng.ids_known && E > 0;
    if (have_ids) {
        ids.resize((size_t)E * 32);
        e = c->eng.get_ids(0, E, ids.data());
        if (e != hipSuccess) return dev_err(err, e, "hgx_save");
    }
    if (c->eng.keys_set) {
        keys.resize((size_t)c->C * 65);
        e = c->eng.get_keys(keys.data());
        if (e != hipSuccess) return dev_err(err, e, "hgx_save");
    }
    if (payload_off) {   // offsets must be non-decreasing from 0
        if (payload_off[0] != 0) {
            set_err(err, HGX_ERR_INVALID, "hgx_save: payload offsets must start at 0");
            return HGX_ERR_INVALID;
        }
        for (int64_t i = 0; i < E; i++)
            if (payload_off[i + 1] < payload_off[i]) {
                set_err(err, HGX_ERR_INVALID, "hgx_save: payload offsets must not decrease");
                return HGX_ERR_INVALID;
            }
    }
    const std::string tmp = std::string(path) + ".tmp";
    FILE* f = std::fopen(tmp.c_str(), "wb");
    if (!f) {
        set_err(err, HGX_ERR_INVALID, std::string("hgx_save: cannot open ") + tmp);
        return HGX_ERR_INVALID;
    }
    CkptWriter w{f};
    const uint32_t version = 2;
    const int32_t flags = (c->rooted ? kCkRooted : 0) | (have_ids ? kCkIds : 0) | (keys.empty() ? 0 : kCkKeys) |
                          (payload_off ? kCkPayloads : 0);
    w.put(kCkptMagic, 8);
    w.put(&version, 4);
    w.put(&c->n, 4);
    w.put(&c->G, 4);
    w.put(&flags, 4);
    w.put(&E, 8);
    if (c->rooted) {
        // the roots, the Root.Others keys and what Reset kept (badger_store.go persists the roots
        // and the blocks; LastConsensusRound & co. are Hashgraph fields Reset leaves in place)
        w.put(c->root_index.data(), (size_t)c->C * 4);
        w.put(c->root_round.data(), (size_t)c->C * 4);
        std::vector<uint8_t> y(c->root_y_ext.begin(), c->root_y_ext.end());
        y.resize(((size_t)c->C + 3) & ~(size_t)3, 0);
        w.put(y.data(), y.size());
        const int64_t no = (int64_t)(c->others_keys.size() / 32);
        w.put(&no, 8);
        w.put(c->others_keys.data(), c->others_keys.size());
        for (int g = 0; g < c->G; g++) {
            const hgx_ctx::Kept k = g < (int)c->reset_kept.size() ? c->reset_kept[g] : hgx_ctx::Kept();
            const int32_t hdr[4] = {k.has_lcr ? 1 : 0, k.lcr, k.lcre, 0};
            const int64_t cnt[2] = {k.consensus_tx, (int64_t)k.blocks.size()};
            w.put(hdr, 16);
            w.put(cnt, 16);
            for (const Block& b : k.blocks) {
                const int32_t a0[2] = {b.rr, b.nev};
                const int32_t a1[2] = {b.tx_nil, b.committed};
                w.put(a0, 8);
                w.put(&b.ntx, 8);
                w.put(a1, 8);
            }
        }
    }
    std::vector<int64_t> wide((size_t)E);
    w.put(creator.data(), (size_t)E * 4);
    for (auto* col : {&index, &sp, &op}) {
        for (int64_t i = 0; i < E; i++) wide[(size_t)i] = (*col)[(size_t)i];
        w.put(wide.data(), (size_t)E * 8);
    }
    w.put(ts.data(), (size_t)E * 8);
    w.put(S.data(), (size_t)E * 32);
    w.put(coin.data(), (size_t)E);
    w.put(ntx.data(), (size_t)E * 4);
    w.put(nil.data(), (size_t)E);
    if (have_ids) w.put(ids.data(), ids.size());
    if (!keys.empty()) w.put(keys.data(), keys.size());
    if (payload_off) {
        w.put(payload_off, (size_t)(E + 1) * 8);
        w.put(payload, (size_t)payload_off[E]);
    }
    const uint64_t sum = w.h;
    w.put(&sum, 8);
    const bool ok_w = w.ok && std::fflush(f) == 0;
    std::fclose(f);
    if (!ok_w || std::rename(tmp.c_str(), path) != 0) {
        std::remove(tmp.c_str());
        set_err(err, HGX_ERR_INVALID, std::string("hgx_save: write failed: ") + path);
        return HGX_ERR_INVALID;
    }
    return ok(err);
}

int32_t hgx_save(hgx_ctx* c, const char* path, hgx_error* err) { return hgx_save_ex(c, path, nullptr, nullptr, err); }

int32_t hgx_bootstrap(hgx_ctx* c, const char* path, hgx_error* err) {
    if (!c || !path) {
        set_err(err, HGX_ERR_INVALID, "hgx_bootstrap: bad arguments");
        return HGX_ERR_INVALID;
    }
    if (group_only_one(c, err, "hgx_bootstrap")) return HGX_ERR_INVALID;
    auto bad = [&](const std::string& why) {
        set_err(err, HGX_ERR_INVALID, "hgx_bootstrap: " + why);
        return HGX_ERR_INVALID;
    };
    if (c->E != 0) return bad("the context already holds events (Bootstrap runs on a fresh Hashgraph)");
    CkptReader r;
    {
        FILE* f = std::fopen(path, "rb");
        if (!f) return bad(std::string("cannot open ") + path);
        uint8_t tmp[1 << 16];
        size_t got;
        while ((got = std::fread(tmp, 1, sizeof tmp, f)) > 0) r.buf.insert(r.buf.end(), tmp, tmp + got);
        std::fclose(f);
    }
    if (r.buf.size() < 8 + 4 + 12 + 8 + 8) return bad("truncated file");
    uint64_t stored = 0;
    std::memcpy(&stored, r.buf.data() + r.buf.size() - 8, 8);
    if (fnv1a(14695981039346656037ull, r.buf.data(), r.buf.size() - 8) != stored) return bad("checksum mismatch");
    r.buf.resize(r.buf.size() - 8);   // (reads past the body fail: truncated sections are caught)
    char magic[8];
    uint32_t version = 0;
    int32_t n = 0, G = 0, flags = 0;
    int64_t E = 0;
    r.get(magic, 8);
    r.get(&version, 4);
    r.get(&n, 4);
    r.get(&G, 4);
    r.get(&flags, 4);
    r.get(&E, 8);
    if (std::memcmp(magic, kCkptMagic, 8) != 0) return bad("not a checkpoint file");
    if (version != 1 && version != 2) return bad("unsupported version " + std::to_string(version));
    if (version == 1 && (flags & ~kCkRooted)) return bad("unsupported flags");
    if (n != c->n || G != c->G)
        return bad("file has " + std::to_string(G) + " x " + std::to_string(n) + " participants, the context " +
                   std::to_string(c->G) + " x " + std::to_string(c->n));
    if (E < 0 || E > (int64_t)(r.buf.size() / 60)) return bad("truncated file");
    if (E > c->eng.cap) return bad("the file has " + std::to_string(E) + " events, the context's capacity is " +
                                   std::to_string(c->eng.cap));
    const size_t Ez = (size_t)E, Cz = (size_t)c->C;
    // every section is parsed and validated into locals first; the context is touched (Reset,
    // Root.Others, the kept state, keys, events) only once the whole file is accepted
    std::vector<uint8_t> others;
    std::vector<hgx_ctx::Kept> kept;
    std::vector<int32_t> ri(Cz), rr(Cz), ry(Cz);
    if (flags & kCkRooted) {
        std::vector<uint8_t> y((Cz + 3) & ~(size_t)3);
        if (!r.get(ri.data(), Cz * 4) || !r.get(rr.data(), Cz * 4) || !r.get(y.data(), y.size())) return bad("truncated file");
        for (size_t p = 0; p < Cz; p++) ry[p] = y[p];
        if (version >= 2) {
            int64_t no = 0;
            if (!r.get(&no, 8) || no < 0 || no > (int64_t)(r.buf.size() / 32)) return bad("truncated file");
            others.resize((size_t)no * 32);
            if (!r.get(others.data(), others.size())) return bad("truncated file");
            kept.resize((size_t)G);
            for (int g = 0; g < G; g++) {
                int32_t hdr[4];
                int64_t cnt[2];
                if (!r.get(hdr, 16) || !r.get(cnt, 16) || cnt[1] < 0 || cnt[1] > (int64_t)(r.buf.size() / 24))
                    return bad("truncated file");
                hgx_ctx::Kept& k = kept[(size_t)g];
                k.has_lcr = hdr[0] != 0;
                k.lcr = hdr[1];
                k.lcre = hdr[2];
                k.consensus_tx = cnt[0];
                k.blocks.resize((size_t)cnt[1]);
                for (Block& b : k.blocks) {
                    int32_t a0[2], a1[2];
                    if (!r.get(a0, 8) || !r.get(&b.ntx, 8) || !r.get(a1, 8)) return bad("truncated file");
                    b.rr = a0[0];
                    b.nev = a0[1];
                    b.tx_nil = a1[0];
                    b.committed = a1[1];
                    b.first = -1;
                }
            }
        }
    }
    std::vector<int32_t> creator(Ez), ntx(Ez), nil(Ez);
    std::vector<int64_t> index(Ez), sp(Ez), op(Ez), ts(Ez);
    std::vector<uint8_t> S(Ez * 32), coin(Ez), nil8(Ez), hash(Ez * 32, 0);
    if (!r.get(creator.data(), Ez * 4) || !r.get(index.data(), Ez * 8) || !r.get(sp.data(), Ez * 8) ||
        !r.get(op.data(), Ez * 8) || !r.get(ts.data(), Ez * 8) || !r.get(S.data(), Ez * 32) ||
        !r.get(coin.data(), Ez) || !r.get(ntx.data(), Ez * 4) || !r.get(nil8.data(), Ez))
        return bad("truncated file");
    const bool have_ids = (flags & kCkIds) != 0;
    if (have_ids) {
        if (!r.get(hash.data(), Ez * 32)) return bad("truncated file");
        for (size_t i = 0; i < Ez; i++)
            if ((hash[32 * i + 16] != 0) != (coin[i] != 0)) return bad("event id and coin disagree at event " + std::to_string(i));
    } else {
        for (size_t i = 0; i < Ez; i++) hash[32 * i + 16] = coin[i] ? 1 : 0;   // the byte middleBit reads (hashgraph.go:1039-1048)
    }
    for (size_t i = 0; i < Ez; i++) nil[i] = nil8[i];
    std::vector<uint8_t> keys;
    if (flags & kCkKeys) {
        keys.resize(Cz * 65);
        if (!r.get(keys.data(), keys.size())) return bad("truncated file");
    }
    std::vector<int64_t> poff;
    std::vector<uint8_t> pblob;
    if (flags & kCkPayloads) {
        poff.resize(Ez + 1);
        if (!r.get(poff.data(), (Ez + 1) * 8) || poff[0] != 0) return bad("truncated file");
        for (size_t i = 0; i < Ez; i++)
            if (poff[i + 1] < poff[i]) return bad("payload offsets decrease");
        if (poff[Ez] < 0 || poff[Ez] > (int64_t)(r.buf.size() - r.pos)) return bad("truncated file");
        pblob.resize((size_t)poff[Ez]);
        if (!r.get(pblob.data(), pblob.size())) return bad("truncated file");
    }
    if (r.pos != r.buf.size()) return bad("size mismatch");
    if (flags & kCkRooted) {
        const int32_t rc = hgx_reset(c, ri.data(), rr.data(), ry.data(), err);
        if (rc) return rc;
        if (!others.empty()) {
            const int32_t rc2 = hgx_set_root_others(c, others.data(), (int64_t)(others.size() / 32), err);
            if (rc2) return rc2;
        }
        if (version >= 2) {   // what Reset kept at the saved context
            for (int g = 0; g < G; g++) {
                GraphState& s = c->gs[g];
                const hgx_ctx::Kept& k = kept[(size_t)g];
                s.has_lcr = k.has_lcr;
                s.lcr = k.lcr;
                s.lcre = k.lcre;
                s.consensus_tx = k.consensus_tx;
                s.blocks = k.blocks;
            }
            c->reset_kept = kept;
        }
    }
    if (!keys.empty()) {
        const int32_t rc = hgx_set_participant_keys(c, keys.data(), err);
        if (rc) return rc;
    }
    hgx_events ev{creator.data(), index.data(), sp.data(), op.data(), ts.data(), hash.data(), S.data(), ntx.data(),
                  nil.data()};
    int64_t inserted = 0;
    // a version-1 file carries no ids: its Root.Others codes were checked when the events were
    // first inserted; a version-2 rooted file brings the keys and the ids, so they are checked again
    c->eng.others_trust = (flags & kCkRooted) && !have_ids;
    int32_t rc = hgx_insert_events(c, &ev, E, &inserted, err);
    c->eng.others_trust = false;
    if (!have_ids) c->eng.ids_known = false;
    c->pl_off = std::move(poff);
    c->pl_blob = std::move(pblob);
    if (rc) return rc;
    return hgx_run_consensus(c, err);
}

int32_t hgx_get_event_id(hgx_ctx* c, int64_t gid, uint8_t* out32, hgx_error* err) {
    if (!c || !out32 || gid < 0 || gid >= c->E) {
        set_err(err, HGX_ERR_KEY_NOT_FOUND, std::to_string(gid) + ", Not Found");
        return HGX_ERR_KEY_NOT_FOUND;
    }
    if (!c->eng.ids_known) {
        set_err(err, HGX_ERR_INVALID, "hgx_get_event_id: the events were inserted without their ids (hgx_events32)");
        return HGX_ERR_INVALID;
    }
    DeviceGuard dg(c);
    const hipError_t e = c->eng.get_ids(gid, 1, out32);
    if (e != hipSuccess) return dev_err(err, e, "hgx_get_event_id");
    return ok(err);
}

int32_t hgx_get_event_payload(hgx_ctx* c, int64_t gid, uint8_t* out, int64_t cap, int64_t* len, hgx_error* err) {
    if (len) *len = 0;
    if (!c || gid < 0 || gid >= c->E) {
        set_err(err, HGX_ERR_KEY_NOT_FOUND, std::to_string(gid) + ", Not Found");
        return HGX_ERR_KEY_NOT_FOUND;
    }
    if (c->pl_off.empty() || gid + 1 >= (int64_t)c->pl_off.size()) {
        set_err(err, HGX_ERR_KEY_NOT_FOUND, std::to_string(gid) + ", Not Found");
        return HGX_ERR_KEY_NOT_FOUND;
    }
    const int64_t a = c->pl_off[(size_t)gid], b = c->pl_off[(size_t)gid + 1];
    if (len) *len = b - a;
    if (out && cap > 0) std::memcpy(out, c->pl_blob.data() + a, (size_t)std::min<int64_t>(cap, b - a));
    return ok(err);
}

// ---- Reset (hashgraph.go:877-895, inmem_store.go:184-192) ---------------------------------
// Store.Reset: new roots, the event / round / consensus caches and the participants'
// RollingIndexes cleared, lastRound = -1 (the block cache is kept). Hashgraph.Reset:
// UndeterminedEvents, UndecidedRounds (empty), PendingLoadedEvents, topologicalIndex and the
// memo caches; LastConsensusRound, LastCommitedRoundEvents and ConsensusTransactions are kept.
int32_t hgx_reset(hgx_ctx* c, const int32_t* root_index, const int32_t* root_round, const int32_t* root_y_is_event,
                  hgx_error* err) {
    if (!c || !root_index || !root_round || !root_y_is_event) {
        set_err(err, HGX_ERR_INVALID, "hgx_reset: bad arguments");
        return HGX_ERR_INVALID;
    }
    if (group_only_one(c, err, "hgx_reset")) return HGX_ERR_INVALID;
    DeviceGuard dg(c);
    std::vector<int32_t> rr(root_round, root_round + c->C);
    std::vector<uint8_t> ye(c->C);
    bool rooted = false;
    for (int p = 0; p < c->C; p++) {
        ye[p] = root_y_is_event[p] ? 1 : 0;
        if (rr[p] >= 0 || ye[p]) rooted = true;
    }
    if (rooted && c->G != 1) {
        set_err(err, HGX_ERR_INVALID, "hgx_reset: roots need a single-graph context");
        return HGX_ERR_INVALID;
    }
    if (c->eng.clear() != hipSuccess || c->eng.set_roots(rr, ye) != hipSuccess ||
        c->eng.set_root_others(nullptr, 0) != hipSuccess)
        return dev_err(err, hipErrorUnknown, "hgx_reset");
    c->root_index.assign(root_index, root_index + c->C);
    c->root_round = rr;
    c->root_y_ext = ye;
    c->rooted = rooted;
    c->others_keys.clear();
    c->pl_off.clear();
    c->pl_blob.clear();
    c->reset_kept.assign(c->G, hgx_ctx::Kept());
    for (int g = 0; g < c->G; g++) {
        const GraphState& s = c->gs[g];
        hgx_ctx::Kept& k = c->reset_kept[g];
        k.has_lcr = s.has_lcr;
        k.lcr = s.lcr;
        k.lcre = s.lcre;
        k.consensus_tx = s.consensus_tx;
        k.blocks = s.blocks;
        for (Block& b : k.blocks) b.first = -1;
    }
    std::fill(c->chain_len.begin(), c->chain_len.end(), 0);
    std::fill(c->chain_base.begin(), c->chain_base.end(), 0);
    std::fill(c->last_gid.begin(), c->last_gid.end(), -1);
    std::fill(c->last_index.begin(), c->last_index.end(), -1);
    for (int g = 0; g < c->G; g++) {
        GraphState& s = c->gs[g];
        s.undecided.clear();
        s.queued_upto = -1;
        s.queued.clear();
        s.pending_loaded = s.undetermined = 0;
        s.last_round = -1;
        s.fame.clear();
        s.round_events.clear();
        for (Block& b : s.blocks) b.first = -1;   // kept (blockCache); their events are gone
        c->order[g] = GraphOrder();
    }
    std::fill(c->g_events.begin(), c->g_events.end(), 0);
    std::fill(c->g_loaded.begin(), c->g_loaded.end(), 0);
    c->arena.used = 0;
    c->E = c->E_div = 0;
    c->divided = false;
    c->fo_prev_valid = false;
    c->mirror_ok = c->chains_ok = false;
    c->rounds_cached = c->recv_cached = false;
    return ok(err);
}

// forward declarations (per-event results, below)
static int32_t ensure_rounds(hgx_ctx* c);
static int32_t round_of(hgx_ctx* c, int64_t x);

// ---- GetFrame (hashgraph.go:897-995) ---------------------------------------------------
// Roots from LastConsensusRound's witnesses (and, for participants without one, from their
// last event), the frame's events in topological order and the Root.Others entries of frame
// events whose other-parent is not an earlier frame event. Encodings as in hgx.h.
int32_t hgx_get_frame(hgx_ctx* c, int64_t* events, int64_t events_cap, int64_t* n_events, int64_t* root_x,
                      int64_t* root_y, int32_t* root_index, int32_t* root_round, int64_t* others_event,
                      int64_t* others_parent, int64_t others_cap, int64_t* n_others, hgx_error* err) {
    if (!c || c->G != 1 || !n_events || !n_others || !root_x || !root_y || !root_index || !root_round) {
        set_err(err, HGX_ERR_INVALID, "hgx_get_frame: bad arguments (single-graph contexts)");
        return HGX_ERR_INVALID;
    }
    const GraphState& s = c->gs[0];
    const int32_t lcr = s.has_lcr ? s.lcr : 0;
    if (!c->divided || lcr < 0 || lcr > s.last_round || s.round_events[(size_t)lcr] == 0) {   // Store.GetRound
        set_err(err, HGX_ERR_KEY_NOT_FOUND, std::to_string(lcr) + ", Not Found");
        return HGX_ERR_KEY_NOT_FOUND;
    }
    DeviceGuard dg(c);
    if (ensure_rounds(c) || ensure_mirror(c) || ensure_chains(c)) return dev_err(err, hipErrorUnknown, "hgx_get_frame");
    const int n = c->n, C = c->C;
    std::vector<int64_t> evs;
    std::vector<uint8_t> has(n, 0);
    auto root_from = [&](int p, int64_t ev) {
        root_x[p] = c->sp[(size_t)ev];
        root_y[p] = c->op[(size_t)ev];
        root_index[p] = c->index32[(size_t)ev] - 1;
        root_round[p] = round_of(c, c->sp[(size_t)ev]);   // Round(Root.X outside the store) = -1
    };
    for (int p = 0; p < n; p++) {   // LastConsensusRound's witnesses
        if (c->rh.wflag[(size_t)lcr * C + p] != 2) continue;
        const int32_t k = c->rh.bm[(size_t)lcr * C + p];
        const int64_t w = c->chain_gids[(size_t)p][(size_t)k];
        has[p] = 1;
        root_from(p, w);
        for (size_t j = (size_t)k; j < c->chain_gids[(size_t)p].size(); j++) evs.push_back(c->chain_gids[(size_t)p][j]);
    }
    for (int p = 0; p < n; p++) {   // participants without a witness there: their last event
        if (has[p]) continue;
        if (c->chain_len[(size_t)p] == 0) {   // LastFrom is the Root: keep it
            root_x[p] = -1;
            root_y[p] = c->root_y_ext[(size_t)p] ? HGX_ROOT_Y : -1;
            root_index[p] = c->root_index[(size_t)p];
            root_round[p] = c->root_round[(size_t)p];
            continue;
        }
        const int64_t ev = c->chain_gids[(size_t)p].back();
        evs.push_back(ev);
        root_from(p, ev);
    }
    std::sort(evs.begin(), evs.end());   // ByTopologicalOrder
    std::vector<uint8_t> treated((size_t)c->E + 1, 0);
    int64_t no = 0;
    for (int64_t ev : evs) {
        treated[(size_t)ev] = 1;
        const int64_t op = c->op[(size_t)ev];
        if (op == -1) continue;
        if (!(op >= 0 && treated[(size_t)op]) && c->sp[(size_t)ev] != root_x[c->creator[(size_t)ev]]) {
            if (no < others_cap && others_event && others_parent) {
                others_event[no] = ev;
                others_parent[no] = op;
            }
            no++;
        }
    }
    *n_others = no;
    *n_events = (int64_t)evs.size();
    for (size_t k = 0; k < evs.size() && (int64_t)k < events_cap && events; k++) events[k] = evs[k];
    return ok(err);
}

// ---- DivideRounds (hashgraph.go:616-646) -----------------------------------------
static int32_t divide_rounds_one(hgx_ctx* c, hgx_error* err) {
    if (!c) { set_err(err, HGX_ERR_INVALID, "null context"); return HGX_ERR_INVALID; }
    if (c->divided && c->E_div == c->E) return ok(err);   // nothing new: AddEvent is idempotent
    DeviceGuard dg(c);
    const bool fo_valid = c->fo_prev_valid;
    c->fo_prev_valid = false;   // (until the call completes; a rebuild starts over)
    hipError_t e = c->eng.divide_rounds(c->E, c->chain_len, c->chain_base, c->rh);
    if (e != hipSuccess) return dev_err(err, e, "hgx_divide_rounds");
    const bool keep_fo = fo_valid && !c->eng.last_rebuild;
    c->divided = true;
    c->E_div = c->E;
    c->rounds_cached = false;
    const int C = c->C, n = c->n;
    for (int g = 0; g < c->G; g++) {
        GraphState& s = c->gs[g];
        const int32_t LR = c->rh.last_round[g];
        s.last_round = LR;
        s.fame.resize((size_t)(LR + 1) * n, 0);
        // rounds below r_lo kept their boundaries (incremental DivideRounds)
        s.round_events.resize(LR + 1, 0);
        for (int32_t r = std::min(c->rh.r_lo, LR + 1); r <= LR; r++) {
            int64_t cnt = 0;
            for (int cl = 0; cl < n; cl++) {
                const int gc = g * n + cl;
                cnt += c->rh.bm[(size_t)(r + 1) * C + gc] - c->rh.bm[(size_t)r * C + gc];
            }
            s.round_events[r] = (int32_t)cnt;
        }
        if (!c->rooted) {
            // rounds first seen in this call are queued in ascending order
            for (int32_t r = s.queued_upto + 1; r <= LR; r++) s.undecided.push_back(r);
            s.queued_upto = std::max(s.queued_upto, LR);
            continue;
        }
        // after a Reset rounds start at the roots' rounds and can first appear out of order:
        // queue the rounds with events not queued yet by their first event (DivideRounds
        // walks UndeterminedEvents in insertion order, hashgraph.go:617-638)
        s.queued.resize(LR + 1, 0);
        std::vector<int32_t> first;
        e = c->eng.round_first_gids(0, first);
        if (e != hipSuccess) return dev_err(err, e, "hgx_divide_rounds");
        std::vector<std::pair<int32_t, int32_t>> fresh;
        for (int32_t r = 0; r <= LR; r++)
            if (!s.queued[r] && s.round_events[r] > 0) fresh.push_back({first[(size_t)r], r});
        std::sort(fresh.begin(), fresh.end());
        for (auto& fr : fresh) {
            s.undecided.push_back(fr.second);
            s.queued[(size_t)fr.second] = 1;
        }
        s.queued_upto = std::max(s.queued_upto, LR);
    }
    c->fo_prev_valid = keep_fo;
    return ok(err);
}

// a chain-sharded context: the shards run DivideRounds together (their recurrence launches hand
// rows to each other)
int32_t hgx_divide_rounds(hgx_ctx* c, hgx_error* err) {
    if (c && c->grp) return on_shards(c, err, [](hgx_ctx* x, hgx_error* e) { return divide_rounds_one(x, e); });
    return divide_rounds_one(c, err);
}

static bool is_witness(const hgx_ctx* c, int32_t r, int gc) {
    return r >= 0 && r < c->rh.R && c->rh.wflag[(size_t)r * c->C + gc] == 2;
}

// RoundInfo.WitnessesDecided (roundInfo.go:64-71); rounds never stored are vacuously decided
static bool witnesses_decided(const hgx_ctx* c, int g, int32_t r) {
    const GraphState& s = c->gs[g];
    if (r < 0 || r > s.last_round) return true;
    for (int cl = 0; cl < c->n; cl++)
        if (is_witness(c, r, g * c->n + cl) && s.fame[(size_t)r * c->n + cl] == 0) return false;
    return true;
}

// ---- DecideFame (hashgraph.go:649-750) -------------------------------------------
static int32_t decide_fame_one(hgx_ctx* c, hgx_error* err) {
    if (!c) { set_err(err, HGX_ERR_INVALID, "null context"); return HGX_ERR_INVALID; }
    DeviceGuard dg(c);
    std::vector<int8_t>& dev = c->fame_dev;   // kept between calls (rows below the first undecided one unused)
    if (c->divided) {
        // decided fame is never revisited: only rounds from the first undecided one
        int32_t f0 = c->rh.R;
        for (int g = 0; g < c->G; g++)
            for (int32_t r : c->gs[g].undecided)
                if (r >= 0 && r <= c->gs[g].last_round) f0 = std::min(f0, r);
        hipError_t e = c->eng.decide_fame(f0, dev);
        if (e != hipSuccess) return dev_err(err, e, "hgx_decide_fame");
    }
    int32_t rc = HGX_OK;
    std::string msg;
    const int n = c->n, C = c->C;
    for (int g = 0; g < c->G; g++) {
        GraphState& s = c->gs[g];
        std::vector<int32_t> decided;
        for (size_t pos = 0; pos < s.undecided.size(); pos++) {
            const int32_t i = s.undecided[pos];
            if (i < 0 || i > s.last_round) {          // Store.GetRound miss -> error
                if (rc == HGX_OK) { rc = HGX_ERR_KEY_NOT_FOUND; msg = std::to_string(i) + ", Not Found"; }
                break;
            }
            for (int cl = 0; cl < n; cl++) {
                const int gc = g * n + cl;
                if (!is_witness(c, i, gc)) continue;
                int8_t& f = s.fame[(size_t)i * n + cl];
                if (f == 0) f = dev[(size_t)i * C + gc];   // SetFame; decided fame is never revisited
            }
            if (witnesses_decided(c, g, i)) {
                decided.push_back(i);
                if (!s.has_lcr || i > s.lcr) {             // setLastConsensusRound (:743-750)
                    s.has_lcr = true;
                    s.lcr = i;
                    s.lcre = (i - 1 >= 0 && i - 1 <= s.last_round) ? s.round_events[i - 1] : 0;
                }
            }
        }
        // deferred updateUndecidedRounds (:733-741): drop every copy of a decided round
        std::vector<uint8_t> is_dec((size_t)std::max(0, s.last_round) + 1, 0);
        for (int32_t r : decided) is_dec[(size_t)r] = 1;
        std::vector<int32_t> keep;
        keep.reserve(s.undecided.size());
        for (int32_t r : s.undecided)
            if (r < 0 || r > s.last_round || !is_dec[(size_t)r]) keep.push_back(r);
        s.undecided.swap(keep);
    }
    if (rc != HGX_OK) { set_err(err, rc, msg); return rc; }
    return ok(err);
}

int32_t hgx_decide_fame(hgx_ctx* c, hgx_error* err) {
    if (c && c->grp) return on_shards(c, err, [](hgx_ctx* x, hgx_error* e) { return decide_fame_one(x, e); });
    return decide_fame_one(c, err);
}

// ---- FindOrder (hashgraph.go:801-858) --------------------------------------------
// In two halves: begin = DecideRoundReceived and the consensus timestamps of this context's
// shard of chains (all chains unless hgx_set_shard); end = the ConsensusSorter order and the
// blocks. A row-sharded graph exchanges the shards' timestamps in between.
static int32_t find_order_begin_one(hgx_ctx* c, hgx_error* err) {
    if (!c) { set_err(err, HGX_ERR_INVALID, "null context"); return HGX_ERR_INVALID; }
    c->fo_open = false;
    if (!c->divided) return ok(err);
    DeviceGuard dg(c);
    const int n = c->n, C = c->C, G = c->G;
    const int32_t R = c->rh.R;
    // Nothing new can be received while every graph's UndecidedRounds[0] is what it was at the
    // last FindOrder: the eligible rounds (decided, below it) are the same or fewer, their famous
    // witnesses are the same events, and an event inserted since is an ancestor of none of them
    // (hashgraph.go:753-799). The call then costs no device work (most calls of the chunked
    // schedule). Not after a Reset (rounds queue out of order) or with an empty queue (the
    // reference's UndecidedRounds[0] panics there), nor when sharded.
    {
        bool same = c->fo_prev_valid && !c->rooted && c->shard_world <= 1 && (int)c->fo_prev_u0.size() == G;
        for (int g = 0; g < G && same; g++)
            same = !c->gs[g].undecided.empty() && c->gs[g].undecided[0] == c->fo_prev_u0[(size_t)g];
        if (same) return ok(err);
    }
    // rounds below r0 cannot be the roundReceived of an event not received yet
    int max_unrecv = 0;
    const int32_t r0 = c->eng.recv_round_lo(c->rh, max_unrecv);
    // the famous flags and eligible rounds: rows below r0 are neither read nor sent (the buffers
    // persist between calls and only rows [r0, R) are cleared: no O(R C) work per call)
    std::vector<uint8_t>& elig = c->fo_elig;
    std::vector<uint8_t>& fw = c->fo_fw;
    std::vector<uint8_t> ure(G, 0);
    elig.assign((size_t)G * std::max(R, 1), 0);
    if (fw.size() < (size_t)std::max(R, 1) * C) fw.resize((size_t)std::max(R, 1) * C, 0);
    if (R > std::max(r0, 0))
        std::memset(fw.data() + (size_t)std::max(r0, 0) * C, 0, (size_t)(R - std::max(r0, 0)) * C);
    for (int g = 0; g < G; g++) {
        const GraphState& s = c->gs[g];
        ure[g] = s.undecided.empty() ? 1 : 0;
        const int32_t U0 = s.undecided.empty() ? -1 : s.undecided[0];
        for (int32_t i = std::max(r0, 0); i <= s.last_round; i++) {
            // one pass over the round's chains: famous witnesses, and WitnessesDecided
            // (roundInfo.go:64-71) for the DecideRoundReceived skip rule (hashgraph.go:763)
            bool decided = true;
            const uint8_t* ws = c->rh.wflag.data() + (size_t)i * C + (size_t)g * n;
            const int8_t* fm = s.fame.data() + (size_t)i * n;
            uint8_t* fwr = fw.data() + (size_t)i * C + (size_t)g * n;
            for (int cl = 0; cl < n; cl++) {
                if (ws[cl] != 2) continue;
                if (fm[cl] == 0) decided = false;
                if (fm[cl] == 1) fwr[cl] = 1;
            }
            elig[(size_t)g * R + i] = (U0 >= 0 && i < U0 && decided) ? 1 : 0;
        }
    }
    hgx::OrderHost& oh = c->fo;
    hipError_t e = c->eng.find_order_begin(elig, fw, ure, r0, max_unrecv, oh);
    if (e != hipSuccess) return dev_err(err, e, "hgx_find_order");
    if (oh.panic) {
        c->fo_prev_valid = false;
        set_err(err, HGX_ERR_PANIC, "runtime error: index out of range [0] with length 0");
        return HGX_ERR_PANIC;
    }
    // the skip rule's UndecidedRounds[0] of this FindOrder: pending until _end commits the
    // order (an _end that fails leaves the skip rule off, so the next FindOrder redoes the work)
    c->fo_prev_valid = false;
    c->fo_pend_u0.assign(G, -1);
    c->fo_pend_valid = true;
    for (int g = 0; g < G; g++) {
        if (c->gs[g].undecided.empty()) c->fo_pend_valid = false;
        else c->fo_pend_u0[(size_t)g] = c->gs[g].undecided[0];
    }
    c->fo_open = true;
    return ok(err);
}

static int32_t find_order_end_one(hgx_ctx* c, hgx_error* err) {
    if (!c) { set_err(err, HGX_ERR_INVALID, "null context"); return HGX_ERR_INVALID; }
    if (!c->fo_open) return ok(err);
    c->fo_open = false;
    DeviceGuard dg(c);
    const int n = c->n, G = c->G;
    (void)n;
    const int32_t R = c->rh.R;
    hgx::OrderHost& oh = c->fo;
    // the m received events' order lands in the arena with the block tables (one round trip)
    const size_t base_off = c->arena.used;
    int32_t* pre = nullptr;
    if (oh.m > 0) {
        if (!c->arena.reserve(base_off + (size_t)oh.m)) {
            set_err(err, HGX_ERR_CAPACITY, "hgx_find_order: out of pinned host memory");
            return HGX_ERR_CAPACITY;
        }
        pre = c->arena.p + base_off;
    }
    hipError_t e = c->eng.find_order_end(oh, pre);
    if (e != hipSuccess) return dev_err(err, e, "hgx_find_order");
    c->recv_cached = false;
    // the device order is graph-major: one D2H copy appends it to the arena and every
    // graph gets its segment
    std::vector<int64_t> seg_at(G, 0), seg_len(G, 0);
    int64_t total = 0;
    for (int g = 0; g < G; g++) {
        int64_t mg = 0;
        for (int32_t rr = 0; rr < R; rr++) mg += oh.blk_cnt[(size_t)g * R + rr];
        seg_at[g] = total;
        seg_len[g] = mg;
        total += mg;
    }
    if (pre && total != (int64_t)oh.m) {   // every received event is in exactly one block
        set_err(err, HGX_ERR_INVALID, "hgx_find_order: block counts differ from the received events");
        return HGX_ERR_INVALID;
    }
    if (total > 0 && !pre) {
        if (!c->arena.reserve(base_off + (size_t)total)) {
            set_err(err, HGX_ERR_CAPACITY, "hgx_find_order: out of pinned host memory");
            return HGX_ERR_CAPACITY;
        }
        e = c->eng.copy_order(c->arena.p + base_off, 0, total);
        if (e != hipSuccess) return dev_err(err, e, "hgx_find_order");
        e = c->eng.sync();
        if (e != hipSuccess) return dev_err(err, e, "hgx_find_order");
    }
    c->arena.used = base_off + (size_t)total;
    // committed blocks (graph, block index): commitCh receives them once the graph state
    // (counters, pending, undetermined) is final for this call
    std::vector<std::pair<int, int64_t>> commits;
    for (int g = 0; g < G; g++) {
        const int64_t mg = seg_len[g];
        if (mg == 0) continue;
        GraphState& s = c->gs[g];
        GraphOrder& o = c->order[g];
        const int64_t base_pos = (int64_t)o.n;
        o.segs.push_back({base_off + (size_t)seg_at[g], (size_t)mg});
        o.n += (size_t)mg;
        s.blocks.reserve(s.blocks.size() + (size_t)R);
        int64_t off = 0;
        for (int32_t rr = 0; rr < R; rr++) {    // one Block per rr, ascending (blockOrder)
            const size_t bi = (size_t)g * R + rr;
            const int32_t cnt = oh.blk_cnt[bi];
            if (!cnt) continue;
            Block b;
            b.rr = rr;
            b.first = base_pos + off;
            b.nev = cnt;
            b.ntx = oh.blk_ntx[bi];
            // NewBlock(rr, first.Transactions()) then append(...): nil iff first nil and nothing appended
            b.tx_nil = (oh.blk_nil[bi] && b.ntx == 0) ? 1 : 0;
            b.committed = b.ntx > 0 ? 1 : 0;   // commitCh only if len(Transactions) > 0
            s.blocks.push_back(b);
            if (b.committed && c->commit_fn) commits.push_back({g, (int64_t)s.blocks.size() - 1});
            s.consensus_tx += b.ntx;
            s.pending_loaded -= oh.blk_loaded[bi];
            off += cnt;
        }
        s.undetermined -= mg;
    }
    c->fo_prev_u0.swap(c->fo_pend_u0);   // the order is committed: the skip rule may use it
    c->fo_prev_valid = c->fo_pend_valid;
    c->fo_pend_valid = false;
    for (const auto& gb : commits) {   // commitCh <- block, in SetBlock order
        const Block& b = c->gs[gb.first].blocks[(size_t)gb.second];
        c->commit_fn(c->commit_user, gb.first, gb.second, b.rr, b.first, b.nev, b.ntx);
    }
    return ok(err);
}

int32_t hgx_find_order_begin(hgx_ctx* c, hgx_error* err) {
    const int32_t rc = group_only_one(c, err, "hgx_find_order_begin");
    return rc ? rc : find_order_begin_one(c, err);
}

int32_t hgx_find_order_end(hgx_ctx* c, hgx_error* err) {
    const int32_t rc = group_only_one(c, err, "hgx_find_order_end");
    return rc ? rc : find_order_end_one(c, err);
}

static int32_t shard_xfer(hgx_ctx* c, int32_t rank, void* buf, int32_t on_device, bool to_buf);

static int32_t grow_dev(hgx_ctx* c, void** p, size_t* cap, size_t bytes) {
    if (bytes <= *cap) return HGX_OK;
    if (*p) (void)hipFree(*p);
    *p = nullptr;
    *cap = 0;
    if (hipMalloc(p, std::max<size_t>(bytes, 1 << 16)) != hipSuccess) return HGX_ERR_DEVICE;
    *cap = std::max<size_t>(bytes, 1 << 16);
    (void)c;
    return HGX_OK;
}

// FindOrder of a chain-sharded context: every shard's begin (round received for every event, the
// consensus timestamps of its own chains' events: its firstDescendants are valid there only), the
// timestamps exchanged (each shard's values copied device to device into every other shard and
// imported there), every shard's end (sort, blocks)
static int32_t group_find_order(hgx_ctx* c, hgx_error* err) {
    int32_t rc = on_shards(c, err, [](hgx_ctx* x, hgx_error* e) { return find_order_begin_one(x, e); });
    if (rc) return rc;
    std::vector<hgx_ctx*> sh{c};
    sh.insert(sh.end(), c->peers.begin(), c->peers.end());
    const int W = (int)sh.size();
    if (c->fo_open) {
        std::vector<int64_t> cnt(W);
        for (int k = 0; k < W; k++) {   // shard k's values into its own device buffer
            hgx_ctx* x = sh[k];
            DeviceGuard dg(x);
            cnt[k] = hgx_shard_values(x, k);
            if (cnt[k] == 0) continue;
            if (grow_dev(x, &x->gx_out, &x->gx_out_cap, (size_t)cnt[k] * 8) ||
                shard_xfer(x, k, x->gx_out, 1, true)) {
                set_err(err, HGX_ERR_DEVICE, "hgx_find_order: shard timestamp export failed");
                return HGX_ERR_DEVICE;
            }
        }
        for (int j = 0; j < W; j++) {   // ... copied to every other shard and imported there
            hgx_ctx* x = sh[j];
            DeviceGuard dg(x);
            for (int k = 0; k < W; k++) {
                if (k == j || cnt[k] == 0) continue;
                // (on the importing engine's stream: a device-to-device copy on the null stream returns
                // before it completes, and the engine's non-blocking stream does not wait for it)
                if (grow_dev(x, &x->gx_in, &x->gx_in_cap, (size_t)cnt[k] * 8) ||
                    hipMemcpyPeerAsync(x->gx_in, x->eng.dev, sh[k]->gx_out, sh[k]->eng.dev, (size_t)cnt[k] * 8,
                                       x->eng.stream) != hipSuccess ||
                    shard_xfer(x, k, x->gx_in, 1, false)) {
                    set_err(err, HGX_ERR_DEVICE, "hgx_find_order: shard timestamp import failed");
                    return HGX_ERR_DEVICE;
                }
            }
        }
    }
    return on_shards(c, err, [](hgx_ctx* x, hgx_error* e) { return find_order_end_one(x, e); });
}

int32_t hgx_find_order(hgx_ctx* c, hgx_error* err) {
    if (c && c->grp) return group_find_order(c, err);
    if (c && c->shard_world > 1) {
        set_err(err, HGX_ERR_INVALID, "hgx_find_order: a sharded context exchanges timestamps between "
                                      "hgx_find_order_begin and hgx_find_order_end");
        return HGX_ERR_INVALID;
    }
    const int32_t rc = find_order_begin_one(c, err);
    if (rc) return rc;
    return find_order_end_one(c, err);
}

// ---- row-sharded graph --------------------------------------------------
static void shard_range(const hgx_ctx* c, int32_t rank, int* lo, int* hi) {
    // (a chain-sharded group's shards use the group's split: every split-dependent piece -- the
    // firstDescendants target range, the recurrence's workgroups, the timestamp tiles and this
    // exchange -- must agree on it)
    if (c->eng.grp && c->eng.grp->W == c->shard_world) {
        *lo = c->eng.grp->c_split[rank];
        *hi = c->eng.grp->c_split[rank + 1];
        return;
    }
    *lo = (int)((int64_t)c->C * rank / c->shard_world);
    *hi = (int)((int64_t)c->C * (rank + 1) / c->shard_world);
}

int32_t hgx_set_shard(hgx_ctx* c, int32_t rank, int32_t world) {
    if (!c || c->grp || world < 1 || rank < 0 || rank >= world || world > c->C) return HGX_ERR_INVALID;
    c->shard_rank = rank;
    c->shard_world = world;
    shard_range(c, rank, &c->eng.shard_lo, &c->eng.shard_hi);
    return HGX_OK;
}

int64_t hgx_shard_values(hgx_ctx* c, int32_t rank) {
    if (!c || rank < 0 || rank >= c->shard_world || !c->fo_open) return 0;
    int lo, hi;
    shard_range(c, rank, &lo, &hi);
    return c->eng.shard_values(lo, hi);
}

static int32_t shard_xfer(hgx_ctx* c, int32_t rank, void* buf, int32_t on_device, bool to_buf) {
    if (!c || rank < 0 || rank >= c->shard_world || (!buf && hgx_shard_values(c, rank) > 0)) return HGX_ERR_INVALID;
    if (!c->fo_open) return HGX_OK;
    DeviceGuard dg(c);
    int lo, hi;
    shard_range(c, rank, &lo, &hi);
    return c->eng.shard_copy(lo, hi, buf, on_device != 0, to_buf) == hipSuccess ? HGX_OK : HGX_ERR_DEVICE;
}

int32_t hgx_shard_export(hgx_ctx* c, void* dst, int32_t dst_on_device) {
    return c ? shard_xfer(c, c->shard_rank, dst, dst_on_device, true) : HGX_ERR_INVALID;
}

int32_t hgx_shard_import(hgx_ctx* c, int32_t src_rank, const void* src, int32_t src_on_device) {
    if (c && src_rank == c->shard_rank) return HGX_OK;
    return shard_xfer(c, src_rank, const_cast<void*>(src), src_on_device, false);
}

int32_t hgx_run_consensus(hgx_ctx* c, hgx_error* err) {
    int32_t rc = hgx_divide_rounds(c, err);
    if (rc) return rc;
    rc = hgx_decide_fame(c, err);
    if (rc) return rc;
    return hgx_find_order(c, err);
}

static int32_t reset_consensus_one(hgx_ctx* c) {
    if (!c) return HGX_ERR_INVALID;
    DeviceGuard dg(c);
    for (int g = 0; g < c->G; g++) {
        GraphState& s = c->gs[g];
        s.reset();
        s.undetermined = c->g_events[g];
        s.pending_loaded = c->g_loaded[g];
        c->order[g] = GraphOrder();
    }
    c->arena.used = 0;
    c->divided = false;
    c->fo_prev_valid = false;
    c->E_div = 0;
    c->rounds_cached = c->recv_cached = false;
    return c->eng.reset_received() == hipSuccess ? HGX_OK : HGX_ERR_DEVICE;
}

int32_t hgx_reset_consensus(hgx_ctx* c) {
    if (c && c->grp) return on_shards(c, nullptr, [](hgx_ctx* x, hgx_error*) { return reset_consensus_one(x); });
    return reset_consensus_one(c);
}

// ---- state getters ----------------------------------------------------------------
static GraphState* graph(hgx_ctx* c, int32_t g) {
    if (!c || g < 0 || g >= c->G) return nullptr;
    return &c->gs[g];
}

int64_t hgx_num_events(hgx_ctx* c) { return c ? c->E : 0; }
int32_t hgx_super_majority(hgx_ctx* c) { return c ? c->sm : 0; }
int64_t hgx_num_undetermined(hgx_ctx* c, int32_t g) { GraphState* s = graph(c, g); return s ? s->undetermined : 0; }
int32_t hgx_undecided_rounds(hgx_ctx* c, int32_t g, int32_t* out, int32_t cap) {
    GraphState* s = graph(c, g);
    if (!s) return 0;
    const int32_t m = (int32_t)s->undecided.size();
    for (int32_t i = 0; i < m && i < cap; i++) out[i] = s->undecided[i];
    return m;
}
int32_t hgx_last_consensus_round(hgx_ctx* c, int32_t g, int32_t* has) {
    GraphState* s = graph(c, g);
    if (has) *has = (s && s->has_lcr) ? 1 : 0;
    return (s && s->has_lcr) ? s->lcr : 0;
}
int32_t hgx_last_commited_round_events(hgx_ctx* c, int32_t g) { GraphState* s = graph(c, g); return s ? s->lcre : 0; }
int64_t hgx_consensus_transactions(hgx_ctx* c, int32_t g) { GraphState* s = graph(c, g); return s ? s->consensus_tx : 0; }
int64_t hgx_pending_loaded_events(hgx_ctx* c, int32_t g) { GraphState* s = graph(c, g); return s ? s->pending_loaded : 0; }
int32_t hgx_last_round(hgx_ctx* c, int32_t g) { GraphState* s = graph(c, g); return s ? s->last_round : -1; }
int32_t hgx_round_event_count(hgx_ctx* c, int32_t g, int32_t r) {
    GraphState* s = graph(c, g);
    if (!s || r < 0 || r > s->last_round) return 0;
    return s->round_events[r];
}
int32_t hgx_round_witnesses(hgx_ctx* c, int32_t g, int32_t r, int64_t* out, int32_t cap) {
    GraphState* s = graph(c, g);
    if (!s || r < 0 || r > s->last_round) return 0;
    DeviceGuard dg(c);
    if (ensure_chains(c)) return 0;
    int32_t m = 0;
    for (int cl = 0; cl < c->n; cl++) {
        const int gc = g * c->n + cl;
        if (!is_witness(c, r, gc)) continue;
        if (m < cap) out[m] = c->chain_gids[gc][c->rh.bm[(size_t)r * c->C + gc]];
        m++;
    }
    return m;
}
int32_t hgx_known(hgx_ctx* c, int32_t g, int32_t* out) {
    if (!graph(c, g)) return HGX_ERR_INVALID;
    for (int cl = 0; cl < c->n; cl++) out[cl] = (int32_t)c->last_index[g * c->n + cl];
    return HGX_OK;
}
int64_t hgx_consensus_events_count(hgx_ctx* c, int32_t g) { return graph(c, g) ? (int64_t)c->order[g].size() : 0; }

int32_t hgx_consensus_events(hgx_ctx* c, int32_t g, int64_t first, int64_t count, int64_t* gids) {
    if (!graph(c, g) || first < 0 || count < 0 || first + count > (int64_t)c->order[g].size()) return HGX_ERR_INVALID;
    walk_order(c, g, first, count, [&](int64_t k, int64_t gid) { gids[k] = gid; });
    return HGX_OK;
}

static int32_t ensure_received(hgx_ctx* c) {
    if (c->recv_cached) return HGX_OK;
    if (c->eng.get_received(c->rr_cache, c->cts_cache) != hipSuccess) return HGX_ERR_DEVICE;
    c->recv_cached = true;
    return HGX_OK;
}

int32_t hgx_consensus_received(hgx_ctx* c, int32_t g, int64_t first, int64_t count, int64_t* gids, int32_t* rr,
                               int64_t* cts) {
    if (!graph(c, g) || first < 0 || count < 0 || first + count > (int64_t)c->order[g].size()) return HGX_ERR_INVALID;
    DeviceGuard dg(c);
    if (ensure_received(c)) return HGX_ERR_DEVICE;
    walk_order(c, g, first, count, [&](int64_t k, int64_t gid) {
        if (gids) gids[k] = gid;
        if (rr) rr[k] = c->rr_cache[(size_t)gid];
        if (cts) cts[k] = c->cts_cache[(size_t)gid];
    });
    return HGX_OK;
}

int64_t hgx_num_blocks(hgx_ctx* c, int32_t g) { GraphState* s = graph(c, g); return s ? (int64_t)s->blocks.size() : 0; }
int32_t hgx_block_info(hgx_ctx* c, int32_t g, int64_t b, int32_t* rr, int64_t* first, int32_t* nev, int64_t* ntx,
                       int32_t* tx_nil, int32_t* committed) {
    GraphState* s = graph(c, g);
    if (!s || b < 0 || b >= (int64_t)s->blocks.size()) return HGX_ERR_INVALID;
    const Block& B = s->blocks[(size_t)b];
    if (rr) *rr = B.rr;
    if (first) *first = B.first;
    if (nev) *nev = B.nev;
    if (ntx) *ntx = B.ntx;
    if (tx_nil) *tx_nil = B.tx_nil;
    if (committed) *committed = B.committed;
    return HGX_OK;
}

// Store.GetBlock(rr) (inmem_store.go:163-169)
int32_t hgx_get_block(hgx_ctx* c, int32_t g, int32_t round_received, int64_t* block, hgx_error* err) {
    GraphState* s = graph(c, g);
    if (!s) { set_err(err, HGX_ERR_INVALID, "hgx_get_block: bad graph"); return HGX_ERR_INVALID; }
    for (size_t b = 0; b < s->blocks.size(); b++)
        if (s->blocks[b].rr == round_received) {
            if (block) *block = (int64_t)b;
            return ok(err);
        }
    set_err(err, HGX_ERR_KEY_NOT_FOUND, std::to_string(round_received) + ", Not Found");
    return HGX_ERR_KEY_NOT_FOUND;
}

// ---- Store: events by participant (inmem_store.go:48-102, caches.go:30-114) -----------
// No eviction (cacheSize >= events): a participant's RollingIndex holds all its
// events, oldest cached Index = its first Index.
static bool valid_participant(const hgx_ctx* c, int32_t p) { return c && p >= 0 && p < c->C; }

int32_t hgx_last_from(hgx_ctx* c, int32_t p, int64_t* gid, int32_t* is_root, hgx_error* err) {
    if (!valid_participant(c, p)) {
        set_err(err, HGX_ERR_KEY_NOT_FOUND, std::to_string(p) + ", Not Found");
        return HGX_ERR_KEY_NOT_FOUND;
    }
    const bool none = c->last_gid[p] < 0;   // no event: the Root's X (genesis: "")
    if (gid) *gid = none ? -1 : c->last_gid[p];
    if (is_root) *is_root = none ? 1 : 0;
    return ok(err);
}

int32_t hgx_participant_events(hgx_ctx* c, int32_t p, int64_t skip, int64_t* gids, int64_t cap, int64_t* count,
                               hgx_error* err) {
    if (count) *count = 0;
    if (!valid_participant(c, p)) {
        set_err(err, HGX_ERR_KEY_NOT_FOUND, std::to_string(p) + ", Not Found");
        return HGX_ERR_KEY_NOT_FOUND;
    }
    const int64_t last = c->last_index[p];
    if (skip > last) return ok(err);   // RollingIndex.Get (common/rolling_index.go:21-38)
    const int64_t items = c->chain_len[p];
    const int64_t oldest = last - items + 1;
    if (skip + 1 < oldest) {
        set_err(err, HGX_ERR_TOO_LATE, go_rune(4 - 1) + ", Too Late");   // NewStoreErr(TooLate, string(SkippedIndex))
        return HGX_ERR_TOO_LATE;
    }
    DeviceGuard dg(c);
    if (ensure_chains(c)) return dev_err(err, hipErrorUnknown, "hgx_participant_events");
    const int64_t start = skip - oldest + 1, m = items - start;
    if (count) *count = m;
    for (int64_t k = 0; k < m && k < cap; k++) gids[k] = c->chain_gids[p][(size_t)(start + k)];
    return ok(err);
}

int32_t hgx_participant_event(hgx_ctx* c, int32_t p, int64_t index, int64_t* gid, hgx_error* err) {
    if (!valid_participant(c, p)) {   // participantEvents[participant] is nil: Go panics
        set_err(err, HGX_ERR_PANIC, "runtime error: invalid memory address or nil pointer dereference");
        return HGX_ERR_PANIC;
    }
    const int64_t last = c->last_index[p], items = c->chain_len[p];
    const int64_t oldest = last - items + 1;   // RollingIndex.GetItem (common/rolling_index.go:40-50)
    if (index < oldest) {
        set_err(err, HGX_ERR_TOO_LATE, go_rune(index) + ", Too Late");
        return HGX_ERR_TOO_LATE;
    }
    if (index - oldest >= items) {
        set_err(err, HGX_ERR_KEY_NOT_FOUND, go_rune(index) + ", Not Found");
        return HGX_ERR_KEY_NOT_FOUND;
    }
    DeviceGuard dg(c);
    if (ensure_chains(c)) return dev_err(err, hipErrorUnknown, "hgx_participant_event");
    if (gid) *gid = c->chain_gids[p][(size_t)(index - oldest)];
    return ok(err);
}

// Store.GetRoot (inmem_store.go:163-169): X = -1 (Root.X: "" for a genesis Root, else the
// event named when hgx_reset installed it), Y = -1 ("") or HGX_ROOT_Y, Index, Round
int32_t hgx_get_root(hgx_ctx* c, int32_t p, int64_t* x, int64_t* y, int32_t* index, int32_t* round, hgx_error* err) {
    if (!valid_participant(c, p)) {
        set_err(err, HGX_ERR_KEY_NOT_FOUND, std::to_string(p) + ", Not Found");
        return HGX_ERR_KEY_NOT_FOUND;
    }
    if (x) *x = -1;
    if (y) *y = c->root_y_ext[(size_t)p] ? HGX_ROOT_Y : -1;
    if (index) *index = c->root_index[(size_t)p];
    if (round) *round = c->root_round[(size_t)p];
    return ok(err);
}

// Store.GetEvent (inmem_store.go:48-55): the DAG fields of one event
int32_t hgx_get_event(hgx_ctx* c, int64_t gid, int32_t* creator, int64_t* index, int64_t* self_parent,
                      int64_t* other_parent, int64_t* timestamp_ns, int32_t* ntx, int32_t* tx_nil, hgx_error* err) {
    if (!c || gid < 0 || gid >= c->E) {
        set_err(err, HGX_ERR_KEY_NOT_FOUND, std::to_string(gid) + ", Not Found");
        return HGX_ERR_KEY_NOT_FOUND;
    }
    DeviceGuard dg(c);
    if (ensure_mirror(c)) return dev_err(err, hipErrorUnknown, "hgx_get_event");
    int64_t ts = 0;
    int32_t nt = 0, nil = 0;
    hipError_t e = c->eng.get_event_fields(gid, &ts, &nt, &nil);
    if (e != hipSuccess) return dev_err(err, e, "hgx_get_event");
    const size_t x = (size_t)gid;
    if (creator) *creator = c->creator[x];
    if (index) *index = c->index32[x];
    if (self_parent) *self_parent = c->sp[x];
    if (other_parent) *other_parent = c->op[x];
    if (timestamp_ns) *timestamp_ns = ts;
    if (ntx) *ntx = nt;
    if (tx_nil) *tx_nil = nil;
    return ok(err);
}

// SetWireInfo (hashgraph.go:532-567): self-parent Index (Root.Index = -1 for a first event),
// other-parent creator id and Index (-1 when ""), per event
int32_t hgx_wire_info(hgx_ctx* c, int64_t first, int64_t count, int32_t* self_parent_index,
                      int32_t* other_parent_creator, int32_t* other_parent_index) {
    if (!c || first < 0 || count < 0 || first + count > c->E) return HGX_ERR_INVALID;
    DeviceGuard dg(c);
    if (ensure_mirror(c)) return HGX_ERR_DEVICE;
    for (int64_t k = 0; k < count; k++) {
        const size_t x = (size_t)(first + k);
        const int32_t sp = c->sp[x], op = c->op[x];
        // a first event's self-parent is the Root: Root.Index (hashgraph.go:537-545)
        if (self_parent_index) self_parent_index[k] = sp >= 0 ? c->index32[(size_t)sp] : c->root_index[(size_t)c->creator[x]];
        if (other_parent_creator) other_parent_creator[k] = op >= 0 ? c->creator[(size_t)op] : -1;
        if (other_parent_index) other_parent_index[k] = op >= 0 ? c->index32[(size_t)op] : -1;
    }
    return HGX_OK;
}

// ReadWireInfo (hashgraph.go:569-614): the parents of a wire event resolved through
// Store.ParticipantEvent
int32_t hgx_read_wire_info(hgx_ctx* c, int32_t creator, int64_t self_parent_index, int32_t other_parent_creator,
                           int64_t other_parent_index, int64_t* self_parent, int64_t* other_parent, hgx_error* err) {
    if (self_parent) *self_parent = -1;
    if (other_parent) *other_parent = -1;
    if (self_parent_index >= 0) {
        const int32_t rc = hgx_participant_event(c, creator, self_parent_index, self_parent, err);
        if (rc) return rc;
    }
    if (other_parent_index >= 0) {
        const int32_t rc = hgx_participant_event(c, other_parent_creator, other_parent_index, other_parent, err);
        if (rc) return rc;
    }
    return ok(err);
}

// ---- per-event results -------------------------------------------------------------
static int32_t ensure_rounds(hgx_ctx* c) {
    if (c->rounds_cached) return HGX_OK;
    if (c->eng.get_rounds(c->round_cache) != hipSuccess) return HGX_ERR_DEVICE;
    c->rounds_cached = true;
    return HGX_OK;
}
static int32_t round_of(hgx_ctx* c, int64_t x) {
    if (x < 0 || x >= (int64_t)c->round_cache.size()) return -1;   // Round("") = -1
    return c->round_cache[(size_t)x];
}
static int32_t witness_of(hgx_ctx* c, int64_t x) {   // Witness (hashgraph.go:265-282)
    if (x < 0 || x >= (int64_t)c->round_cache.size()) return 0;
    // the creator's first event on its Root: SelfParent == Root.X && OtherParent == Root.Y
    const int32_t sp = c->sp[(size_t)x], op = c->op[(size_t)x];
    const bool yext = c->root_y_ext[(size_t)c->creator[(size_t)x]] != 0;
    if (sp == -1 && ((op == -1 && !yext) || op == HGX_ROOT_Y)) return 1;
    return round_of(c, x) > round_of(c, sp) ? 1 : 0;   // Round(Root.X) = -1
}

int32_t hgx_get_rounds(hgx_ctx* c, int64_t first, int64_t count, int32_t* round, int8_t* witness, int8_t* famous) {
    if (!c || first < 0 || count < 0 || first + count > c->E) return HGX_ERR_INVALID;
    DeviceGuard dg(c);
    if (ensure_rounds(c) || ensure_mirror(c)) return HGX_ERR_DEVICE;
    for (int64_t k = 0; k < count; k++) {
        const int64_t x = first + k;
        const int32_t r = round_of(c, x);
        const int32_t w = witness_of(c, x);
        if (round) round[k] = r;
        if (witness) witness[k] = (int8_t)w;
        if (famous) {
            int8_t f = 0;
            if (w && r >= 0) {
                const int gc = c->creator[(size_t)x];
                const GraphState& s = c->gs[gc / c->n];
                if (r <= s.last_round) f = s.fame[(size_t)r * c->n + gc % c->n];
            }
            famous[k] = f;
        }
    }
    return HGX_OK;
}

int32_t hgx_get_received(hgx_ctx* c, int64_t first, int64_t count, int32_t* rr, int64_t* cts) {
    if (!c || first < 0 || count < 0 || first + count > c->E) return HGX_ERR_INVALID;
    DeviceGuard dg(c);
    if (ensure_received(c)) return HGX_ERR_DEVICE;
    for (int64_t k = 0; k < count; k++) {
        const size_t x = (size_t)(first + k);
        const bool have = x < c->rr_cache.size();
        if (rr) rr[k] = have ? c->rr_cache[x] : -1;
        if (cts) cts[k] = (have && c->rr_cache[x] >= 0) ? c->cts_cache[x] : 0;
    }
    return HGX_OK;
}

int32_t hgx_get_coords(hgx_ctx* c, int64_t gid, int32_t* la, int32_t* fd) {
    if (!c || gid < 0 || gid >= c->E_div || !c->divided) return HGX_ERR_INVALID;
    DeviceGuard dg(c);
    return c->eng.get_coords(gid, la, fd) == hipSuccess ? HGX_OK : HGX_ERR_DEVICE;
}

// ---- primitives (hashgraph.go:73-339) ----------------------------------------------
// Events of different graphs of a batched context never see each other.
static bool known_div(hgx_ctx* c, int64_t x) { return c && x >= 0 && x < c->E_div && c->divided; }
static bool same_graph(hgx_ctx* c, int64_t x, int64_t y) { return graph_of(c, x) == graph_of(c, y); }

int32_t hgx_ancestor(hgx_ctx* c, int64_t x, int64_t y) {
    if (x == y) return 1;
    if (!known_div(c, x) || !known_div(c, y)) return 0;
    DeviceGuard dg(c);
    if (ensure_mirror(c) || !same_graph(c, x, y)) return 0;
    std::vector<int32_t> la(c->n), fd(c->n);
    if (c->eng.get_coords(x, la.data(), fd.data()) != hipSuccess) return 0;
    return la[c->creator[(size_t)y] % c->n] >= c->index32[(size_t)y] ? 1 : 0;
}
int32_t hgx_self_ancestor(hgx_ctx* c, int64_t x, int64_t y) {
    if (x == y) return 1;
    if (!c || x < 0 || y < 0 || x >= c->E || y >= c->E) return 0;
    DeviceGuard dg(c);
    if (ensure_mirror(c)) return 0;
    return (c->creator[(size_t)x] == c->creator[(size_t)y] && c->index32[(size_t)x] >= c->index32[(size_t)y]) ? 1 : 0;
}
int32_t hgx_see(hgx_ctx* c, int64_t x, int64_t y) { return hgx_ancestor(c, x, y); }
int32_t hgx_strongly_see(hgx_ctx* c, int64_t x, int64_t y) {
    if (!known_div(c, x) || !known_div(c, y)) return 0;
    DeviceGuard dg(c);
    if (ensure_mirror(c) || !same_graph(c, x, y)) return 0;
    std::vector<int32_t> lx(c->n), fx(c->n), ly(c->n), fy(c->n);
    if (c->eng.get_coords(x, lx.data(), fx.data()) != hipSuccess) return 0;
    if (c->eng.get_coords(y, ly.data(), fy.data()) != hipSuccess) return 0;
    int cnt = 0;
    for (int i = 0; i < c->n; i++) cnt += lx[i] >= fy[i];
    return cnt >= c->sm ? 1 : 0;
}
int64_t hgx_oldest_self_ancestor_to_see(hgx_ctx* c, int64_t x, int64_t y) {
    if (!known_div(c, x) || !known_div(c, y)) return -1;
    DeviceGuard dg(c);
    if (ensure_chains(c) || !same_graph(c, x, y)) return -1;
    std::vector<int32_t> la(c->n), fd(c->n);
    if (c->eng.get_coords(y, la.data(), fd.data()) != hipSuccess) return -1;
    const int cx = c->creator[(size_t)x];
    const int32_t a = fd[cx % c->n];
    if (a <= c->index32[(size_t)x]) return c->chain_gids[cx][(size_t)(a - c->chain_base[cx])];
    return -1;
}
int32_t hgx_round(hgx_ctx* c, int64_t x) {
    if (!c) return -1;
    DeviceGuard dg(c);
    if (ensure_rounds(c)) return -1;
    return round_of(c, x);
}
int32_t hgx_witness(hgx_ctx* c, int64_t x) {
    if (!c) return 0;
    DeviceGuard dg(c);
    if (ensure_rounds(c) || ensure_mirror(c)) return 0;
    return witness_of(c, x);
}

// ---- instrumentation / knobs ----------------------------------------------------------
int32_t hgx_phase_times(hgx_ctx* c, double* out, int32_t cap) {
    if (!c || !out) return 0;
    const int32_t m = std::min<int32_t>(cap, 22);
    double v[22] = {c->eng.phase_ms[0], c->eng.phase_ms[1], c->eng.phase_ms[2], c->eng.phase_ms[3],
                    (double)c->eng.la_sweeps, (double)c->eng.R, (double)c->eng.compact,
                    (double)c->eng.la_rows, c->eng.last_rebuild ? 1.0 : 0.0, (double)c->rh.r_lo,
                    c->eng.la_wave_used ? 1.0 : 0.0, (double)c->eng.la_wave_fallbacks,
                    (double)(c->eng.la_wave_used ? c->eng.la_wave_segs : 0), (double)c->eng.round_p_runs,
                    (double)c->eng.round_p_fallbacks, (double)c->eng.round_p_ovf,
                    (double)c->eng.round_p_fail_round, (double)c->eng.round_p_fail_chain,
                    (double)c->eng.round_g_runs, c->eng.la_small_used ? 1.0 : 0.0,
                    c->eng.la_verified ? 1.0 : 0.0, (double)c->eng.sort_seg_runs};
    for (int32_t i = 0; i < m; i++) out[i] = v[i];
    return m;
}

static const char* kKernelNames[hgx::K_NUM] = {"layout", "la_sweep", "fd_build", "round_gather", "round_search",
                                              "fame", "threshold", "round_received", "cts_median", "order_sort"};

int32_t hgx_kernel_stats(hgx_ctx* c, int32_t k, char* name, int32_t name_cap, double* ms, int64_t* launches,
                         double* bytes) {
    if (!c || k < 0 || k >= hgx::K_NUM) return HGX_ERR_INVALID;
    if (name && name_cap > 0) std::snprintf(name, (size_t)name_cap, "%s", kKernelNames[k]);
    const hgx::KernelStat& ks = c->eng.kstat[k];
    // summed device time of all launches, extrapolated from the timed sample
    if (ms) *ms = (ks.timed > 0 && ks.timed < ks.launches) ? ks.ms * (double)ks.launches / (double)ks.timed : ks.ms;
    if (launches) *launches = c->eng.kstat[k].launches;
    if (bytes) *bytes = c->eng.kstat[k].bytes;
    return HGX_OK;
}

int32_t hgx_reset_stats(hgx_ctx* c) {
    if (!c) return HGX_ERR_INVALID;
    for (auto& s : c->eng.kstat) s = hgx::KernelStat();
    return HGX_OK;
}

int32_t hgx_set_coord_storage(hgx_ctx* c, int32_t mode) {
    if (!c || mode < 0 || mode > 1) return HGX_ERR_INVALID;
    each_shard(c, [&](hgx_ctx* x) { x->eng.force_coord32 = mode == 1; });
    return HGX_OK;
}

int32_t hgx_set_kernel_timing(hgx_ctx* c, int32_t on) {
    if (!c) return HGX_ERR_INVALID;
    each_shard(c, [&](hgx_ctx* x) { x->eng.time_mask = (uint32_t)on; });
    return HGX_OK;
}

int32_t hgx_set_fame_tally(hgx_ctx* c, int32_t mode) {
    if (!c || mode < 0 || mode > 2) return HGX_ERR_INVALID;
    each_shard(c, [&](hgx_ctx* x) { x->eng.fame_tally = mode; });
    return HGX_OK;
}

// ---- device buffers for callers without their own allocator (bench, tests) ---------
int32_t hgx_device_alloc(int32_t device, int64_t bytes, void** ptr) {
    if (!ptr || bytes < 0) return HGX_ERR_INVALID;
    *ptr = nullptr;
    int prev = -1;
    (void)hipGetDevice(&prev);
    if (hipSetDevice(device) != hipSuccess) return HGX_ERR_DEVICE;
    const hipError_t e = hipMalloc(ptr, (size_t)std::max<int64_t>(bytes, 1));
    if (prev >= 0 && prev != device) (void)hipSetDevice(prev);
    return e == hipSuccess ? HGX_OK : HGX_ERR_DEVICE;
}

int32_t hgx_device_free(int32_t device, void* ptr) {
    int prev = -1;
    (void)hipGetDevice(&prev);
    if (hipSetDevice(device) != hipSuccess) return HGX_ERR_DEVICE;
    const hipError_t e = ptr ? hipFree(ptr) : hipSuccess;
    if (prev >= 0 && prev != device) (void)hipSetDevice(prev);
    return e == hipSuccess ? HGX_OK : HGX_ERR_DEVICE;
}

int32_t hgx_device_copy(int32_t device, void* dst, const void* src, int64_t bytes, int32_t to_device) {
    if (bytes < 0 || (bytes > 0 && (!dst || !src))) return HGX_ERR_INVALID;
    int prev = -1;
    (void)hipGetDevice(&prev);
    if (hipSetDevice(device) != hipSuccess) return HGX_ERR_DEVICE;
    const hipError_t e = bytes ? hipMemcpy(dst, src, (size_t)bytes, to_device ? hipMemcpyHostToDevice
                                                                               : hipMemcpyDeviceToHost)
                               : hipSuccess;
    if (prev >= 0 && prev != device) (void)hipSetDevice(prev);
    return e == hipSuccess ? HGX_OK : HGX_ERR_DEVICE;
}

int32_t hgx_set_la_kernel(hgx_ctx* c, int32_t mode) {
    if (!c || mode < 0 || mode > 1026) return HGX_ERR_INVALID;
    each_shard(c, [&](hgx_ctx* x) {
        x->eng.la_kernel = mode == 1 ? 1 : 0;
        x->eng.la_segs_override = (mode >= 2 && mode <= 1024) ? mode : 0;
        x->eng.la_small_override = mode == 1025 ? 0 : -1;
        x->eng.la_verify_always = mode == 1026;
    });
    return HGX_OK;
}

int32_t hgx_set_root_others(hgx_ctx* c, const uint8_t* event_hash32, int64_t count, hgx_error* err) {
    if (!c || count < 0 || (count > 0 && !event_hash32)) {
        set_err(err, HGX_ERR_INVALID, "hgx_set_root_others: bad arguments");
        return HGX_ERR_INVALID;
    }
    if (group_only_one(c, err, "hgx_set_root_others")) return HGX_ERR_INVALID;
    if (!c->rooted && count > 0) {
        set_err(err, HGX_ERR_INVALID, "hgx_set_root_others: no roots installed (hgx_reset)");
        return HGX_ERR_INVALID;
    }
    DeviceGuard dg(c);
    const hipError_t e = c->eng.set_root_others(event_hash32, count);
    if (e != hipSuccess) return dev_err(err, e, "hgx_set_root_others");
    c->others_keys.assign(event_hash32, event_hash32 + (size_t)count * 32);
    return ok(err);
}

int32_t hgx_set_sort_kernel(hgx_ctx* c, int32_t mode) {
    if (!c || mode < 0 || mode > 1) return HGX_ERR_INVALID;
    each_shard(c, [&](hgx_ctx* x) { x->eng.sort_seg_enabled = mode == 0; });
    return HGX_OK;
}

int32_t hgx_set_round_kernel(hgx_ctx* c, int32_t mode) {
    if (!c || mode < 0 || mode > 5) return HGX_ERR_INVALID;
    each_shard(c, [&](hgx_ctx* x) {
        x->eng.round_kernel = mode == 5 ? 0 : mode;
        x->eng.round_pb_enabled = mode != 5;
    });
    return HGX_OK;
}

// The first chain of shard k of W: C k / W (every split-dependent piece reads c_split or shard_range)
static int32_t shard_split(int32_t C, int32_t W, int32_t k) {
    return (int32_t)((int64_t)C * k / W);
}

// W shards of one graph: shard 0 is `c` (on devs[0] == its device), shard k a new
// context on devs[k]; every shard holds the whole DAG, shard k owns chains [C k / W, C (k + 1) / W)
static int32_t setup_group(hgx_ctx* c, int32_t W, const int32_t* devs, hgx_error* err) {
    auto bad = [&](const std::string& why) {
        set_err(err, HGX_ERR_INVALID, "chain-sharded context: " + why);
        return HGX_ERR_INVALID;
    };
    if (W < 1 || W > hgx::kMaxShards) return bad("1 to 8 shards");
    if (c->E != 0) return bad("shards are set up on an empty context (before the first insert)");
    if (W == 1) {
        drop_group(c);
        return ok(err);
    }
    if (c->G != 1) return bad("one graph per context (hgx_create)");
    if (c->rooted) return bad("not after a Reset");
    if (W > c->C || c->n > 256) return bad("at most one shard per chain and n <= 256 (the persistent recurrence)");
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess) return bad("no HIP device");
    if (devs[0] != c->eng.dev) return bad("shard 0 runs on the context's own device");
    // every shard's launch of the recurrence waits for the others' granules, so the shards that share
    // a device need a hardware queue each besides the ones HIP keeps for itself
    const char* qenv = std::getenv("GPU_MAX_HW_QUEUES");
    const int queues = qenv ? std::max(1, std::atoi(qenv)) : 4;
    for (int k = 0; k < W; k++) {
        if (devs[k] < 0 || devs[k] >= ndev) return bad("invalid device ordinal " + std::to_string(devs[k]));
        int same = 0;
        for (int j = 0; j < W; j++) same += devs[j] == devs[k];
        if (same > 1 && same > queues - 2)
            return bad(std::to_string(same) + " shards on device " + std::to_string(devs[k]) +
                       " need GPU_MAX_HW_QUEUES >= " + std::to_string(same + 2) + " (set before the HIP runtime starts)");
    }
    // peer mappings between the shards' devices (window stores, round-row and timestamp copies)
    int prev = -1;
    (void)hipGetDevice(&prev);
    for (int a = 0; a < W; a++)
        for (int b = 0; b < W; b++) {
            if (devs[a] == devs[b]) continue;
            int can = 0;
            if (hipDeviceCanAccessPeer(&can, devs[a], devs[b]) != hipSuccess || !can) {
                if (prev >= 0) (void)hipSetDevice(prev);
                return bad("device " + std::to_string(devs[a]) + " cannot map device " + std::to_string(devs[b]));
            }
            (void)hipSetDevice(devs[a]);
            const hipError_t e = hipDeviceEnablePeerAccess(devs[b], 0);
            if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) {
                if (prev >= 0) (void)hipSetDevice(prev);
                return dev_err(err, e, "hipDeviceEnablePeerAccess");
            }
            (void)hipGetLastError();
        }
    if (prev >= 0) (void)hipSetDevice(prev);
    drop_group(c);
    auto* g = new (std::nothrow) hgx::ShardGroup();
    if (!g) return bad("out of host memory");
    g->W = W;
    for (int k = 0; k < W; k++) {
        g->dev[k] = devs[k];
        g->c_split[k] = shard_split(c->C, W, k);
    }
    g->c_split[W] = c->C;
    c->grp = g;
    for (int k = 1; k < W; k++) {
        hgx_ctx* q = hgx_create_batch(1, c->n, c->cap, devs[k], err);
        if (!q) {
            drop_group(c);
            return err ? err->code : HGX_ERR_DEVICE;
        }
        // the shard 0 settings (hgx_set_*) so far: every Engine field an hgx_set_* call writes
        // through each_shard
        q->eng.force_coord32 = c->eng.force_coord32;
        q->eng.la_verify_always = c->eng.la_verify_always;
        q->eng.time_mask = c->eng.time_mask;
        q->eng.fame_tally = c->eng.fame_tally;
        q->eng.la_kernel = c->eng.la_kernel;
        q->eng.la_segs_override = c->eng.la_segs_override;
        q->eng.la_small_override = c->eng.la_small_override;
        q->eng.round_kernel = c->eng.round_kernel;
        q->eng.round_pb_enabled = c->eng.round_pb_enabled;
        q->eng.sort_seg_enabled = c->eng.sort_seg_enabled;
        q->eng.cts_kernel = c->eng.cts_kernel;
        q->eng.incremental = c->eng.incremental;
        q->grp = nullptr;
        c->peers.push_back(q);
    }
    std::vector<hgx_ctx*> sh{c};
    sh.insert(sh.end(), c->peers.begin(), c->peers.end());
    for (int k = 0; k < W; k++) {
        g->eng[k] = &sh[k]->eng;
        sh[k]->eng.grp = g;
        sh[k]->eng.shard = k;
        sh[k]->shard_rank = k;
        sh[k]->shard_world = W;
        sh[k]->eng.shard_lo = g->c_split[k];
        sh[k]->eng.shard_hi = g->c_split[k + 1];
    }
    return ok(err);
}

int32_t hgx_set_shard_remote(hgx_ctx* c, int32_t on) {
    if (!c || !c->grp || on < 0 || on > 1) return HGX_ERR_INVALID;
    c->grp->force_remote = on != 0;
    return HGX_OK;
}

int32_t hgx_set_round_shards(hgx_ctx* c, int32_t shards) {
    if (!c || shards < 1 || shards > hgx::kMaxShards) return HGX_ERR_INVALID;
    if (shards == (c->grp ? c->grp->W : 1)) return HGX_OK;
    std::vector<int32_t> devs((size_t)shards, c->eng.dev);   // every shard on this context's device
    return setup_group(c, shards, devs.data(), nullptr);
}

hgx_ctx* hgx_create_sharded(int32_t n_participants, int64_t capacity_events, int32_t n_shards, const int32_t* devices,
                            hgx_error* err) {
    if (n_shards < 1 || n_shards > hgx::kMaxShards || !devices) {
        set_err(err, HGX_ERR_INVALID, "hgx_create_sharded: 1 to 8 shards, one device ordinal each");
        return nullptr;
    }
    hgx_ctx* c = hgx_create_batch(1, n_participants, capacity_events, devices[0], err);
    if (!c) return nullptr;
    if (setup_group(c, n_shards, devices, err) != HGX_OK) {
        hgx_destroy(c);
        return nullptr;
    }
    return c;
}

int32_t hgx_set_cts_kernel(hgx_ctx* c, int32_t mode) {
    if (!c || mode < 0 || mode > 2) return HGX_ERR_INVALID;
    each_shard(c, [&](hgx_ctx* x) { x->eng.cts_kernel = mode == 0 ? 1 : mode; });
    return HGX_OK;
}

int32_t hgx_set_commit_callback(hgx_ctx* c, hgx_commit_fn fn, void* user) {
    if (!c) return HGX_ERR_INVALID;
    c->commit_fn = fn;
    c->commit_user = user;
    return HGX_OK;
}

int32_t hgx_set_incremental(hgx_ctx* c, int32_t on) {
    if (!c || on < 0 || on > 1) return HGX_ERR_INVALID;
    each_shard(c, [&](hgx_ctx* x) { x->eng.incremental = on != 0; });
    return HGX_OK;
}

int32_t hgx_reserve_rounds(hgx_ctx* c, int32_t rounds) {
    if (!c || rounds < 1 || c->divided) return HGX_ERR_INVALID;   // before the first DivideRounds only
    int32_t rc = HGX_OK;
    each_shard(c, [&](hgx_ctx* x) {
        DeviceGuard dg(x);
        if (x->eng.reserve_rounds(rounds) != hipSuccess) rc = HGX_ERR_DEVICE;
        x->rounds_cached = x->recv_cached = false;
    });
    return rc;
}

}  // extern "C"
