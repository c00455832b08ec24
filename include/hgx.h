/*
 * hgx.h -- C ABI of the MI355X-native Hashgraph consensus engine (libhgx.so).
 *
 * Drop-in boundary for the reference's consensus hot path (datatypevoid/babble
 * v0.2.0, package hashgraph). A thin cgo shim keeps the Go API
 *   (*Hashgraph).InsertEvent(Event, bool) error   hashgraph/hashgraph.go:356
 *   (*Hashgraph).DivideRounds() error             hashgraph/hashgraph.go:616
 *   (*Hashgraph).DecideFame() error               hashgraph/hashgraph.go:649
 *   (*Hashgraph).FindOrder() error                hashgraph/hashgraph.go:801
 * and the exported state Core reads (UndeterminedEvents, PendingLoadedEvents,
 * LastConsensusRound, LastCommitedRoundEvents, ConsensusTransactions;
 * hashgraph.go:15-37, node/core.go:335-369), mapping event hex ids to dense ids.
 *
 * Conventions
 *  - Events get dense ids ("gid") in insertion order (the reference's
 *    topologicalIndex, hashgraph.go:373). A parent that is "" is -1; a parent
 *    hash the shim cannot resolve is HGX_UNKNOWN_PARENT.
 *  - Participants are ids 0..n-1 (Hashgraph.Participants, hashgraph.go:16).
 *    A batched context holds n_graphs independent hashgraphs; graph g owns
 *    participant ids [g*n, (g+1)*n).
 *  - All input arrays are copied before the call returns; no caller pointer is
 *    retained (cgo pointer rules). Output arrays are caller-allocated.
 *  - Every entry point returns HGX_OK (0) or an error code; the message of the
 *    last error is written to hgx_error.msg verbatim as the Go error string.
 *  - A context is single-caller (the reference serialises calls under
 *    node.coreLock, node/node.go:226-237); it owns one HIP stream.
 *  - The library fails loudly (HGX_ERR_DEVICE) when no gfx950 device is usable:
 *    there is no CPU fallback.
 */
#ifndef HGX_H
#define HGX_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define HGX_ABI_VERSION 6   /* 6: hgx_host_alloc / hgx_host_free (page-locked caller buffers);
                              5: hgx_events_packed (hgx_insert_events_packed, hgx_insert_and_run_packed,
                                 hgx_pack_events32);
                              4: hgx_create_sharded (chain-sharded recurrence over devices);
                              3: HGX_ROOT_OTHER needs its key registered (hgx_set_root_others) */

/* Error codes. 1..5 mirror common.StoreErrType + 1 (common/errors.go:7-13). */
enum {
    HGX_OK = 0,
    HGX_ERR_KEY_NOT_FOUND = 1,  /* "%s, Not Found"        errors.go:27 */
    HGX_ERR_TOO_LATE = 2,       /* "%s, Too Late"         errors.go:29 */
    HGX_ERR_PASSED_INDEX = 3,   /* "%s, Passed Index"     errors.go:31 */
    HGX_ERR_SKIPPED_INDEX = 4,  /* "%s, Skipped Index"    errors.go:33 */
    HGX_ERR_NO_ROOT = 5,        /* "%s, No Root"          errors.go:35 */
    HGX_ERR_SELF_PARENT = 100,  /* "CheckSelfParent: Self-parent not last known event by creator" hashgraph.go:366,416 */
    HGX_ERR_OTHER_PARENT = 101, /* "CheckOtherParent: Other-parent not known" hashgraph.go:370,441 */
    HGX_ERR_INVALID = 102,      /* bad argument to the C ABI itself */
    HGX_ERR_CAPACITY = 103,     /* context capacity exceeded */
    HGX_ERR_SIGNATURE = 104,    /* "Invalid signature" hashgraph.go:358-363 (Event.Verify false) */
    HGX_ERR_DEVICE = 200,       /* HIP error / no gfx950 device */
    HGX_ERR_PANIC = 300         /* the reference would panic here (e.g. UndecidedRounds[0] on empty) */
};

#define HGX_UNKNOWN_PARENT (-2)
/* After hgx_reset, other-parents outside the store that CheckOtherParent accepts through the
 * creator's Root (hashgraph.go:430-440): */
#define HGX_ROOT_Y (-3)       /* Root.Y (the creator's first event, self-parent = Root.X = -1) */
#define HGX_ROOT_OTHER (-4)   /* Root.Others[event]: the event's hash must be a key registered with
                                 hgx_set_root_others (the caller checked the entry's value) */

typedef struct {
    int32_t code;
    char msg[252];
} hgx_error;

typedef struct hgx_ctx hgx_ctx;

/* Event batch, structure of arrays, `count` entries each (hashgraph/event.go:14-76). */
typedef struct {
    const int32_t* creator;       /* participant id (global id in a batched ctx) */
    const int64_t* index;         /* Body.Index */
    const int64_t* self_parent;   /* gid, -1 for "" */
    const int64_t* other_parent;  /* gid, -1 for "", HGX_UNKNOWN_PARENT if not known */
    const int64_t* timestamp_ns;  /* Body.Timestamp as Unix ns (UTC) */
    const uint8_t* hash;          /* 32 bytes per event: SHA-256 event id (Event.Hash) */
    const uint8_t* sig_s;         /* 32 bytes per event: signature S, big-endian, zero-padded */
    const int32_t* ntx;           /* len(Body.Transactions) */
    const int32_t* tx_nil;        /* 1 if Body.Transactions == nil */
} hgx_events;

/* ---- lifecycle ------------------------------------------------------------ */
int32_t hgx_abi_version(void);
/* NewHashgraph(participants, store, ...) (hashgraph.go:39-66) with an InmemStore of
 * cacheSize >= capacity_events (no eviction). device = HIP device ordinal. The context pins
 * 4 bytes of host memory per event of capacity (at most 64 MB up front, grown on demand) for
 * the consensus order, which FindOrder writes there directly. */
hgx_ctx* hgx_create(int32_t n_participants, int64_t capacity_events, int32_t device, hgx_error* err);
/* n_graphs independent hashgraphs of n_participants each (seed-sharded simulations) */
hgx_ctx* hgx_create_batch(int32_t n_graphs, int32_t n_participants, int64_t capacity_events,
                          int32_t device, hgx_error* err);
/* One graph whose round recurrence is chain-sharded over n_shards devices (the north star's
 * single-graph mode; no reference counterpart: the Go Hashgraph is one object on one
 * core). devices[k] = shard k's HIP device (ordinals may repeat: shards that share a device need
 * GPU_MAX_HW_QUEUES >= shards on it + 2, set before the HIP runtime starts); shard 0 is the returned
 * context. Every shard holds the whole DAG (inserts, lastAncestors, fame, round received, sort:
 * replicated); shard k owns chains [C k / W, C (k + 1) / W): it builds their events'
 * firstDescendants, runs their workgroups of the persistent recurrence (writing each candidate row and
 * granule write-through into every shard's window, over the peer mapping when the shard lies on
 * another device) and their events' consensus timestamps, which FindOrder exchanges device to device.
 * The drop-in calls and getters work as on one context, with the same results; n <= 256, one graph;
 * hgx_reset, hgx_bootstrap, verified and wire inserts, hgx_set_shard and the public FindOrder halves
 * return HGX_ERR_INVALID on it. */
hgx_ctx* hgx_create_sharded(int32_t n_participants, int64_t capacity_events, int32_t n_shards,
                            const int32_t* devices, hgx_error* err);
void hgx_destroy(hgx_ctx* ctx);

/* ---- the four drop-in calls ------------------------------------------------ */
/* InsertEvent(e, true) for each event in order (hashgraph.go:356-401); stops at the first
 * failure like Core.Sync (node/core.go:199-211): *n_inserted = events accepted, err = the
 * Go error of the first rejected event. The batch is copied to HBM and validated there
 * (CheckSelfParent :404-420, CheckOtherParent :423-445, RollingIndex.Add
 * common/rolling_index.go:54-68) by data-parallel kernels; a whole Core.Sync batch is one call.
 * Event.Verify (the signature) stays with the caller. */
int32_t hgx_insert_events(hgx_ctx* ctx, const hgx_events* ev, int64_t count, int64_t* n_inserted,
                          hgx_error* err);
/* The compact form of the same batch (61 instead of 108 bytes per event cross PCIe): Index and
 * parents as int32 (gids are < 2^31 by hgx_create's capacity), the one byte of the event id that
 * consensus reads instead of the 32-byte id, and len(Body.Transactions) with -1 for nil. */
typedef struct {
    const int32_t* creator;       /* participant id (global id in a batched ctx) */
    const int32_t* index;         /* Body.Index */
    const int32_t* self_parent;   /* gid, -1 for "" */
    const int32_t* other_parent;  /* gid, -1 for "", HGX_UNKNOWN_PARENT / HGX_ROOT_Y as in hgx_events */
    const int64_t* timestamp_ns;  /* Body.Timestamp as Unix ns (UTC) */
    const uint8_t* coin;          /* 1 byte per event: middleBit (hashgraph.go:1039-1048), i.e. byte 16 of
                                     Event.Hash() is not 0 -- the coin of DecideFame's coin rounds */
    const uint8_t* sig_s;         /* 32 bytes per event: signature S, big-endian, zero-padded */
    const int32_t* ntx;           /* len(Body.Transactions); -1 if Body.Transactions == nil */
} hgx_events32;
/* hgx_insert_events / hgx_insert_and_run with hgx_events32 host columns. Same results, errors and
 * counters. Not after hgx_reset (the Root.Others check reads the 32-byte id): HGX_ERR_INVALID. */
int32_t hgx_insert_events32(hgx_ctx* ctx, const hgx_events32* ev, int64_t count, int64_t* n_inserted, hgx_error* err);
int32_t hgx_insert_and_run32(hgx_ctx* ctx, const hgx_events32* ev, int64_t count, int64_t* n_inserted,
                             hgx_error* err);
/* The same batch with its structure columns in 10 instead of 16 bytes per event (what
 * validation and DivideRounds wait for; the payload columns are those of hgx_events32). Event k
 * of the batch gets gid base + k, base = hgx_num_events(ctx) at the call. A parent is stored as
 * its distance back from that gid: 0 = "" (-1), 1..65534 = gid base + k - d, HGX_PARENT_ESCAPE =
 * the event's entry in the exception list (exc_pos: batch positions, distinct, any order;
 * exc_self_parent / exc_other_parent: both parents as hgx_events32 holds them, HGX_UNKNOWN_PARENT
 * included). An escaped parent without an entry reads as HGX_UNKNOWN_PARENT. The columns are
 * decoded on the device into the hgx_events32 form, so results, errors and counters are those of
 * hgx_insert_events32 / hgx_insert_and_run32 on the decoded batch. hgx_pack_events32 builds them. */
#define HGX_PARENT_ESCAPE 0xFFFF
typedef struct {
    const uint16_t* creator;            /* participant id (global id in a batched ctx), < 65536 */
    const int32_t* index;               /* Body.Index */
    const uint16_t* self_parent_back;   /* distance back, 0 = "", HGX_PARENT_ESCAPE */
    const uint16_t* other_parent_back;
    int64_t n_exc;                      /* exception list (host memory) */
    const int64_t* exc_pos;
    const int32_t* exc_self_parent;
    const int32_t* exc_other_parent;
    const int64_t* timestamp_ns;        /* the payload columns, as in hgx_events32 */
    const uint8_t* coin;
    const uint8_t* sig_s;
    const int32_t* ntx;
} hgx_events_packed;
int32_t hgx_insert_events_packed(hgx_ctx* ctx, const hgx_events_packed* ev, int64_t count, int64_t* n_inserted,
                                 hgx_error* err);
int32_t hgx_insert_and_run_packed(hgx_ctx* ctx, const hgx_events_packed* ev, int64_t count, int64_t* n_inserted,
                                  hgx_error* err);
/* Host helper (no device): the packed structure columns of an hgx_events32 batch whose first
 * event will get gid `base`. Writes creator16 / sp_back / op_back (count each) and up to exc_cap
 * exceptions; *n_exc = the number needed (HGX_ERR_INVALID "exception list full" if > exc_cap,
 * HGX_ERR_INVALID "creator outside 0..65535" for a creator the form cannot hold). */
int32_t hgx_pack_events32(const hgx_events32* ev, int64_t count, int64_t base, uint16_t* creator16, uint16_t* sp_back,
                          uint16_t* op_back, int64_t* exc_pos, int32_t* exc_self_parent, int32_t* exc_other_parent,
                          int64_t exc_cap, int64_t* n_exc, hgx_error* err);
/* Page-locked host memory for the caller's event columns (Core's sync buffers, allocated once and
 * reused: C memory, so cgo may hand Go slices over it with unsafe.Slice). Every insert call accepts
 * pageable memory as well; from page-locked memory the column copies are DMA transfers at the host
 * link's rate instead of staged copies. NULL on failure or bytes <= 0; hgx_host_free(NULL) is a no-op.
 * Usable with a context on any device. */
void* hgx_host_alloc(int64_t bytes);
void hgx_host_free(void* p);
/* The same with every hgx_events column a DEVICE pointer on the context's device (events
 * decoded / hashed on the GPU, or a trace resident in HBM). hash and sig_s must be
 * 16-byte aligned. Synchronous: the columns may be reused when the call returns. */
int32_t hgx_insert_events_device(hgx_ctx* ctx, const hgx_events* ev, int64_t count, int64_t* n_inserted,
                                 hgx_error* err);
/* Participants' public keys for Event.Verify: C = graphs * n_participants entries of 65 bytes
 * (Body.Creator: the uncompressed P-256 point 0x04|X|Y, participant id order). The device
 * window tables are built once here. A key that is not a P-256 point is accepted; an event it
 * signs then fails as in the reference, where elliptic.Unmarshal returns nil and
 * ecdsa.Verify dereferences it: HGX_ERR_PANIC "runtime error: invalid memory address or nil
 * pointer dereference". */
int32_t hgx_set_participant_keys(hgx_ctx* ctx, const uint8_t* keys65, hgx_error* err);
/* InsertEvent including Event.Verify (hashgraph.go:356-363, event.go:142-152): every event's
 * signature (R = sig_r32, S = ev->sig_s, 32 bytes big-endian each) is checked on the device
 * against its creator's key (hgx_set_participant_keys) and its body digest digest32
 * (EventBody.Hash: SHA-256 of the body JSON, event.go:48-54; hgx_sha256_batch computes it),
 * in the same data-parallel pass as the parent checks. The batch stops at the first failing
 * event; at one event the signature's failure ("Invalid signature", HGX_ERR_SIGNATURE) comes
 * before its parent checks, as in the reference. Host pointers (copied to HBM), or device
 * pointers (_device). HGX_ERR_INVALID "participant keys not set" without keys. */
int32_t hgx_insert_events_verified(hgx_ctx* ctx, const hgx_events* ev, const uint8_t* digest32, const uint8_t* sig_r32,
                                   int64_t count, int64_t* n_inserted, hgx_error* err);
int32_t hgx_insert_events_verified_device(hgx_ctx* ctx, const hgx_events* ev, const uint8_t* digest32,
                                          const uint8_t* sig_r32, int64_t count, int64_t* n_inserted, hgx_error* err);
/* WireEvents (event.go:252-267) as a SyncResponse carries them (net/commands.go:10-15), the
 * caller having decoded the JSON: the participants' ids instead of hashes. */
typedef struct {
    const int32_t* creator_id;            /* WireBody.CreatorID */
    const int64_t* index;                 /* WireBody.Index */
    const int64_t* self_parent_index;     /* WireBody.SelfParentIndex (-1: no self-parent) */
    const int32_t* other_parent_creator;  /* WireBody.OtherParentCreatorID */
    const int64_t* other_parent_index;    /* WireBody.OtherParentIndex (-1: "") */
    const int64_t* timestamp_ns;
    const uint8_t* hash;                  /* 32 bytes per event: the event id (Event.Hash) */
    const uint8_t* sig_s;                 /* 32 bytes per event: S, big-endian */
    const int32_t* ntx;
    const int32_t* tx_nil;
} hgx_wire_events;
/* Core.Sync's insert loop (node/core.go:199-211) in one call: per event ReadWireInfo
 * (hashgraph.go:569-614: parents through Store.ParticipantEvent, which sees the batch's earlier
 * events) then InsertEvent(ev, false); stops at the first error with Go's string (the
 * ReadWireInfo errors "<index>, Too Late" / "<index>, Not Found" included). */
int32_t hgx_insert_wire_events(hgx_ctx* ctx, const hgx_wire_events* ev, int64_t count, int64_t* n_inserted,
                               hgx_error* err);
int32_t hgx_divide_rounds(hgx_ctx* ctx, hgx_error* err);
int32_t hgx_decide_fame(hgx_ctx* ctx, hgx_error* err);
int32_t hgx_find_order(hgx_ctx* ctx, hgx_error* err);
/* FindOrder in two halves (hgx_find_order = begin + end): begin = DecideRoundReceived and the
 * consensus timestamps of the context's shard of chains; end = the ConsensusSorter order and
 * the blocks. A row-sharded graph exchanges the shards' timestamps in between. */
int32_t hgx_find_order_begin(hgx_ctx* ctx, hgx_error* err);
int32_t hgx_find_order_end(hgx_ctx* ctx, hgx_error* err);
/* One graph row-sharded over `world` ranks: every rank holds
 * the whole DAG and runs the replicated phases (lastAncestors, firstDescendants, the round
 * steps, fame, roundReceived); the consensus-timestamp medians of the events newly received
 * are computed by the rank owning their creator (chains [C*rank/world, C*(rank+1)/world)) and
 * all-gathered between hgx_find_order_begin and _end: hgx_shard_values(ctx, r) = how many int64
 * values rank r contributes, hgx_shard_export writes this rank's, hgx_shard_import reads rank
 * r's (device pointers on the context's device, e.g. RCCL buffers, or host pointers, e.g.
 * gloo). hgx_find_order refuses a sharded context. */
int32_t hgx_set_shard(hgx_ctx* ctx, int32_t rank, int32_t world);
int64_t hgx_shard_values(hgx_ctx* ctx, int32_t rank);
int32_t hgx_shard_export(hgx_ctx* ctx, void* dst, int32_t dst_on_device);
int32_t hgx_shard_import(hgx_ctx* ctx, int32_t src_rank, const void* src, int32_t src_on_device);
/* Bootstrap from host columns / Core.Sync followed by Core.RunConsensus (hashgraph.go:1008-1037,
 * node/core.go:190-303): hgx_insert_events for the batch, then hgx_run_consensus, in one call.
 * For batches of 65 536 events and more (single-graph or batched contexts without roots, not
 * row-sharded) the timestamps, hashes, S and transaction columns are copied to HBM while
 * DivideRounds runs (they are read from FindOrder on); the result, the errors and the
 * counters equal the two calls'. On an insert error the accepted prefix stays inserted and
 * consensus does not run (the error is returned). The host buffers are read before it returns. */
int32_t hgx_insert_and_run(hgx_ctx* ctx, const hgx_events* ev, int64_t count, int64_t* n_inserted, hgx_error* err);
/* Core.RunConsensus (node/core.go:277-303): the three calls in sequence */
int32_t hgx_run_consensus(hgx_ctx* ctx, hgx_error* err);
/* Forget every consensus result but keep the inserted events resident in HBM:
 * the state of a fresh NewHashgraph after InsertEvent of the same events
 * (Bootstrap replay, hashgraph.go:1008-1022). Used to repeat timed passes. */
int32_t hgx_reset_consensus(hgx_ctx* ctx);
/* Forget every event as well: the state of a fresh NewHashgraph (hashgraph.go:39-66) with
 * the device allocations kept. */
int32_t hgx_clear(hgx_ctx* ctx);

/* ---- persistence: checkpoint file + Bootstrap (hashgraph.go:1008-1037) ----- */
/* The reference persists the DAG in its BadgerStore (events under topological-index keys with
 * their bodies and signatures, the participants, the roots and the blocks; badger_store.go:103-125,
 * 309-343, 540) and Hashgraph.Bootstrap replays the events in topological order through
 * InsertEvent, then runs DivideRounds / DecideFame / FindOrder once (dbTopologicalEvents,
 * badger_store.go:345-386). The equivalent here is a binary SoA file of the resident events in
 * gid (= topological) order, little-endian (version 2; version-1 files are still read):
 *   "HGXCKPT1" | u32 version 2 | i32 n | i32 graphs | i32 flags | i64 E
 *     flags: 1 rooted, 2 event ids, 4 participant keys, 8 payloads
 *   | rooted: i32 root_index[C], i32 root_round[C], u8 root_y_is_event[C], zero pad to 4
 *     | i64 n_others | u8 others[n_others][32] (the Root.Others keys, hgx_set_root_others)
 *     | per graph, what Reset kept (hashgraph.go:877-895): i32 has_lcr, i32 LastConsensusRound,
 *       i32 LastCommitedRoundEvents, i32 0, i64 ConsensusTransactions, i64 n_blocks, then per block
 *       i32 RoundReceived, i32 events, i64 transactions, i32 nil, i32 committed
 *   | i32 creator[E] | i64 index[E] | i64 self_parent[E] | i64 other_parent[E]
 *   | i64 timestamp_ns[E] | u8 sig_s[E][32] | u8 coin[E] (Event.Hash byte 16 != 0)
 *   | i32 ntx[E] | u8 tx_nil[E]
 *   | ids: u8 id[E][32] (Event.Hash), when every event was inserted with its id (hgx_events)
 *   | keys: u8 key[C][65] (hgx_set_participant_keys)
 *   | payloads: i64 off[E+1] | u8 bytes[off[E]] (the caller's per-event bytes, e.g. the body's
 *     transactions as the shim serialises them; opaque to libhgx)
 *   | u64 FNV-1a of every preceding byte
 * (C = graphs * n). hgx_save writes it atomically (a temporary file renamed over `path`);
 * hgx_save_ex also stores the caller's payloads (payload_off: E + 1 non-decreasing offsets from
 * 0 into payload, or NULL). hgx_bootstrap = Bootstrap on a fresh context (no events inserted):
 * checks the file (magic, version, n, graphs, sizes, checksum: HGX_ERR_INVALID "<reason>"),
 * installs the roots, the Root.Others keys and the kept state of a rooted file, the participant
 * keys, inserts every event in order (hgx_insert_events with the ids when the file has them:
 * their Go error if one is rejected), keeps the payloads (hgx_get_event_payload) and runs the
 * three consensus calls once (hgx_run_consensus). */
int32_t hgx_save(hgx_ctx* ctx, const char* path, hgx_error* err);
int32_t hgx_save_ex(hgx_ctx* ctx, const char* path, const int64_t* payload_off, const uint8_t* payload,
                    hgx_error* err);
/* the file's checksum: 64-bit FNV-1a of `bytes` bytes (host function, no device) */
uint64_t hgx_checksum(const void* data, int64_t bytes);
int32_t hgx_bootstrap(hgx_ctx* ctx, const char* path, hgx_error* err);
/* The id (Event.Hash, 32 bytes) of an inserted event: known when every event was inserted with
 * hgx_events (or bootstrapped from a file with ids); else HGX_ERR_INVALID. */
int32_t hgx_get_event_id(hgx_ctx* ctx, int64_t gid, uint8_t* out32, hgx_error* err);
/* The payload bytes of a bootstrapped event (hgx_save_ex): *len = its size, the first min(cap,
 * len) bytes to out; HGX_ERR_KEY_NOT_FOUND "<gid>, Not Found" without one. */
int32_t hgx_get_event_payload(hgx_ctx* ctx, int64_t gid, uint8_t* out, int64_t cap, int64_t* len, hgx_error* err);

/* ---- persistence: Reset / GetFrame (hashgraph.go:877-995, root.go) -------- */
/* Hashgraph.Reset(roots): forget the events and rounds (keeping LastConsensusRound,
 * LastCommitedRoundEvents, ConsensusTransactions and the blocks, like the reference) and
 * install one Root per participant: Index, Round and whether Root.Y names an event (1) or is
 * "" (0). Inserted events then name Root.X as self-parent -1 and Root.Y / Root.Others as
 * HGX_ROOT_Y / HGX_ROOT_OTHER. Single-graph contexts. */
int32_t hgx_reset(hgx_ctx* ctx, const int32_t* root_index, const int32_t* root_round, const int32_t* root_y_is_event,
                  hgx_error* err);
/* The keys of the roots' Others maps (root.go: Others[event hex] = other-parent hex,
 * hashgraph.go:437-440): the 32-byte ids of the events allowed to name HGX_ROOT_OTHER. After
 * hgx_reset the set is empty; an event inserted with HGX_ROOT_OTHER whose hash (hgx_events.hash)
 * is not a key fails with "CheckOtherParent: Other-parent not known", as in the reference. The
 * value (which other-parent the entry names) stays the shim's check, since the other-parent is
 * outside the store. hgx_bootstrap re-checks the HGX_ROOT_OTHER events of a rooted version-2
 * checkpoint against its keys and ids (a version-1 file, without ids, is trusted). */
int32_t hgx_set_root_others(hgx_ctx* ctx, const uint8_t* event_hash32, int64_t count, hgx_error* err);
/* Hashgraph.GetFrame: per participant root_x / root_y (gid; -1 = the current Root.X / ""; 
 * HGX_ROOT_Y / HGX_ROOT_OTHER as inserted), root_index, root_round; the frame's events (gids,
 * topological order) and Root.Others pairs (event, other-parent). Counts are returned in full;
 * arrays get the first `cap`. "<r>, Not Found" when LastConsensusRound's round is not stored. */
int32_t hgx_get_frame(hgx_ctx* ctx, int64_t* events, int64_t events_cap, int64_t* n_events, int64_t* root_x,
                      int64_t* root_y, int32_t* root_index, int32_t* root_round, int64_t* others_event,
                      int64_t* others_parent, int64_t others_cap, int64_t* n_others, hgx_error* err);

/* ---- Hashgraph state (hashgraph.go:15-37) --------------------------------- */
int64_t hgx_num_events(hgx_ctx* ctx);
int32_t hgx_super_majority(hgx_ctx* ctx);
int64_t hgx_num_undetermined(hgx_ctx* ctx, int32_t graph);
int32_t hgx_undecided_rounds(hgx_ctx* ctx, int32_t graph, int32_t* out, int32_t cap); /* returns length */
int32_t hgx_last_consensus_round(hgx_ctx* ctx, int32_t graph, int32_t* has_value);
int32_t hgx_last_commited_round_events(hgx_ctx* ctx, int32_t graph);
int64_t hgx_consensus_transactions(hgx_ctx* ctx, int32_t graph);
int64_t hgx_pending_loaded_events(hgx_ctx* ctx, int32_t graph);

/* ---- Store views (hashgraph/store.go:3-25) -------------------------------- */
int32_t hgx_last_round(hgx_ctx* ctx, int32_t graph);                       /* Store.LastRound */
int32_t hgx_round_event_count(hgx_ctx* ctx, int32_t graph, int32_t r);     /* Store.RoundEvents */
int32_t hgx_round_witnesses(hgx_ctx* ctx, int32_t graph, int32_t r, int64_t* out, int32_t cap);
int32_t hgx_known(hgx_ctx* ctx, int32_t graph, int32_t* last_index);     /* Store.Known */
int64_t hgx_consensus_events_count(hgx_ctx* ctx, int32_t graph);         /* Store.ConsensusEventsCount */
/* full consensus order (AddConsensusEvent sequence) of one graph: gids */
int32_t hgx_consensus_events(hgx_ctx* ctx, int32_t graph, int64_t first, int64_t count, int64_t* gids);
/* Blocks in SetBlock order (hashgraph.go:826-854): rr, first position in the
 * graph's consensus order, number of events, number of transactions, nil flag,
 * committed (sent on commitCh: len(Transactions) > 0). */
int64_t hgx_num_blocks(hgx_ctx* ctx, int32_t graph);
int32_t hgx_block_info(hgx_ctx* ctx, int32_t graph, int64_t b, int32_t* round_received, int64_t* first,
                       int32_t* n_events, int64_t* n_tx, int32_t* tx_nil, int32_t* committed);
/* commitCh (hashgraph.go:848-854, node/node.go:150-154 -> AppProxy.CommitBlock): fn is called
 * from hgx_find_order for every new block with transactions, in SetBlock order, after the
 * block's state is recorded (graph, block index b, RoundReceived, first position and number of
 * its events in the graph's consensus order, transactions). NULL removes it. */
typedef void (*hgx_commit_fn)(void* user, int32_t graph, int64_t b, int32_t round_received, int64_t first,
                              int32_t n_events, int64_t n_tx);
int32_t hgx_set_commit_callback(hgx_ctx* ctx, hgx_commit_fn fn, void* user);
/* Store.GetBlock(rr) (inmem_store.go:163-169): index b of the block with RoundReceived rr,
 * else HGX_ERR_KEY_NOT_FOUND "<rr>, Not Found" */
int32_t hgx_get_block(hgx_ctx* ctx, int32_t graph, int32_t round_received, int64_t* b, hgx_error* err);
/* positions [first, first+count) of a graph's consensus order: gid, RoundReceived and
 * consensusTimestamp (ns) of each, in one call (any output may be NULL) */
int32_t hgx_consensus_received(hgx_ctx* ctx, int32_t graph, int64_t first, int64_t count, int64_t* gids,
                               int32_t* round_received, int64_t* consensus_ts);

/* ---- Store: events by participant (store.go:3-25, inmem_store.go:48-161) ---
 * Participant ids are the context's creator ids (global ids in a batched context). The
 * RollingIndex never evicts (cacheSize >= events). Errors carry Go's strings. */
/* LastFrom: gid of the participant's last event; none: gid -1 and is_root 1 (Root.X = "") */
int32_t hgx_last_from(hgx_ctx* ctx, int32_t participant, int64_t* gid, int32_t* is_root, hgx_error* err);
/* ParticipantEvents(p, skip) (caches.go:54-72): the events with Index > skip, in Index
 * order; *count = how many (gids gets the first min(count, cap)) */
int32_t hgx_participant_events(hgx_ctx* ctx, int32_t participant, int64_t skip, int64_t* gids, int64_t cap,
                               int64_t* count, hgx_error* err);
/* ParticipantEvent(p, index) (caches.go:74-80): "<index>, Too Late" / "<index>, Not Found" */
int32_t hgx_participant_event(hgx_ctx* ctx, int32_t participant, int64_t index, int64_t* gid, hgx_error* err);
/* GetRoot (inmem_store.go:163-169): X = -1 (Root.X), Y = -1 ("") or HGX_ROOT_Y, Index, Round
 * (the genesis Root: Index = Round = -1, or the one hgx_reset installed) */
int32_t hgx_get_root(hgx_ctx* ctx, int32_t participant, int64_t* x, int64_t* y, int32_t* index, int32_t* round,
                     hgx_error* err);
/* GetEvent (inmem_store.go:48-55): the DAG fields of an inserted event (bodies stay with the caller) */
int32_t hgx_get_event(hgx_ctx* ctx, int64_t gid, int32_t* creator, int64_t* index, int64_t* self_parent,
                      int64_t* other_parent, int64_t* timestamp_ns, int32_t* ntx, int32_t* tx_nil, hgx_error* err);
/* SetWireInfo (hashgraph.go:532-567) of events [first, first+count): self-parent Index
 * (Root.Index -1 for a first event), other-parent creator id and Index (-1 for "") */
int32_t hgx_wire_info(hgx_ctx* ctx, int64_t first, int64_t count, int32_t* self_parent_index,
                      int32_t* other_parent_creator, int32_t* other_parent_index);
/* ReadWireInfo (hashgraph.go:569-614): parents of a wire event as gids (-1 for an index < 0),
 * through ParticipantEvent (its errors) */
int32_t hgx_read_wire_info(hgx_ctx* ctx, int32_t creator, int64_t self_parent_index, int32_t other_parent_creator,
                           int64_t other_parent_index, int64_t* self_parent, int64_t* other_parent, hgx_error* err);

/* ---- per-event results (bulk) --------------------------------------------- */
/* round (Round), witness (Witness), famous (RoundEvent.Famous: 0 Undefined,1 True,2 False) */
int32_t hgx_get_rounds(hgx_ctx* ctx, int64_t first, int64_t count, int32_t* round, int8_t* witness,
                       int8_t* famous);
/* RoundReceived (-1 = nil) and consensusTimestamp (Unix ns) */
int32_t hgx_get_received(hgx_ctx* ctx, int64_t first, int64_t count, int32_t* round_received,
                         int64_t* consensus_ts);
/* lastAncestors / firstDescendants indexes of one event (n values each) */
int32_t hgx_get_coords(hgx_ctx* ctx, int64_t gid, int32_t* last_ancestors, int32_t* first_descendants);

/* ---- primitives (hashgraph.go:73-339), valid after hgx_divide_rounds ------ */
int32_t hgx_ancestor(hgx_ctx* ctx, int64_t x, int64_t y);
int32_t hgx_self_ancestor(hgx_ctx* ctx, int64_t x, int64_t y);
int32_t hgx_see(hgx_ctx* ctx, int64_t x, int64_t y);
int32_t hgx_strongly_see(hgx_ctx* ctx, int64_t x, int64_t y);
int64_t hgx_oldest_self_ancestor_to_see(hgx_ctx* ctx, int64_t x, int64_t y);
int32_t hgx_round(hgx_ctx* ctx, int64_t x);
int32_t hgx_witness(hgx_ctx* ctx, int64_t x);

/* ---- Go encodings (parity unpinned) -------------------- */
/* SHA256(json.Encoder(Block)) with Block{RoundReceived, Transactions} (block.go:26-53) */
int32_t hgx_block_hash(int64_t round_received, int32_t ntx, const uint8_t* const* tx, const int64_t* tx_len,
                       int32_t tx_nil, uint8_t* out32);

/* ---- ingest front end: batched SHA-256 ----------------- */
/* crypto.SHA256 (crypto/utils.go:11-16) of `count` messages in one launch, message i =
 * data[offsets[i], offsets[i+1]) (offsets has count+1 non-decreasing entries). Replaces the
 * per-event calls Event.Hash (hashgraph/event.go:171-180; the event id of Hex() :183-188),
 * EventBody.Hash (:48-54, the bytes Verify checks :142-152) and Block.Hash (block.go:44-53)
 * over a whole sync batch (node/core.go:199-211). Host buffers, copied to HBM; out32 gets
 * 32 bytes per message. HGX_ERR_DEVICE without a gfx950 device (no CPU fallback). */
int32_t hgx_sha256_batch(int32_t device, const uint8_t* data, const int64_t* offsets, int64_t count,
                         uint8_t* out32, hgx_error* err);
/* The same on device-resident buffers, enqueued on `stream` (a hipStream_t; NULL = null
 * stream) without synchronising. d_out32 must be 4-byte aligned. Message bytes are read
 * with 16-byte loads from the 16-byte-aligned span of each message: up to 15 bytes before
 * d_data + offsets[i] and past d_data + offsets[i+1] may be read (harmless inside one
 * allocation; the caller keeps that span mapped). */
int32_t hgx_sha256_batch_device(const uint8_t* d_data, const int64_t* d_offsets, int64_t count,
                                uint8_t* d_out32, void* stream);
/* Measurement: `count` synthetic messages resident in HBM (message i has length
 * min_len + splitmix64(~seed + i) % (max_len - min_len + 1); packed 8-byte word j of the
 * data is splitmix64(seed + j)), hashed warmup + iters times; *ms_per_launch from HIP
 * events on the launch stream; digests of the first n_sample messages to sample32. */
int32_t hgx_sha256_bench(int32_t device, int64_t count, int32_t min_len, int32_t max_len, uint64_t seed,
                         int32_t warmup, int32_t iters, double* ms_per_launch, int64_t* total_bytes,
                         int64_t* n_blocks, int64_t n_sample, uint8_t* sample32);

/* Measurement (bench.py roofline.latency): the exchange floor of one round of the persistent
 * recurrence -- `chains` resident workgroups of k_round_p's geometry at n coordinates (16 < n <= 256,
 * chains <= the device's CUs) that per round only publish their n-byte candidate row and granule
 * (write-through) and poll every other one's (sc1), no search. *us_per_round from HIP events over one
 * launch of `rounds` rounds after a warm-up launch; chains = 2 is one 1-to-1 hand-off each way. */
int32_t hgx_exchange_floor_bench(int32_t device, int32_t chains, int32_t n, int32_t rounds, double* us_per_round);

/* ---- ingest front end: batched ECDSA P-256 verify ------ */
/* Event.Verify (hashgraph/event.go:142-152) for a whole sync batch: crypto.ToECDSAPub of
 * Body.Creator (crypto/utils.go:22-28) and crypto.Verify (crypto/utils.go:41-43) = Go's
 * ecdsa.Verify on P-256. keys65: n_keys public keys, 65 bytes each (0x04 || X || Y, the
 * bytes of Body.Creator); key_idx[i]: the key of signature i; digest32: EventBody.Hash
 * (SHA-256 of the body, hgx_sha256_batch); r32, s32: R and S big-endian, zero-padded.
 * out[i] = 1 valid, 0 invalid, 2 the key is not a P-256 point (Go's elliptic.Unmarshal
 * returns nil there). Pinned by libcrypto answers (oracle/p256_ref.c). */
int32_t hgx_p256_verify_batch(int32_t device, const uint8_t* keys65, int32_t n_keys, const int32_t* key_idx,
                              const uint8_t* digest32, const uint8_t* r32, const uint8_t* s32, int64_t count,
                              uint8_t* out, hgx_error* err);
/* bench.py: the same batch resident in HBM; the key tables built once (as a context does when its
 * keys are set), then the verify launch warmup + iters times, device time per verify launch from
 * HIP events; out = the results of the last launch */
int32_t hgx_p256_verify_bench(int32_t device, const uint8_t* keys65, int32_t n_keys, const int32_t* key_idx,
                              const uint8_t* digest32, const uint8_t* r32, const uint8_t* s32, int64_t count,
                              int32_t warmup, int32_t iters, uint8_t* out, double* ms_per_launch);

/* ---- timing / instrumentation --------------------------------------------- */
/* per-phase device times (ms) of the last calls: coords, rounds, fame, order; then
 * LA sweeps, rounds, 1 if the coordinates were stored compact (uint16); then of the last
 * DivideRounds: lastAncestors rows recomputed, 1 if it rebuilt the layout (0: incremental),
 * the first round step it ran, 1 if the lastAncestors pass was the dataflow kernel; then
 * the number of dataflow passes that gave up and were redone by the sweeps, and the time
 * segments of the last dataflow pass; then the persistent round launches so far and the
 * DivideRounds calls whose persistent launch gave up and were redone per round, and the
 * candidate rows it counted with exact compares (over 8 bits), the round and chain of the last
 * persistent launch that gave up, then the whole-graph round launches so far (up to 19 values) */
int32_t hgx_phase_times(hgx_ctx* ctx, double* out, int32_t cap);
/* dominant-kernel accounting for the roofline line of bench.py:
 * name of the kernel, summed device ms (the round steps time one hipGraph replay in four and
 * scale the sample to every launch), launches, algorithmic bytes moved */
int32_t hgx_kernel_stats(hgx_ctx* ctx, int32_t k, char* name, int32_t name_cap, double* ms, int64_t* launches,
                         double* bytes);
int32_t hgx_reset_stats(hgx_ctx* ctx);
/* time the kernels in bitmask `mask` (bit k = kernel id of hgx_kernel_stats; -1 = all) with HIP events on the context stream (bench.py roofline) */
int32_t hgx_set_kernel_timing(hgx_ctx* ctx, int32_t mask);

/* coordinate storage of later DivideRounds calls: 0 = auto (uint16 when every Index
 * <= 65533 and n is even, else int32), 1 = always int32. Same results either way. */
int32_t hgx_set_coord_storage(hgx_ctx* ctx, int32_t mode);
/* DecideFame vote tally: 0 = witness-tiled popcount (default), 1 = per-round popcount
 * kernel, 2 = witness-tiled int8 MFMA. Same results; for measurement. */
int32_t hgx_set_fame_tally(hgx_ctx* ctx, int32_t mode);
/* DivideRounds lastAncestors: 0 = one dataflow pass per (graph, column block) where it
 * applies (default: n <= 896, chains < 2^21 rows; hgx_la_wave.hip), and for a small graph
 * (n <= 32 compact / 16 int32, its rows within 150 KB) the pass with the whole graph in one
 * workgroup's LDS; 1 = Gauss-Seidel sweeps to the fixed point (hgx_kernels.hip), 2 <= m <= 1024 =
 * the dataflow pass with m time segments on a rebuild (measurement), 1025 = the dataflow pass
 * without the small-graph form, 1026 = the default with the verify sweep after every time-segmented
 * pass (by default it runs only when the segments' exactness check fails). Same results
 * (DESIGN.md §3.1). */
int32_t hgx_set_la_kernel(hgx_ctx* ctx, int32_t mode);
/* DivideRounds rounds: 0 = default: the persistent recurrence (hgx_round_p.hip, one resident
 * workgroup per chain runs every round in one launch) where it applies (n <= 256, at most one
 * chain per compute unit, no roots; for 256 < n <= 1024 and one graph hgx_round_pb.hip, one
 * resident workgroup per chain with events) on a call that lays the DAG out anew (a call resuming after
 * a few inserts runs a few rounds: one launch per round of mode 2 there, and wherever the
 * persistent launch does not apply); 3 = the persistent recurrence on every call where it
 * applies;
 * 1 = block binary search per round (hgx_rounds.hip; per-candidate search over streamed rows
 * above n = 256); 2 = one launch per round, one lane per candidate, 8-bit rebased compares
 * (hgx_round_k.hip; candidates in chunks of 128 above n = 256); 4 = the whole-graph recurrence
 * (hgx_round_g.hip: one workgroup per graph runs every round in one launch, n <= 16), which mode 0
 * also uses on every call where it applies; 5 = mode 0 without hgx_round_pb.hip (n > 256: the
 * steps of mode 2). Same results. */
int32_t hgx_set_round_kernel(hgx_ctx* ctx, int32_t mode);
/* FindOrder's sort of the received events by (graph, roundReceived, consensus timestamp, S): 0 =
 * default: bucketed by (graph, roundReceived) and every bucket sorted in one workgroup's LDS where
 * every bucket holds at most 8 192 events (else as 1); 1 = LSD radix passes over the whole list.
 * Same results. */
int32_t hgx_set_sort_kernel(hgx_ctx* ctx, int32_t mode);
/* hgx_create_sharded's shards on this context's own device: shards = W in [1, 8] (1 = back to one
 * context), on an empty context only (before the first insert). W shards on one device need
 * GPU_MAX_HW_QUEUES >= W + 2 (HGX_ERR_INVALID otherwise). Same results. */
int32_t hgx_set_round_shards(hgx_ctx* ctx, int32_t shards);
/* Test switch of a chain-sharded context (hgx_create_sharded / hgx_set_round_shards): on = 1 writes
 * every other shard's window as a window on another device (system-scope write-through stores, the
 * peer path), also where the shards share a device, so a one-GPU box runs the instructions the
 * shards of an 8-GPU node run. HGX_ERR_INVALID on a context without shards. Same results. */
int32_t hgx_set_shard_remote(hgx_ctx* ctx, int32_t on);
/* FindOrder consensus timestamps: 0 = default = 1: one tile of 8 positions per block (k_cts_small /
 * k_cts_tile, hgx_kernels.hip); 2 = resident blocks with three tiles' loads in flight behind the
 * selects of a fourth (hgx_cts.hip) where it applies (32 < n <= 512, at most 4096 chains),
 * otherwise mode 1 (measured slower at c3: 12.6 against 8.9 ms). Same results. */
int32_t hgx_set_cts_kernel(hgx_ctx* ctx, int32_t mode);
/* DivideRounds schedule: 1 = incremental (default: a call after more InsertEvents extends
 * lastAncestors/firstDescendants for the new events only and resumes the round steps at the
 * lowest round that can change; FindOrder works on the events not yet received), 0 = every
 * call recomputes from the whole DAG. Same results. */
int32_t hgx_set_incremental(hgx_ctx* ctx, int32_t on);
/* Size the per-round device tables for `rounds` rounds (they grow on demand during
 * DivideRounds); before the first DivideRounds only. A small value exercises the growth path. */
int32_t hgx_reserve_rounds(hgx_ctx* ctx, int32_t rounds);

/* ---- device buffers (for callers without a device allocator: bench, tests) ---- */
int32_t hgx_device_alloc(int32_t device, int64_t bytes, void** ptr);
int32_t hgx_device_free(int32_t device, void* ptr);
/* synchronous copy; to_device 1: host src -> device dst, 0: device src -> host dst */
int32_t hgx_device_copy(int32_t device, void* dst, const void* src, int64_t bytes, int32_t to_device);

/* ---- synthetic gossip traces (BASELINE.md / SURVEY 8d generator) ---------- */
/* Seeded random gossip modelled on node/core_test.go:514-537: every active peer
 * emits a genesis event, then each step a uniformly chosen `to` emits
 * (sp = head[to], op = head[from]); ts = t0 + step*1000 ns; w.p. 1/2 one
 * 16-byte-class payload "p%03d tx %08d", else an empty non-nil payload; S and
 * the event id are PRNG bytes (synthetic ids). Silent peers are the last
 * `n_silent` ids (never to/from, no genesis). With probability stale_prob the
 * `from` head is replaced by one of from's last stale_depth events. Fills
 * caller arrays of length n_events (index/parents as in hgx_events; tx_seq =
 * per-creator payload counter or -1). Returns HGX_OK. */
int32_t hgx_trace_gossip(int32_t n_participants, int32_t n_silent, int64_t n_events, uint64_t seed,
                         double stale_prob, int32_t stale_depth,
                         int32_t* creator, int64_t* index, int64_t* self_parent, int64_t* other_parent,
                         int64_t* timestamp_ns, uint8_t* hash, uint8_t* sig_s, int32_t* ntx, int32_t* tx_nil,
                         int64_t* tx_seq);
/* payload bytes of generated transaction (creator, seq); returns length */
int32_t hgx_trace_tx_payload(int32_t creator, int64_t seq, uint8_t* out, int32_t cap);

#ifdef __cplusplus
}
#endif
#endif /* HGX_H */
