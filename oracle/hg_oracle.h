/*
 * hg_oracle.h -- TEST INFRASTRUCTURE. CPU restatement of the reference Hashgraph
 * consensus path (datatypevoid/babble v0.2.0, hashgraph/hashgraph.go) used ONLY as
 * the parity checker by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
 * leg. It is never linked into or called by the product library (babble_amd/libhgx.so).
 *
 * Pinning: checked against every structural known-answer assertion of the
 * reference's own tests (hashgraph/hashgraph_test.go, node/core_test.go) via the
 * fixtures in tests/golden/ (see tests/test_oracle_kat.py). Event/block hash bytes
 * follow SURVEY.md Appendix B and are "parity unpinned" (no reference test pins a hash).
 *
 * Identity: events are dense ids (gid) in insertion order; "" (no parent) is -1,
 * an unknown parent hash is HGO_UNKNOWN (-2). Participants are ids 0..n-1.
 * Only the genesis Root (X=Y="", Index=-1, Round=-1; hashgraph/root.go:70-77) is
 * supported: Reset/Frame (hashgraph.go:879-1002) is out of scope.
 */
#ifndef HG_ORACLE_H
#define HG_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define HGO_UNKNOWN (-2)

typedef struct hgo hgo;

hgo* hgo_new(int n_participants);
void hgo_free(hgo* h);

/* InsertEvent(event, setWireInfo=true) (hashgraph.go:356-401). Returns 0 on success,
 * else a StoreErr-like kind code (>0) with the Go error string in err (if non-NULL).
 * txs: ntx payloads concatenated in tx_data with lengths tx_len (may be NULL if ntx==0). */
int hgo_insert(hgo* h, int creator, int64_t index, int64_t self_parent, int64_t other_parent,
               int64_t ts_ns, const uint8_t* hash32, const uint8_t* s32, int ntx, int tx_nil,
               const uint8_t* tx_data, const int32_t* tx_len, char* err, int errlen);

/* hgo_insert over a batch (structure of arrays), stopping at the first failure; payloads
 * of event k: the next ntx[k] lengths of tx_len, bytes consecutive in tx_blob */
int64_t hgo_insert_batch(hgo* h, int64_t m, const int32_t* creator, const int64_t* index, const int64_t* sp,
                         const int64_t* op, const int64_t* ts, const uint8_t* hash, const uint8_t* S,
                         const int32_t* ntx, const int32_t* tx_nil, const uint8_t* tx_blob, const int32_t* tx_len,
                         int* rc, char* err, int errlen);

/* other-parent codes for events whose other-parent is outside the store after a Reset
   (CheckOtherParent through the creator's Root, hashgraph.go:430-440) */
#define HGO_ROOT_Y (-3)      /* Root.Y */
#define HGO_ROOT_OTHER (-4)  /* Root.Others[event] */
/* Hashgraph.Reset(roots) (hashgraph.go:877-895): per participant Root.Index, Root.Round and
   whether Root.Y names an event (1) or is "" (0); a first event's self-parent -1 is Root.X */
int hgo_reset(hgo* h, const int32_t* root_index, const int32_t* root_round, const uint8_t* root_y_ext);
void hgo_get_root(hgo* h, int p, int32_t* index, int32_t* round, int* y_ext);
/* Hashgraph.GetFrame (hashgraph.go:897-995); see hg_oracle.c for the encodings */
int hgo_get_frame(hgo* h, int64_t* ev_out, int64_t ev_cap, int64_t* n_ev, int64_t* root_x, int64_t* root_y,
                  int32_t* root_index, int32_t* root_round, int64_t* oth_ev, int64_t* oth_op, int64_t oth_cap,
                  int64_t* n_oth);
int hgo_divide_rounds(hgo* h);                       /* hashgraph.go:616-646 */
int hgo_decide_fame(hgo* h, char* err, int errlen);  /* hashgraph.go:649-730 */
int hgo_decide_round_received(hgo* h, char* err, int errlen); /* :753-799 */
int hgo_find_order(hgo* h, char* err, int errlen);   /* hashgraph.go:801-858 */

/* primitives (hashgraph.go:73-339); gids, -1 = "" */
int hgo_ancestor(hgo* h, int64_t x, int64_t y);
int hgo_self_ancestor(hgo* h, int64_t x, int64_t y);
int hgo_see(hgo* h, int64_t x, int64_t y);
int hgo_strongly_see(hgo* h, int64_t x, int64_t y);
int64_t hgo_oldest_self_ancestor_to_see(hgo* h, int64_t x, int64_t y);
int hgo_parent_round(hgo* h, int64_t x, int* is_root);
int hgo_round_inc(hgo* h, int64_t x);
int hgo_round(hgo* h, int64_t x);
int hgo_witness(hgo* h, int64_t x);

/* state / getters */
int64_t hgo_num_events(hgo* h);
int hgo_super_majority(hgo* h);
int hgo_last_round(hgo* h);
int hgo_round_event_count(hgo* h, int r);
int hgo_round_witnesses(hgo* h, int r, int64_t* out, int cap);
int hgo_famous(hgo* h, int64_t x);            /* 0 Undefined, 1 True, 2 False (roundInfo.go:9-15) */
int hgo_round_received(hgo* h, int64_t x);    /* -1 = nil */
int64_t hgo_consensus_timestamp(hgo* h, int64_t x);
void hgo_coords(hgo* h, int64_t x, int32_t* la, int32_t* fd);
void hgo_wire_info(hgo* h, int64_t x, int32_t* sp_index, int32_t* op_creator, int32_t* op_index);
int hgo_undecided_rounds(hgo* h, int32_t* out, int cap);
int hgo_last_consensus_round(hgo* h, int* has);   /* value, has=0 => nil */
int hgo_last_commited_round_events(hgo* h);
int64_t hgo_consensus_transactions(hgo* h);
int64_t hgo_pending_loaded_events(hgo* h);
int64_t hgo_consensus_events(hgo* h, int64_t* out, int64_t cap); /* full order, all FindOrder calls */
void hgo_known(hgo* h, int32_t* out);   /* [participant] -> last index (-1 none) */
/* blocks produced by FindOrder, in SetBlock order */
int64_t hgo_num_blocks(hgo* h);
void hgo_block(hgo* h, int64_t b, int32_t* rr, int32_t* ntx, int32_t* tx_nil,
               int32_t* committed, uint8_t* hash32);
int64_t hgo_block_tx(hgo* h, int64_t b, int32_t t, uint8_t* out, int64_t cap);

#ifdef __cplusplus
}
#endif
#endif
