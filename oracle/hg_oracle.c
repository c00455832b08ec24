/*
 * hg_oracle.c -- TEST INFRASTRUCTURE: CPU restatement of the reference consensus
 * path (datatypevoid/babble v0.2.0). Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg load this; the product never does.
 *
 * Follows, function by function and loop by loop:
 *   hashgraph/hashgraph.go:39-868,1039-1055   (Hashgraph)
 *   hashgraph/roundInfo.go:39-98             (RoundInfo / RoundEvent / Trilean)
 *   hashgraph/consensus_sorter.go:5-52       (ConsensusSorter; whitening word is 0)
 *   hashgraph/block.go:11-61                 (Block, Hash)
 *   hashgraph/inmem_store.go:9-196           (InmemStore, cacheSize >= E so no eviction)
 *   common/rolling_index.go:54-68, common/errors.go:5-47 (index rules, StoreErr strings)
 * Differences that do not change results: gids instead of hex strings, witness
 * lists iterated in AddEvent order instead of Go map order (result-invariant,
 * SURVEY A.5), LRU memo caches are unbounded memo tables (pure functions).
 */
#include "hg_oracle.h"

#include <limits.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "goenc.h"

#define MAXI32 2147483647

/* ---------------- small containers ---------------- */
typedef struct { int64_t* a; int64_t n, cap; } vec64;
static void v_push(vec64* v, int64_t x) {
    if (v->n == v->cap) {
        v->cap = v->cap ? v->cap * 2 : 16;
        v->a = (int64_t*)realloc(v->a, (size_t)v->cap * sizeof(int64_t));
    }
    v->a[v->n++] = x;
}

/* open-addressing map int64 key -> uint8 value (key -1 = empty slot) */
typedef struct { int64_t* k; uint8_t* v; int64_t cap, n; } hmap;
static uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
    return z ^ (z >> 31);
}
static void hm_init(hmap* m, int64_t cap) {
    m->cap = cap; m->n = 0;
    m->k = (int64_t*)malloc((size_t)cap * sizeof(int64_t));
    m->v = (uint8_t*)malloc((size_t)cap);
    for (int64_t i = 0; i < cap; i++) m->k[i] = -1;
}
static void hm_free(hmap* m) { free(m->k); free(m->v); m->k = NULL; m->v = NULL; m->cap = m->n = 0; }
static int hm_get(const hmap* m, int64_t key, uint8_t* val) {
    uint64_t i = mix64((uint64_t)key) & (uint64_t)(m->cap - 1);
    for (;;) {
        if (m->k[i] == -1) return 0;
        if (m->k[i] == key) { *val = m->v[i]; return 1; }
        i = (i + 1) & (uint64_t)(m->cap - 1);
    }
}
static void hm_put(hmap* m, int64_t key, uint8_t val);
static void hm_grow(hmap* m) {
    hmap o = *m;
    hm_init(m, o.cap * 2);
    for (int64_t i = 0; i < o.cap; i++) if (o.k[i] != -1) hm_put(m, o.k[i], o.v[i]);
    hm_free(&o);
}
static void hm_clear(hmap* m) {
    for (int64_t i = 0; i < m->cap; i++) m->k[i] = -1;
    m->n = 0;
}
static void hm_put(hmap* m, int64_t key, uint8_t val) {
    if (2 * (m->n + 1) > m->cap) hm_grow(m);
    uint64_t i = mix64((uint64_t)key) & (uint64_t)(m->cap - 1);
    for (;;) {
        if (m->k[i] == -1) { m->k[i] = key; m->v[i] = val; m->n++; return; }
        if (m->k[i] == key) { m->v[i] = val; return; }
        i = (i + 1) & (uint64_t)(m->cap - 1);
    }
}
static int64_t pair_key(int64_t a, int64_t b) { return (a << 31) ^ b; }

/* ---------------- state ---------------- */
typedef struct {
    int exists;      /* SetRound called (InmemStore.roundCache has it) */
    int queued;      /* RoundInfo.queued (unexported) */
    vec64 events;    /* keys of RoundInfo.Events in AddEvent order */
    vec64 witnesses; /* subset with RoundEvent.Witness */
} round_info;

typedef struct { int32_t rr; int64_t first; int32_t nev; int32_t ntx; int tx_nil; int committed; uint8_t hash[32]; } block_t;

struct hgo {
    int n, sm;
    int64_t E, cap;
    int32_t* creator; int64_t* index; int64_t* sp; int64_t* op; int64_t* ts;
    uint8_t* hash; uint8_t* S; int32_t* ntx; uint8_t* txnil; int64_t* tx_first;
    int64_t* topo;
    int32_t* la; int32_t* fd;
    int32_t *w_spi, *w_opc, *w_opi;
    int32_t* round_memo; uint8_t* round_known;
    int32_t* pr_round; uint8_t* pr_root; uint8_t* pr_known;
    int8_t* famous;       /* RoundEvent.Famous of x in round(x) */
    uint8_t* in_round;    /* AddEvent done */
    int32_t* rr; int64_t* cts;
    /* tx storage */
    vec64 tx_off; vec64 tx_len; uint8_t* txblob; int64_t txblob_n, txblob_cap;
    /* participant event caches (ParticipantEventsCache / RollingIndex without roll) */
    vec64* chain; int64_t* chain_base; int64_t* last_index;
    /* Roots (root.go:62-67): Index, Round, and whether Y names an event outside the store
       (genesis: X = Y = "", Index = Round = -1). Parent codes: self-parent -1 = Root.X; other
       parent -1 = "", HGO_ROOT_Y = Root.Y (outside the store), HGO_ROOT_OTHER = the event's
       Root.Others entry (outside the store) */
    int32_t* root_index; int32_t* root_round; uint8_t* root_y_ext;
    /* Hashgraph fields (hashgraph.go:15-37) */
    vec64 undetermined;
    vec64 undecided;
    int has_lcr; int lcr; int lcre;
    int64_t consensus_tx, pending_loaded, topo_counter;
    round_info* rounds; int64_t rounds_cap; int last_round;
    hmap ss_memo;
    vec64 consensus;
    block_t* blocks; int64_t nblocks, blocks_cap;
    vec64 block_tx;  /* per block: tx indices (into tx_off/tx_len), concatenated */
    vec64 block_tx_first;
};

hgo* hgo_new(int n) {
    hgo* h = (hgo*)calloc(1, sizeof(hgo));
    h->n = n;
    h->sm = 2 * n / 3 + 1;                           /* hashgraph.go:63 */
    h->chain = (vec64*)calloc((size_t)n, sizeof(vec64));
    h->chain_base = (int64_t*)calloc((size_t)n, sizeof(int64_t));
    h->last_index = (int64_t*)malloc((size_t)n * sizeof(int64_t));
    for (int i = 0; i < n; i++) h->last_index[i] = -1;  /* RollingIndex.lastIndex = -1 */
    h->root_index = (int32_t*)malloc((size_t)n * sizeof(int32_t));
    h->root_round = (int32_t*)malloc((size_t)n * sizeof(int32_t));
    h->root_y_ext = (uint8_t*)calloc((size_t)n, 1);
    for (int i = 0; i < n; i++) { h->root_index[i] = -1; h->root_round[i] = -1; }  /* NewBaseRoot */
    v_push(&h->undecided, 0);                          /* UndecidedRounds: []int{0} (:64) */
    h->last_round = -1;                                /* InmemStore.lastRound = -1 */
    hm_init(&h->ss_memo, 1 << 12);
    return h;
}

void hgo_free(hgo* h) {
    if (!h) return;
    free(h->creator); free(h->index); free(h->sp); free(h->op); free(h->ts);
    free(h->hash); free(h->S); free(h->ntx); free(h->txnil); free(h->tx_first); free(h->topo);
    free(h->la); free(h->fd); free(h->w_spi); free(h->w_opc); free(h->w_opi);
    free(h->round_memo); free(h->round_known); free(h->pr_round); free(h->pr_root); free(h->pr_known);
    free(h->famous); free(h->in_round); free(h->rr); free(h->cts);
    free(h->tx_off.a); free(h->tx_len.a); free(h->txblob);
    for (int i = 0; i < h->n; i++) free(h->chain[i].a);
    free(h->chain); free(h->chain_base); free(h->last_index);
    free(h->root_index); free(h->root_round); free(h->root_y_ext);
    free(h->undetermined.a); free(h->undecided.a);
    for (int64_t r = 0; r < h->rounds_cap; r++) { free(h->rounds[r].events.a); free(h->rounds[r].witnesses.a); }
    free(h->rounds);
    hm_free(&h->ss_memo);
    free(h->consensus.a); free(h->blocks); free(h->block_tx.a); free(h->block_tx_first.a);
    free(h);
}

static void grow_events(hgo* h) {
    if (h->E < h->cap) return;
    int64_t c = h->cap ? h->cap * 2 : 64, n = h->n;
#define RE(p, T, k) p = (T*)realloc(p, (size_t)(c * (k)) * sizeof(T))
    RE(h->creator, int32_t, 1); RE(h->index, int64_t, 1); RE(h->sp, int64_t, 1); RE(h->op, int64_t, 1);
    RE(h->ts, int64_t, 1); RE(h->hash, uint8_t, 32); RE(h->S, uint8_t, 32); RE(h->ntx, int32_t, 1);
    RE(h->txnil, uint8_t, 1); RE(h->tx_first, int64_t, 1); RE(h->topo, int64_t, 1);
    RE(h->la, int32_t, n); RE(h->fd, int32_t, n);
    RE(h->w_spi, int32_t, 1); RE(h->w_opc, int32_t, 1); RE(h->w_opi, int32_t, 1);
    RE(h->round_memo, int32_t, 1); RE(h->round_known, uint8_t, 1);
    RE(h->pr_round, int32_t, 1); RE(h->pr_root, uint8_t, 1); RE(h->pr_known, uint8_t, 1);
    RE(h->famous, int8_t, 1); RE(h->in_round, uint8_t, 1); RE(h->rr, int32_t, 1); RE(h->cts, int64_t, 1);
#undef RE
    h->cap = c;
}

static round_info* get_round_slot(hgo* h, int r) {
    if (r >= h->rounds_cap) {
        int64_t c = h->rounds_cap ? h->rounds_cap : 16;
        while (c <= r) c *= 2;
        h->rounds = (round_info*)realloc(h->rounds, (size_t)c * sizeof(round_info));
        memset(h->rounds + h->rounds_cap, 0, (size_t)(c - h->rounds_cap) * sizeof(round_info));
        h->rounds_cap = c;
    }
    return &h->rounds[r];
}

/* store.GetEvent succeeds? */
static int known(const hgo* h, int64_t x) { return x >= 0 && x < h->E; }
/* participant event at (creator c, index k) -> gid, -1 if none */
static int64_t chain_gid(const hgo* h, int c, int64_t k) {
    int64_t off = k - h->chain_base[c];
    if (off < 0 || off >= h->chain[c].n) return -1;
    return h->chain[c].a[off];
}

/* ---------------- primitives (hashgraph.go:73-339) ---------------- */
int hgo_ancestor(hgo* h, int64_t x, int64_t y) {        /* :82-101 */
    if (x == y) return 1;
    if (!known(h, x) || !known(h, y)) return 0;
    return h->la[x * h->n + h->creator[y]] >= h->index[y];
}
int hgo_self_ancestor(hgo* h, int64_t x, int64_t y) {   /* :113-130 */
    if (x == y) return 1;
    if (!known(h, x) || !known(h, y)) return 0;
    return h->creator[x] == h->creator[y] && h->index[x] >= h->index[y];
}
int hgo_see(hgo* h, int64_t x, int64_t y) { return hgo_ancestor(h, x, y); } /* :133-138 */

int64_t hgo_oldest_self_ancestor_to_see(hgo* h, int64_t x, int64_t y) { /* :150-167 */
    if (!known(h, x) || !known(h, y)) return -1;
    int32_t a = h->fd[y * h->n + h->creator[x]];
    if (a <= h->index[x]) return chain_gid(h, h->creator[x], a);
    return -1;
}

static int strongly_see_raw(const hgo* h, int64_t x, int64_t y) { /* :179-198 */
    if (!known(h, x) || !known(h, y)) return 0;
    const int32_t* lx = h->la + x * h->n;
    const int32_t* fy = h->fd + y * h->n;
    int c = 0;
    for (int i = 0; i < h->n; i++) if (lx[i] >= fy[i]) c++;
    return c >= h->sm;
}
/* The memo is a bounded cache like the reference's stronglySeeCache (an LRU of cacheSize entries,
 * hashgraph.go:170-177): StronglySee is a pure function of the DAG, so dropping entries changes no
 * result. Bounded at 2^25 entries (~600 MB) so a 10 M-event trace fits the build container. */
#ifndef HGO_SS_MEMO_MAX
#define HGO_SS_MEMO_MAX ((int64_t)1 << 25)
#endif
int hgo_strongly_see(hgo* h, int64_t x, int64_t y) {    /* :170-177 (memoised) */
    uint8_t v;
    int64_t key = pair_key(x + 2, y + 2);
    if (hm_get(&h->ss_memo, key, &v)) return v;
    int s = strongly_see_raw(h, x, y);
    if (h->ss_memo.n >= HGO_SS_MEMO_MAX) hm_clear(&h->ss_memo);
    hm_put(&h->ss_memo, key, (uint8_t)s);
    return s;
}

int hgo_round(hgo* h, int64_t x);

int hgo_parent_round(hgo* h, int64_t x, int* is_root) {  /* :202-262 */
    if (known(h, x) && h->pr_known[x]) { *is_root = h->pr_root[x]; return h->pr_round[x]; }
    int res_round = -1, res_root = 0;                    /* NewBaseParentRoundInfo */
    if (!known(h, x)) { *is_root = 0; return -1; }
    const int c = h->creator[x];
    const int rr0 = h->root_round[c];
    int spRound, spRoot, opRound = -1, opRoot = 0;
    if (h->sp[x] == -1) { spRound = rr0; spRoot = 1; }    /* SelfParent == Root.X */
    else { spRound = hgo_round(h, h->sp[x]); spRoot = 0; }
    if (known(h, h->op[x])) opRound = hgo_round(h, h->op[x]);
    else if ((h->op[x] == -1 && !h->root_y_ext[c]) || h->op[x] == HGO_ROOT_Y) { opRound = rr0; opRoot = 1; }
    else if (h->op[x] == HGO_ROOT_OTHER) { opRound = rr0; opRoot = 0; }   /* Root.Others */
    res_round = spRound; res_root = spRoot;
    if (spRound < opRound) { res_round = opRound; res_root = opRoot; }
    h->pr_known[x] = 1; h->pr_round[x] = res_round; h->pr_root[x] = (uint8_t)res_root;
    *is_root = res_root;
    return res_round;
}

static const vec64* round_witnesses(hgo* h, int r) {     /* InmemStore.RoundWitnesses */
    static const vec64 empty = {0, 0, 0};
    if (r < 0 || r >= h->rounds_cap || !h->rounds[r].exists) return &empty;
    return &h->rounds[r].witnesses;
}

int hgo_round_inc(hgo* h, int64_t x) {                   /* :285-305 */
    int root;
    int pr = hgo_parent_round(h, x, &root);
    if (root) return 1;
    const vec64* ws = round_witnesses(h, pr);
    int c = 0;
    for (int64_t k = 0; k < ws->n; k++) if (hgo_strongly_see(h, x, ws->a[k])) c++;
    return c >= h->sm;
}

int hgo_round(hgo* h, int64_t x) {                       /* :320-339 (memoised) */
    if (known(h, x) && h->round_known[x]) return h->round_memo[x];
    int root;
    int r = hgo_parent_round(h, x, &root);
    if (hgo_round_inc(h, x)) r++;
    if (known(h, x)) { h->round_known[x] = 1; h->round_memo[x] = r; }
    return r;
}

int hgo_witness(hgo* h, int64_t x) {                     /* :265-282 */
    if (!known(h, x)) return 0;
    /* SelfParent == Root.X && OtherParent == Root.Y */
    if (h->sp[x] == -1 && ((h->op[x] == -1 && !h->root_y_ext[h->creator[x]]) || h->op[x] == HGO_ROOT_Y)) return 1;
    return hgo_round(h, x) > hgo_round(h, h->sp[x]);
}

/* ---------------- InsertEvent (hashgraph.go:356-530) ---------------- */
static void set_err(char* err, int errlen, const char* msg) {
    if (err && errlen > 0) { strncpy(err, msg, (size_t)errlen - 1); err[errlen - 1] = 0; }
}
/* Go string(int) -> UTF-8 of the rune (rolling_index.go passes string(index)) */
static int go_rune_string(int64_t v, char* out) {
    uint32_t r = (v < 0 || v > 0x10FFFF || (v >= 0xD800 && v <= 0xDFFF)) ? 0xFFFD : (uint32_t)v;
    if (r < 0x80) { out[0] = (char)r; return 1; }
    if (r < 0x800) { out[0] = (char)(0xC0 | (r >> 6)); out[1] = (char)(0x80 | (r & 63)); return 2; }
    if (r < 0x10000) { out[0] = (char)(0xE0 | (r >> 12)); out[1] = (char)(0x80 | ((r >> 6) & 63));
                       out[2] = (char)(0x80 | (r & 63)); return 3; }
    out[0] = (char)(0xF0 | (r >> 18)); out[1] = (char)(0x80 | ((r >> 12) & 63));
    out[2] = (char)(0x80 | ((r >> 6) & 63)); out[3] = (char)(0x80 | (r & 63)); return 4;
}

int hgo_insert(hgo* h, int creator, int64_t index, int64_t sp, int64_t op, int64_t ts_ns,
               const uint8_t* hash32, const uint8_t* s32, int ntx, int tx_nil,
               const uint8_t* tx_data, const int32_t* tx_len, char* err, int errlen) {
    char msg[256];
    const int n = h->n;
    /* event.Verify(): signatures are not modelled (ingest front-end) */
    /* CheckSelfParent (:404-420): LastFrom(creator) */
    if (creator < 0 || creator >= n) {
        snprintf(msg, sizeof msg, "CheckSelfParent: %d, Not Found", creator);
        set_err(err, errlen, msg);
        return 1; /* KeyNotFound */
    }
    int64_t last = h->chain[creator].n ? h->chain[creator].a[h->chain[creator].n - 1] : -1;
    if (sp != last) {
        set_err(err, errlen, "CheckSelfParent: Self-parent not last known event by creator");
        return 100;
    }
    /* CheckOtherParent (:423-445): unknown other-parents only through the creator's Root:
       Root.X == SelfParent && Root.Y == OtherParent, or Root.Others[event] == OtherParent */
    if (op != -1 && !known(h, op)) {
        const int via_root = (op == HGO_ROOT_Y && sp == -1 && h->root_y_ext[creator]) || op == HGO_ROOT_OTHER;
        if (!via_root) {
            set_err(err, errlen, "CheckOtherParent: Other-parent not known");
            return 101;
        }
    }
    /* topologicalIndex++ (:373-374) is consumed even if SetEvent fails below */
    int64_t topo = h->topo_counter++;
    /* InmemStore.SetEvent -> RollingIndex.Add (rolling_index.go:54-68): checked before storing */
    int64_t li = h->last_index[creator];
    if (index <= li || (li >= 0 && index > li + 1)) {
        char rs[8]; int l = go_rune_string(index, rs); rs[l] = 0;
        snprintf(msg, sizeof msg, "SetEvent: %s, %s", rs, index <= li ? "Passed Index" : "Skipped Index");
        set_err(err, errlen, msg);
        return index <= li ? 3 : 4;
    }
    grow_events(h);
    int64_t x = h->E;
    h->creator[x] = creator; h->index[x] = index; h->sp[x] = sp; h->op[x] = op; h->ts[x] = ts_ns;
    memcpy(h->hash + 32 * x, hash32, 32); memcpy(h->S + 32 * x, s32, 32);
    h->ntx[x] = ntx; h->txnil[x] = (uint8_t)(tx_nil != 0); h->topo[x] = topo;
    h->tx_first[x] = h->tx_off.n;
    int64_t pos = 0;
    for (int t = 0; t < ntx; t++) {
        int32_t l = tx_len[t];
        if (h->txblob_n + l > h->txblob_cap) {
            h->txblob_cap = (h->txblob_cap + l) * 2 + 1024;
            h->txblob = (uint8_t*)realloc(h->txblob, (size_t)h->txblob_cap);
        }
        memcpy(h->txblob + h->txblob_n, tx_data + pos, (size_t)l);
        v_push(&h->tx_off, h->txblob_n); v_push(&h->tx_len, l);
        h->txblob_n += l; pos += l;
    }
    h->round_known[x] = 0; h->pr_known[x] = 0; h->famous[x] = 0; h->in_round[x] = 0;
    h->rr[x] = -1; h->cts[x] = 0;
    /* SetWireInfo (:532-567) */
    h->w_spi[x] = (sp == -1) ? h->root_index[creator] : (int32_t)h->index[sp];
    h->w_opc[x] = known(h, op) ? h->creator[op] : -1;
    h->w_opi[x] = known(h, op) ? (int32_t)h->index[op] : -1;
    /* InitEventCoordinates (:448-499) */
    int32_t* la = h->la + x * n;
    int32_t* fd = h->fd + x * n;
    for (int i = 0; i < n; i++) fd[i] = MAXI32;
    int spk = known(h, sp), opk = known(h, op);
    if (!spk && !opk) { for (int i = 0; i < n; i++) la[i] = -1; }
    else if (!spk) memcpy(la, h->la + op * n, (size_t)n * 4);
    else if (!opk) memcpy(la, h->la + sp * n, (size_t)n * 4);
    else {
        memcpy(la, h->la + sp * n, (size_t)n * 4);
        const int32_t* lo = h->la + op * n;
        for (int i = 0; i < n; i++) if (la[i] < lo[i]) la[i] = lo[i];
    }
    fd[creator] = (int32_t)index;
    la[creator] = (int32_t)index;
    /* Store.SetEvent (:386): participant cache */
    if (h->chain[creator].n == 0) h->chain_base[creator] = index;
    v_push(&h->chain[creator], x);
    h->last_index[creator] = index;
    h->E++;
    /* UpdateAncestorFirstDescendant (:502-530) */
    for (int i = 0; i < n; i++) {
        int64_t ah = (la[i] >= 0) ? chain_gid(h, i, la[i]) : -1;
        while (ah != -1) {
            int32_t* afd = h->fd + ah * n;
            if (afd[creator] == MAXI32) {
                afd[creator] = (int32_t)index;
                ah = h->sp[ah];
            } else break;
        }
    }
    v_push(&h->undetermined, x);
    /* IsLoaded (event.go:119-126) */
    if (index == 0 || (!tx_nil && ntx > 0)) h->pending_loaded++;
    return 0;
}

/* ---------------- Reset (hashgraph.go:877-895, inmem_store.go:184-192) ---------------- */
int hgo_reset(hgo* h, const int32_t* root_index, const int32_t* root_round, const uint8_t* root_y_ext) {
    /* Store.Reset: new roots; event, round and consensus caches and the participant
       RollingIndexes cleared; lastRound = -1. The block cache is kept. */
    for (int i = 0; i < h->n; i++) {
        h->root_index[i] = root_index[i];
        h->root_round[i] = root_round[i];
        h->root_y_ext[i] = root_y_ext[i] ? 1 : 0;
        h->chain[i].n = 0;
        h->chain_base[i] = 0;
        h->last_index[i] = -1;
    }
    h->E = 0;
    for (int64_t r = 0; r < h->rounds_cap; r++) {
        h->rounds[r].exists = 0; h->rounds[r].queued = 0;
        h->rounds[r].events.n = 0; h->rounds[r].witnesses.n = 0;
    }
    h->last_round = -1;
    hm_free(&h->ss_memo);
    hm_init(&h->ss_memo, 1 << 12);
    h->consensus.n = 0;
    /* Hashgraph.Reset: UndeterminedEvents, UndecidedRounds (empty, not [0]), PendingLoadedEvents,
       topologicalIndex and the memo caches; LastConsensusRound, LastCommitedRoundEvents and
       ConsensusTransactions are kept */
    h->undetermined.n = 0;
    h->undecided.n = 0;
    h->pending_loaded = 0;
    h->topo_counter = 0;
    return 0;
}

void hgo_get_root(hgo* h, int p, int32_t* index, int32_t* round, int* y_ext) {
    *index = h->root_index[p];
    *round = h->root_round[p];
    *y_ext = h->root_y_ext[p];
}

/* ---------------- GetFrame (hashgraph.go:897-995) ----------------
   Roots: X = the root event's self-parent (gid, or -1 = the participant's current Root.X),
   Y = its other-parent (gid, -1 = "", HGO_ROOT_Y / HGO_ROOT_OTHER = outside the store as
   inserted), Index = Index - 1, Round = Round(self-parent). Others: (event, other-parent)
   pairs for frame events whose other-parent is not an earlier frame event. Events: gids in
   topological (= insertion) order. Returns 0, or 1 (GetRound(LastConsensusRound) not found). */
static int cmp_i64(const void* a, const void* b);

int hgo_get_frame(hgo* h, int64_t* ev_out, int64_t ev_cap, int64_t* n_ev, int64_t* root_x, int64_t* root_y,
                  int32_t* root_index, int32_t* root_round, int64_t* oth_ev, int64_t* oth_op, int64_t oth_cap,
                  int64_t* n_oth) {
    const int n = h->n;
    const int lcr = h->has_lcr ? h->lcr : 0;
    if (lcr < 0 || lcr >= h->rounds_cap || !h->rounds[lcr].exists) return 1;
    vec64 evs = {0, 0, 0};
    uint8_t* has_root = (uint8_t*)calloc((size_t)n, 1);
    const vec64* ws = &h->rounds[lcr].witnesses;
    for (int64_t k = 0; k < ws->n; k++) {
        const int64_t w = ws->a[k];
        const int c = h->creator[w];
        v_push(&evs, w);
        has_root[c] = 1;
        root_x[c] = h->sp[w];
        root_y[c] = h->op[w];
        root_index[c] = (int32_t)(h->index[w] - 1);
        root_round[c] = hgo_round(h, h->sp[w]);
        /* ParticipantEvents(creator, w.Index()): the creator's events after w */
        for (int64_t j = h->index[w] + 1 - h->chain_base[c]; j < h->chain[c].n; j++) v_push(&evs, h->chain[c].a[j]);
    }
    for (int p = 0; p < n; p++) {
        if (has_root[p]) continue;
        if (h->chain[p].n == 0) {   /* LastFrom is the Root: keep it */
            root_x[p] = -1;
            root_y[p] = h->root_y_ext[p] ? HGO_ROOT_Y : -1;
            root_index[p] = h->root_index[p];
            root_round[p] = h->root_round[p];
        } else {
            const int64_t ev = h->chain[p].a[h->chain[p].n - 1];
            v_push(&evs, ev);
            root_x[p] = h->sp[ev];
            root_y[p] = h->op[ev];
            root_index[p] = (int32_t)(h->index[ev] - 1);
            root_round[p] = hgo_round(h, h->sp[ev]);
        }
    }
    qsort(evs.a, (size_t)evs.n, sizeof(int64_t), cmp_i64);   /* ByTopologicalOrder */
    uint8_t* treated = (uint8_t*)calloc((size_t)(h->E + 1), 1);
    int64_t no = 0;
    for (int64_t k = 0; k < evs.n; k++) {
        const int64_t ev = evs.a[k];
        treated[ev] = 1;
        const int64_t op = h->op[ev];
        if (op == -1) continue;
        if (!(known(h, op) && treated[op]) && h->sp[ev] != root_x[h->creator[ev]]) {
            if (no < oth_cap) { oth_ev[no] = ev; oth_op[no] = op; }
            no++;
        }
    }
    *n_oth = no;
    *n_ev = evs.n;
    for (int64_t k = 0; k < evs.n && k < ev_cap; k++) ev_out[k] = evs.a[k];
    free(evs.a);
    free(has_root);
    free(treated);
    return 0;
}

/* ---------------- DivideRounds (hashgraph.go:616-646) ---------------- */
int hgo_divide_rounds(hgo* h) {
    for (int64_t k = 0; k < h->undetermined.n; k++) {
        int64_t x = h->undetermined.a[k];
        int r = hgo_round(h, x);
        int w = hgo_witness(h, x);
        round_info* ri = get_round_slot(h, r);  /* GetRound miss => fresh RoundInfo, queued=false */
        if (!ri->queued) { v_push(&h->undecided, r); ri->queued = 1; }
        if (!h->in_round[x]) {                   /* RoundInfo.AddEvent (roundInfo.go:39-46) */
            h->in_round[x] = 1;
            v_push(&ri->events, x);
            if (w) v_push(&ri->witnesses, x);
            h->famous[x] = 0;
        }
        ri->exists = 1;                          /* SetRound */
        if (r > h->last_round) h->last_round = r;
    }
    return 0;
}

/* ---------------- DecideFame (hashgraph.go:649-750) ---------------- */
static int middle_bit(const hgo* h, int64_t y) {          /* :1039-1048 */
    return h->hash[32 * y + 16] != 0;
}

static int witnesses_decided(const hgo* h, int r) {       /* roundInfo.go:64-71 */
    if (r < 0 || r >= h->rounds_cap || !h->rounds[r].exists) return 1; /* empty RoundInfo */
    const vec64* ws = &h->rounds[r].witnesses;
    for (int64_t k = 0; k < ws->n; k++) if (h->famous[ws->a[k]] == 0) return 0;
    return 1;
}
static int round_events(const hgo* h, int r) {             /* InmemStore.RoundEvents */
    if (r < 0 || r >= h->rounds_cap || !h->rounds[r].exists) return 0;
    return (int)h->rounds[r].events.n;
}

int hgo_decide_fame(hgo* h, char* err, int errlen) {
    hmap votes;                                          /* [y][x] => vote */
    hm_init(&votes, 1 << 10);
    int64_t nur = h->undecided.n;
    int32_t* ur = (int32_t*)malloc((size_t)(nur + 1) * sizeof(int32_t));
    for (int64_t p = 0; p < nur; p++) ur[p] = (int32_t)h->undecided.a[p];
    uint8_t* decided_pos = (uint8_t*)calloc((size_t)(nur + 1), 1);
    int rc = 0;
    for (int64_t pos = 0; pos < nur; pos++) {
        int i = ur[pos];
        if (i < 0 || i >= h->rounds_cap || !h->rounds[i].exists) {  /* GetRound error */
            char msg[64]; snprintf(msg, sizeof msg, "%d, Not Found", i);
            set_err(err, errlen, msg);
            rc = 1;
            break;
        }
        round_info* ri = &h->rounds[i];
        for (int64_t xi = 0; xi < ri->witnesses.n; xi++) {
            int64_t x = ri->witnesses.a[xi];
            if (h->famous[x] != 0) continue;             /* IsDecided */
            int done = 0;
            for (int j = i + 1; j <= h->last_round && !done; j++) {
                const vec64* wj = round_witnesses(h, j);
                for (int64_t yi = 0; yi < wj->n; yi++) {
                    int64_t y = wj->a[yi];
                    int diff = j - i;
                    if (diff == 1) {
                        hm_put(&votes, pair_key(y, x), (uint8_t)hgo_see(h, y, x));
                    } else {
                        const vec64* wp = round_witnesses(h, j - 1);
                        int yays = 0, nays = 0;
                        for (int64_t wi = 0; wi < wp->n; wi++) {
                            int64_t w = wp->a[wi];
                            if (!hgo_strongly_see(h, y, w)) continue;
                            uint8_t v = 0;
                            hm_get(&votes, pair_key(w, x), &v);   /* missing => false */
                            if (v) yays++; else nays++;
                        }
                        int v = 0, t = nays;
                        if (yays >= nays) { v = 1; t = yays; }
                        if (diff % h->n > 0) {           /* math.Mod(diff, n) > 0: normal round */
                            if (t >= h->sm) {
                                h->famous[x] = v ? 1 : 2;          /* SetFame */
                                hm_put(&votes, pair_key(y, x), (uint8_t)v);
                                done = 1;
                                break;                   /* break X */
                            } else {
                                hm_put(&votes, pair_key(y, x), (uint8_t)v);
                            }
                        } else {                          /* coin round */
                            if (t >= h->sm) hm_put(&votes, pair_key(y, x), (uint8_t)v);
                            else hm_put(&votes, pair_key(y, x), (uint8_t)middle_bit(h, y));
                        }
                    }
                }
            }
        }
        /* votes[y][x] is only ever read for the x it was written for (:671-716), and every x of
         * round i is done here: Go's one map per call, restated per round so that a call over
         * thousands of rounds holds one round's votes (same results) */
        hm_free(&votes);
        hm_init(&votes, 1 << 10);
        if (witnesses_decided(h, i)) {
            decided_pos[pos] = 1;
            if (!h->has_lcr || i > h->lcr) {            /* setLastConsensusRound (:743-750) */
                h->has_lcr = 1; h->lcr = i;
                h->lcre = round_events(h, i - 1);
            }
        }
        /* SetRound(i, roundInfo): already in place */
    }
    /* deferred updateUndecidedRounds (:733-741): drop every copy of a decided round */
    vec64 nu = {0, 0, 0};
    for (int64_t p = 0; p < nur; p++) {
        int r = ur[p], dec = 0;
        for (int64_t q = 0; q < nur; q++) if (decided_pos[q] && ur[q] == r) { dec = 1; break; }
        if (!dec) v_push(&nu, r);
    }
    free(h->undecided.a);
    h->undecided = nu;
    free(ur); free(decided_pos);
    hm_free(&votes);
    return rc;
}

/* ---------------- DecideRoundReceived / FindOrder (hashgraph.go:753-868) ---------------- */
static int cmp_i64(const void* a, const void* b) {
    int64_t x = *(const int64_t*)a, y = *(const int64_t*)b;
    return x < y ? -1 : x > y;
}

int hgo_decide_round_received(hgo* h, char* err, int errlen) {
    const int n = h->n;
    int64_t* t = (int64_t*)malloc((size_t)(n + 1) * sizeof(int64_t));
    for (int64_t k = 0; k < h->undetermined.n; k++) {
        int64_t x = h->undetermined.a[k];
        int r = hgo_round(h, x);
        for (int i = r + 1; i <= h->last_round; i++) {
            if (h->undecided.n == 0) {  /* Go: h.UndecidedRounds[0] index out of range */
                set_err(err, errlen, "runtime error: index out of range");
                free(t);
                return 2;
            }
            if (!(witnesses_decided(h, i) && h->undecided.a[0] > i)) continue;
            const vec64* ws = round_witnesses(h, i);
            int64_t nfw = 0, ns = 0;
            for (int64_t wi = 0; wi < ws->n; wi++) {
                int64_t w = ws->a[wi];
                if (h->famous[w] != 1) continue;          /* FamousWitnesses */
                nfw++;
                if (hgo_see(h, w, x)) {
                    int64_t a = hgo_oldest_self_ancestor_to_see(h, w, x);
                    t[ns++] = (a >= 0) ? h->ts[a] : INT64_MIN; /* MedianTimestamp GetEvent("") => zero Time */
                }
            }
            if (ns > nfw / 2) {
                h->rr[x] = i;                              /* SetRoundReceived */
                qsort(t, (size_t)ns, sizeof(int64_t), cmp_i64);  /* sort.Sort(ByTimestamp) */
                h->cts[x] = t[ns / 2];
                break;
            }
        }
    }
    free(t);
    return 0;
}

static const hgo* g_sort_h;
static int cmp_consensus(const void* pa, const void* pb) { /* consensus_sorter.go:23-43 */
    const hgo* h = g_sort_h;
    int64_t a = *(const int64_t*)pa, b = *(const int64_t*)pb;
    if (h->rr[a] != h->rr[b]) return h->rr[a] < h->rr[b] ? -1 : 1;
    if (h->cts[a] != h->cts[b]) return h->cts[a] < h->cts[b] ? -1 : 1;
    return memcmp(h->S + 32 * a, h->S + 32 * b, 32);      /* S XOR 0, big-endian Cmp */
}

int hgo_find_order(hgo* h, char* err, int errlen) {
    int rc = hgo_decide_round_received(h, err, errlen);
    if (rc) return rc;
    vec64 newc = {0, 0, 0}, newu = {0, 0, 0};
    for (int64_t k = 0; k < h->undetermined.n; k++) {
        int64_t x = h->undetermined.a[k];
        if (h->rr[x] >= 0) v_push(&newc, x); else v_push(&newu, x);
    }
    free(h->undetermined.a);
    h->undetermined = newu;
    g_sort_h = h;
    if (newc.n > 1) qsort(newc.a, (size_t)newc.n, sizeof(int64_t), cmp_consensus);
    /* block assembly (:826-854): one Block per rr in first-appearance order */
    int64_t first_block = h->nblocks;
    for (int64_t k = 0; k < newc.n; k++) {
        int64_t e = newc.a[k];
        v_push(&h->consensus, e);                          /* AddConsensusEvent */
        h->consensus_tx += h->ntx[e];
        if (h->index[e] == 0 || (!h->txnil[e] && h->ntx[e] > 0)) h->pending_loaded--;
        /* blockMap[rr]: newc is sorted by rr, so an existing block is the last one */
        int64_t b = (h->nblocks > first_block && h->blocks[h->nblocks - 1].rr == h->rr[e])
                        ? h->nblocks - 1 : -1;
        if (b < 0) {
            if (h->nblocks == h->blocks_cap) {
                h->blocks_cap = h->blocks_cap ? 2 * h->blocks_cap : 16;
                h->blocks = (block_t*)realloc(h->blocks, (size_t)h->blocks_cap * sizeof(block_t));
            }
            b = h->nblocks++;
            block_t* B = &h->blocks[b];
            memset(B, 0, sizeof(*B));
            B->rr = h->rr[e]; B->first = k;
            B->tx_nil = h->txnil[e];                       /* NewBlock(rr, e.Transactions()) */
            v_push(&h->block_tx_first, h->block_tx.n);
        }
        block_t* B = &h->blocks[b];
        B->nev++;
        for (int t = 0; t < h->ntx[e]; t++) v_push(&h->block_tx, h->tx_first[e] + t);
        B->ntx += h->ntx[e];
        if (h->ntx[e] > 0) B->tx_nil = 0;                  /* append of >=1 element => non-nil */
    }
    /* SetBlock + commit; compute Block.Hash (block.go:44-53) */
    for (int64_t b = first_block; b < h->nblocks; b++) {
        block_t* B = &h->blocks[b];
        int64_t tf = h->block_tx_first.a[b];
        const uint8_t** txp = (const uint8_t**)malloc((size_t)(B->ntx + 1) * sizeof(uint8_t*));
        size_t* txl = (size_t*)malloc((size_t)(B->ntx + 1) * sizeof(size_t));
        for (int t = 0; t < B->ntx; t++) {
            int64_t ti = h->block_tx.a[tf + t];
            txp[t] = h->txblob + h->tx_off.a[ti];
            txl[t] = (size_t)h->tx_len.a[ti];
        }
        size_t cap = goenc_block_json_bound(B->ntx, txl);
        char* js = (char*)malloc(cap);
        size_t len = goenc_block_json(B->rr, B->ntx, txp, txl, B->tx_nil, js);
        goenc_sha256((const uint8_t*)js, len, B->hash);
        B->committed = B->ntx > 0;                          /* commitCh only if len(tx) > 0 */
        free(js); free(txp); free(txl);
    }
    free(newc.a);
    return 0;
}

/* ---------------- getters ---------------- */
int64_t hgo_num_events(hgo* h) { return h->E; }
int hgo_super_majority(hgo* h) { return h->sm; }
int hgo_last_round(hgo* h) { return h->last_round; }
int hgo_round_event_count(hgo* h, int r) { return round_events(h, r); }
int hgo_round_witnesses(hgo* h, int r, int64_t* out, int cap) {
    const vec64* ws = round_witnesses(h, r);
    int m = (int)ws->n < cap ? (int)ws->n : cap;
    for (int k = 0; k < m; k++) out[k] = ws->a[k];
    return (int)ws->n;
}
int hgo_famous(hgo* h, int64_t x) { return known(h, x) ? h->famous[x] : 0; }
int hgo_round_received(hgo* h, int64_t x) { return known(h, x) ? h->rr[x] : -1; }
int64_t hgo_consensus_timestamp(hgo* h, int64_t x) { return known(h, x) ? h->cts[x] : 0; }
void hgo_coords(hgo* h, int64_t x, int32_t* la, int32_t* fd) {
    memcpy(la, h->la + x * h->n, (size_t)h->n * 4);
    memcpy(fd, h->fd + x * h->n, (size_t)h->n * 4);
}
void hgo_wire_info(hgo* h, int64_t x, int32_t* spi, int32_t* opc, int32_t* opi) {
    *spi = h->w_spi[x]; *opc = h->w_opc[x]; *opi = h->w_opi[x];
}
int hgo_undecided_rounds(hgo* h, int32_t* out, int cap) {
    int m = (int)h->undecided.n < cap ? (int)h->undecided.n : cap;
    for (int k = 0; k < m; k++) out[k] = (int32_t)h->undecided.a[k];
    return (int)h->undecided.n;
}
int hgo_last_consensus_round(hgo* h, int* has) { *has = h->has_lcr; return h->lcr; }
int hgo_last_commited_round_events(hgo* h) { return h->lcre; }
int64_t hgo_consensus_transactions(hgo* h) { return h->consensus_tx; }
int64_t hgo_pending_loaded_events(hgo* h) { return h->pending_loaded; }
int64_t hgo_consensus_events(hgo* h, int64_t* out, int64_t cap) {
    int64_t m = h->consensus.n < cap ? h->consensus.n : cap;
    if (out) memcpy(out, h->consensus.a, (size_t)m * sizeof(int64_t));
    return h->consensus.n;
}
void hgo_known(hgo* h, int32_t* out) {
    for (int i = 0; i < h->n; i++) out[i] = (int32_t)h->last_index[i];
}
int64_t hgo_num_blocks(hgo* h) { return h->nblocks; }
void hgo_block(hgo* h, int64_t b, int32_t* rr, int32_t* ntx, int32_t* tx_nil, int32_t* committed,
               uint8_t* hash32) {
    block_t* B = &h->blocks[b];
    *rr = B->rr; *ntx = B->ntx; *tx_nil = B->tx_nil; *committed = B->committed;
    memcpy(hash32, B->hash, 32);
}
int64_t hgo_block_tx(hgo* h, int64_t b, int32_t t, uint8_t* out, int64_t cap) {
    int64_t ti = h->block_tx.a[h->block_tx_first.a[b] + t];
    int64_t l = h->tx_len.a[ti];
    if (out) memcpy(out, h->txblob + h->tx_off.a[ti], (size_t)(l < cap ? l : cap));
    return l;
}

/* Core.Sync-style batch (node/core.go:199-211): hgo_insert for events 0..m-1 in order,
 * stopping at the first rejected event. Payloads of event k are the next ntx[k] entries of
 * tx_len, their bytes consecutive in tx_blob. Returns the number of events inserted; the
 * error of the rejected event (if any) is in err / *rc. */
int64_t hgo_insert_batch(hgo* h, int64_t m, const int32_t* creator, const int64_t* index, const int64_t* sp,
                         const int64_t* op, const int64_t* ts, const uint8_t* hash, const uint8_t* S,
                         const int32_t* ntx, const int32_t* tx_nil, const uint8_t* tx_blob, const int32_t* tx_len,
                         int* rc, char* err, int errlen) {
    int64_t tpos = 0, bpos = 0;
    *rc = 0;
    for (int64_t k = 0; k < m; k++) {
        const int r = hgo_insert(h, creator[k], index[k], sp[k], op[k], ts[k], hash + 32 * k, S + 32 * k, ntx[k],
                                 tx_nil[k], tx_blob ? tx_blob + bpos : NULL, tx_len ? tx_len + tpos : NULL, err,
                                 errlen);
        if (r) {
            *rc = r;
            return k;
        }
        for (int t = 0; t < ntx[k]; t++) bpos += tx_len[tpos + t];
        tpos += ntx[k];
    }
    return m;
}
