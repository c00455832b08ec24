// Synthetic gossip traces (host side of libhgx). Models the reference's
// deterministic gossip test harness: node/core_test.go:514-537 (synchronizeCores:
// `to` learns `from`'s events, then creates an event with self-parent = its head
// and other-parent = from's head, node/core.go:215-227), genesis per participant
// (node/core.go:79-85, nil transactions). See BASELINE.md "trace generator".
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <vector>

#include "hgx.h"

namespace {

struct SplitMix64 {
    uint64_t s;
    explicit SplitMix64(uint64_t seed) : s(seed) {}
    uint64_t next() {
        uint64_t z = (s += 0x9E3779B97F4A7C15ULL);
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
        return z ^ (z >> 31);
    }
    uint64_t below(uint64_t m) { return (uint64_t)(((unsigned __int128)next() * m) >> 64); }
    double unit() { return (double)(next() >> 11) * (1.0 / 9007199254740992.0); }
    void bytes32(uint8_t* out) {
        for (int w = 0; w < 4; w++) {
            uint64_t v = next();
            for (int b = 0; b < 8; b++) out[8 * w + b] = (uint8_t)(v >> (56 - 8 * b));
        }
    }
};

constexpr int64_t kT0 = 1500000000000000000LL;  // 2017-07-14T02:40:00Z

}  // namespace

extern "C" int32_t hgx_trace_gossip(int32_t n, int32_t n_silent, int64_t n_events, uint64_t seed,
                                    double stale_prob, int32_t stale_depth, int32_t* creator,
                                    int64_t* index, int64_t* self_parent, int64_t* other_parent,
                                    int64_t* timestamp_ns, uint8_t* hash, uint8_t* sig_s, int32_t* ntx,
                                    int32_t* tx_nil, int64_t* tx_seq) {
    if (n <= 0 || n_silent < 0 || n_silent >= n || n_events < 0) return HGX_ERR_INVALID;
    if (stale_depth < 1) stale_depth = 1;
    const int active = n - n_silent;
    SplitMix64 rng(seed);
    std::vector<int64_t> head(active, -1), head_idx(active, -1), txcount(active, 0);
    // per-creator recent history for stale other-parents (ring of stale_depth+1)
    const int ring = stale_depth + 1;
    std::vector<int64_t> hist((size_t)active * ring, -1);
    int64_t e = 0;
    auto emit = [&](int to, int64_t sp, int64_t op, int nt, int nil) {
        creator[e] = to;
        index[e] = head_idx[to] + 1;
        self_parent[e] = sp;
        other_parent[e] = op;
        timestamp_ns[e] = kT0 + e * 1000;
        ntx[e] = nt;
        tx_nil[e] = nil;
        tx_seq[e] = nt ? txcount[to]++ : -1;
        rng.bytes32(sig_s + 32 * e);
        rng.bytes32(hash + 32 * e);
        head[to] = e;
        head_idx[to] += 1;
        hist[(size_t)to * ring + (size_t)(head_idx[to] % ring)] = e;
        e++;
    };
    for (int p = 0; p < active && e < n_events; p++) emit(p, -1, -1, 0, 1);
    while (e < n_events) {
        int to = (int)rng.below((uint64_t)active);
        int64_t op = -1;
        if (active > 1) {
            int from = (int)rng.below((uint64_t)(active - 1));
            if (from >= to) from++;
            op = head[from];
            if (stale_prob > 0.0 && rng.unit() < stale_prob) {
                int64_t d = 1 + (int64_t)rng.below((uint64_t)stale_depth);
                int64_t k = head_idx[from] - d;
                if (k < 0) k = 0;
                int64_t g = hist[(size_t)from * ring + (size_t)(k % ring)];
                if (g >= 0 && index[g] == k) op = g;
            }
        }
        int has_tx = (int)(rng.next() & 1);
        emit(to, head[to], op, has_tx, 0);
    }
    return HGX_OK;
}

extern "C" int32_t hgx_trace_tx_payload(int32_t creator, int64_t seq, uint8_t* out, int32_t cap) {
    char buf[64];
    int l = snprintf(buf, sizeof buf, "p%03d tx %08lld", creator, (long long)seq);
    if (out && cap > 0) memcpy(out, buf, (size_t)(l < cap ? l : cap));
    return l;
}
