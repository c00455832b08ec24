// Engine host code: device allocation, per-call orchestration of the kernels,
// D2H of the small per-round tables the Go-semantics bookkeeping needs.
#include "hgx_engine.h"

#include <algorithm>
#include <array>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>

namespace hgx {

#define HGX_TRY(x)                              \
    do {                                        \
        hipError_t _e = (x);                    \
        if (_e != hipSuccess) return _e;        \
    } while (0)

template <typename T>
hipError_t DBuf<T>::alloc(size_t count) {
    release();
    if (count == 0) count = 1;
    hipError_t e = hipMalloc((void**)&p, count * sizeof(T));
    if (e == hipSuccess) n = count; else p = nullptr;
    return e;
}

template <typename T>
hipError_t DBuf<T>::grow_copy(size_t count, size_t keep, hipStream_t s) {
    if (count <= n) return hipSuccess;
    T* q = nullptr;
    HGX_TRY(hipMalloc((void**)&q, count * sizeof(T)));
    if (p && keep) {
        HGX_TRY(hipMemcpyAsync(q, p, std::min(keep, n) * sizeof(T), hipMemcpyDeviceToDevice, s));
        HGX_TRY(hipStreamSynchronize(s));
    }
    if (p) (void)hipFree(p);
    p = q;
    n = count;
    return hipSuccess;
}

template <typename T>
void DBuf<T>::release() {
    if (p && own) (void)hipFree(p);
    p = nullptr;
    n = 0;
    own = true;
}

template struct DBuf<int32_t>;
template struct DBuf<int64_t>;
template struct DBuf<uint8_t>;
template struct DBuf<int8_t>;
template struct DBuf<uint32_t>;
template struct DBuf<uint64_t>;
template struct DBuf<unsigned long long>;

static int bitlen(uint64_t v) {
    int b = 0;
    while (v) { b++; v >>= 1; }
    return b;
}

// ---- chain-sharded group -------------------------------------------------
bool ShardGroup::wait() {
    std::unique_lock<std::mutex> lk(m);
    if (broken) return false;
    const uint64_t g = gen;
    if (++count == W) {
        count = 0;
        gen++;
        cv.notify_all();
        return true;
    }
    // (a shard that failed breaks the barrier; the time limit only guards against a lost thread)
    if (!cv.wait_for(lk, std::chrono::seconds(120), [&] { return gen != g || broken; })) broken = true;
    if (broken) cv.notify_all();
    return !broken;
}

void ShardGroup::fail() {
    std::lock_guard<std::mutex> lk(m);
    broken = true;
    cv.notify_all();
}

void ShardGroup::rearm() {
    std::lock_guard<std::mutex> lk(m);
    broken = false;
    count = 0;
}

hipError_t Engine::share_round_rows(int32_t r_a, int32_t r_b) {
    if (!grp || grp->W < 2) return hipSuccess;
    const int lo = grp->c_split[shard], hi = grp->c_split[shard + 1];
    if (hi <= lo || r_b < r_a) return hipSuccess;
    const int32_t r_s = std::min(r_b, r_cap - 1);   // rows of the [r_cap x C] tables
    const size_t Cz = (size_t)C, w = (size_t)(hi - lo);
    for (int k = 0; k < grp->W; k++) {
        if (k == shard) continue;
        Engine* q = grp->eng[k];
        // the peer's tables have the same shapes (identical calls, identical growth)
        if (q->r_cap != r_cap) return hipErrorInvalidValue;
        HGX_TRY(hipMemcpy2DAsync(q->Bm.p + (size_t)r_a * Cz + lo, Cz * 4, Bm.p + (size_t)r_a * Cz + lo, Cz * 4, w * 4,
                                 (size_t)(r_b - r_a + 1), hipMemcpyDefault, stream));
        if (r_s >= r_a) {
            const size_t rows = (size_t)(r_s - r_a + 1);
            HGX_TRY(hipMemcpy2DAsync(q->Smat.p + ((size_t)r_a * Cz + lo) * nw, Cz * nw * 8, Smat.p + ((size_t)r_a * Cz + lo) * nw,
                                     Cz * nw * 8, w * nw * 8, rows, hipMemcpyDefault, stream));
            HGX_TRY(hipMemcpy2DAsync(q->wstat.p + (size_t)r_a * Cz + lo, Cz, wstat.p + (size_t)r_a * Cz + lo, Cz, w, rows,
                                     hipMemcpyDefault, stream));
            HGX_TRY(hipMemcpy2DAsync(q->wflag.p + (size_t)r_a * Cz + lo, Cz, wflag.p + (size_t)r_a * Cz + lo, Cz, w, rows,
                                     hipMemcpyDefault, stream));
        }
    }
    return hipStreamSynchronize(stream);
}

Engine::~Engine() {
    if (pay_thread.joinable()) pay_thread.join();
    if (stream2) (void)hipStreamSynchronize(stream2);
    if (ev_pay) (void)hipEventDestroy(ev_pay);
    if (stream2) (void)hipStreamDestroy(stream2);
    if (stream) (void)hipStreamSynchronize(stream);
    for (auto e : kev) (void)hipEventDestroy(e);
    if (ph0) (void)hipEventDestroy(ph0);
    if (ph1) (void)hipEventDestroy(ph1);
    if (ph2) (void)hipEventDestroy(ph2);
    if (h_small) (void)hipHostFree(h_small);
    if (h_pack) (void)hipHostFree(h_pack);
    if (h_stage) (void)hipHostFree(h_stage);
    if (h_ins) (void)hipHostFree(h_ins);
    if (h_cpar) (void)hipHostFree(h_cpar);
    if (h_flag) (void)hipHostFree(h_flag);
    if (h_segc) (void)hipHostFree(h_segc);
    if (stream_o) (void)hipStreamSynchronize(stream_o);
    for (auto e : ev_o)
        if (e) (void)hipEventDestroy(e);
    if (stream_o) (void)hipStreamDestroy(stream_o);
    for (auto e : flag_ev)
        if (e) (void)hipEventDestroy(e);
    for (auto e : la_ev)
        if (e) (void)hipEventDestroy(e);
    drop_step_graph();
    if (stream) (void)hipStreamDestroy(stream);
}

hipError_t Engine::init(int device, int n_graphs, int n_part, int64_t cap_events, std::string& why) {
    int count = 0;
    hipError_t e = hipGetDeviceCount(&count);
    if (e != hipSuccess || count <= 0) {
        why = "no HIP device available (libhgx has no CPU fallback)";
        return e != hipSuccess ? e : hipErrorNoDevice;
    }
    if (device < 0 || device >= count) {
        why = "invalid HIP device ordinal";
        return hipErrorInvalidDevice;
    }
    hipDeviceProp_t prop;
    HGX_TRY(hipGetDeviceProperties(&prop, device));
    num_cus = std::max(1, prop.multiProcessorCount);
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) {
        why = std::string("device is ") + prop.gcnArchName + ", libhgx is built for gfx950 (MI355X) only";
        return hipErrorInvalidDeviceFunction;
    }
    dev = device;
    HGX_TRY(hipSetDevice(dev));
    HGX_TRY(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
    HGX_TRY(hipEventCreate(&ph0));
    HGX_TRY(hipEventCreate(&ph1));
    HGX_TRY(hipEventCreate(&ph2));
    G = n_graphs;
    n = n_part;
    C = G * n;
    sm = 2 * n / 3 + 1;   // hashgraph.go:63
    shard_lo = 0;
    shard_hi = C;
    nw = (n + 63) / 64;
    cap = std::max<int64_t>(cap_events, 1);
    const size_t P = (size_t)cap;
    // positions: the events plus slack for chains to grow in place between DivideRounds
    Ppos = cap + std::max<int64_t>(cap / 2, (int64_t)256 * C);
    const size_t PP = (size_t)Ppos;
    HGX_TRY(g_creator.alloc(P)); HGX_TRY(g_index.alloc(P)); HGX_TRY(g_sp.alloc(P)); HGX_TRY(g_op.alloc(P));
    HGX_TRY(g_ntx.alloc(P)); HGX_TRY(g_rr.alloc(P)); HGX_TRY(g_pos.alloc(P)); HGX_TRY(g_ts.alloc(P));
    HGX_TRY(g_cts.alloc(P)); HGX_TRY(g_ck.alloc(P)); HGX_TRY(g_S.alloc(P * 32)); HGX_TRY(g_coin.alloc(P)); HGX_TRY(g_loaded.alloc(P));
    HGX_TRY(g_txnil.alloc(P)); HGX_TRY(g_id.alloc(P * 32));
    // insert state: no claims, no events per creator
    HGX_TRY(succ.alloc(P)); HGX_TRY(first_none.alloc(C));
    ins_gl_off = ((size_t)3 * C + 1) & ~(size_t)1;
    HGX_TRY(ins_blk.alloc(ins_gl_off + (size_t)2 * G));
    last_gid_d.view(ins_blk.p, C);
    last_index_d.view(ins_blk.p + C, C);
    chain_base_d.view(ins_blk.p + 2 * C, C);
    graph_loaded_d.view((unsigned long long*)(ins_blk.p + ins_gl_off), G);
    HGX_TRY(ins_fail.alloc(1));
    HGX_TRY(hipMemsetAsync(ins_fail.p, 0xFF, 8, stream));   // re-armed after every read
    HGX_TRY(hipHostMalloc((void**)&h_ins, ins_blk.n * sizeof(int32_t), hipHostMallocDefault));
    HGX_TRY(cpar_blk.alloc((size_t)3 * C));
    HGX_TRY(hipHostMalloc((void**)&h_cpar, (size_t)3 * C * sizeof(int32_t), hipHostMallocDefault));
    HGX_TRY(hipMemsetAsync(succ.p, 0xFF, P * 4, stream));
    HGX_TRY(hipMemsetAsync(first_none.p, 0xFF, (size_t)C * 4, stream));
    HGX_TRY(hipMemsetAsync(last_gid_d.p, 0xFF, (size_t)C * 8, stream));   // last_gid, last_index
    HGX_TRY(hipMemsetAsync(chain_base_d.p, 0, (ins_blk.n - (size_t)2 * C) * 4, stream));   // chain_base, graph_loaded
    HGX_TRY(c_off.alloc(C + 1));
    c_len.view(cpar_blk.p, C);
    c_base.view(cpar_blk.p + C, C);
    c_old.view(cpar_blk.p + 2 * C, C);
    HGX_TRY(fu.alloc(C)); HGX_TRY(rcnt.alloc(C));
    HGX_TRY(root_round_d.alloc(C)); HGX_TRY(root_y_ext_d.alloc(C));
    HGX_TRY(hipMemsetAsync(root_round_d.p, 0xFF, (size_t)C * 4, stream));   // genesis: Round -1, Y ""
    HGX_TRY(hipMemsetAsync(root_y_ext_d.p, 0, (size_t)C, stream));
    HGX_TRY(p_gid.alloc(PP)); HGX_TRY(p_chain.alloc(PP)); HGX_TRY(p_op.alloc(PP)); HGX_TRY(p_opu.alloc(PP));
    HGX_TRY(p_opk.alloc(PP));
    HGX_TRY(p_round.alloc(PP)); HGX_TRY(p_rr.alloc(PP)); HGX_TRY(p_ts.alloc(PP)); HGX_TRY(p_cts.alloc(PP));
    fd_ld = (Ppos + 31) & ~(int64_t)31;   // firstDescendants columns: 64-byte aligned 32-position segments
    HGX_TRY(LA.alloc(PP * n));
    HGX_TRY(FDT.alloc((size_t)fd_ld * n + 128));   // slack: compact window staging reads past a column
    HGX_TRY(recv_list.alloc(P)); HGX_TRY(counters.alloc(8 + 4 * kLaRing));
    HGX_TRY(hipMemsetAsync(counters.p, 0, (8 + 4 * kLaRing) * 4, stream)); HGX_TRY(order_gid.alloc(P));
    HGX_TRY(scan_part.alloc((size_t)256 * ((P + 2047) / 2048 + 1) / 2048 + 64));
    HGX_TRY(key_a.alloc(P)); HGX_TRY(key_b.alloc(P)); HGX_TRY(val_a.alloc(P)); HGX_TRY(val_b.alloc(P));
    HGX_TRY(hist.alloc((size_t)256 * ((P + 2047) / 2048 + 1)));
    HGX_TRY(minmax.alloc(3));
    HGX_TRY(lr.alloc(G));
    for (auto& e : la_ev) HGX_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    HGX_TRY(hipEventCreateWithFlags(&flag_ev[0], hipEventDisableTiming));
    HGX_TRY(hipEventCreateWithFlags(&flag_ev[1], hipEventDisableTiming));
    HGX_TRY(hipHostMalloc((void**)&h_small, 64 * sizeof(int32_t), hipHostMallocDefault));
    HGX_TRY(hipHostMalloc((void**)&h_flag, 16 * sizeof(int32_t), hipHostMallocMapped | hipHostMallocCoherent));
    HGX_TRY(hipHostGetDevicePointer((void**)&d_flag, h_flag, 0));
    // rounds: initial guess, grown on demand
    const int lg = std::max(1, bitlen((uint64_t)n));
    // rounds of the largest graph: ~events per graph / (n log n) (SURVEY §8 estimate), x2
    const int64_t per_graph = (cap + G - 1) / G;
    int32_t guess = (int32_t)std::min<int64_t>(1 << 20, std::max<int64_t>(64, 2 * per_graph / std::max(1, n * lg) + 16));
    HGX_TRY(ensure_round_cap(guess));
    return hipStreamSynchronize(stream);
}

hipError_t Engine::ensure_round_cap(int32_t need) {
    if (need <= r_cap) return hipSuccess;
    const int32_t old = r_cap;
    int32_t nc = std::max<int32_t>(need, old * 2);
    const size_t Cz = (size_t)C;
    HGX_TRY(Bm.grow_copy((size_t)(nc + 1) * Cz, (size_t)(old + 1) * Cz, stream));
    HGX_TRY(WLA.grow_copy((size_t)nc * Cz * n, (size_t)old * Cz * n, stream));
    HGX_TRY(WFD.grow_copy((size_t)nc * Cz * n, (size_t)old * Cz * n, stream));
    HGX_TRY(wflag.grow_copy((size_t)nc * Cz, (size_t)old * Cz, stream));
    HGX_TRY(wstat.grow_copy((size_t)nc * Cz, (size_t)old * Cz, stream));
    drop_step_graph();
    HGX_TRY(wcoin.grow_copy((size_t)nc * Cz, (size_t)old * Cz, stream));
    HGX_TRY(active.grow_copy((size_t)nc + 1, (size_t)old + 1, stream));
    HGX_TRY(ovf.grow_copy((size_t)nc + 2, (size_t)old + 2, stream));
    HGX_TRY(Tthr.grow_copy((size_t)nc * Cz, 0, stream));
    HGX_TRY(fw.grow_copy((size_t)nc * Cz, 0, stream));
    HGX_TRY(elig.grow_copy((size_t)nc * G, 0, stream));
    HGX_TRY(ur_empty.grow_copy((size_t)G, 0, stream));
    // S rows of earlier rounds were written by the round steps of this DivideRounds (the
    // growth happens between step batches) and are read by DecideFame: keep them
    HGX_TRY(Smat.grow_copy((size_t)nc * Cz * nw, (size_t)old * Cz * nw, stream));
    HGX_TRY(Vbuf.grow_copy((size_t)nc * 2 * Cz * nw, 0, stream));
    HGX_TRY(fame.grow_copy((size_t)nc * Cz, 0, stream));
    HGX_TRY(blk_cnt.grow_copy((size_t)nc * G, 0, stream));
    HGX_TRY(blk_loaded.grow_copy((size_t)nc * G, 0, stream));
    HGX_TRY(blk_ntx.grow_copy((size_t)nc * G, 0, stream));
    HGX_TRY(blk_nil.grow_copy((size_t)nc * G, 0, stream));
    if (old < nc) {
        HGX_TRY(hipMemsetAsync(active.p + old + 1, 0, (size_t)(nc - old) * sizeof(int32_t), stream));
        HGX_TRY(hipMemsetAsync(ovf.p + old + 2, 0, (size_t)(nc - old) * sizeof(int32_t), stream));
    }
    r_cap = nc;
    return hipSuccess;
}

DevArrays Engine::arrays() {
    DevArrays a;
    a.g_creator = g_creator.p; a.g_index = g_index.p; a.g_op = g_op.p; a.g_ntx = g_ntx.p;
    a.g_ts = g_ts.p; a.g_S = g_S.p; a.g_coin = g_coin.p; a.g_loaded = g_loaded.p; a.g_txnil = g_txnil.p;
    a.g_rr = g_rr.p; a.g_pos = g_pos.p; a.g_cts = g_cts.p; a.g_ck = g_ck.p;
    a.c_off = c_off.p; a.c_len = c_len.p; a.c_base = c_base.p;
    a.p_gid = p_gid.p; a.p_chain = p_chain.p; a.p_op = p_op.p; a.p_opu = p_opu.p; a.p_opk = p_opk.p; a.p_round = p_round.p; a.p_rr = p_rr.p;
    a.p_ts = p_ts.p; a.p_cts = p_cts.p;
    a.LA = LA.p; a.FDT = FDT.p; a.compact = compact;
    a.Bm = Bm.p; a.wflag = wflag.p; a.wstat = wstat.p; a.wcoin = wcoin.p; a.WLA = WLA.p; a.WFD = WFD.p; a.WLAT = WLAT.p;
    a.active = active.p; a.lr = lr.p;
    a.Smat = Smat.p; a.Vbuf = Vbuf.p; a.fame = fame.p;
    a.elig = elig.p; a.fw = fw.p; a.ur_empty = ur_empty.p; a.T = Tthr.p;
    a.recv_list = recv_list.p; a.counters = counters.p; a.fu = fu.p; a.rcnt = rcnt.p; a.scan_part = scan_part.p;
    a.key_a = key_a.p; a.key_b = key_b.p; a.val_a = val_a.p; a.val_b = val_b.p; a.hist = hist.p;
    a.minmax = minmax.p; a.order_gid = order_gid.p;
    a.blk_cnt = blk_cnt.p; a.blk_loaded = blk_loaded.p; a.blk_ntx = blk_ntx.p; a.blk_nil = blk_nil.p;
    return a;
}

// ---- per-kernel timing (only when time_kernels) ---------------------------------
// count = launches the window covers (a hipGraph replay of round steps); sample = false
// counts them without timing (a per-launch average from the timed sample: KernelStat.timed)
// HGX_HOST_TIME_KERNELS=1 (diagnostic): every timed window also drained and timed by the host clock,
// one stderr line per window (a cross-check of the HIP-event and profiler kernel times)
static const bool g_host_time = getenv("HGX_HOST_TIME_KERNELS") != nullptr;
static std::chrono::steady_clock::time_point g_host_t0;

void Engine::kbeg(int k, bool sample, int64_t count) {
    kstat[k].launches += count;
    if (!((time_mask >> k) & 1u) || !sample) return;
    if (g_host_time) {
        (void)hipStreamSynchronize(stream);
        g_host_t0 = std::chrono::steady_clock::now();
    }
    while (kev.size() < kev_used + 2) {
        hipEvent_t e;
        // timing only (nothing on the host waits on them): no system-scope fences, so that the
        // events bracketing every round-step replay cost the timed region as little as possible
        if (hipEventCreateWithFlags(&e, hipEventDisableSystemFence) != hipSuccess) return;
        kev.push_back(e);
    }
    (void)hipEventRecord(kev[kev_used], stream);
    kopen.push_back({k, kev_used, 0, count});
    kev_used += 2;
}

void Engine::kend(int k, double bytes) {
    kstat[k].bytes += bytes;
    if (!((time_mask >> k) & 1u) || kopen.empty() || kopen.back().k != k) return;
    Open& o = kopen.back();
    o.bytes = bytes;
    (void)hipEventRecord(kev[o.e0 + 1], stream);
    if (g_host_time) {
        (void)hipStreamSynchronize(stream);
        const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - g_host_t0).count();
        float ev = 0.f;
        (void)hipEventElapsedTime(&ev, kev[o.e0], kev[o.e0 + 1]);
        fprintf(stderr, "[hgx host-timed] kernel %d host %.4f ms events %.4f ms\n", k, ms, (double)ev);
    }
}

// bytes known only after the launch completed (attributed to the last open launch of k)
void Engine::kadd_bytes(int k, double bytes) {
    kstat[k].bytes += bytes;
    for (auto it = kopen.rbegin(); it != kopen.rend(); ++it)
        if (it->k == k) { it->bytes += bytes; break; }
}

hipError_t Engine::stage_reserve(size_t bytes) {
    const size_t need = stage_used + ((bytes + 63) & ~(size_t)63);
    if (need <= stage_cap) return hipSuccess;
    // grow: nothing staged may still be in flight, and staged D2H data is copied out first
    HGX_TRY(hipStreamSynchronize(stream));
    size_t cap = std::max(need, std::max((size_t)1 << 20, 2 * stage_cap));
    uint8_t* q = nullptr;
    HGX_TRY(hipHostMalloc((void**)&q, cap, hipHostMallocDefault));
    if (h_stage) {
        std::memcpy(q, h_stage, stage_used);
        (void)hipHostFree(h_stage);
    }
    h_stage = q;
    stage_cap = cap;
    return hipHostGetDevicePointer((void**)&d_stage, h_stage, 0);
}

hipError_t Engine::stage_h2d(void* dev, const void* host, size_t bytes) {
    if (bytes == 0) return hipSuccess;
    HGX_TRY(stage_reserve(bytes));
    std::memcpy(h_stage + stage_used, host, bytes);
    pend.push_back({0, stage_used, dev, nullptr, nullptr, bytes});
    stage_used += (bytes + 63) & ~(size_t)63;
    return hipSuccess;
}

hipError_t Engine::stage_d2h(void* host, const void* dev, size_t bytes) {
    if (bytes == 0) return hipSuccess;
    HGX_TRY(stage_reserve(bytes));
    stage_out.push_back({host, stage_used, bytes});
    pend.push_back({1, stage_used, dev, nullptr, nullptr, bytes});
    stage_used += (bytes + 63) & ~(size_t)63;
    return hipSuccess;
}

hipError_t Engine::copy_to_pinned(void* pinned_dst, const void* dev, size_t bytes, int reset) {
    if (bytes == 0) return hipSuccess;
    void* d = nullptr;
    HGX_TRY(hipHostGetDevicePointer(&d, pinned_dst, 0));
    PendCopy p{2, 0, dev, pinned_dst, d, bytes};
    p.reset = reset;
    pend.push_back(p);
    return hipSuccess;
}

hipError_t Engine::copy_from_pinned(void* dev, const void* pinned_src, size_t bytes) {
    if (bytes == 0) return hipSuccess;
    void* d = nullptr;
    HGX_TRY(hipHostGetDevicePointer(&d, const_cast<void*>(pinned_src), 0));
    PendCopy p{3, 0, dev, nullptr, nullptr, bytes};
    p.host_src = pinned_src;
    p.dev_src = d;
    pend.push_back(p);
    return hipSuccess;
}

hipError_t Engine::stage_issue() {
    if (pend.empty()) return hipSuccess;
    size_t total = 0;
    for (const PendCopy& p : pend) total += p.bytes;
    if (pend.size() <= (size_t)kCopyMax && total <= kCopyKernelMax) {
        CopyRange r[kCopyMax];
        int k = 0;
        for (const PendCopy& p : pend) {
            if (p.kind == 0) r[k++] = {d_stage + p.off, const_cast<void*>(p.dev), (uint32_t)p.bytes};
            else if (p.kind == 1) r[k++] = {p.dev, d_stage + p.off, (uint32_t)p.bytes};
            else if (p.kind == 2) r[k++] = {p.dev, p.dev_dst, (uint32_t)p.bytes, p.reset};
            else r[k++] = {p.dev_src, const_cast<void*>(p.dev), (uint32_t)p.bytes};
        }
        launch_copy_many(stream, r, k);
        pend.clear();
        return hipGetLastError();
    }
    for (const PendCopy& p : pend) {
        if (p.kind == 0) HGX_TRY(hipMemcpyAsync(const_cast<void*>(p.dev), h_stage + p.off, p.bytes, hipMemcpyHostToDevice, stream));
        else if (p.kind == 1) HGX_TRY(hipMemcpyAsync(h_stage + p.off, p.dev, p.bytes, hipMemcpyDeviceToHost, stream));
        else if (p.kind == 2) {
            HGX_TRY(hipMemcpyAsync(p.host_dst, p.dev, p.bytes, hipMemcpyDeviceToHost, stream));
            if (p.reset >= 0) HGX_TRY(hipMemsetAsync(const_cast<void*>(p.dev), p.reset, p.bytes, stream));
        }
        else HGX_TRY(hipMemcpyAsync(const_cast<void*>(p.dev), p.host_src, p.bytes, hipMemcpyHostToDevice, stream));
    }
    pend.clear();
    return hipSuccess;
}

void Engine::stage_flush() {
    for (const StagedD2H& d : stage_out) std::memcpy(d.dst, h_stage + d.off, d.bytes);
    stage_out.clear();
    stage_used = 0;
}

hipError_t Engine::collect_kernel_times() {
    if (kopen.empty()) return hipSuccess;
    HGX_TRY(hipStreamSynchronize(stream));
    for (const Open& o : kopen) {
        float ms = 0;
        if (hipEventElapsedTime(&ms, kev[o.e0], kev[o.e0 + 1]) == hipSuccess) {
            kstat[o.k].ms += ms;
            kstat[o.k].timed += o.count;
        }
    }
    kopen.clear();
    kev_used = 0;
    return hipSuccess;
}

// ---- inputs: InsertEvent batches (hgx_insert.hip) ----------------------------------
InsertState Engine::insert_state() {
    InsertState st;
    st.g_creator = g_creator.p; st.g_index = g_index.p; st.g_sp = g_sp.p; st.g_op = g_op.p; st.g_ntx = g_ntx.p;
    st.g_rr = g_rr.p; st.g_ts = g_ts.p; st.g_cts = g_cts.p; st.g_S = g_S.p; st.g_coin = g_coin.p;
    st.g_loaded = g_loaded.p; st.g_txnil = g_txnil.p; st.g_id = g_id.p;
    st.succ = succ.p; st.first_none = first_none.p;
    st.last_gid = last_gid_d.p; st.last_index = last_index_d.p; st.chain_base = chain_base_d.p;
    st.fail = ins_fail.p; st.graph_loaded = graph_loaded_d.p;
    st.root_y_ext = root_y_ext_d.p; st.rooted = rooted ? 1 : 0;
    st.others = others_d.p; st.n_others = n_others; st.others_trust = others_trust ? 1 : 0;
    return st;
}

template <typename T>
static hipError_t stage_col(DBuf<T>& b, const T* src, size_t count, size_t per, hipStream_t s) {
    if (b.n < count * per) HGX_TRY(b.alloc(count * per));
    return hipMemcpyAsync(b.p, src, count * per * sizeof(T), hipMemcpyHostToDevice, s);
}

// a sync-sized batch (at most kPackEvents): the k host columns packed into pinned memory and sent as
// one copy into st_pack (k pageable copies cost a staged, blocking transfer each); off[i] = column i's
// byte offset in st_pack
hipError_t Engine::stage_pinned(int k, const void* const* src, const size_t* bytes, size_t* off) {
    size_t total = 0;
    for (int i = 0; i < k; i++) {
        off[i] = total;
        total += (bytes[i] + 255) & ~(size_t)255;
    }
    if (st_pack.n < total) HGX_TRY(st_pack.alloc(std::max(total, (size_t)2 * st_pack.n)));
    if (h_pack_cap < total) {   // (every insert synchronized before returning: the buffer is free)
        if (h_pack) (void)hipHostFree(h_pack);
        h_pack = nullptr;
        h_pack_cap = 0;
        HGX_TRY(hipHostMalloc((void**)&h_pack, std::max(total, (size_t)2 * st_pack.n), hipHostMallocDefault));
        h_pack_cap = std::max(total, (size_t)2 * st_pack.n);
    }
    for (int i = 0; i < k; i++)
        if (bytes[i]) std::memcpy(h_pack + off[i], src[i], bytes[i]);
    return hipMemcpyAsync(st_pack.p, h_pack, total, hipMemcpyHostToDevice, stream);
}

hipError_t Engine::stage_host(const int32_t* creator, const int64_t* index, const int64_t* sp, const int64_t* op,
                              const int64_t* ts, const uint8_t* hash, const uint8_t* S, const int32_t* ntx,
                              const int32_t* nil, int64_t count, InsertIn& in) {
    const size_t c = (size_t)count;
    if (count <= kPackEvents) {
        const void* src[9] = {creator, index, sp, op, ts, hash, S, ntx, nil};
        const size_t bytes[9] = {4 * c, 8 * c, 8 * c, 8 * c, 8 * c, 32 * c, 32 * c, 4 * c, 4 * c};
        size_t off[9];
        HGX_TRY(stage_pinned(9, src, bytes, off));
        uint8_t* d = st_pack.p;
        in.creator = (const int32_t*)(d + off[0]); in.index = (const int64_t*)(d + off[1]);
        in.sp = (const int64_t*)(d + off[2]); in.op = (const int64_t*)(d + off[3]); in.ts = (const int64_t*)(d + off[4]);
        in.hash = d + off[5]; in.S = d + off[6]; in.ntx = (const int32_t*)(d + off[7]); in.nil = (const int32_t*)(d + off[8]);
        return hipSuccess;
    }
    HGX_TRY(stage_col(st_creator, creator, c, 1, stream));
    HGX_TRY(stage_col(st_index, index, c, 1, stream));
    HGX_TRY(stage_col(st_sp, sp, c, 1, stream));
    HGX_TRY(stage_col(st_op, op, c, 1, stream));
    HGX_TRY(stage_col(st_ts, ts, c, 1, stream));
    HGX_TRY(stage_col(st_hash, hash, c, 32, stream));
    HGX_TRY(stage_col(st_S, S, c, 32, stream));
    HGX_TRY(stage_col(st_ntx, ntx, c, 1, stream));
    HGX_TRY(stage_col(st_nil, nil, c, 1, stream));
    in.creator = st_creator.p; in.index = st_index.p; in.sp = st_sp.p; in.op = st_op.p; in.ts = st_ts.p;
    in.hash = st_hash.p; in.S = st_S.p; in.ntx = st_ntx.p; in.nil = st_nil.p;
    return hipSuccess;
}

hipError_t Engine::stage_host32(const int32_t* creator, const int32_t* index, const int32_t* sp, const int32_t* op,
                                const int64_t* ts, const uint8_t* coin, const uint8_t* S, const int32_t* ntx,
                                int64_t count, InsertIn& in) {
    const size_t c = (size_t)count;
    in = InsertIn{};
    if (count <= kPackEvents) {   // one pinned packed copy (as stage_host)
        const void* src[8] = {creator, index, sp, op, ts, coin, S, ntx};
        const size_t bytes[8] = {4 * c, 4 * c, 4 * c, 4 * c, 8 * c, c, 32 * c, 4 * c};
        size_t off[8];
        HGX_TRY(stage_pinned(8, src, bytes, off));
        uint8_t* d = st_pack.p;
        in.creator = (const int32_t*)(d + off[0]); in.index32 = (const int32_t*)(d + off[1]);
        in.sp32 = (const int32_t*)(d + off[2]); in.op32 = (const int32_t*)(d + off[3]);
        in.ts = (const int64_t*)(d + off[4]); in.coin = d + off[5]; in.S = d + off[6];
        in.ntx = (const int32_t*)(d + off[7]);
        if (count > 0) ids_known = false;
        return hipSuccess;
    }
    HGX_TRY(stage_col(st_creator, creator, c, 1, stream));
    HGX_TRY(stage_col(st_index32, index, c, 1, stream));
    HGX_TRY(stage_col(st_sp32, sp, c, 1, stream));
    HGX_TRY(stage_col(st_op32, op, c, 1, stream));
    HGX_TRY(stage_col(st_ts, ts, c, 1, stream));
    HGX_TRY(stage_col(st_coin, coin, c, 1, stream));
    HGX_TRY(stage_col(st_S, S, c, 32, stream));
    HGX_TRY(stage_col(st_ntx, ntx, c, 1, stream));
    in.creator = st_creator.p; in.index32 = st_index32.p; in.sp32 = st_sp32.p; in.op32 = st_op32.p;
    in.ts = st_ts.p; in.coin = st_coin.p; in.S = st_S.p; in.ntx = st_ntx.p;
    if (count > 0) ids_known = false;
    return hipSuccess;
}

hipError_t Engine::set_keys(const uint8_t* keys65) {
    HGX_TRY(pk_keys.alloc((size_t)C * 65 + 1));
    HGX_TRY(pk_valid.alloc((size_t)C + 1));
    HGX_TRY(pk_tab.alloc(p256_table_bytes(C) / 4 + 1));
    HGX_TRY(hipMemcpyAsync(pk_keys.p, keys65, (size_t)C * 65, hipMemcpyHostToDevice, stream));
    launch_p256_tables(stream, C, pk_keys.p, pk_tab.p, pk_valid.p);
    HGX_TRY(hipGetLastError());
    HGX_TRY(hipStreamSynchronize(stream));
    keys_set = true;
    return hipSuccess;
}

hipError_t Engine::stage_sig(const uint8_t* digest, const uint8_t* r, int64_t count, const uint8_t** d_digest,
                             const uint8_t** d_r) {
    const size_t c = (size_t)count * 32;
    if (st_dig.n < c) HGX_TRY(st_dig.alloc(c));
    if (st_r.n < c) HGX_TRY(st_r.alloc(c));
    if (c) {
        HGX_TRY(hipMemcpyAsync(st_dig.p, digest, c, hipMemcpyHostToDevice, stream));
        HGX_TRY(hipMemcpyAsync(st_r.p, r, c, hipMemcpyHostToDevice, stream));
    }
    *d_digest = st_dig.p;
    *d_r = st_r.p;
    return hipSuccess;
}

hipError_t Engine::insert_verified(const InsertIn& in, const uint8_t* digest, const uint8_t* r, int64_t count,
                                   InsertOut& out) {
    if (!keys_set) return hipErrorNotReady;
    if (count > 0) {
        if (pk_out.n < (size_t)count) HGX_TRY(pk_out.alloc((size_t)count));
        if (ins_fail_sig.n < 1) HGX_TRY(ins_fail_sig.alloc(1));
        HGX_TRY(hipMemsetAsync(ins_fail_sig.p, 0xFF, 8, stream));
        // Event.Verify of the whole batch (hgx_p256.hip; key = the creator's), then its first failure
        launch_p256_verify(stream, count, C, in.creator, digest, r, in.S, pk_tab.p, pk_valid.p, pk_out.p);
        launch_insert_sig_first(stream, count, C, in.creator, pk_out.p, ins_fail_sig.p);
        HGX_TRY(hipGetLastError());
    }
    return insert_impl(in, count, out, count > 0 ? ins_fail_sig.p : nullptr);
}

hipError_t Engine::insert(const InsertIn& in, int64_t count, InsertOut& out) {
    return insert_impl(in, count, out, nullptr);
}

hipError_t Engine::insert_split_begin(const int32_t* creator, const int64_t* index, const int64_t* sp,
                                      const int64_t* op, int64_t count, InsertOut& out) {
    const size_t c = (size_t)count;
    HGX_TRY(stage_col(st_creator, creator, c, 1, stream));
    HGX_TRY(stage_col(st_index, index, c, 1, stream));
    HGX_TRY(stage_col(st_sp, sp, c, 1, stream));
    HGX_TRY(stage_col(st_op, op, c, 1, stream));
    InsertIn in{};
    in.creator = st_creator.p; in.index = st_index.p; in.sp = st_sp.p; in.op = st_op.p;   // no payload yet
    split32 = false;
    return insert_impl(in, count, out, nullptr, kCommitStructure);
}

hipError_t Engine::insert_split_begin32(const int32_t* creator, const int32_t* index, const int32_t* sp,
                                        const int32_t* op, int64_t count, InsertOut& out) {
    const size_t c = (size_t)count;
    HGX_TRY(stage_col(st_creator, creator, c, 1, stream));
    HGX_TRY(stage_col(st_index32, index, c, 1, stream));
    HGX_TRY(stage_col(st_sp32, sp, c, 1, stream));
    HGX_TRY(stage_col(st_op32, op, c, 1, stream));
    InsertIn in{};
    in.creator = st_creator.p; in.index32 = st_index32.p; in.sp32 = st_sp32.p; in.op32 = st_op32.p;
    split32 = true;
    return insert_impl(in, count, out, nullptr, kCommitStructure);
}

hipError_t Engine::stage_packed(const Packed& pk, int64_t count, InsertIn& in, const int64_t* ts, const uint8_t* coin,
                                const uint8_t* S, const int32_t* ntx) {
    const size_t c = (size_t)count, x = (size_t)pk.n_exc;
    in = InsertIn{};
    if (st_creator.n < c) HGX_TRY(st_creator.alloc(c));
    if (st_sp32.n < c) HGX_TRY(st_sp32.alloc(c));
    if (st_op32.n < c) HGX_TRY(st_op32.alloc(c));
    if (ts && count <= kPackEvents) {   // a sync-sized batch: one pinned packed copy (as stage_host32)
        const void* src[11] = {pk.creator, pk.index, pk.spb, pk.opb, ts, coin, S, ntx, pk.exc_pos, pk.exc_sp, pk.exc_op};
        const size_t bytes[11] = {2 * c, 4 * c, 2 * c, 2 * c, 8 * c, c, 32 * c, 4 * c, 8 * x, 4 * x, 4 * x};
        size_t off[11];
        HGX_TRY(stage_pinned(11, src, bytes, off));
        uint8_t* d = st_pack.p;
        launch_unpack_packed(stream, count, E, (const uint16_t*)(d + off[0]), (const uint16_t*)(d + off[2]),
                             (const uint16_t*)(d + off[3]), pk.n_exc, (const int64_t*)(d + off[8]),
                             (const int32_t*)(d + off[9]), (const int32_t*)(d + off[10]), st_creator.p, st_sp32.p,
                             st_op32.p);
        HGX_TRY(hipGetLastError());
        in.creator = st_creator.p; in.index32 = (const int32_t*)(d + off[1]); in.sp32 = st_sp32.p;
        in.op32 = st_op32.p; in.ts = (const int64_t*)(d + off[4]); in.coin = d + off[5]; in.S = d + off[6];
        in.ntx = (const int32_t*)(d + off[7]);
        if (count > 0) ids_known = false;
        return hipSuccess;
    }
    HGX_TRY(stage_col(st_c16, pk.creator, c, 1, stream));
    HGX_TRY(stage_col(st_index32, pk.index, c, 1, stream));
    HGX_TRY(stage_col(st_spb, pk.spb, c, 1, stream));
    HGX_TRY(stage_col(st_opb, pk.opb, c, 1, stream));
    if (x) {
        HGX_TRY(stage_col(st_exc_pos, pk.exc_pos, x, 1, stream));
        HGX_TRY(stage_col(st_exc_sp, pk.exc_sp, x, 1, stream));
        HGX_TRY(stage_col(st_exc_op, pk.exc_op, x, 1, stream));
    }
    launch_unpack_packed(stream, count, E, st_c16.p, st_spb.p, st_opb.p, pk.n_exc, st_exc_pos.p, st_exc_sp.p,
                         st_exc_op.p, st_creator.p, st_sp32.p, st_op32.p);
    HGX_TRY(hipGetLastError());
    in.creator = st_creator.p; in.index32 = st_index32.p; in.sp32 = st_sp32.p; in.op32 = st_op32.p;
    if (ts) {
        HGX_TRY(stage_col(st_ts, ts, c, 1, stream));
        HGX_TRY(stage_col(st_coin, coin, c, 1, stream));
        HGX_TRY(stage_col(st_S, S, c, 32, stream));
        HGX_TRY(stage_col(st_ntx, ntx, c, 1, stream));
        in.ts = st_ts.p; in.coin = st_coin.p; in.S = st_S.p; in.ntx = st_ntx.p;
        if (count > 0) ids_known = false;
    }
    return hipSuccess;
}

hipError_t Engine::insert_split_begin_packed(const Packed& pk, int64_t count, InsertOut& out) {
    InsertIn in;
    HGX_TRY(stage_packed(pk, count, in));   // (no payload yet)
    split32 = true;
    return insert_impl(in, count, out, nullptr, kCommitStructure);
}

hipError_t Engine::payload_begin32(const int64_t* ts, const uint8_t* coin, const uint8_t* S, const int32_t* ntx,
                                   int64_t m_ok) {
    if (!stream2) {
        HGX_TRY(hipStreamCreateWithFlags(&stream2, hipStreamNonBlocking));
        HGX_TRY(hipEventCreateWithFlags(&ev_pay, hipEventDisableTiming));
    }
    const size_t c = (size_t)m_ok;
    if (st_ts.n < c) HGX_TRY(st_ts.alloc(c));
    if (st_coin.n < c) HGX_TRY(st_coin.alloc(c));
    if (st_ntx.n < c) HGX_TRY(st_ntx.alloc(c));
    if (!ev_pay_S) HGX_TRY(hipEventCreateWithFlags(&ev_pay_S, hipEventDisableTiming));
    if (pay_thread.joinable()) pay_thread.join();
    pay_err = hipSuccess;
    pay32 = true;
    pay_stage = 0;
    pay_S_pending = true;
    if (m_ok > 0) ids_known = false;
    uint8_t* S_dst = g_S.p + 32 * (size_t)(E - m_ok);   // the accepted prefix (just appended): gids E - m_ok ..
    pay_thread = std::thread([=]() {
        hipError_t e = hipSetDevice(dev);
        if (c && e == hipSuccess) e = hipMemcpyAsync(st_ts.p, ts, c * 8, hipMemcpyHostToDevice, stream2);
        if (c && e == hipSuccess) e = hipMemcpyAsync(st_coin.p, coin, c, hipMemcpyHostToDevice, stream2);
        if (c && e == hipSuccess) e = hipMemcpyAsync(st_ntx.p, ntx, c * 4, hipMemcpyHostToDevice, stream2);
        if (e == hipSuccess) e = hipEventRecord(ev_pay, stream2);
        pay_err_a = e;
        pay_stage.store(1, std::memory_order_release);
        if (c && e == hipSuccess) e = hipMemcpyAsync(S_dst, S, c * 32, hipMemcpyHostToDevice, stream2);
        if (e == hipSuccess) e = hipEventRecord(ev_pay_S, stream2);
        if (e == hipSuccess) e = hipStreamSynchronize(stream2);
        pay_err = e;
    });
    return hipSuccess;
}

hipError_t Engine::payload_begin(const int64_t* ts, const uint8_t* hash, const uint8_t* S, const int32_t* ntx,
                                 const int32_t* nil, int64_t m_ok) {
    if (!stream2) {
        HGX_TRY(hipStreamCreateWithFlags(&stream2, hipStreamNonBlocking));
        HGX_TRY(hipEventCreateWithFlags(&ev_pay, hipEventDisableTiming));
    }
    const size_t c = (size_t)m_ok;   // the accepted prefix only
    if (st_ts.n < c) HGX_TRY(st_ts.alloc(c));
    if (st_hash.n < 32 * c) HGX_TRY(st_hash.alloc(32 * c));
    if (st_S.n < 32 * c) HGX_TRY(st_S.alloc(32 * c));
    if (st_ntx.n < c) HGX_TRY(st_ntx.alloc(c));
    if (st_nil.n < c) HGX_TRY(st_nil.alloc(c));
    if (pay_thread.joinable()) pay_thread.join();
    pay_err = hipSuccess;
    pay32 = false;
    pay_S_pending = false;
    // pageable host memory: each copy returns once its source has been consumed, so the copies
    // run on their own host thread (and stream) beside the DivideRounds launches
    pay_thread = std::thread([=]() {
        hipError_t e = hipSetDevice(dev);
        if (c && e == hipSuccess) e = hipMemcpyAsync(st_ts.p, ts, c * 8, hipMemcpyHostToDevice, stream2);
        if (c && e == hipSuccess) e = hipMemcpyAsync(st_hash.p, hash, c * 32, hipMemcpyHostToDevice, stream2);
        if (c && e == hipSuccess) e = hipMemcpyAsync(st_S.p, S, c * 32, hipMemcpyHostToDevice, stream2);
        if (c && e == hipSuccess) e = hipMemcpyAsync(st_ntx.p, ntx, c * 4, hipMemcpyHostToDevice, stream2);
        if (c && e == hipSuccess) e = hipMemcpyAsync(st_nil.p, nil, c * 4, hipMemcpyHostToDevice, stream2);
        if (e == hipSuccess) e = hipEventRecord(ev_pay, stream2);
        if (e == hipSuccess) e = hipStreamSynchronize(stream2);   // the caller's buffers are read completely
        pay_err = e;
    });
    return hipSuccess;
}

hipError_t Engine::payload_end(int64_t E0, int64_t m_ok, bool laid_out_new, int32_t wcoin_r0,
                               std::vector<uint64_t>& loaded) {
    if (pay_S_pending) {   // the compact payload: its first stage only (S lands in g_S later)
        while (pay_stage.load(std::memory_order_acquire) == 0) std::this_thread::yield();
        HGX_TRY(pay_err_a);
    } else {
        if (pay_thread.joinable()) pay_thread.join();
        HGX_TRY(pay_err);
    }
    HGX_TRY(hipStreamWaitEvent(stream, ev_pay, 0));
    InsertIn in{};
    in.creator = st_creator.p; in.ts = st_ts.p; in.S = pay_S_pending ? nullptr : st_S.p; in.ntx = st_ntx.p;
    if (split32) { in.index32 = st_index32.p; in.sp32 = st_sp32.p; in.op32 = st_op32.p; }
    else { in.index = st_index.p; in.sp = st_sp.p; in.op = st_op.p; }
    if (pay32) in.coin = st_coin.p;
    else { in.hash = st_hash.p; in.nil = st_nil.p; }
    split32 = false;
    launch_insert_commit(stream, m_ok, nullptr, nullptr, E0, n, in, insert_state(), kCommitPayload);
    if (laid_out_new) {   // the layout ran before the timestamps and coins were committed
        launch_ts_to_pos(stream, E0, m_ok, g_pos.p, g_ts.p, p_ts.p);
        if (R > wcoin_r0) launch_wcoin(stream, arrays(), wcoin_r0, R, C);
    }
    HGX_TRY(hipGetLastError());
    HGX_TRY(hipMemcpyAsync(h_ins, ins_blk.p, ins_blk.n * sizeof(int32_t), hipMemcpyDeviceToHost, stream));
    HGX_TRY(hipStreamSynchronize(stream));
    loaded.resize(G);
    std::memcpy(loaded.data(), h_ins + ins_gl_off, (size_t)G * 8);
    return hipSuccess;
}

hipError_t Engine::payload_wait_S() {
    if (!pay_S_pending) return hipSuccess;
    pay_S_pending = false;
    if (pay_thread.joinable()) pay_thread.join();
    HGX_TRY(pay_err);
    return hipStreamWaitEvent(stream, ev_pay_S, 0);
}

hipError_t Engine::insert_impl(const InsertIn& in, int64_t count, InsertOut& out, const unsigned long long* fail_sig,
                               int commit_mode) {
    out = InsertOut();
    const int64_t E0 = E;
    InsertState st = insert_state();
    if (count > 0) {
        // checks, then the commit of the accepted prefix and the withdrawal of the rest's claims:
        // the kernels take the prefix from the first-failure words, so the batch costs one host
        // round trip (the chunked schedule inserts 1 000 events per call)
        // (ins_fail is ~0 here: set at creation, re-armed by the read-back below)
        if (!launch_insert_fused(stream, count, fail_sig, E0, cap, C, n, in, st, commit_mode)) {
            launch_insert_claim(stream, count, E0, cap, C, in, st);
            launch_insert_check(stream, count, E0, cap, C, n, in, st);
            launch_insert_commit(stream, count, ins_fail.p, fail_sig, E0, n, in, st, commit_mode);
            launch_insert_unclaim(stream, count, ins_fail.p, fail_sig, E0, cap, C, in, st);
        }
        HGX_TRY(copy_to_pinned(h_small, ins_fail.p, 8, 0xFF));
        if (fail_sig) HGX_TRY(copy_to_pinned(h_small + 2, fail_sig, 8));
    }
    out.last_gid.resize(C);
    out.last_index.resize(C);
    out.chain_base.resize(C);
    out.graph_loaded.resize(G);
    // the first-failure words and the whole state block into pinned memory (one launch), then
    // the host mirrors
    HGX_TRY(copy_to_pinned(h_ins, ins_blk.p, ins_blk.n * sizeof(int32_t)));
    HGX_TRY(stage_issue());
    HGX_TRY(hipStreamSynchronize(stream));
    if (count > 0) {
        unsigned long long fail = 0, fsig = ~0ull;
        std::memcpy(&fail, h_small, 8);
        if (fail_sig) std::memcpy(&fsig, h_small + 2, 8);
        // Verify comes first in InsertEvent: at the same event the signature's failure wins
        // (the kernels' accepted_prefix)
        if ((fsig >> 8) <= (fail >> 8) && fsig != ~0ull) fail = fsig;
        const int64_t m_ok = (fail == ~0ull) ? count : (int64_t)(fail >> 8);
        out.accepted = m_ok;
        out.code = (fail == ~0ull) ? 0 : (int)(fail & 0xFF);
        if (out.code) {   // the failing event's creator and Index for the error string
            HGX_TRY(hipMemcpyAsync(&out.fail_creator, in.creator + m_ok, 4, hipMemcpyDeviceToHost, stream));
            if (in.index32) {
                int32_t fi = 0;
                HGX_TRY(hipMemcpyAsync(&fi, in.index32 + m_ok, 4, hipMemcpyDeviceToHost, stream));
                HGX_TRY(hipStreamSynchronize(stream));
                out.fail_index = fi;
            } else {
                HGX_TRY(hipMemcpyAsync(&out.fail_index, in.index + m_ok, 8, hipMemcpyDeviceToHost, stream));
            }
            HGX_TRY(hipStreamSynchronize(stream));
        }
        E = E0 + m_ok;
    }
    std::memcpy(out.last_gid.data(), h_ins, (size_t)C * 4);
    std::memcpy(out.last_index.data(), h_ins + C, (size_t)C * 4);
    std::memcpy(out.chain_base.data(), h_ins + 2 * C, (size_t)C * 4);
    std::memcpy(out.graph_loaded.data(), h_ins + ins_gl_off, (size_t)G * 8);
    return hipSuccess;
}

hipError_t Engine::clear() {
    HGX_TRY(payload_wait_S());
    if (E > 0) HGX_TRY(hipMemsetAsync(succ.p, 0xFF, (size_t)E * 4, stream));
    HGX_TRY(hipMemsetAsync(first_none.p, 0xFF, (size_t)C * 4, stream));
    HGX_TRY(hipMemsetAsync(last_gid_d.p, 0xFF, (size_t)C * 8, stream));   // last_gid, last_index
    HGX_TRY(hipMemsetAsync(chain_base_d.p, 0, (ins_blk.n - (size_t)2 * C) * 4, stream));   // chain_base, graph_loaded
    E = 0;
    E_div = 0;
    R = 0;
    laid_out = false;
    ids_known = true;
    return hipStreamSynchronize(stream);
}

hipError_t Engine::get_ids(int64_t first, int64_t count, uint8_t* out32) {
    if (!ids_known || first < 0 || first + count > E) return hipErrorInvalidValue;
    if (count <= 0) return hipSuccess;
    HGX_TRY(hipMemcpyAsync(out32, g_id.p + 32 * first, (size_t)count * 32, hipMemcpyDeviceToHost, stream));
    return hipStreamSynchronize(stream);
}

hipError_t Engine::get_keys(uint8_t* out65) {
    if (!keys_set) return hipErrorNotReady;
    HGX_TRY(hipMemcpyAsync(out65, pk_keys.p, (size_t)C * 65, hipMemcpyDeviceToHost, stream));
    return hipStreamSynchronize(stream);
}

hipError_t Engine::set_roots(const std::vector<int32_t>& round, const std::vector<uint8_t>& y_ext) {
    rooted = false;
    root_gmax = -1;
    for (int c = 0; c < C; c++) {
        if (round[c] >= 0 || y_ext[c]) rooted = true;
        root_gmax = std::max(root_gmax, round[c] + 1);
    }
    if (!rooted) root_gmax = -1;
    HGX_TRY(hipMemcpyAsync(root_round_d.p, round.data(), (size_t)C * 4, hipMemcpyHostToDevice, stream));
    HGX_TRY(hipMemcpyAsync(root_y_ext_d.p, y_ext.data(), (size_t)C, hipMemcpyHostToDevice, stream));
    return hipStreamSynchronize(stream);
}

// Root.Others keys (event ids, 32 bytes each): sorted as 4 big-endian words for k_insert_check
hipError_t Engine::set_root_others(const uint8_t* keys32, int64_t count) {
    std::vector<std::array<uint64_t, 4>> k((size_t)count);
    for (int64_t i = 0; i < count; i++)
        for (int w = 0; w < 4; w++) {
            uint64_t x = 0;
            for (int b = 0; b < 8; b++) x = (x << 8) | keys32[32 * i + 8 * w + b];
            k[(size_t)i][w] = x;
        }
    std::sort(k.begin(), k.end());
    k.erase(std::unique(k.begin(), k.end()), k.end());
    n_others = (int64_t)k.size();
    if (others_d.n < (size_t)std::max<int64_t>(1, 4 * n_others)) HGX_TRY(others_d.alloc((size_t)std::max<int64_t>(1, 4 * n_others)));
    if (n_others) HGX_TRY(hipMemcpyAsync(others_d.p, k.data(), (size_t)n_others * 32, hipMemcpyHostToDevice, stream));
    return hipStreamSynchronize(stream);
}

hipError_t Engine::round_first_gids(int32_t r0, std::vector<int32_t>& out) {
    out.assign((size_t)std::max(0, R - r0), 0x7FFFFFFF);
    if (R <= r0) return hipSuccess;
    if (rfirst.n < (size_t)(R - r0)) HGX_TRY(rfirst.alloc((size_t)std::max(R - r0, 2 * (int)rfirst.n)));
    HGX_TRY(hipMemsetAsync(rfirst.p, 0x7F, (size_t)(R - r0) * 4, stream));
    launch_round_first_gid(stream, arrays(), r0, R, C, rfirst.p);
    HGX_TRY(hipMemcpyAsync(out.data(), rfirst.p, (size_t)(R - r0) * 4, hipMemcpyDeviceToHost, stream));
    return hipStreamSynchronize(stream);
}

hipError_t Engine::get_events(std::vector<int32_t>& creator, std::vector<int32_t>& index, std::vector<int32_t>& sp,
                              std::vector<int32_t>& op) {
    creator.resize((size_t)E);
    index.resize((size_t)E);
    sp.resize((size_t)E);
    op.resize((size_t)E);
    if (E == 0) return hipSuccess;
    HGX_TRY(hipMemcpyAsync(creator.data(), g_creator.p, (size_t)E * 4, hipMemcpyDeviceToHost, stream));
    HGX_TRY(hipMemcpyAsync(index.data(), g_index.p, (size_t)E * 4, hipMemcpyDeviceToHost, stream));
    HGX_TRY(hipMemcpyAsync(sp.data(), g_sp.p, (size_t)E * 4, hipMemcpyDeviceToHost, stream));
    HGX_TRY(hipMemcpyAsync(op.data(), g_op.p, (size_t)E * 4, hipMemcpyDeviceToHost, stream));
    return hipStreamSynchronize(stream);
}

hipError_t Engine::get_columns(std::vector<int32_t>& creator, std::vector<int32_t>& index, std::vector<int32_t>& sp,
                               std::vector<int32_t>& op, std::vector<int64_t>& ts, std::vector<uint8_t>& S,
                               std::vector<uint8_t>& coin, std::vector<int32_t>& ntx, std::vector<uint8_t>& txnil) {
    HGX_TRY(payload_wait_S());
    HGX_TRY(get_events(creator, index, sp, op));
    const size_t e = (size_t)E;
    ts.resize(e);
    S.resize(e * 32);
    coin.resize(e);
    ntx.resize(e);
    txnil.resize(e);
    if (e == 0) return hipSuccess;
    HGX_TRY(hipMemcpyAsync(ts.data(), g_ts.p, e * 8, hipMemcpyDeviceToHost, stream));
    HGX_TRY(hipMemcpyAsync(S.data(), g_S.p, e * 32, hipMemcpyDeviceToHost, stream));
    HGX_TRY(hipMemcpyAsync(coin.data(), g_coin.p, e, hipMemcpyDeviceToHost, stream));
    HGX_TRY(hipMemcpyAsync(ntx.data(), g_ntx.p, e * 4, hipMemcpyDeviceToHost, stream));
    HGX_TRY(hipMemcpyAsync(txnil.data(), g_txnil.p, e, hipMemcpyDeviceToHost, stream));
    return hipStreamSynchronize(stream);
}

hipError_t Engine::get_event_fields(int64_t gid, int64_t* ts, int32_t* ntx, int32_t* tx_nil) {
    uint8_t nil = 0;
    HGX_TRY(hipMemcpyAsync(ts, g_ts.p + gid, 8, hipMemcpyDeviceToHost, stream));
    HGX_TRY(hipMemcpyAsync(ntx, g_ntx.p + gid, 4, hipMemcpyDeviceToHost, stream));
    HGX_TRY(hipMemcpyAsync(&nil, g_txnil.p + gid, 1, hipMemcpyDeviceToHost, stream));
    HGX_TRY(hipStreamSynchronize(stream));
    *tx_nil = nil;
    return hipSuccess;
}

hipError_t Engine::reserve_rounds(int32_t rounds) {
    rounds = std::max<int32_t>(rounds, 1);
    drop_step_graph();
    Bm.release(); WLA.release(); WFD.release(); wflag.release(); wstat.release(); wcoin.release();
    active.release(); Tthr.release(); fw.release(); elig.release(); ur_empty.release(); Smat.release();
    Vbuf.release(); fame.release(); blk_cnt.release(); blk_loaded.release(); blk_ntx.release(); blk_nil.release();
    ovf.release();
    WLAT.release();
    r_cap = 0;
    R = 0;
    E_div = 0;
    HGX_TRY(ensure_round_cap(rounds));
    return hipStreamSynchronize(stream);
}

// nb round-step nodes captured as one hipGraph (their round arguments are rewritten per replay)
hipError_t Engine::capture_steps(StepGraph& sgr, const RoundArgs& args, int kern, int nb) {
    sgr.drop();
    sgr.args = args;
    sgr.kernel = kern;
    sgr.compact = compact;
    sgr.nb = nb;
    HGX_TRY(hipStreamBeginCapture(stream, hipStreamCaptureModeThreadLocal));
    hipError_t le = hipSuccess;   // a failed launch ends the capture, then is reported
    for (int k = 0; k < nb && le == hipSuccess; k++) le = launch_round_step(stream, sgr.args, k, kern);
    const hipError_t ce = hipStreamEndCapture(stream, &sgr.graph);
    if (le != hipSuccess) {
        if (ce == hipSuccess && sgr.graph) (void)hipGraphDestroy(sgr.graph);
        sgr.graph = nullptr;
        return le;
    }
    HGX_TRY(ce);
    HGX_TRY(hipGraphInstantiate(&sgr.exec, sgr.graph, nullptr, nullptr, 0));
    // the step nodes in launch order (a linear chain)
    size_t nn = 0;
    HGX_TRY(hipGraphGetNodes(sgr.graph, nullptr, &nn));
    std::vector<hipGraphNode_t> nodes(nn);
    HGX_TRY(hipGraphGetNodes(sgr.graph, nodes.data(), &nn));
    sgr.nodes.clear();
    sgr.params.clear();
    hipGraphNode_t nd_cur = nullptr;
    for (auto nd : nodes) {
        size_t nd_deps = 0;
        HGX_TRY(hipGraphNodeGetDependencies(nd, nullptr, &nd_deps));
        if (nd_deps == 0) nd_cur = nd;
    }
    while (nd_cur) {
        hipKernelNodeParams kp;
        HGX_TRY(hipGraphKernelNodeGetParams(nd_cur, &kp));
        sgr.nodes.push_back(nd_cur);
        sgr.params.push_back(kp);
        size_t nd_out = 0;
        HGX_TRY(hipGraphNodeGetDependentNodes(nd_cur, nullptr, &nd_out));
        if (nd_out == 0) break;
        std::vector<hipGraphNode_t> outs(nd_out);
        HGX_TRY(hipGraphNodeGetDependentNodes(nd_cur, outs.data(), &nd_out));
        nd_cur = outs[0];
    }
    if ((int)sgr.nodes.size() != nb) return hipErrorUnknown;
    return hipSuccess;
}

// ---- DivideRounds ---------------------------------------------------------------
// Chains are laid out with slack (positions [c_off[c], c_off[c] + slot)), so that a call
// after more InsertEvents only appends rows: the events of earlier calls keep their
// positions, lastAncestors rows and rounds, and the call works on the new events (DESIGN.md
// §3.7). The layout is rebuilt (and everything recomputed) when a chain outgrows its slot,
// the coordinate storage changes, or after reset_received / reserve_rounds / clear.
hipError_t Engine::divide_rounds(int64_t En, const std::vector<int32_t>& chain_len,
                                 const std::vector<int32_t>& chain_base, RoundsHost& out) {
    stage_out.clear();   // every earlier call synchronized: the staging is free
    pend.clear();
    stage_used = 0;
    int32_t max_index = -1;
    int new_max_len = 0;
    for (int c = 0; c < C; c++) {
        if (chain_len[c] > 0) max_index = std::max(max_index, chain_base[c] + chain_len[c] - 1);
        new_max_len = std::max(new_max_len, chain_len[c]);
    }
    // compact (uint16) coordinates when every Index fits below the sentinels
    // (Coord<uint16_t>, hgx_device.h) and rows are whole dwords
    const int new_compact = (!force_coord32 && (n % 2) == 0 && max_index <= 65533) ? 1 : 0;
    bool rebuild = !laid_out || E_div == 0 || new_compact != compact || !incremental;
    if (!rebuild)
        for (int c = 0; c < C; c++)
            if (chain_len[c] > h_off[c + 1] - h_off[c]) { rebuild = true; break; }
    const int64_t E0 = rebuild ? 0 : E_div;
    E = En;
    compact = new_compact;
    max_len = new_max_len;
    const size_t csz = compact ? 2 : 4;
    if (rebuild) {
        // slack in shares: two for a chain with events, one for a chain without (a silent peer, or
        // one that has not created an event yet). With even shares c5's 341 silent peers held a
        // third of the slack and the live chains outgrew theirs two thirds through the run (an
        // 18.8 ms rebuild call)
        int act = 0;
        for (int c = 0; c < C; c++) act += chain_len[c] > 0 ? 1 : 0;
        const int64_t share = (Ppos - En) / (2 * (int64_t)act + (C - act));
        h_off.assign(C + 1, 0);
        // slots of multiples of 32 positions (a share >= 128 > 31: Ppos >= capacity + 256 C): every
        // chain starts 64-byte aligned in the firstDescendants columns (the round kernels' staging)
        for (int c = 0; c < C; c++)
            h_off[c + 1] = h_off[c] + ((chain_len[c] + (int32_t)((chain_len[c] > 0 ? 2 : 1) * share)) & ~31);
        HGX_TRY(hipMemcpyAsync(c_off.p, h_off.data(), (C + 1) * 4, hipMemcpyHostToDevice, stream));
        h_len_div.assign(C, 0);
        last_rebuild = true;
    } else {
        last_rebuild = false;
    }
    // c_len | c_base | c_old in one copy from pinned staging (the previous call's copy has
    // completed: every call synchronizes before returning)
    std::memcpy(h_cpar, chain_len.data(), (size_t)C * 4);
    std::memcpy(h_cpar + C, chain_base.data(), (size_t)C * 4);
    std::memcpy(h_cpar + 2 * C, h_len_div.data(), (size_t)C * 4);
    HGX_TRY(copy_from_pinned(cpar_blk.p, h_cpar, (size_t)3 * C * 4));
    HGX_TRY(stage_issue());
    // first round whose step can change: the lowest round of the last old event of a chain
    // that got new events (every boundary below it is among old events)
    int32_t r_lo = 0;
    if (!rebuild) {
        r_lo = 0x7FFFFFFF;
        const int32_t Rp = out.R;
        for (int c = 0; c < C && r_lo > 0; c++) {
            if (chain_len[c] <= h_len_div[c]) continue;
            const int32_t last = h_len_div[c] - 1;
            if (last < 0 || Rp == 0) { r_lo = 0; break; }
            int32_t lo = 0, hi = Rp;   // largest r in [0, Rp] with bm[r][c] <= last
            while (lo < hi) {
                const int32_t mid = (lo + hi + 1) / 2;
                if (out.bm[(size_t)mid * C + c] <= last) lo = mid; else hi = mid - 1;
            }
            r_lo = std::min(r_lo, lo);
        }
        if (r_lo == 0x7FFFFFFF) r_lo = 0;
    }
    int max_new = 0;
    for (int c = 0; c < C; c++) max_new = std::max(max_new, chain_len[c] - h_len_div[c]);
    DevArrays a = arrays();
    HGX_TRY(hipEventRecord(ph0, stream));
    const int seg = kLaSeg;
    kbeg(K_LAYOUT);
    launch_layout(stream, E0, En, a, C, n, seg);
    kend(K_LAYOUT, (double)(En - E0) * 64);
    // lastAncestors: fixed point from all -1 (new rows), dirty-tracked sweeps (k_la_sweep)
    const size_t nunits = (size_t)((max_len + seg - 1) / seg) * C;
    int64_t u0 = 0;
    // above 896 chains a workgroup cannot give every chain a lane: one graph gets lanes for
    // the chains that have events only (silent peers have none)
    int la_na = n;
    const int32_t* la_map = nullptr;
    if (n > 896 && G == 1) {
        h_lmap.clear();
        for (int c = 0; c < C; c++)
            if (chain_len[c] > 0) h_lmap.push_back(c);
        la_na = (int)h_lmap.size();
        if (la_na <= 896) {
            if (la_lmap.n < (size_t)std::max(1, la_na)) HGX_TRY(la_lmap.alloc((size_t)n));
            HGX_TRY(hipMemcpyAsync(la_lmap.p, h_lmap.data(), (size_t)la_na * 4, hipMemcpyHostToDevice, stream));
            la_map = la_lmap.p;
        }
    }
    la_wave_used = la_kernel == 0 && la_wave_ok(n, max_len, la_na) && (n <= 896 || la_map);
    // a rebuild of one large graph runs the wavefront on time segments in parallel (their
    // rows are lower bounds), then a verify sweep and the dirty sweeps complete them
    la_wave_segs = 1;
    if (la_wave_used && rebuild && G == 1 && En >= (int64_t)kLaSegMinRows * C) {
        // as many segments as the CUs hold, of at least 2 x kLaHeadRows rows per chain: c2 (64 chains
        // of 16 384 rows, 4 column blocks) took 2.04 ms at 16 segments, 0.69 at 128, and at 192 its
        // exactness check failed (the verify sweep ran); c3 keeps its LDS-bound 16 (profiles/r05/b28_*, b29_*)
        // (the round-4 cap of kLaMaxSegs alone: c2 2.04 ms)
        const int cap = (int)std::max<int64_t>(kLaMaxSegs, En / C / (2 * kLaHeadRows));
        la_wave_segs = la_segs_override > 0 ? la_segs_override : la_wave_segments(n, compact, num_cus, cap);
    }
    if (rebuild) {   // (the wavefront writes every row it builds before anything reads it)
        if (!la_wave_used) HGX_TRY(hipMemsetAsync(LA.p, compact ? 0x00 : 0xFF, (size_t)h_off[C] * n * csz, stream));
    } else {
        launch_init_new(stream, a, E0, En - E0, n, fd_ld);
        int32_t smin = 0x7FFFFFFF;
        for (int c = 0; c < C; c++)
            if (chain_len[c] > h_len_div[c]) smin = std::min(smin, h_len_div[c] / seg);
        u0 = (int64_t)smin * C;
    }
    if (la_chg.n < nunits) {   // change stamps: new units start at 0, a stamp no sweep uses
        const size_t old = la_chg.n;
        HGX_TRY(la_chg.grow_copy(std::max(nunits, 2 * la_chg.n), old, stream));
        HGX_TRY(hipMemsetAsync(la_chg.p + old, 0, (la_chg.n - old) * 4, stream));
    }
    if (la_usum.n < nunits) HGX_TRY(la_usum.grow_copy(std::max(nunits, 2 * la_usum.n), la_usum.n, stream));
    const int32_t* cold = rebuild ? nullptr : c_old.p;
    la_sweeps = 0;
    la_rows = 0;
    auto run_sweeps = [&](int first_mode) -> hipError_t {
        // sweep k's counters in ring slot k % kLaRing; up to kLaAhead sweeps are queued
        // before the host reads the oldest one's "units changed" (a sweep after the one that
        // changed nothing finds no dirty unit and does nothing)
        // dirty flags are sweep stamps (monotone over calls: stale ones never match), so a
        // sweep is one kernel, one 8-byte read-back and one event
        int launched_s = 0;
        HGX_TRY(hipMemsetAsync(counters.p + 8, 0, 16, stream));
        auto launch_sweep = [&]() -> hipError_t {
            const int slot = launched_s % kLaRing;
            int32_t* cnt = counters.p + 8 + 4 * slot;
            int32_t* cnt_next = counters.p + 8 + 4 * ((launched_s + 1) % kLaRing);
            kbeg(K_LA_SWEEP);
            launch_la_sweep(stream, a, C, n, max_len, seg, launched_s == 0 ? first_mode : 0, la_chg.p, ++la_stamp,
                            la_usum.p, cnt, cnt_next, cold, u0);
            kend(K_LA_SWEEP, 0);
            HGX_TRY(hipMemcpyAsync(h_small + 16 + 4 * slot, cnt, 8, hipMemcpyDeviceToHost, stream));
            HGX_TRY(hipEventRecord(la_ev[slot], stream));
            launched_s++;
            return hipSuccess;
        };
        for (;;) {
            // a verify sweep usually finds nothing to redo: wait for it before queueing more
            const int ahead = (first_mode == 2 && la_sweeps == 0) ? 1 : kLaAhead;
            while (launched_s < la_sweeps + ahead) HGX_TRY(launch_sweep());
            const int slot = la_sweeps % kLaRing;
            HGX_TRY(hipEventSynchronize(la_ev[slot]));
            const int32_t rows = h_small[16 + 4 * slot], changed = h_small[16 + 4 * slot + 1];
            // algorithmic bytes of the rows this sweep recomputed (read the two
            // parent rows, write the row, 12n + 16; the self-parent row is the register carry)
            la_rows += rows;
            kadd_bytes(K_LA_SWEEP, (double)rows * (3.0 * csz * n + 16));
            la_sweeps++;
            if (changed == 0) break;
            if (la_sweeps > 100000) return hipErrorUnknown;
        }
        return hipSuccess;
    };
    if (la_wave_used) {
        // one dataflow pass (k_la_wave); its error flag is read with the phase clock below
        // the error flag is 0 here: zeroed at creation, re-armed by every read
        kbeg(K_LA_SWEEP);
        // a small graph (c1) entirely in one workgroup's LDS
        int64_t gpos = 0;   // the most events of a graph
        for (int g = 0; g < G && la_wave_segs == 1 && !la_map; g++) {
            int64_t e = 0;
            for (int c = 0; c < n; c++) e += chain_len[(size_t)g * n + c];
            gpos = std::max(gpos, e);
        }
        const size_t small_lds = (la_wave_segs == 1 && !la_map && la_small_override != 0) ? la_small_bytes(n, compact, gpos) : 0;
        la_small_used = small_lds > 0;
        if (la_small_used) HGX_TRY(launch_la_small(stream, a, G, n, cold, small_lds, counters.p + 6));
        else
            HGX_TRY(launch_la_wave(stream, a, G, n, cold, En, la_wave_segs, 0, counters.p + 6, la_map, la_na,
                                   !rebuild && (En - E0) <= 8 * (int64_t)C));
        if (la_wave_segs > 1)
            HGX_TRY(launch_la_wave(stream, a, G, n, nullptr, En, la_wave_segs, kLaHeadRows, counters.p + 6, la_map, la_na));
        const double rows = (double)(En - E0);
        kend(K_LA_SWEEP, rows * (3.0 * csz * n + 16));
        if (rebuild) {
            HGX_TRY(hipMemcpyAsync(h_small + 48, counters.p + 6, 4, hipMemcpyDeviceToHost, stream));
            HGX_TRY(hipMemsetAsync(counters.p + 6, 0, 4, stream));
        }
        if (la_wave_segs > 1) {
            // the verify sweep (+ dirty sweeps, counted there) only when the segments' exactness check
            // fails (k_la_seg_check): c3 1.6 ms per pass otherwise
            const size_t nt = (size_t)(la_wave_segs + 1) * n;
            if (la_chk.n < nt + 1) HGX_TRY(la_chk.alloc(nt + 1));
            HGX_TRY(hipMemsetAsync(la_chk.p, 0, 4, stream));
            HGX_TRY(launch_la_seg_check(stream, a, n, En, la_wave_segs, kLaHeadRows, la_chk.p + 1, la_chk.p));
            HGX_TRY(hipMemcpyAsync(h_small + 50, la_chk.p, 4, hipMemcpyDeviceToHost, stream));
            HGX_TRY(hipStreamSynchronize(stream));
            la_verified = h_small[50] != 0 || la_verify_always;
            if (la_verified) HGX_TRY(run_sweeps(2));
        }
        la_sweeps++;
        la_rows += (int64_t)rows;
    } else {
        HGX_TRY(run_sweeps(1));
    }
    kbeg(K_FD_BUILD);
    if (grp) {   // a chain-sharded group (one graph): the firstDescendants of this shard's chains' events
        launch_fd_build(stream, a, C, n, max_len, fd_ld, cold, max_new, grp->c_split[shard], grp->c_split[shard + 1]);
    } else {
        launch_fd_build(stream, a, C, n, max_len, fd_ld, cold, max_new);
    }
    kend(K_FD_BUILD, (double)(En - E0) * 2.0 * csz * n);
    if (rooted) {   // root floors of every position (after a Reset)
        if (gfl.n < (size_t)Ppos) HGX_TRY(gfl.alloc((size_t)Ppos));
        const size_t need = (size_t)(root_gmax + 1) * C;
        if (gB.n < need) {
            HGX_TRY(gB.alloc(need));
            drop_step_graph();
        }
        launch_root_floor(stream, a, root_round_d.p, gfl.p, gB.p, root_gmax, C, n, max_len);
    }
    if (rebuild) {   // events received before the rebuild (a prefix of every chain)
        HGX_TRY(hipMemsetAsync(fu.p, 0, (size_t)C * 4, stream));
        launch_fu_count(stream, a, En);
        h_fu.assign(C, 0);
        HGX_TRY(hipMemcpyAsync(h_fu.data(), fu.p, (size_t)C * 4, hipMemcpyDeviceToHost, stream));
    }
    // a call resuming the state (not a rebuild) makes one host round trip: the wavefront's
    // error flag is read with the rounds' results, and a lane that gave up (never seen in
    // practice) redoes the call as a rebuild with the sweeps
    const bool one_trip = !rebuild;
    if (one_trip) {
        HGX_TRY(hipEventRecord(ph2, stream));
    } else {
        HGX_TRY(hipEventRecord(ph1, stream));
        HGX_TRY(hipEventSynchronize(ph1));
        if (la_wave_used && h_small[48] != 0) {
            // a wavefront lane gave up waiting (bounded spins): redo lastAncestors and the
            // firstDescendants built from them with the sweeps
            la_wave_used = false;
            la_wave_fallbacks++;
            HGX_TRY(hipMemsetAsync(LA.p, compact ? 0x00 : 0xFF, (size_t)h_off[C] * n * csz, stream));
            HGX_TRY(run_sweeps(1));
            launch_fd_build(stream, a, C, n, max_len, fd_ld, cold, max_new);
            if (rooted) launch_root_floor(stream, a, root_round_d.p, gfl.p, gB.p, root_gmax, C, n, max_len);
            HGX_TRY(hipEventRecord(ph1, stream));
            HGX_TRY(hipEventSynchronize(ph1));
        }
        float ms = 0;
        HGX_TRY(hipEventElapsedTime(&ms, ph0, ph1));
        phase_ms[0] = ms;
    }
    h_len_div = chain_len;
    E_div = En;
    laid_out = true;

    // rounds, step by step from r_lo
    if (!one_trip) HGX_TRY(hipEventRecord(ph0, stream));
    HGX_TRY(ensure_round_cap(r_lo + 2 * kStepBatch + 2));
    a = arrays();
    {   // one launch for the round tables' resets
        FillRange fr[4] = {{lr.p, (uint32_t)((size_t)G * 4), 0xFF},
                           {active.p + r_lo, (uint32_t)((size_t)(r_cap + 1 - r_lo) * 4), 0},
                           {ovf.p + r_lo, (uint32_t)((size_t)(r_cap + 2 - r_lo) * 4), 0},
                           {Bm.p, (uint32_t)((size_t)C * 4), 0}};
        launch_fill_many(stream, fr, r_lo == 0 ? 4 : 3);
        HGX_TRY(hipGetLastError());
    }
    {
        const size_t need = (size_t)2 * C * round_k_ndw(n);
        if (FD8.n < need) {
            HGX_TRY(FD8.alloc(need));
            drop_step_graph();
        }
    }
    auto round_args = [&]() {
        RoundArgs A{};
        A.n = n; A.C = C; A.sm = sm; A.nw = nw; A.Pcap = fd_ld;
        A.c_len = c_len.p; A.c_off = c_off.p; A.c_base = c_base.p; A.LA = LA.p; A.FDT = FDT.p; A.compact = compact;
        A.p_gid = p_gid.p; A.g_coin = g_coin.p; A.FD8 = FD8.p; A.ovf = ovf.p;
        A.Bm = Bm.p; A.WLA = WLA.p; A.WFD = WFD.p; A.p_round = p_round.p; A.active = active.p;
        A.lr = lr.p; A.wflag = wflag.p; A.wstat = wstat.p; A.wcoin = wcoin.p; A.Smat = Smat.p;
        A.gB = rooted ? gB.p : c_len.p;   // (any int array without roots: read, never used)
        A.gmax = rooted ? root_gmax : -1;
        return A;
    };
    // the tail of the call: every graph's last round over the rounds stepped so far, and the rows
    // [r_lo, r_hi] of the boundaries / [r_lo, r_hi) of the witness flags for the host copies
    // (rows beyond the last round are copied and dropped), then ph1
    const int r_scan = rebuild ? 0 : r_lo;
    const std::vector<int32_t> prev_last = out.last_round;
    bool tail_ready = false, la_flag_read = false;
    auto enqueue_tail = [&](int32_t r_hi) -> hipError_t {
        stage_out.clear();   // (a tail queued before more steps were needed is superseded)
        pend.clear();
        stage_used = 0;
        launch_last_round(stream, r_scan, r_hi, G, C, n, wstat.p, lr.p);
        h_lr.assign(G, -1);
        HGX_TRY(stage_d2h(h_lr.data(), lr.p, (size_t)G * 4));
        const size_t b0 = (size_t)r_lo * C;
        if (out.bm.size() < (size_t)(r_hi + 1) * C) out.bm.resize((size_t)(r_hi + 1) * C);
        if (out.wflag.size() < (size_t)r_hi * C) out.wflag.resize((size_t)r_hi * C);
        HGX_TRY(stage_d2h(out.bm.data() + b0, Bm.p + b0, ((size_t)(r_hi + 1) * C - b0) * 4));
        if (r_hi > r_lo) HGX_TRY(stage_d2h(out.wflag.data() + b0, wstat.p + b0, (size_t)r_hi * C - b0));
        if (one_trip && la_wave_used && !la_flag_read) {   // (read and re-armed once)
            HGX_TRY(copy_to_pinned(h_small + 48, counters.p + 6, 4, 0));
            la_flag_read = true;
        }
        HGX_TRY(stage_issue());
        return hipEventRecord(ph1, stream);
    };
    kbeg(K_ROUND_GATHER);
    launch_round_gather(stream, a, r_lo, C, n, fd_ld);   // W'_{r_lo}: round 0 = first event of every chain
    kend(K_ROUND_GATHER, (double)C * n * 16);
    int launched = 0, checked = 0;
    // the persistent recurrence (hgx_round_p.hip): every round in one launch; r_done = rounds
    // [r_lo, r_done) written (the last one empty)
    int32_t r_done = -1;
    auto run_persistent = [&]() -> hipError_t {
        const int ndw = round_k_ndw(n);
        if (FD8p.n < (size_t)kRoundPBufs * C * ndw) HGX_TRY(FD8p.alloc((size_t)kRoundPBufs * C * ndw));
        if (rp_gran.n < (size_t)4 * C) HGX_TRY(rp_gran.alloc((size_t)4 * C));
        if (rp_st.n < (size_t)4 + G) HGX_TRY(rp_st.alloc((size_t)4 + G));
        int32_t* fin = rp_st.p + 4;
        HGX_TRY(hipMemsetAsync(rp_gran.p, 0, (size_t)4 * C * 8, stream));   // no tag survives a call
        HGX_TRY(hipMemsetAsync(fin, 0xFF, (size_t)G * 4, stream));          // no graph finished yet
        // a chain-sharded group: this shard's chain block, its candidate rows and granules written into
        // every shard's window; the host threads of the W shards meet at the barriers
        const bool sh = grp && grp->W > 1;
        int c_lo = 0, c_hi = C;
        RoundPWindows win;
        auto gwait = [&]() -> hipError_t { return grp->wait() ? hipSuccess : hipErrorUnknown; };
        if (sh) {
            c_lo = grp->c_split[shard];
            c_hi = grp->c_split[shard + 1];
            HGX_TRY(hipStreamSynchronize(stream));
            HGX_TRY(gwait());   // every window is cleared and registered (its engine's FD8p / gran / st)
            win.nwin = grp->W;
            for (int k = 0; k <= grp->W; k++) win.c_split[k] = grp->c_split[k];
            for (int k = 0; k < grp->W; k++) {
                Engine* q = grp->eng[k];
                win.FD8p[k] = q->FD8p.p;
                win.gran[k] = q->rp_gran.p;
                win.st[k] = q->rp_st.p;
                win.FDT[k] = q->FDT.p;
                if (grp->dev[k] != dev || (grp->force_remote && k != shard)) win.remote |= 1u << k;
            }
            if (rp_win.n < sizeof(RoundPWindows)) HGX_TRY(rp_win.alloc(sizeof(RoundPWindows)));
            HGX_TRY(hipMemcpyAsync(rp_win.p, &win, sizeof(RoundPWindows), hipMemcpyHostToDevice, stream));
            HGX_TRY(hipStreamSynchronize(stream));
        }
        const RoundPWindows* win_d = sh ? (const RoundPWindows*)rp_win.p : nullptr;
        // n > 256 (one graph): k_round_pb, a workgroup per chain with events (hgx_round_pb.hip)
        const bool big = n > 256;
        int na = 0;
        if (big) {
            h_amap.clear();
            for (int c = 0; c < C; c++)
                if (chain_len[c] > 0) h_amap.push_back(c);
            na = (int)h_amap.size();
            if (na == 0) return hipErrorCooperativeLaunchTooLarge;   // (nothing to step: the steps' path)
            if (rp_amap.n < (size_t)C) HGX_TRY(rp_amap.alloc((size_t)C));
            HGX_TRY(hipMemcpyAsync(rp_amap.p, h_amap.data(), (size_t)na * 4, hipMemcpyHostToDevice, stream));
        }
        int32_t s = r_lo, last = -1;
        int finished = 0;
        for (int init = 1;; init = 0) {
            if (r_cap - 1 <= s + 1) {
                HGX_TRY(ensure_round_cap(s + 64));
                a = arrays();
            }
            HGX_TRY(hipMemsetAsync(rp_st.p, 0, 16, stream));
            if (big) {
                kbeg(K_ROUND_SEARCH);
                HGX_TRY(launch_round_pb(stream, round_args(), FD8p.p, rp_gran.p, rp_st.p, fin, rp_amap.p, na, s, r_cap - 1,
                                        num_cus, init != 0));
                kend(K_ROUND_SEARCH, 0);
            } else if (sh && init) {
                // W'_{r_lo} of this shard's chains into every window; every shard's launch starts once
                // every window holds the whole W'_{r_lo}
                HGX_TRY(launch_round_p(stream, round_args(), FD8p.p, rp_gran.p, rp_st.p, fin, s, r_cap - 1, 2, num_cus,
                                       c_lo, c_hi, win_d, win.nwin));
                HGX_TRY(hipStreamSynchronize(stream));
                HGX_TRY(gwait());
            }
            if (!big) {
                kbeg(K_ROUND_SEARCH);
                HGX_TRY(launch_round_p(stream, round_args(), FD8p.p, rp_gran.p, rp_st.p, fin, s, r_cap - 1, sh ? 0 : init,
                                       num_cus, c_lo, c_hi, win_d, sh ? win.nwin : 1));
                kend(K_ROUND_SEARCH, 0);
            }
            HGX_TRY(hipMemcpyAsync(h_small + 56, rp_st.p, 16, hipMemcpyDeviceToHost, stream));
            HGX_TRY(hipStreamSynchronize(stream));
            round_p_runs++;
            round_p_ovf += h_small[59];
            int32_t st0 = h_small[56], st1 = h_small[57], st2 = h_small[58], st3 = h_small[59];
            if (sh) {
                // every shard's outcome; then this shard's round rows into every shard's tables
                for (int k = 0; k < 4; k++) grp->st[shard][k] = h_small[56 + k];
                HGX_TRY(gwait());
                for (int k = 0; k < grp->W; k++) {
                    if (grp->st[k][0] != 0 && st0 == 0) {
                        st0 = grp->st[k][0];
                        st3 = grp->st[k][3];
                    }
                    st1 = std::max(st1, grp->st[k][1]);
                    st2 = std::max(st2, grp->st[k][2]);
                }
                if (st0 == 0) HGX_TRY(share_round_rows(s, std::min(st1 + 1, r_cap)));
                HGX_TRY(gwait());
            }
            if (st0 != 0) {   // a workgroup gave up waiting: st[0] = 1 + its chain, st[3] its round
                round_p_fail_chain = st0 - 1;
                round_p_fail_round = st3;
                return hipErrorLaunchTimeOut;
            }
            last = std::max(last, st1);
            finished += st2;
            if (finished >= G) {
                r_done = last + 1;
                // graphs that finished earlier: empty rows up to the last round (k_last_round,
                // fame and the host copies read every graph's rows of every round)
                launch_round_p_tail(stream, round_args(), fin, last);
                if (big) launch_round_pb_silent(stream, round_args(), r_lo, last);
                kbeg(K_ROUND_GATHER);
                launch_round_p_post(stream, round_args(), r_lo, last);
                kend(K_ROUND_GATHER, (double)(last - r_lo + 1) * C * n * (sizeof(int32_t) + (compact ? 2 : 4)));
                return hipGetLastError();
            }
            s = st1;   // the round tables' capacity: continue from there
        }
    };
    // the whole-graph recurrence (hgx_round_g.hip, n <= 16): one workgroup per graph, every round
    // in one launch, nothing shared between workgroups; relaunched from the round tables'
    // capacity (its prologue rebuilds a round's state from Bm alone)
    auto run_graph = [&]() -> hipError_t {
        if (rp_st.n < (size_t)4 + G) HGX_TRY(rp_st.alloc((size_t)4 + G));
        int32_t* fin = rp_st.p + 4;
        HGX_TRY(hipMemsetAsync(fin, 0xFF, (size_t)G * 4, stream));
        int32_t s = r_lo, last = -1;
        int finished = 0;
        for (;;) {
            if (r_cap - 1 <= s + 1) {
                HGX_TRY(ensure_round_cap(s + 64));
                a = arrays();
            }
            HGX_TRY(hipMemsetAsync(rp_st.p, 0, 16, stream));
            kbeg(K_ROUND_SEARCH);
            HGX_TRY(launch_round_g(stream, round_args(), rp_st.p, fin, s, r_cap - 1));
            kend(K_ROUND_SEARCH, 0);
            HGX_TRY(hipMemcpyAsync(h_small + 56, rp_st.p, 16, hipMemcpyDeviceToHost, stream));
            HGX_TRY(hipStreamSynchronize(stream));
            round_g_runs++;
            round_p_ovf += h_small[59];
            last = std::max(last, h_small[57]);
            finished += h_small[58];
            if (finished >= G) {
                r_done = last + 1;
                launch_round_p_tail(stream, round_args(), fin, last);
                kbeg(K_ROUND_GATHER);
                launch_round_p_post(stream, round_args(), r_lo, last);
                kend(K_ROUND_GATHER, (double)(last - r_lo + 1) * C * n * (sizeof(int32_t) + (compact ? 2 : 4)));
                return hipGetLastError();
            }
            s = h_small[57];   // the round tables' capacity: continue from there
        }
    };
    const bool graph_ok = !rooted && round_g_ok(n, nw) && (round_kernel == 0 || round_kernel == 4) && !grp;
    if (graph_ok) HGX_TRY(run_graph());
    // the persistent launch pays a fixed cost (every chain's window staged, 256 resident
    // workgroups) that a call resuming for a few rounds does not recover: those use the steps
    // (a chain-sharded group always runs it: its shards build firstDescendants for their own chains only)
    if (!graph_ok && !rooted && (round_kernel == 3 || (round_kernel == 0 && rebuild) || grp) &&
        (round_p_ok(n, C, num_cus) || (round_pb_ok(n, G) && !grp && round_pb_enabled))) {
        const hipError_t pe = run_persistent();
        if (pe != hipSuccess) {
            // redo the rounds with the per-launch steps (a timed-out launch left partial rows)
            (void)hipGetLastError();
            if (pe != hipErrorLaunchTimeOut && pe != hipErrorCooperativeLaunchTooLarge) return pe;
            round_p_fallbacks++;
            r_done = -1;
            if (grp) {
                // the steps read every candidate's firstDescendants: this shard built its own chains'
                // only, so the whole table is rebuilt here, and W'_{r_lo} gathered again from it
                launch_fd_build(stream, a, C, n, max_len, fd_ld, nullptr, 0);
                launch_round_gather(stream, a, r_lo, C, n, fd_ld);
            }
        }
    }
    if (r_done >= 0 && rebuild && !graph_ok && !rooted && round_kernel == 0) {
        // the resumed calls that follow use the per-launch steps: their hipGraphs are captured and
        // instantiated now, inside this (long) rebuild call, not in the first short resumed one
        // (c2: a 7 ms first resumed call)
        for (int i = 1; i <= 2; i++)
            if (!step_g[i].exec) HGX_TRY(capture_steps(step_g[i], round_args(), 0, i == 1 ? kStepBatchSmall : 2 * kStepBatchSmall));
    }
    if (r_done < 0) launch_round_k_gather(stream, round_args(), r_lo);   // W'_{r_lo} rebased for k_round_k
    // a rebuild replays kStepBatch steps per hipGraph; a resumed call (a few rounds) 2 or 4: a
    // round holds ~10-14 events per chain, so fewer than 6 new events per chain rarely take
    // more than two steps (a second batch costs another host round trip)
    const bool few = (En - E0) < 6 * (int64_t)C;
    StepGraph& sgr = step_g[rebuild ? 0 : few ? 1 : 2];
    const int nb = rebuild ? kStepBatch : few ? kStepBatchSmall : 2 * kStepBatchSmall;
    if (r_done < 0) {   // n <= 1024 (hgx_create's limit)
        // nb step nodes replayed as one hipGraph; before each replay the nodes' round
        // arguments are rewritten (hipGraphExecKernelNodeSetParams), so a step knows its
        // round without a dependent device load. Batch i+1 is queued before the host looks
        // at batch i's "any candidate left" flag (pipelined check).
        auto launch_batch = [&]() -> hipError_t {
            const int need = r_lo + (launched + 2) * nb + 2;
            if (need > r_cap) {
                HGX_TRY(ensure_round_cap(need));
                a = arrays();
            }
            const int kern = (rooted || round_kernel != 1) ? 0 : 1;   // root floors: per-candidate step only
            const RoundArgs cur = round_args();
            if (!sgr.exec || sgr.kernel != kern || sgr.compact != compact || sgr.nb != nb || sgr.args.gB != cur.gB ||
                sgr.args.gmax != cur.gmax)
                HGX_TRY(capture_steps(sgr, cur, kern, nb));
            const int slot = launched & 1;
            // the batch's last step writes round + 1 into this slot's host-mapped flag when a
            // chain still has events beyond its boundary (no D2H copy between the replays)
            sgr.args_last[slot] = sgr.args;
            sgr.args_last[slot].hflag = d_flag + slot;
            h_flag[slot] = 0;
            for (int k = 0; k < nb; k++) {
                sgr.round[k] = r_lo + launched * nb + k;
                void* args[2] = {(void*)(k == nb - 1 ? &sgr.args_last[slot] : &sgr.args), (void*)&sgr.round[k]};
                hipKernelNodeParams kp = sgr.params[k];
                kp.kernelParams = args;
                kp.extra = nullptr;
                HGX_TRY(hipGraphExecKernelNodeSetParams(sgr.exec, sgr.nodes[k], &kp));
            }
            // nb step kernels per replay, every replay bracketed by timing events when the round
            // search is timed (a sample of replays misjudged the pass: the first replays' rounds hold
            // most of the events, the last ones' steps find little left -- c5: 19.4 ms sampled
            // against 12.8 ms in the rocprofv3 trace)
            const bool sample = true;
            kbeg(K_ROUND_SEARCH, sample, nb);
            HGX_TRY(hipGraphLaunch(sgr.exec, stream));
            if (sample) kend(K_ROUND_SEARCH, 0);
            HGX_TRY(hipEventRecord(flag_ev[slot], stream));
            launched++;
            return hipSuccess;
        };
        // a rebuild keeps two batches in flight; a resumed call usually ends within its first
        // batch, so it waits for that batch's flag before queueing another
        HGX_TRY(launch_batch());
        if (rebuild) HGX_TRY(launch_batch());
        if (one_trip) {
            // the tail queued right behind the first batch: when that batch ends the rounds (the
            // usual resumed call), the call has made its only host round trip here
            HGX_TRY(enqueue_tail(r_lo + launched * nb));
            HGX_TRY(hipEventSynchronize(ph1));
            const int more = __atomic_load_n(&h_flag[0], __ATOMIC_ACQUIRE);
            checked = 1;
            if (!more) tail_ready = true;
            else {
                if (launched == checked) HGX_TRY(launch_batch());
                HGX_TRY(launch_batch());
            }
        }
        while (!tail_ready) {
            HGX_TRY(hipEventSynchronize(flag_ev[checked & 1]));
            const int more = __atomic_load_n(&h_flag[checked & 1], __ATOMIC_ACQUIRE);
            checked++;
            if (!more) break;
            if (launched == checked) HGX_TRY(launch_batch());   // no batch in flight
            HGX_TRY(launch_batch());
        }
    }
    if (!tail_ready) {
        HGX_TRY(enqueue_tail(r_done >= 0 ? r_done : r_lo + launched * nb));
        HGX_TRY(hipEventSynchronize(ph1));
    }
    if (one_trip && la_wave_used && h_small[48] != 0) {
        // a wavefront lane gave up waiting (bounded spins): the call again as a rebuild, with
        // the sweeps for lastAncestors
        la_wave_fallbacks++;
        laid_out = false;
        stage_out.clear();
        const int keep = la_kernel;
        la_kernel = 1;
        const hipError_t re = divide_rounds(En, chain_len, chain_base, out);
        la_kernel = keep;
        return re;
    }
    stage_flush();
    // rounds below r_lo are unchanged and every round up to a graph's last one has witnesses,
    // so only [r_lo, R) is scanned: last = max(that, min(previous last, r_lo - 1))
    if (r_scan > 0)
        for (int g = 0; g < G; g++) {
            const int32_t pl = g < (int)prev_last.size() ? prev_last[g] : -1;
            h_lr[g] = std::max(h_lr[g], std::min(pl, r_scan - 1));
        }
    out.last_round.assign(h_lr.begin(), h_lr.end());
    int32_t mx = -1;
    for (int g = 0; g < G; g++) mx = std::max(mx, out.last_round[g]);
    R = mx + 1;
    out.R = R;
    out.r_lo = std::min(r_lo, R);
    // the host copies keep the rows below r_lo (rows the tail copied beyond R are dropped)
    out.bm.resize((size_t)(R + 1) * C);
    out.wflag.resize((size_t)R * C);
    launch_wcoin(stream, a, out.r_lo, R, C);   // (DecideFame reads the coins on this stream)
    HGX_TRY(hipGetLastError());
    float ms = 0;
    if (one_trip) {
        HGX_TRY(hipEventElapsedTime(&ms, ph0, ph2));
        phase_ms[0] = ms;
        HGX_TRY(hipEventElapsedTime(&ms, ph2, ph1));
    } else {
        HGX_TRY(hipEventElapsedTime(&ms, ph0, ph1));
    }
    phase_ms[1] = ms;
    step_prof_dump();   // -DHGX_STEP_PROF builds only
    return collect_kernel_times();
}

// 1 + the lowest round of an event not yet received (rounds below it cannot be a
// roundReceived any more), R when every event is received; max_unrecv = most unreceived
// events of one chain
int32_t Engine::recv_round_lo(const RoundsHost& rh, int& max_unrecv) const {
    int32_t lo = R;
    max_unrecv = 0;
    if (E_div == 0 || rh.R == 0) return lo;
    for (int c = 0; c < C; c++) {
        const int32_t k = h_fu[c], len = h_len_div[c];
        if (k >= len) continue;
        max_unrecv = std::max(max_unrecv, len - k);
        int32_t a = 0, b = rh.R;   // round of offset k: largest r with bm[r][c] <= k
        while (a < b) {
            const int32_t mid = (a + b + 1) / 2;
            if (rh.bm[(size_t)mid * C + c] <= k) a = mid; else b = mid - 1;
        }
        lo = std::min(lo, a + 1);
    }
    return lo;
}

// ---- DecideFame -----------------------------------------------------------------
hipError_t Engine::decide_fame(int32_t r0, std::vector<int8_t>& fame_out) {
    stage_out.clear();   // every earlier call synchronized: the staging is free
    pend.clear();
    stage_used = 0;
    // rows [r0, R) are copied back below; the caller reads no row below r0, so the buffer only
    // grows (no O(R C) clear per call: the chunked schedule calls this thousands of times)
    if (fame_out.size() < (size_t)R * C) fame_out.resize((size_t)R * C, 0);
    r0 = std::max(r0, 0);
    if (R <= r0) return hipSuccess;
    DevArrays a = arrays();
    HGX_TRY(hipEventRecord(ph0, stream));
    HGX_TRY(hipGetLastError());   // (an error left by DivideRounds' launches surfaces there, not here)
    kbeg(K_FAME);
    launch_fame(stream, a, r0, R, C, n, nw, sm, G, fame_tally);
    kend(K_FAME, 0);
    HGX_TRY(hipGetLastError());
    const size_t o = (size_t)r0 * C;
    HGX_TRY(stage_d2h(fame_out.data() + o, fame.p + o, fame_out.size() - o));
    HGX_TRY(stage_issue());
    HGX_TRY(hipEventRecord(ph1, stream));
    HGX_TRY(hipEventSynchronize(ph1));
    stage_flush();
    float ms = 0;
    HGX_TRY(hipEventElapsedTime(&ms, ph0, ph1));
    phase_ms[2] = ms;
    return collect_kernel_times();
}

// ---- FindOrder ------------------------------------------------------------------
hipError_t Engine::find_order(const std::vector<uint8_t>& el, const std::vector<uint8_t>& famous,
                              const std::vector<uint8_t>& ure, int32_t r0, int max_unrecv, OrderHost& out) {
    HGX_TRY(find_order_begin(el, famous, ure, r0, max_unrecv, out));
    return find_order_end(out, nullptr);
}

// threshold and roundReceived (every chain), consensus timestamps of the shard's chains
hipError_t Engine::find_order_begin(const std::vector<uint8_t>& el, const std::vector<uint8_t>& famous,
                                    const std::vector<uint8_t>& ure, int32_t r0, int max_unrecv, OrderHost& out) {
    stage_out.clear();   // every earlier call synchronized: the staging is free
    pend.clear();
    stage_used = 0;
    out = OrderHost();
    fo_m = 0;
    fo_cnt.assign(C, 0);
    if (R == 0 || E_div == 0 || max_unrecv == 0 || r0 >= R) return hipSuccess;
    DevArrays a = arrays();
    HGX_TRY(hipEventRecord(ph0, stream));
    const size_t o = (size_t)r0 * C;
    HGX_TRY(stage_h2d(elig.p, el.data(), (size_t)G * R));
    HGX_TRY(stage_h2d(fw.p + o, famous.data() + o, (size_t)R * C - o));
    HGX_TRY(stage_h2d(ur_empty.p, ure.data(), (size_t)G));
    HGX_TRY(stage_issue());
    if (WLAT.n < (size_t)R * C * n) {   // grown geometrically: R grows by a round or two per call
        // the first allocation covers the round tables' capacity (at most 256 M entries): each
        // later doubling was a synchronous free + allocation inside one FindOrder of the chunked
        // schedule (0.6-0.9 ms outliers)
        const size_t want = (size_t)R * C * n + (size_t)C * n;
        const size_t first = WLAT.n ? 0 : std::min((size_t)r_cap * C * n, (size_t)1 << 28);
        HGX_TRY(WLAT.alloc(std::max(want, std::max(2 * WLAT.n, first))));
        a = arrays();
    }
    kbeg(K_THRESHOLD);
    launch_wla_transpose(stream, a, r0, R, G, C, n);
    launch_threshold(stream, a, r0, R, C, n);
    kend(K_THRESHOLD, 0);
    {
        FillRange fr[2] = {{counters.p, 8, 0}, {rcnt.p, (uint32_t)((size_t)C * 4), 0}};
        launch_fill_many(stream, fr, 2);
        HGX_TRY(hipGetLastError());
    }
    kbeg(K_ROUND_RECEIVED);
    launch_round_received(stream, a, R, C, n, max_unrecv);
    kend(K_ROUND_RECEIVED, 0);
    HGX_TRY(copy_to_pinned(h_small, counters.p, 8));
    HGX_TRY(stage_d2h(fo_cnt.data(), rcnt.p, (size_t)C * 4));
    HGX_TRY(stage_issue());
    HGX_TRY(hipStreamSynchronize(stream));
    stage_flush();
    fo_m = h_small[0];
    out.panic = h_small[1] != 0;
    out.m = fo_m;
    int max_cnt = 0, unrecv = 0;
    for (int c = 0; c < C; c++) unrecv += h_len_div[c] - h_fu[c];
    for (int c = shard_lo; c < shard_hi; c++) max_cnt = std::max(max_cnt, fo_cnt[c]);
    kadd_bytes(K_ROUND_RECEIVED, (double)unrecv * 16);
    if (out.panic || fo_m == 0) {
        fo_m = 0;
        return collect_kernel_times();
    }
    kbeg(K_CTS);
    if (cts_kernel != 2 || !launch_cts_pipe(stream, a, shard_lo, shard_hi - shard_lo, C, n, fd_ld, max_cnt))
        launch_cts(stream, a, shard_lo, shard_hi - shard_lo, C, n, fd_ld, max_cnt);
    int64_t own = 0;
    for (int c = shard_lo; c < shard_hi; c++) own += fo_cnt[c];
    kend(K_CTS, (double)own * (4.0 * n + 8.0 * n));
    return hipSuccess;
}

// the consensus timestamps of the events newly received on chains [lo, hi), chain-major
// ([fu, fu + rcnt) of each chain): the values a shard exchanges
int64_t Engine::shard_values(int lo, int hi) const {
    int64_t k = 0;
    for (int c = lo; c < hi && c < (int)fo_cnt.size(); c++) k += fo_cnt[c];
    return k;
}

hipError_t Engine::shard_copy(int lo, int hi, void* buf, bool on_device, bool to_buf) {
    const int64_t cnt = shard_values(lo, hi);
    if (cnt == 0) return hipSuccess;
    std::vector<int32_t> offs(C + 1, 0);   // exclusive scan of the counts over [lo, hi)
    for (int c = lo; c < hi; c++) offs[c + 1] = offs[c] + fo_cnt[c];
    if (sh_off.n < (size_t)C + 1) HGX_TRY(sh_off.alloc((size_t)C + 1));
    HGX_TRY(hipMemcpyAsync(sh_off.p, offs.data(), (size_t)(C + 1) * 4, hipMemcpyHostToDevice, stream));
    int64_t* dev = (int64_t*)buf;
    if (!on_device) {
        if (sh_buf.n < (size_t)cnt) HGX_TRY(sh_buf.alloc((size_t)cnt));
        dev = sh_buf.p;
        if (!to_buf) HGX_TRY(hipMemcpyAsync(dev, buf, (size_t)cnt * 8, hipMemcpyHostToDevice, stream));
    }
    launch_cts_shard_copy(stream, arrays(), lo, hi, sh_off.p, dev, to_buf ? 1 : 0);
    if (!on_device && to_buf) HGX_TRY(hipMemcpyAsync(buf, dev, (size_t)cnt * 8, hipMemcpyDeviceToHost, stream));
    return hipStreamSynchronize(stream);
}

// sort by (graph, rr, cts, S), blocks
// order_dst (pinned, room for the m received events): the order is copied there with the block
// tables, in the same host round trip
hipError_t Engine::find_order_end(OrderHost& out, int32_t* order_dst) {
    HGX_TRY(payload_wait_S());   // (the sort's tie-break reads S)
    out.blk_cnt.assign((size_t)G * std::max(R, 1), 0);
    out.blk_ntx.assign((size_t)G * std::max(R, 1), 0);
    out.blk_loaded.assign((size_t)G * std::max(R, 1), 0);
    out.blk_nil.assign((size_t)G * std::max(R, 1), 0);
    const int32_t m = fo_m;
    if (m == 0) return hipSuccess;
    fo_m = 0;
    DevArrays a = arrays();
    uint32_t* vals = nullptr;
    const bool small = sort_small_ok(m);
    {   // one launch for the per-(graph, rr) block tables (and the small sort's ranks)
        FillRange fr[5] = {{blk_cnt.p, (uint32_t)((size_t)G * R * 4), 0},
                           {blk_loaded.p, (uint32_t)((size_t)G * R * 4), 0},
                           {blk_ntx.p, (uint32_t)((size_t)G * R * 8), 0},
                           {blk_nil.p, (uint32_t)((size_t)G * R), 0},
                           {val_b.p, (uint32_t)((size_t)m * 4), 0}};
        launch_fill_many(stream, fr, small ? 5 : 4);
        HGX_TRY(hipGetLastError());
    }
    // a large order (a full pass: 40 MB at c3) is written straight into the pinned host arena
    // (coalesced writes over the host link while the kernel runs) instead of a D2H copy after it --
    // by the bucket sort itself, which finishes every bucket it places (k_seg_sort, SortFinish: its
    // host-link writes overlap the other buckets' sorting), or by k_finish_order after the other
    // sorts; a small one comes back with the block tables in the copy launch
    // A large order into a pinned order_dst: the bucket sort runs in kOrderParts parts of about equal
    // event counts, each part's order copied to the host (DMA on stream_o) while the next part sorts
    // (round 6: the sort writing the gids over the host link itself took as long as sorting and copying
    // one after the other, c3 1.0 + 0.85 ms); the other sorts write the order straight into the arena.
    void* dst_dev = nullptr;
    const bool big_dst = order_dst && (size_t)m * 4 > kCopyKernelMax &&
                         hipHostGetDevicePointer(&dst_dev, order_dst, 0) == hipSuccess && dst_dev;
    if (order_dst && !big_dst) (void)hipGetLastError();   // (a pageable order_dst: the query's error is not sticky)
    bool direct = false, finished = false, piped = false;
    auto go_direct = [&]() {
        if (big_dst) {
            a.order_gid = (int32_t*)dst_dev;
            direct = true;
        }
    };
    if (small) {
        go_direct();
        kbeg(K_SORT);
        launch_sort_small(stream, a, m, n, &vals);
        kend(K_SORT, (double)m * 24.0);
    } else {
        // sort keys: cts range, then (graph, rr); and the (graph, rr) buckets' sizes (the segmented
        // sort's condition), read back in the same round trip
        const unsigned long long init[3] = {~0ull, 0ull, 0ull};
        HGX_TRY(hipMemcpyAsync(minmax.p, init, 24, hipMemcpyHostToDevice, stream));
        const int64_t nseg64 = (int64_t)G * R;
        const bool seg_try = sort_seg_enabled && nseg64 >= 1 && nseg64 <= (int64_t)1 << 24;
        const int nseg = (int)nseg64;
        if (seg_try) {   // (the bucket counts with the timestamp range, one pass)
            // sized for the round tables' capacity (then doubled): an exact-size reallocation whenever R
            // had grown since the last bucket sort was a hipFree + hipMalloc inside a chunked-schedule
            // FindOrder (1-2 ms calls)
            if (seg_off.n < (size_t)nseg + 1) {
                const size_t cap = std::max({(size_t)nseg + 1, (size_t)G * std::max(r_cap, 1) + 1, 2 * seg_off.n});
                HGX_TRY(seg_off.alloc(cap));
                HGX_TRY(seg_cur.alloc(cap));
            }
            HGX_TRY(hipMemsetAsync(seg_off.p, 0, (size_t)nseg * 4, stream));
            launch_seg_count(stream, a, m, R, n, nseg, seg_off.p, (unsigned long long*)minmax.p + 2);
        } else {
            launch_minmax(stream, a, m);
        }
        // (the bucket counts come back in the same round trip; below kOrderPipeMin the parts' launch tails
        // cost more than the copy they hide -- c2, 4 MB: order sort 0.23 -> 0.43 ms -- and the sort writes
        // the order straight into the arena)
        const bool want_cuts = seg_try && big_dst && (size_t)m * 4 >= kOrderPipeMin;
        if (want_cuts && h_segc_n < (size_t)nseg) {
            if (h_segc) HGX_TRY(hipHostFree(h_segc));
            h_segc = nullptr;
            h_segc_n = 0;
            const size_t cap = std::max((size_t)nseg, (size_t)G * std::max(r_cap, 1));
            HGX_TRY(hipHostMalloc((void**)&h_segc, cap * 4, hipHostMallocDefault));
            h_segc_n = cap;
        }
        if (want_cuts) HGX_TRY(hipMemcpyAsync(h_segc, seg_off.p, (size_t)nseg * 4, hipMemcpyDeviceToHost, stream));
        unsigned long long mm[3];
        HGX_TRY(hipMemcpyAsync(mm, minmax.p, 24, hipMemcpyDeviceToHost, stream));
        HGX_TRY(hipStreamSynchronize(stream));
        const int64_t cmin = (int64_t)(mm[0] ^ 0x8000000000000000ull);
        const int64_t cmax = (int64_t)(mm[1] ^ 0x8000000000000000ull);
        const int cts_bits = bitlen((uint64_t)(cmax - cmin));
        const int seg_bits = bitlen((uint64_t)G * (uint64_t)R - 1);
        uint64_t* keys = nullptr;
        kbeg(K_SORT);
        // (a refused LDS limit for the 1 024-thread bucket sort is reported before anything is
        // launched, and the radix passes run instead)
        const bool seg_ok = seg_try && cts_bits + seg_bits <= 64 && mm[2] >= 1 &&
                            mm[2] <= (unsigned long long)seg_sort_cap();
        // parts: cuts[k] = the first bucket of part k, off[k] = its first element of the order
        std::vector<int> cuts;
        std::vector<int64_t> off;
        if (seg_ok && want_cuts) {
            cuts.push_back(0);
            off.push_back(0);
            int64_t cum = 0;
            for (int sg = 0; sg < nseg && (int)cuts.size() < kOrderParts; sg++) {
                cum += h_segc[sg];
                if (cum * kOrderParts >= (int64_t)m * (int64_t)cuts.size() && sg + 1 < nseg) {
                    cuts.push_back(sg + 1);
                    off.push_back(cum);
                }
            }
            cuts.push_back(nseg);
            off.push_back(m);
            piped = cuts.size() > 2;
            if (piped && !stream_o) {
                HGX_TRY(hipStreamCreateWithFlags(&stream_o, hipStreamNonBlocking));
                for (auto& e : ev_o) HGX_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
            }
        }
        // (a failure here is fatal, not a fallback to the radix passes: earlier parts' copies are queued)
        hipError_t part_err = hipSuccess;
        const std::function<hipError_t(int)> copy_part = [&](int k) -> hipError_t {
            const int64_t o0 = off[k], cnt = off[k + 1] - off[k];
            if (cnt <= 0) return hipSuccess;
            part_err = hipEventRecord(ev_o[k], stream);
            if (part_err == hipSuccess) part_err = hipStreamWaitEvent(stream_o, ev_o[k], 0);
            if (part_err == hipSuccess)
                part_err = hipMemcpyAsync(order_dst + o0, order_gid.p + o0, (size_t)cnt * 4, hipMemcpyDeviceToHost,
                                          stream_o);
            return part_err;
        };
        if (seg_ok && !piped) go_direct();
        const bool seg = seg_ok && launch_sort_seg(stream, a, m, cmin, cts_bits, R, n, nseg, seg_off.p, seg_cur.p,
                                                   (int)mm[2], &vals, &keys, piped ? &cuts : nullptr,
                                                   piped ? copy_part : nullptr) == hipSuccess;
        HGX_TRY(part_err);
        if (seg) {
            sort_seg_runs++;
            finished = true;
            if (piped) {   // the stream waits for the last part's copy
                HGX_TRY(hipEventRecord(ev_o[kOrderParts], stream_o));
                HGX_TRY(hipStreamWaitEvent(stream, ev_o[kOrderParts], 0));
            }
            kend(K_SORT, (double)m * 24.0 * 2);   // (bucket scatter + in-LDS sort: two passes' bytes)
        } else {
            (void)hipGetLastError();
            piped = false;
            direct = false;
            a.order_gid = order_gid.p;
            go_direct();
            launch_sort(stream, a, m, cmin, cts_bits, R, n, seg_bits, &vals, &keys);
            kend(K_SORT, (double)m * 24.0 *
                             (cts_bits + seg_bits <= 64 ? (cts_bits + seg_bits + 7) / 8
                                                        : (cts_bits + 7) / 8 + (seg_bits + 7) / 8));
        }
    }
    if (!finished) launch_finish_order(stream, a, m, vals, R, n);
    launch_fu_advance(stream, a, C);
    for (int c = 0; c < C; c++) h_fu[c] += fo_cnt[c];
    stage_out.clear();
    pend.clear();
    stage_used = 0;
    HGX_TRY(stage_d2h(out.blk_cnt.data(), blk_cnt.p, (size_t)G * R * 4));
    HGX_TRY(stage_d2h(out.blk_ntx.data(), blk_ntx.p, (size_t)G * R * 8));
    HGX_TRY(stage_d2h(out.blk_loaded.data(), blk_loaded.p, (size_t)G * R * 4));
    HGX_TRY(stage_d2h(out.blk_nil.data(), blk_nil.p, (size_t)G * R));
    if (order_dst && !direct && !piped) HGX_TRY(copy_to_pinned(order_dst, order_gid.p, (size_t)m * 4));
    HGX_TRY(stage_issue());
    HGX_TRY(hipEventRecord(ph1, stream));
    HGX_TRY(hipEventSynchronize(ph1));
    stage_flush();
    float ms = 0;
    HGX_TRY(hipEventElapsedTime(&ms, ph0, ph1));
    phase_ms[3] = ms;
    return collect_kernel_times();
}

hipError_t Engine::copy_order(int32_t* dst, int64_t first, int64_t count) {
    if (count <= 0) return hipSuccess;
    return hipMemcpyAsync(dst, order_gid.p + first, (size_t)count * 4, hipMemcpyDeviceToHost, stream);
}

hipError_t Engine::reset_received() {
    if (E > 0) {
        HGX_TRY(hipMemsetAsync(g_rr.p, 0xFF, (size_t)E * 4, stream));
        HGX_TRY(hipMemsetAsync(g_cts.p, 0, (size_t)E * 8, stream));
    }
    E_div = 0;
    R = 0;
    laid_out = false;
    return hipStreamSynchronize(stream);
}

// ---- getters --------------------------------------------------------------------
hipError_t Engine::get_rounds(std::vector<int32_t>& round_by_gid) {
    round_by_gid.assign((size_t)E_div, -1);
    if (E_div == 0) return hipSuccess;
    launch_gather_i32(stream, E_div, p_round.p, g_pos.p, recv_list.p);
    HGX_TRY(hipMemcpyAsync(round_by_gid.data(), recv_list.p, (size_t)E_div * 4, hipMemcpyDeviceToHost, stream));
    return hipStreamSynchronize(stream);
}

hipError_t Engine::get_received(std::vector<int32_t>& rr, std::vector<int64_t>& cts) {
    rr.assign((size_t)E, -1);
    cts.assign((size_t)E, 0);
    if (E == 0) return hipSuccess;
    HGX_TRY(hipMemcpyAsync(rr.data(), g_rr.p, (size_t)E * 4, hipMemcpyDeviceToHost, stream));
    HGX_TRY(hipMemcpyAsync(cts.data(), g_cts.p, (size_t)E * 8, hipMemcpyDeviceToHost, stream));
    return hipStreamSynchronize(stream);
}

hipError_t Engine::get_coords(int64_t gid, int32_t* la, int32_t* fd) {
    int32_t pos = 0;
    HGX_TRY(hipMemcpyAsync(&pos, g_pos.p + gid, 4, hipMemcpyDeviceToHost, stream));
    HGX_TRY(hipStreamSynchronize(stream));
    if (!compact) {
        HGX_TRY(hipMemcpyAsync(la, LA.p + (size_t)pos * n, (size_t)n * 4, hipMemcpyDeviceToHost, stream));
        HGX_TRY(hipMemcpy2DAsync(fd, 4, FDT.p + pos, (size_t)fd_ld * 4, 4, (size_t)n, hipMemcpyDeviceToHost, stream));
        return hipStreamSynchronize(stream);
    }
    std::vector<uint16_t> l16(n), f16(n);
    const uint16_t* la16 = (const uint16_t*)LA.p;
    const uint16_t* fd16 = (const uint16_t*)FDT.p;
    HGX_TRY(hipMemcpyAsync(l16.data(), la16 + (size_t)pos * n, (size_t)n * 2, hipMemcpyDeviceToHost, stream));
    HGX_TRY(hipMemcpy2DAsync(f16.data(), 2, fd16 + pos, (size_t)fd_ld * 2, 2, (size_t)n, hipMemcpyDeviceToHost, stream));
    HGX_TRY(hipStreamSynchronize(stream));
    for (int i = 0; i < n; i++) {   // Coord<uint16_t> decode
        la[i] = (int32_t)l16[i] - 1;
        fd[i] = f16[i] == 0xFFFF ? 2147483647 : (int32_t)f16[i];
    }
    return hipSuccess;
}

}  // namespace hgx


namespace hgx {
void StepGraph::drop() {
    if (exec) (void)hipGraphExecDestroy(exec);
    if (graph) (void)hipGraphDestroy(graph);
    exec = nullptr;
    graph = nullptr;
}

void Engine::drop_step_graph() {
    for (auto& g : step_g) g.drop();
}
}  // namespace hgx
