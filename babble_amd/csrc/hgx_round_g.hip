// Whole-graph round recurrence for small graphs (n <= 16 chains): ONE workgroup runs every
// round of one graph's DivideRounds (RoundInc, hashgraph.go:285-305; StronglySee :170-198;
// DivideRounds :616-646) with nothing but LDS between the chains. DESIGN.md §3.3b.
//
// Same result as k_round_k / k_round_p: round s of chain c finds Bm[s+1][c] = the first offset
// k >= Bm[s][c] whose event strongly sees >= SM candidates of W'_s, by a 5-level binary search per
// candidate over a window of 31 probe rows, then the first probe where #{K(w) <= p} >= SM. What
// changes is the geometry:
//  * lane (c, w) = 16 c + w searches candidate w over chain c's window, so the 16 lanes of a chain
//    sit in one wave: the chain's staging ring, its K(w) values and any later window are private
//    to that wave (LDS, no barrier);
//  * the probe rows are compared RAW, straight from the staging ring: n <= 16 coordinates are at
//    most 8 packed u16 dwords (or 16 int32), so the search needs no rebased 8-bit window (the
//    per-round rebase of 31 rows, of which the search reads 5, and the exact-compare fallback for
//    rows over 8 bits both disappear). Compact coordinates: lastAncestor + 1 >= firstDescendant + 1
//    by a packed saturating subtract (v_pk_sub_u16 clamp, zero = seen), exact for every value;
//  * what crosses chains is W'_{s+1} (each new candidate's firstDescendants row and position):
//    written to LDS by the chain's own lanes at the end of round s, read by every wave after ONE
//    workgroup barrier, buffers by round parity;
//  * the raw lastAncestors rows and firstDescendants columns of each chain are staged by LDS-DMA
//    into a per-chain ring of 4 segments (128 positions, 64 with int32 coordinates), one round
//    ahead: round s waits only for the segments round s - 2 issued (s_waitcnt vmcnt(#DMA
//    instructions of round s - 1): the counter retires in order), so the DMA latency (~1 us from
//    HBM) hides behind the round;
//  * Bm and the S rows go to an LDS ring flushed every 32 rounds (no global store in the loop).
// Used for n <= 16 without roots (c1: 1 graph of 4 chains, c4: 512 graphs of 16): one workgroup
// per graph, no inter-workgroup wait of any kind, so any number of graphs.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

#include "hgx_device.h"
#include "hgx_kernels.h"

namespace hgx {

// Optional phase clocks (-DHGX_STEP_PROF, build variant "prof"): thread 0 of each workgroup adds
// s_memtime deltas per phase of every round, flushed once at the end of the launch. Slots: 1 round
// start (W'_s rows from LDS), 2 search levels, 3 boundary scan + later windows, 4 S row + staging
// wait + staging issue, 5 candidate row of W'_{s+1}, 7 flush + barrier; 15 = workgroup-rounds
#ifdef HGX_STEP_PROF
__device__ unsigned long long hgx_rg_prof[16];
#define RG_PROF_BEGIN() long long _pt = clock64(); unsigned long long _pa[16] = {}
#define RG_PROF(i)                                              \
    do {                                                        \
        if (threadIdx.x == 0) {                                 \
            const long long _t = clock64();                     \
            _pa[i] += (unsigned long long)(_t - _pt);           \
            _pt = _t;                                           \
            if ((i) == 7) _pa[15] += 1;                         \
            if ((i) == 11) _pa[12] += 1;                        \
        }                                                       \
    } while (0)
#define RG_PROF_END()                                                              \
    do {                                                                           \
        if (threadIdx.x == 0)                                                      \
            for (int _i = 0; _i < 16; _i++)                                        \
                if (_pa[_i]) atomicAdd(&hgx_rg_prof[_i], _pa[_i]);                 \
    } while (0)
void round_g_prof_dump() {
    unsigned long long h[16];
    if (hipMemcpyFromSymbol(h, HIP_SYMBOL(hgx_rg_prof), sizeof(h)) != hipSuccess) return;
    const double r = h[15] ? (double)h[15] : 1.0;
    fprintf(stderr, "[hgx] k_round_g clk per workgroup-round (thread 0): start %.0f search %.0f scan %.0f "
            "outputs %.0f stage-issue %.0f wait %.0f cand-row %.0f flush+barrier %.0f | workgroup-rounds %llu; "
            "DMA instructions: %llu, clk in them %.0f each\n",
            h[1] / r, h[2] / r, h[3] / r, h[8] / r, h[9] / r, h[4] / r, h[5] / r, h[7] / r, h[15], h[12],
            h[12] ? (double)h[11] / (double)h[12] : 0.0);
    unsigned long long z[16] = {};
    (void)hipMemcpyToSymbol(HIP_SYMBOL(hgx_rg_prof), z, sizeof(z));
}
#else
#define RG_PROF_BEGIN() (void)0
#define RG_PROF(i) (void)0
#define RG_PROF_END() (void)0
void round_g_prof_dump() {}
#endif

namespace {

constexpr int kGP = 31;      // probes per window (K in [0, 31], 5 binary-search levels)
constexpr int kGN = 16;      // chains per graph at most
constexpr int kGSeg = 4;     // ring segments per chain
// bytes of one firstDescendants column piece of a segment: SEG = SEGB / sizeof(CT) positions. 64
// (32 compact positions, 128 per ring, 512 n^2 bytes) except for compact rows of 9..16
// coordinates (ND = 8): 32 (16 positions, 64 per ring, 256 n^2 bytes: two workgroups per CU at n = 16)
template <typename CT, int ND>
constexpr int g_segb() { return (sizeof(CT) == 2 && ND == 8) ? 32 : 64; }
constexpr int kGOut = 32;    // rounds of Bm / S rows held in LDS between flushes

struct RoundGArgs {
    RoundArgs A;
    int32_t* st;    // [1] max over graphs of the round each stopped at, [2] graphs finished (W'_s
                    // empty) in this launch
    int32_t* fin;   // [G] the round at which graph g found W'_s empty (-1: not yet, this call)
    int r0, r_end;  // rounds [r0, r_end) at most
};

// LDS carve (bytes), n chains, nd dwords per candidate row, SEGB-byte column pieces; every offset
// 16-aligned
struct GLds {
    int segb, rawb, chb;   // per segment (raw rows | FD columns), raw part, per chain ring
    int o_cand, o_kk, o_curb, o_ob, o_os, o_seq, total;
    __host__ __device__ GLds(int n, int nseg, int nd, int seg_bytes) {
        rawb = seg_bytes * n;       // SEG raw rows of n coordinates = SEGB n bytes whatever the width
        segb = 2 * rawb;            // + n firstDescendants column pieces of SEGB bytes
        chb = nseg * segb;
        o_cand = n * chb;                      // [2][16][nd] dwords: W'_r rows by parity
        o_kk = o_cand + 2 * kGN * nd * 4;      // [16][16] bytes K(w)
        o_curb = o_kk + kGN * kGN;             // [2][16] int32 Bm[r], by parity
        o_ob = o_curb + 2 * kGN * 4;           // [kGOut][16] int32 Bm[r + 1]
        o_os = o_ob + kGOut * kGN * 4;         // [kGOut][16] uint16 S rows
        o_seq = o_os + kGOut * kGN * 2;        // [16][nseg] int32: issue count after each slot's DMA
        total = o_seq + kGN * nseg * 4;
    }
};

// 16 bytes per lane from global memory into LDS at m0 + 16 * lane (LDS-DMA). In asm so that the
// compiler does not put a vmcnt(0) before the next LDS access it cannot tell apart (the wait is
// this kernel's own, counted per round); m0 restored for the compiler.
__device__ __forceinline__ void g_dma16(const void* src, uint32_t lds_base) {
    uint32_t save;
    asm volatile(
        "s_mov_b32 %0, m0\n\t"
        "s_mov_b32 m0, %2\n\t"
        "s_nop 0\n\t"
        "global_load_lds_dwordx4 %1, off\n\t"
        "s_mov_b32 m0, %0"
        : "=&s"(save)
        : "v"(src), "s"(lds_base)
        : "memory");
}

// wait until at most k vector-memory instructions of this wave are outstanding (wave-uniform k;
// a smaller immediate waits for more: always safe)
__device__ __forceinline__ void g_vm_wait(int k) {
    switch (k < 0 ? 0 : k) {
        case 0: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
        case 1: asm volatile("s_waitcnt vmcnt(1)" ::: "memory"); break;
        case 2: asm volatile("s_waitcnt vmcnt(2)" ::: "memory"); break;
        case 3: asm volatile("s_waitcnt vmcnt(3)" ::: "memory"); break;
        case 4: asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); break;
        case 5: asm volatile("s_waitcnt vmcnt(5)" ::: "memory"); break;
        case 6: asm volatile("s_waitcnt vmcnt(6)" ::: "memory"); break;
        case 7: asm volatile("s_waitcnt vmcnt(7)" ::: "memory"); break;
        case 8: asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); break;
        case 9: asm volatile("s_waitcnt vmcnt(9)" ::: "memory"); break;
        case 10: asm volatile("s_waitcnt vmcnt(10)" ::: "memory"); break;
        case 11: asm volatile("s_waitcnt vmcnt(11)" ::: "memory"); break;
        default: asm volatile("s_waitcnt vmcnt(12)" ::: "memory"); break;
    }
}

__device__ __forceinline__ void g_lds_row4(const void* p, uint32_t (&v)[4]) {
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    u32x4 r;
    asm volatile("ds_read_b128 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=&v"(r) : "v"((uint32_t)(uintptr_t)p) : "memory");
    v[0] = r.x; v[1] = r.y; v[2] = r.z; v[3] = r.w;
}

// ND dwords of a row at p (RW = 16: 16-byte aligned rows, read as ND / 4 ds_read_b128; RW = 4:
// the first ndr dwords one by one, the rest zero)
template <int ND, int RW>
__device__ __forceinline__ void g_row(const uint8_t* p, int ndr, uint32_t (&v)[ND]) {
    if constexpr (RW == 16) {
#pragma unroll
        for (int k = 0; k < ND / 4; k++) {
            const uint4 q = ((const uint4*)p)[k];
            v[4 * k] = q.x; v[4 * k + 1] = q.y; v[4 * k + 2] = q.z; v[4 * k + 3] = q.w;
        }
    } else {
#pragma unroll
        for (int d = 0; d < ND; d++) v[d] = d < ndr ? ((const uint32_t*)p)[d] : 0u;
    }
}

// coordinates of probe row L that reach the candidate's row F (StronglySee, hashgraph.go:191-197:
// lastAncestors[i] >= firstDescendants[i])
template <typename CT, int ND>
__device__ __forceinline__ int g_count(const uint32_t (&L)[ND], const uint32_t (&F)[ND]) {
    if constexpr (sizeof(CT) == 2) {
        // stored lastAncestor + 1 >= firstDescendant + 1 (F; none = 0xFFFF, never reached):
        // sub_sat(F, L) == 0; min(., 1) adds 1 per unseen half. In asm: the compiler folds
        // min(sub_sat(F, L), 1) back into per-half compares and selects (5 instructions a dword).
        typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
        const uint32_t one = 0x00010001u;
        u16x2 x[ND];
#pragma unroll
        for (int d = 0; d < ND; d++) {
            uint32_t y;
            asm("v_pk_sub_u16 %0, %1, %2 clamp\n\tv_pk_min_u16 %0, %0, %3" : "=&v"(y) : "v"(F[d]), "v"(L[d]), "v"(one));
            x[d] = __builtin_bit_cast(u16x2, y);
        }
#pragma unroll
        for (int h = ND / 2; h >= 1; h /= 2)   // pairwise packed sums (<= 16 per half)
#pragma unroll
            for (int d = 0; d < h; d++) x[d] += x[d + h];
        return 2 * ND - (int)x[0].x - (int)x[0].y;
    } else {
        int cnt = 0;
#pragma unroll
        for (int d = 0; d < ND; d++) cnt += (int32_t)L[d] >= (int32_t)F[d] ? 1 : 0;
        return cnt;
    }
}

template <typename CT, int ND, int RW>
__global__ void __launch_bounds__(256) k_round_g(RoundGArgs P) {
    constexpr int CSZ = (int)sizeof(CT), SEGB = g_segb<CT, ND>(), SEG = SEGB / CSZ, NSEG = kGSeg;
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    const RoundArgs& A = P.A;
    const int n = A.n, C = A.C, sm = A.sm;
    const int g = blockIdx.x, g0 = g * n;
    const int t = threadIdx.x, lane = lane_id(), wave = t >> 6;
    const int c = t >> 4, w = t & 15, csh = 16 * (c & 3);   // chain searched, candidate, chain's lane base
    const bool cv = c < n, wv = w < n;
    const int rb = n * CSZ, ndr = rb / 4;   // bytes / dwords of a raw row (n even when compact)
    const GLds L(n, NSEG, ND, SEGB);
    uint32_t* cand = (uint32_t*)(lds + L.o_cand);
    uint8_t* kk = lds + L.o_kk;
    int32_t* curb = (int32_t*)(lds + L.o_curb);
    int32_t* ob = (int32_t*)(lds + L.o_ob);
    uint16_t* os = (uint16_t*)(lds + L.o_os);
    int32_t* seqs = (int32_t*)(lds + L.o_seq);
    uint8_t* ring = lds + (cv ? c : 0) * L.chb;

    if (P.fin[g] >= 0) return;   // the graph finished in an earlier launch of this DivideRounds
    RG_PROF_BEGIN();
    const int len = cv ? A.c_len[g0 + c] : 0, off = cv ? A.c_off[g0 + c] : 0;
    const int lenw = wv ? A.c_len[g0 + w] : 0;
    const int last_seg = len > 0 ? (len - 1) / SEG : -1;
    int b = cv ? A.Bm[(size_t)P.r0 * C + g0 + c] : 0;

    // ---- staging: segment m of chain c = its raw rows [SEG m, SEG m + SEG) (SEGB n bytes) followed by
    // the n firstDescendants column pieces of those positions (SEGB bytes each) in ring slot m % NSEG,
    // 16 bytes per lane (lane k < SEGB n / 16: raw chunk k; then column (k - SEGB n / 16) / (SEGB / 16));
    // one instruction per 64 lanes (one per segment compact). Chain offsets are multiples of 32
    // (hgx_engine.cpp layout): every segment is aligned in both arrays; rows past the chain's end lie
    // in its slot's slack (read, never used). The wave that owns chains 4 wave .. 4 wave + 3 issues
    // their DMA. nis counts this wave's DMA instructions; seqs[c][slot] = nis after a segment's DMA:
    // that segment has landed once at most nis_now - seqs[..] instructions are outstanding (the
    // counter retires in order).
    int sh1 = -1;      // highest segment issued (chain c)
    int landed = -1;   // highest segment known to have landed (chain c)
    int nis = 0;       // DMA instructions this wave issued (wave-uniform)
    constexpr int RAWC = SEGB / 16;   // (x n: raw chunks of a segment; as many column chunks)
    auto seg_of = [&](int p) { return ring + ((p / SEG) % NSEG) * L.segb; };
    auto stage = [&](bool want, int lo, int hi) {
        if (!__any(want && hi > sh1)) return;   // (most rounds: nothing new for any chain of the wave)
        for (int k = 0; k < 4; k++) {
            const int cc = wave * 4 + k;
            if (cc >= n) break;
            if (!__builtin_amdgcn_readlane((int)want, 16 * k)) continue;
            const int lo_k = __builtin_amdgcn_readlane(lo, 16 * k), hi_k = __builtin_amdgcn_readlane(hi, 16 * k);
            const int sh_k = __builtin_amdgcn_readlane(sh1, 16 * k), off_k = __builtin_amdgcn_readlane(off, 16 * k);
            for (int m = max(sh_k + 1, lo_k); m <= hi_k; m++) {
                const uint32_t dst = __builtin_amdgcn_readfirstlane(
                    (uint32_t)(uintptr_t)(lds + cc * L.chb + (m % NSEG) * L.segb));
                const size_t pos = (size_t)off_k + (size_t)m * SEG;
                const int rawc = RAWC * n;
#pragma unroll
                for (int k0 = 0; k0 < 2 * RAWC * kGN; k0 += 64) {
                    if (k0 >= 2 * rawc) break;
                    const int q = k0 + lane;
                    const uint8_t* src = nullptr;
                    if (q < rawc) {
                        src = (const uint8_t*)A.LA + pos * n * CSZ + 16 * q;
                    } else if (q < 2 * rawc) {
                        const int qq = q - rawc;
                        src = (const uint8_t*)A.FDT + ((size_t)(qq / RAWC) * A.Pcap + pos) * CSZ + 16 * (qq % RAWC);
                    }
                    RG_PROF(10);
                    if (src) g_dma16(src, dst + 16 * k0);
                    RG_PROF(11);
                    nis++;
                }
                if (lane == 0) seqs[cc * NSEG + m % NSEG] = nis;
            }
        }
        if (want) sh1 = max(sh1, hi);
    };
    // chain c's candidate row of W'_r (the event at offset pos), buffer r & 1: lane w' = coordinate
    // w' (compact: firstDescendant + 1, none 0xFFFF; int32: firstDescendant, none MaxInt32; the
    // padding never reached)
    auto cand_row = [&](int par, bool exists, int pos) {
        if (!cv) return;
        const uint8_t* col = seg_of(pos) + L.rawb + (pos % SEG) * CSZ;   // + SEGB i: column i
        if constexpr (CSZ == 2) {
            uint32_t f = 0xFFFFu;
            if (exists && wv) f = min((uint32_t)*(const uint16_t*)(col + w * SEGB) + 1u, 0xFFFFu);
            if (w < 2 * ND) ((uint16_t*)(cand + (par * kGN + c) * ND))[w] = (uint16_t)f;
        } else {
            int32_t f = kMaxI32;
            if (exists && wv) f = *(const int32_t*)(col + w * SEGB);
            if (w < ND) ((int32_t*)(cand + (par * kGN + c) * ND))[w] = f;
        }
    };
    // Bm / S rows of rounds [lo, hi] from the LDS ring to global memory (this chain's lanes)
    auto flush = [&](int lo, int hi) {
        if (!cv) return;
        for (int r = lo + w; r <= hi; r += 16) {
            const int kst = ob[(r % kGOut) * kGN + c];
            A.Bm[(size_t)(r + 1) * C + g0 + c] = kst;
            if (kst < len) A.Smat[((size_t)(r + 1) * C + g0 + c) * A.nw] = (uint64_t)os[(r % kGOut) * kGN + c];
        }
    };

    // ---- prologue: round r0's windows staged, W'_{r0} rows
    const int r0 = P.r0;
    if (cv && w == 0) curb[(r0 & 1) * kGN + c] = b;
    {
        const bool have = b < len;
        stage(have, b / SEG, min(b / SEG + NSEG - 1, last_seg));
        g_vm_wait(0);
        landed = sh1;
    }
    cand_row(r0 & 1, b < len, b);
    __syncthreads();

    int s = r0, flo = r0;
    bool empty = false;
    for (;; s++) {
        if (s >= P.r_end) break;   // capacity: the host continues from round s
        const int par = s & 1;
        // W'_s: candidate w exists iff Bm[s][w] < len_w (every wave sees every w)
        const bool candw = wv && curb[par * kGN + w] < lenw;
        if (__ballot(candw) == 0) { empty = true; break; }   // no round s (every wave agrees)
        const bool act = cv && candw;
        uint32_t fd[ND];
        {
            const uint32_t* cp = cand + (par * kGN + w) * ND;
            if constexpr (ND >= 4) {
#pragma unroll
                for (int k = 0; k < ND / 4; k++) {
                    const uint4 q = ((const uint4*)cp)[k];
                    fd[4 * k] = q.x; fd[4 * k + 1] = q.y; fd[4 * k + 2] = q.z; fd[4 * k + 3] = q.w;
                }
            } else {
#pragma unroll
                for (int d = 0; d < ND; d++) fd[d] = cp[d];
            }
        }
        RG_PROF(1);

        // search, window after window (a later window is rare, and private to the chain's wave)
        const bool have = b < len;
        int kb = b, np = have ? min(kGP, len - b) : 0, carried = 0, B = -1, Klast = kGP, kstar = len;
        bool done = false, need = have;
        for (;;) {
            int lo = 0, hi = kGP;
            if (need && act) {
#pragma unroll 1
                for (int it = 0; it < 5; it++) {
                    const int mid = (lo + hi) >> 1;
                    const uint32_t p = (uint32_t)(kb + mid);
                    uint32_t v[ND];
                    g_row<ND, RW>(ring + __umul24((p / SEG) % NSEG, L.segb) + __umul24(p % SEG, rb), ndr, v);
                    const int cnt = g_count<CT, ND>(v, fd);
                    const bool seen = done || mid >= np || (cnt >= sm && !(w == c && (int)p == b));
                    if (seen) hi = mid; else lo = mid + 1;
                }
            }
            RG_PROF(2);
            if (need) kk[c * kGN + w] = (act && !done && lo < np) ? (uint8_t)lo : (uint8_t)127;
            // the boundary: first probe p with carried + #{K(w) <= p} >= SM (lane w: p = w, w + 16);
            // K bytes in [0, 31] or 127 (not counted): x <= p  <=>  bit 7 of (0x80 | p) - x, 4 per dword
            uint32_t kq[4];
            g_lds_row4(kk + (cv ? c : 0) * kGN, kq);
            const uint32_t p1 = 0x80808080u | (0x01010101u * (uint32_t)w), p2 = p1 + 0x10101010u;
            const uint32_t pt = 0x80808080u | (0x01010101u * (uint32_t)(np - 1));   // x < np (np >= 1 here)
            int c1 = carried, c2 = carried, tot = carried;
#pragma unroll
            for (int d = 0; d < 4; d++) {
                c1 += __builtin_popcount((p1 - kq[d]) & 0x80808080u);
                c2 += __builtin_popcount((p2 - kq[d]) & 0x80808080u);
                tot += __builtin_popcount((pt - kq[d]) & 0x80808080u);
            }
            const uint32_t m1 = (uint32_t)((__ballot(need && w < np && c1 >= sm) >> csh) & 0xFFFFull);
            const uint32_t m2 = (uint32_t)((__ballot(need && w + 16 < np && c2 >= sm) >> csh) & 0xFFFFull);
            bool more = false;
            if (need) {
                Klast = lo;
                if (m1 | m2) {
                    B = m1 ? (int)__builtin_ctz(m1) : 16 + (int)__builtin_ctz(m2);
                    kstar = kb + B;
                    need = false;
                } else {
                    carried = tot;
                    if (act && lo < np) done = true;
                    kb += np;
                    if (kb >= len) need = false;
                    else { np = min(kGP, len - kb); more = true; }
                }
            }
            if (!__any(more)) break;
            // the next window of the chains that go on, staged synchronously
            stage(more, kb / SEG, min(kb / SEG + NSEG - 1, last_seg));
            g_vm_wait(0);
            landed = sh1;
        }
        RG_PROF(3);

        // round s's outputs (LDS ring) and W'_{s+1} of chain c: the next window staged one round
        // ahead (waiting only for the DMA round s - 2 issued, unless the window jumped past it)
        const bool nx = kstar < len;
        const uint32_t srow = (uint32_t)((__ballot(have && nx && act && (done || Klast <= B)) >> csh) & 0xFFFFull);
        if (cv && w == 0) {
            ob[(s % kGOut) * kGN + c] = kstar;
            os[(s % kGOut) * kGN + c] = (uint16_t)srow;
        }
        const int np1 = nx ? min(kGP, len - kstar) : 0;
        RG_PROF(8);
        // the ring ahead first, then a wait only for the segment the next window ends in, counted
        // from its own DMA (usually issued rounds ago: no wait)
        {
            const int lo = kstar / SEG;
            stage(nx, lo, min(lo + NSEG - 1, last_seg));
        }
        RG_PROF(9);
        {
            const int m_need = nx ? (kstar + np1 - 1) / SEG : -1;
            const bool nw = m_need > landed;
            if (__any(nw)) {
                int kc = nw ? nis - seqs[c * NSEG + m_need % NSEG] : 64;
                kc = min(kc, __shfl_xor(kc, 16));
                kc = min(kc, __shfl_xor(kc, 32));
                g_vm_wait(kc);
                if (nw) landed = m_need;
            }
        }
        RG_PROF(4);
        cand_row(par ^ 1, nx, kstar);
        if (cv && w == 0) curb[(par ^ 1) * kGN + c] = kstar;
        b = kstar;
        RG_PROF(5);
        if ((s - flo) == kGOut - 1) {
            flush(flo, s);
            flo = s + 1;
        }
        // W'_{s+1} complete (LDS only: __syncthreads would also wait for the DMA in flight)
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        RG_PROF(7);
    }
    RG_PROF_END();
    flush(flo, s - 1);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // no LDS-DMA outlives the workgroup
    if (empty && cv && w == 0) {   // W'_s empty: round s has no events (the per-launch step's outputs)
        A.wstat[(size_t)s * C + g0 + c] = 0;
        A.wflag[(size_t)(s + 1) * C + g0 + c] = 0;
        A.Bm[(size_t)(s + 1) * C + g0 + c] = len;
    }
    if (t == 0) {
        if (empty) {
            P.fin[g] = s;
            atomicAdd(&P.st[2], 1);
        }
        atomicMax(&P.st[1], s);
    }
}

template <typename CT, int ND, int RW>
hipError_t rg_launch(hipStream_t st, const RoundGArgs& P) {
    const GLds L(P.A.n, kGSeg, ND, g_segb<CT, ND>());
    if (L.total > 160 * 1024) return hipErrorInvalidValue;
    const void* f = (const void*)k_round_g<CT, ND, RW>;
    const hipError_t e = ensure_lds_limit(f, (size_t)L.total);
    if (e != hipSuccess) return e;
    const int T = 64 * ((P.A.n + 3) / 4);
    hipLaunchKernelGGL((k_round_g<CT, ND, RW>), dim3(P.A.C / P.A.n), dim3(T), L.total, st, P);
    return hipGetLastError();
}

// the instantiation for n coordinates of CT: ND = dwords of a row rounded up to a power of two,
// 16-byte reads when rows are 16-byte aligned
template <typename CT>
hipError_t rg_launch_t(hipStream_t st, const RoundGArgs& P) {
    const int rb = P.A.n * (int)sizeof(CT), nd = (rb + 3) / 4;
    const bool a16 = rb % 16 == 0 && (nd & (nd - 1)) == 0;   // (16-byte reads never run past a row)
    if (nd <= 1) return rg_launch<CT, 1, 4>(st, P);
    if (nd <= 2) return rg_launch<CT, 2, 4>(st, P);
    if (nd <= 4) return a16 ? rg_launch<CT, 4, 16>(st, P) : rg_launch<CT, 4, 4>(st, P);
    if (nd <= 8) return a16 ? rg_launch<CT, 8, 16>(st, P) : rg_launch<CT, 8, 4>(st, P);
    if constexpr (sizeof(CT) == 4) {
        if (nd <= 16) return a16 ? rg_launch<CT, 16, 16>(st, P) : rg_launch<CT, 16, 4>(st, P);
    }
    return hipErrorInvalidValue;
}

}  // namespace

bool round_g_ok(int n, int nw) { return n >= 1 && n <= kGN && nw == 1; }

hipError_t launch_round_g(hipStream_t st, const RoundArgs& A, int32_t* status, int32_t* fin, int r0, int r_end) {
    if (!round_g_ok(A.n, A.nw) || A.C % A.n) return hipErrorInvalidValue;
    RoundGArgs P{};
    P.A = A;
    P.st = status;
    P.fin = fin;
    P.r0 = r0;
    P.r_end = r_end;
    return A.compact ? rg_launch_t<uint16_t>(st, P) : rg_launch_t<int32_t>(st, P);
}

}  // namespace hgx
