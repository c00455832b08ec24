// Round step with one lane per candidate (RoundInc, hashgraph.go:285-305; StronglySee
// hashgraph.go:170-198). DESIGN.md §3.3.
//
// Step s finds, for chain c, the boundary Bm[s+1][c] = first offset k >= Bm[s][c] whose
// event strongly sees >= SM candidates w of W'_s (the first event of each chain with round
// >= s; its own candidate does not count at the probe that is itself). Strongly seeing w is
// monotone along the chain (lastAncestors only grow), so every candidate has a first
// strongly-seeing probe K(w) in a window of P probe rows, and the boundary is the SM-th
// smallest K(w): each lane binary-searches its own candidate's K(w), an LDS histogram of
// the K(w) gives the boundary. No barrier per search level, and the per-(probe, candidate)
// count never leaves the lane.
//
// The count #{i : LA[x][i] >= FD[w][i]} runs on 8-bit SWAR: every coordinate is rebased
// per round to base_i = Index of the candidate of round s-1 on chain i (c_base + Bm[s-1][i]).
// A candidate of round s has FD[w][i] >= base_i (its descendants have round >= s, so they sit
// at or after Bm[s][i] >= Bm[s-1][i]), so FD' = FD - base + 1 is in [1, 126] when the
// candidate's first descendants are within 125 events of base (127 = none), and the probe
// values are LA' = clamp(LA - base + 1, 0, 126) with the byte's top bit set: per byte,
// (0x80 | LA') - FD' never borrows and its bit 7 is [LA' >= FD'] = [LA >= FD]. One v_sub,
// one v_and, one v_bcnt per 4 coordinates. The producer of a candidate row (the step that
// found it) writes it rebased and flags the round if a value does not fit; a flagged round
// runs the exact int32 compare instead (same search, slower).
//
// The step also writes what the next step needs: the new candidate's rows (WLA, raw WFD,
// rebased FD8) and its strongly-seen bitmask, DecideFame's S row (hashgraph.go:688-705).
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

#include "hgx_device.h"
#include "hgx_kernels.h"

namespace hgx {

// Optional phase clocks (-DHGX_STEP_PROF, build variant "prof"): thread 0 of each block adds
// s_memtime deltas per phase to hgx_rk_prof[] once, at the end of the step.
#ifdef HGX_STEP_PROF
__device__ unsigned long long hgx_rk_prof[8];
#define RK_PROF_BEGIN() long long _pt = clock64(); unsigned long long _pa[8] = {0, 0, 0, 0, 0, 0, 0, 0}
#define RK_PROF(i)                                                \
    do {                                                          \
        if (threadIdx.x == 0) {                                   \
            const long long _t = clock64();                       \
            _pa[i] += (unsigned long long)(_t - _pt);             \
            _pt = _t;                                             \
        }                                                         \
    } while (0)
#define RK_PROF_END()                                                              \
    do {                                                                           \
        if (threadIdx.x == 0) {                                                    \
            _pa[7] += 1;                                                           \
            for (int _i = 0; _i < 8; _i++)                                         \
                if (_pa[_i]) atomicAdd(&hgx_rk_prof[_i], _pa[_i]);                 \
        }                                                                          \
    } while (0)
void round_k_prof_dump() {
    unsigned long long h[8];
    if (hipMemcpyFromSymbol(h, HIP_SYMBOL(hgx_rk_prof), sizeof(h)) != hipSuccess) return;
    fprintf(stderr, "[hgx] k_round_k phases (clk sums): head %llu window %llu convert %llu search %llu boundary %llu "
            "outputs: S row %llu, candidate rows %llu | block-steps %llu\n", h[0], h[1], h[2], h[3], h[4], h[6], h[5],
            h[7]);
}
#else
#define RK_PROF_BEGIN() (void)0
#define RK_PROF(i) (void)0
#define RK_PROF_END() (void)0
void round_k_prof_dump() {}
#endif

constexpr int kWinP = 31;   // probes per window: K in [0, 31], 5 binary-search levels

// window row stride in dwords: even (8-byte reads) and == 2 mod 4, so that 32 lanes reading
// 32 different rows at the same column hit 32 distinct bank pairs (MI355X_MICROARCH.md, LDS)
__host__ __device__ constexpr int win_stride(int ndw) { return (ndw % 4 == 0) ? ndw + 2 : ndw + 4; }

struct RoundKLds {
    int win, raw, fdc, base, bm1, hist, total;
};

// one chain group's LDS: rebased byte window | raw LA rows | FD columns (stg) | bases | histogram
__host__ __device__ inline RoundKLds round_k_lds(int n, int ndw, int csz, bool stg) {
    RoundKLds L{};
    int o = 0;
    L.win = o;
    o += kWinP * win_stride(ndw) * 4;
    L.raw = o;
    if (stg) o += ((kWinP * n * csz + 15) / 16) * 16;
    L.fdc = o;
    if (stg) {   // FD columns in groups of one LDS-DMA instruction (64 dwords) + 1 pad dword
        const int cpi = (csz == 2) ? 4 : 2;
        o += ((n + cpi - 1) / cpi) * 65 * 4;
    }
    L.base = o;
    o += n * 4;
    L.bm1 = o;
    o += n * 4;
    L.hist = o;
    o += 32 * 4;
    L.total = (o + 15) & ~15;
    return L;
}

// HD dwords of an LDS row as plain ds_read_b64 (2 cycles, 256 B/clk, 64-bank rule), all in
// flight before one wait. Left to itself the compiler fuses pairs into ds_read2_b64 (8 cycles,
// 128 B/clk, 32-bank rule: rows 16 apart conflict), which halves the search's LDS bandwidth
// (MI355X_MICROARCH.md, LDS table).
template <int HD>
__device__ __forceinline__ void lds_read_row(const uint32_t* p, uint32_t (&v)[HD]) {
    static_assert(HD % 2 == 0 && HD <= 64, "row width");
    const uint32_t a = (uint32_t)(uintptr_t)p;   // LDS byte address
    uint64_t r[HD / 2];
#define RK_RD(k) asm volatile("ds_read_b64 %0, %1 offset:%2" : "=v"(r[k]) : "v"(a), "i"(8 * (k)))
    RK_RD(0);
    if constexpr (HD >= 4) RK_RD(1);
    if constexpr (HD >= 8) { RK_RD(2); RK_RD(3); }
    if constexpr (HD >= 16) { RK_RD(4); RK_RD(5); RK_RD(6); RK_RD(7); }
    if constexpr (HD >= 32) { RK_RD(8); RK_RD(9); RK_RD(10); RK_RD(11); RK_RD(12); RK_RD(13); RK_RD(14); RK_RD(15); }
    if constexpr (HD >= 64) {
        RK_RD(16); RK_RD(17); RK_RD(18); RK_RD(19); RK_RD(20); RK_RD(21); RK_RD(22); RK_RD(23);
        RK_RD(24); RK_RD(25); RK_RD(26); RK_RD(27); RK_RD(28); RK_RD(29); RK_RD(30); RK_RD(31);
    }
#undef RK_RD
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
    for (int k = 0; k < HD / 2; k++) {
        asm volatile("" : "+v"(r[k]));   // the values exist only after the wait
        v[2 * k] = (uint32_t)r[k];
        v[2 * k + 1] = (uint32_t)(r[k] >> 32);
    }
}

// CG waves of 64 candidates each; every candidate's row is split over H waves (coordinate
// dwords [h*NDW/H, (h+1)*NDW/H)), whose partial counts meet in LDS once per search level, so
// that two waves share each SIMD; GPB chain groups per block when a group is one wave.
template <typename CT, int NDW, int CG, int H, int GPB, bool STG>
__global__ void __launch_bounds__(64 * CG * H * GPB) k_round_k(RoundArgs A, int s) {
    constexpr int P = kWinP;
    constexpr int GW = CG * H;           // waves of one chain group
    constexpr int GL = 64 * GW;          // threads of one chain group
    constexpr int HD = NDW / H;          // candidate-row dwords per wave
    constexpr int WS = win_stride(NDW);
    constexpr int FDW = P / 2 + 1;       // dwords per compact FD column (32 positions from an even start)
    constexpr int CW = (sizeof(CT) == 2) ? FDW : 32;   // dwords per staged FD column
    constexpr int CPI = 64 / CW;                        // FD columns per LDS-DMA wave instruction
    static_assert(GPB == 1 || GW == 1, "several chain groups per block only with one-wave groups");
    static_assert(NDW % (2 * H) == 0, "row split");
    typedef __attribute__((address_space(3))) void* lds_ptr_t;
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    __shared__ int s_B[GPB], s_tot[GPB];
    __shared__ int pc[(H > 1) ? 2 * H * 64 * CG : 1];   // partial counts by level parity

    const int n = A.n, C = A.C, sm = A.sm;
    const int lane = lane_id(), wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int grp = wave / GW, wh = wave % GW, h = wh / CG, cw = wh % CG;
    const int gt = wh * 64 + lane;       // thread within the chain group
    const int gc = blockIdx.x * GPB + grp;
    if (gc >= C) return;   // group-uniform; block barriers are only used when GPB == 1
    RK_PROF_BEGIN();
    const RoundKLds L = round_k_lds(n, NDW, (int)sizeof(CT), STG);
    uint8_t* gl = lds + (size_t)grp * L.total;
    uint32_t* win = (uint32_t*)(gl + L.win);
    CT* raw = (CT*)(gl + L.raw);
    CT* fdc = (CT*)(gl + L.fdc);
    int32_t* base = (int32_t*)(gl + L.base);
    int32_t* bm1 = (int32_t*)(gl + L.bm1);
    int32_t* hist = (int32_t*)(gl + L.hist);
    auto gsync = [&]() {
        if constexpr (GW == 1) wave_lds_fence();
        else __syncthreads();
    };

    const int g = gc / n, cl = gc % n;
    const int par = s & 1;
    const size_t wrow = (size_t)s * C + (size_t)g * n;
    // every load that does not depend on this chain's boundary is issued first, so their
    // latencies overlap the boundary load: the boundary, this lane's part of its candidate's
    // rebased row (written by the step that found the candidate), the flags and the bases
    const int b = A.Bm[(size_t)s * C + gc];
    const int len = A.c_len[gc], off = A.c_off[gc];
    // root floor (after hgx_reset): offsets >= gk have round >= s+1 whatever they strongly see
    const int gk = (s + 1 <= A.gmax) ? A.gB[(size_t)(s + 1) * C + gc] : len;
    const int j = cw * 64 + lane;        // this lane's candidate
    const int jj = j < n ? j : 0;
    uint32_t fd[HD];
    {
        const uint32_t* __restrict__ row = A.FD8 + ((size_t)par * C + (size_t)g * n + jj) * NDW + h * HD;
        if constexpr (HD % 4 == 0) {
#pragma unroll
            for (int d = 0; d < HD; d += 4) {
                const uint4 v = *(const uint4*)(row + d);
                fd[d] = v.x; fd[d + 1] = v.y; fd[d + 2] = v.z; fd[d + 3] = v.w;
            }
        } else {
#pragma unroll
            for (int d = 0; d < HD; d += 2) {
                const uint2 v = *(const uint2*)(row + d);
                fd[d] = v.x; fd[d + 1] = v.y;
            }
        }
    }
    const uint8_t wfl = A.wflag[wrow + jj];
    const int ovf_s = A.ovf[s];
    constexpr int BPT = (256 + GL - 1) / GL;   // base coordinates per thread (n <= 256)
    int cbv[BPT], bmp[BPT], bmc[BPT];
#pragma unroll
    for (int u = 0; u < BPT; u++) {
        const int i = gt + u * GL;
        const int ii = i < n ? i : 0;
        cbv[u] = A.c_base[g * n + ii];
        bmp[u] = s > 0 ? A.Bm[wrow - C + ii] : 0;
        bmc[u] = A.Bm[wrow + ii];
    }
    if (b >= len) {
        if (gt == 0) {
            A.wstat[(size_t)s * C + gc] = 0;
            A.wflag[(size_t)(s + 1) * C + gc] = 0;
            A.Bm[(size_t)(s + 1) * C + gc] = len;
        }
        return;
    }

    // the window: raw LA rows [kbase, kbase+np) (contiguous) and, when staged, the window's
    // FD columns (the new candidate's FD row comes from there), by LDS-DMA
    int fsh = 0;
    auto stage = [&](int kbase, int np) {
        if constexpr (STG) {
            const int nel = (int)((size_t)np * n * sizeof(CT) / 4);
            const uint32_t* __restrict__ src = (const uint32_t*)A.LA + (size_t)(off + kbase) * n * sizeof(CT) / 4;
            uint32_t* raw_w = (uint32_t*)raw;
            if (((n * (int)sizeof(CT)) & 15) == 0) {
                for (int c0 = wh * 256; c0 < nel; c0 += GW * 256) {
                    const int t = c0 + lane * 4;
                    if (t < nel)
                        __builtin_amdgcn_global_load_lds((const void*)(src + t), (lds_ptr_t)(raw_w + c0), 16, 0, 0);
                }
            } else {
                for (int c0 = wh * 64; c0 < nel; c0 += GW * 64) {
                    const int t = c0 + lane;
                    if (t < nel) __builtin_amdgcn_global_load_lds((const void*)(src + t), (lds_ptr_t)(raw_w + c0), 4, 0, 0);
                }
            }
            // FD columns: one wave instruction stages CPI columns of CW dwords each (positions
            // [kbase, kbase+np) for int32; the 2*FDW positions from the even start below kbase for
            // uint16) into a 64-dword group; groups are 65 dwords apart (bank spread)
            uint32_t* fd_w = (uint32_t*)fdc;
            const int pcol = lane % CW, icol = lane / CW;
            const uint32_t* __restrict__ fsrc;
            size_t cstride;
            bool pok;
            if constexpr (sizeof(CT) == 4) {
                fsrc = (const uint32_t*)A.FDT + off + kbase + pcol;
                cstride = (size_t)A.Pcap;
                pok = pcol < np;
            } else {
                const int64_t p0 = (off + kbase) & ~1;
                fsh = (off + kbase) & 1;
                fsrc = (const uint32_t*)((const CT*)A.FDT + p0) + pcol;
                cstride = (size_t)(A.Pcap / 2);
                pok = true;
            }
            for (int i0 = wh * CPI; i0 < n; i0 += GW * CPI) {
                const int i = i0 + icol;
                if (i < n && pok)
                    __builtin_amdgcn_global_load_lds((const void*)(fsrc + (size_t)i * cstride),
                                                     (lds_ptr_t)(fd_w + (size_t)(i0 / CPI) * 65), 4, 0, 0);
            }
        }
    };
    auto la_at = [&](int kbase, int p, int i) -> int32_t {   // decoded lastAncestors of window row p
        if constexpr (STG) return Coord<CT>::la(raw[p * n + i]);
        else return Coord<CT>::la(((const CT*)A.LA)[(size_t)(off + kbase + p) * n + i]);
    };
    // rebased byte window: (0x80 | LA') per coordinate, padding coordinates LA' = 0. A thread
    // keeps one dword column d (4 coordinates, their bases in registers) over rows p.
    typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
    auto convert = [&](int kbase, int np) {
        constexpr int RS = (GL >= NDW) ? GL / NDW : 1;   // rows per pass
        constexpr int NP = (P + RS - 1) / RS;              // passes (fixed trip count)
        for (int d = gt % NDW; d < NDW; d += GL) {
            const int i0 = 4 * d;
            if constexpr (STG && sizeof(CT) == 2) {
                // packed: LA' = min(sat(raw - base), 126) on coordinate pairs (raw = LA + 1)
                u16x2 b01 = {0, 0}, b23 = {0, 0};
                if (i0 < n) b01 = u16x2{(unsigned short)base[i0], (unsigned short)base[i0 + 1]};
                if (i0 + 2 < n) b23 = u16x2{(unsigned short)base[i0 + 2], (unsigned short)base[i0 + 3]};
                const u16x2 cap = {126, 126};
#pragma unroll
                for (int u = 0; u < NP; u++) {
                    const int p = gt / NDW + u * RS;
                    if (p < np) {
                        const uint32_t* rp = (const uint32_t*)(raw + p * n + i0);
                        const uint32_t r01 = i0 < n ? rp[0] : 0u, r23 = i0 + 2 < n ? rp[1] : 0u;
                        const u16x2 y01 = __builtin_elementwise_min(
                            __builtin_elementwise_sub_sat(__builtin_bit_cast(u16x2, r01), b01), cap);
                        const u16x2 y23 = __builtin_elementwise_min(
                            __builtin_elementwise_sub_sat(__builtin_bit_cast(u16x2, r23), b23), cap);
                        const uint32_t w = __builtin_amdgcn_perm(__builtin_bit_cast(uint32_t, y23),
                                                                 __builtin_bit_cast(uint32_t, y01), 0x06040200u);
                        win[p * WS + d] = w | 0x80808080u;
                    }
                }
            } else {
                int32_t bq[4];
#pragma unroll
                for (int q = 0; q < 4; q++) bq[q] = (i0 + q < n) ? base[i0 + q] : 0;
                for (int p = gt / NDW; p < np; p += RS) {
                    uint32_t w = 0x80808080u;
#pragma unroll
                    for (int q = 0; q < 4; q++) {
                        const int i = i0 + q;
                        if (i < n) {
                            const int32_t x = la_at(kbase, p, i) - bq[q] + 1;
                            w |= (uint32_t)min(max(x, 0), 126) << (8 * q);
                        }
                    }
                    win[p * WS + d] = w;
                }
            }
        }
    };
    // total count over the H waves of this candidate (partial counts meet in LDS)
    auto combine = [&](uint32_t part, int it) -> uint32_t {
        if constexpr (H == 1) {
            return part;
        } else {
            int* pcb = pc + (it & 1) * (H * 64 * CG);
            pcb[h * 64 * CG + j] = (int)part;
            gsync();
            uint32_t t = 0;
#pragma unroll
            for (int q = 0; q < H; q++) t += (uint32_t)pcb[q * 64 * CG + j];
            return t;
        }
    };

    int kbase = b, np = min(P, len - b), kstar = len, carried = 0, B = -1, K = P;
    bool done = false;   // seen in an earlier window: seen at every later probe
    // the first window's staging depends on the boundary only: issue it now, so the candidate
    // rows and the bases are still in flight while it lands
    stage(kbase, np);
    const bool exact = ovf_s != 0;   // a candidate row of this round did not fit 8 bits
    const bool cand = j < n && wfl == 1;
#pragma unroll
    for (int u = 0; u < BPT; u++) {
        const int i = gt + u * GL;
        if (i < n) {
            base[i] = cbv[u] + bmp[u];   // base(s): Index of round s-1's candidate on chain i
            bm1[i] = cbv[u] + bmc[u];    // base(s+1)
        }
    }
    if (gt < 32) hist[gt] = 0;
    RK_PROF(0);
    bool staged = true;
    for (;;) {
        if (!staged) stage(kbase, np);
        staged = false;
        __builtin_amdgcn_s_waitcnt(0);
        gsync();
        RK_PROF(1);
        convert(kbase, np);
        gsync();
        RK_PROF(2);
        // first probe of the window that strongly sees this lane's candidate (np: none);
        // probes past the window's end count as seeing (keeps the predicate monotone)
        int lo = 0, hi = P;
        if (!exact) {
            uint32_t f[HD];
#pragma unroll
            for (int d = 0; d < HD; d++) f[d] = cand ? fd[d] : 0x7F7F7F7Fu;
#pragma unroll
            for (int it = 0; it < 5; it++) {
                const int mid = (lo + hi) >> 1;
                const uint32_t* row = win + mid * WS + h * HD;
                uint32_t v[HD];
                lds_read_row<HD>(row, v);
                uint32_t c4[4] = {0, 0, 0, 0};
#pragma unroll
                for (int d = 0; d < HD; d++) c4[d & 3] += __builtin_popcount((v[d] - f[d]) & 0x80808080u);
                uint32_t cnt = (c4[0] + c4[1]) + (c4[2] + c4[3]);
                cnt = combine(cnt, it);
                const bool seen = done || mid >= np || ((int)cnt >= sm && !(j == cl && kbase + mid == b));
                if (seen) hi = mid; else lo = mid + 1;
            }
        } else {
            // exact int32 compares against the raw candidate row (rounds flagged by the producer)
            const int i_lo = h * HD * 4, i_hi = min(n, (h + 1) * HD * 4);
            for (int it = 0; it < 5; it++) {
                const int mid = (lo + hi) >> 1;
                uint32_t cnt = 0;
                if (cand && !done && mid < np) {
                    for (int i = i_lo; i < i_hi; i++) {
                        const int32_t fdv = (sizeof(CT) == 2)
                                                ? Coord<uint16_t>::fd(((const uint16_t*)A.WFD)[(wrow + jj) * n + i])
                                                : A.WFD[(wrow + jj) * n + i];
                        const int32_t lav = min(la_at(kbase, mid, i), kMaxI32 - 1);
                        cnt += lav >= fdv ? 1u : 0u;
                    }
                }
                cnt = combine(cnt, it);
                const bool seen = done || mid >= np || (cand && (int)cnt >= sm && !(j == cl && kbase + mid == b));
                if (seen) hi = mid; else lo = mid + 1;
            }
        }
        K = lo;
        RK_PROF(3);
        if (h == 0 && K < np && cand && !done) atomicAdd(&hist[K], 1);   // earlier windows are in `carried`
        gsync();
        if (wh == 0) {   // boundary: first probe where #{K <= p} (+ candidates seen earlier) >= SM
            const uint32_t v = lane < np ? (uint32_t)hist[lane] : 0u;
            const uint32_t inc = wave_scan_add_u32(v) + (uint32_t)carried;
            const uint64_t m = __ballot(lane < np && ((int)inc >= sm || kbase + lane >= gk));
            const int tot = __builtin_amdgcn_readlane((int)inc, 63);
            if (lane == 0) {
                s_B[grp] = m ? (int)__builtin_ctzll(m) : -1;
                s_tot[grp] = tot;
            }
        }
        gsync();
        B = s_B[grp];
        RK_PROF(4);
        if (B >= 0) {
            kstar = kbase + B;
            break;
        }
        carried = s_tot[grp];
        done = done || (cand && K < np);
        if (gt < 32) hist[gt] = 0;
        kbase += np;
        if (kbase >= len) {
            kstar = len;
            break;
        }
        np = min(P, len - kbase);
        gsync();
    }

    // outputs of round s for this chain
    for (int k = b + gt; k < kstar; k += GL) A.p_round[off + k] = s;
    if (gt == 0) {
        A.wstat[(size_t)s * C + gc] = (kstar > b) ? 2 : 1;
        if (kstar < len) A.active[s] = 1;   // same value from every writer: a plain store
        A.Bm[(size_t)(s + 1) * C + gc] = kstar;
    }
    if (kstar < len) {
        const int pk = kstar - kbase;   // inside the staged window
        // S row of the boundary event: the candidates it strongly sees (bit j of word j/64)
        const uint64_t bits = __ballot(cand && K <= B);
        const size_t srow = ((size_t)(s + 1) * C + gc) * A.nw;
        if (h == 0 && lane == 0 && cw < A.nw) A.Smat[srow + cw] = bits;
        RK_PROF(6);
        // the new candidate's rows for round s+1
        const size_t nrow = ((size_t)(s + 1) * C + gc) * n;
        auto fd_raw = [&](int i) -> CT {
            if constexpr (STG) {
                const int col = (i / CPI) * 65 + (i % CPI) * CW;   // dword offset of column i
                if constexpr (sizeof(CT) == 2) return fdc[2 * col + fsh + pk];
                else return fdc[col + pk];
            } else {
                return ((const CT*)A.FDT)[(size_t)i * A.Pcap + off + kstar];
            }
        };
        for (int i = gt; i < n; i += GL) {
            A.WLA[nrow + i] = la_at(kbase, pk, i);
            const CT f = fd_raw(i);
            if constexpr (sizeof(CT) == 2) ((uint16_t*)A.WFD)[nrow + i] = f;
            else A.WFD[nrow + i] = f;
        }
        // rebased FD row (base(s+1) = Index of this round's candidates) for the next step
        uint32_t* nfd = A.FD8 + ((size_t)(par ^ 1) * C + gc) * NDW;
        bool of = false;
        for (int d = gt; d < NDW; d += GL) {
            uint32_t w = 0;
#pragma unroll
            for (int q = 0; q < 4; q++) {
                const int i = 4 * d + q;
                uint32_t v = 127u;
                if (i < n) {
                    const int32_t f = Coord<CT>::fd(fd_raw(i));
                    if (f != kMaxI32) {
                        const int32_t x = f - bm1[i] + 1;
                        if (x > 126) of = true;
                        else v = (uint32_t)x;
                    }
                }
                w |= v << (8 * q);
            }
            nfd[d] = w;
        }
        if (of) A.ovf[s + 1] = 1;   // same value from every writer
        if (gt == 0) A.wflag[(size_t)(s + 1) * C + gc] = 1;
    } else if (gt == 0) {
        A.wflag[(size_t)(s + 1) * C + gc] = 0;
    }
    RK_PROF(5);
    RK_PROF_END();
}

// round r's candidate rows (round 0: the first event of every chain; r > 0: the restart
// round of an incremental DivideRounds), rebased to base(r) = c_base + Bm[r-1], from the
// row-major WFD rows k_round_gather has just written (raw uint16 or int32 FD)
template <typename CT>
__global__ void k_round_k_gather(RoundArgs A, int ndw, int r) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= (int64_t)A.C * ndw) return;
    const int gc = (int)(t / ndw), d = (int)(t % ndw);
    const int n = A.n, C = A.C, g = gc / n;
    uint32_t w = 0;
    bool of = false;
    const bool have = A.wflag[(size_t)r * C + gc] != 0;
    const CT* __restrict__ row = (const CT*)A.WFD + ((size_t)r * C + gc) * n;
    for (int q = 0; q < 4; q++) {
        const int i = 4 * d + q;
        uint32_t v = 127u;
        if (have && i < n) {
            const int32_t f = Coord<CT>::fd(row[i]);
            if (f != kMaxI32) {
                const int32_t bs = A.c_base[g * n + i] + (r > 0 ? A.Bm[(size_t)(r - 1) * C + g * n + i] : 0);
                const int32_t x = f - bs + 1;
                if (x > 126) of = true;
                else v = (uint32_t)x;
            }
        }
        w |= v << (8 * q);
    }
    A.FD8[((size_t)(r & 1) * C + gc) * ndw + d] = w;
    if (of) A.ovf[r] = 1;
}

int round_k_ndw(int n) {
    int d = (n + 3) / 4;
    int p = 2;
    while (p < d) p *= 2;
    return p;
}

template <typename CT, int NDW, int CG, int H, int GPB, bool STG>
static hipError_t round_k_launch_v(hipStream_t st, const RoundArgs& A, int s) {
    const void* f = (const void*)k_round_k<CT, NDW, CG, H, GPB, STG>;
    const RoundKLds L = round_k_lds(A.n, NDW, (int)sizeof(CT), STG);
    const size_t lds = (size_t)L.total * GPB;
    static bool attr = false;
    if (!attr) {
        const hipError_t e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024 - 8192);
        if (e != hipSuccess) return e;
        attr = true;
    }
    const unsigned grid = (unsigned)((A.C + GPB - 1) / GPB);
    hipLaunchKernelGGL((k_round_k<CT, NDW, CG, H, GPB, STG>), dim3(grid), dim3(64 * CG * H * GPB), lds, st, A, s);
    return hipGetLastError();
}

template <typename CT, int NDW, int CG, int H, int GPB>
static hipError_t round_k_launch(hipStream_t st, const RoundArgs& A, int s) {
    const RoundKLds L = round_k_lds(A.n, NDW, (int)sizeof(CT), true);
    if ((size_t)L.total * GPB <= 140 * 1024) return round_k_launch_v<CT, NDW, CG, H, GPB, true>(st, A, s);
    return round_k_launch_v<CT, NDW, CG, H, GPB, false>(st, A, s);
}

// one wave per chain, four chains per block, when chains are many (batched simulations);
// otherwise one chain per block with its rows split over 8 waves (two per SIMD)
template <typename CT>
static hipError_t launch_round_k_t(hipStream_t st, const RoundArgs& A, int s) {
    const bool many = A.C >= 1024;
    switch (round_k_ndw(A.n)) {
        case 2: return many ? round_k_launch<CT, 2, 1, 1, 4>(st, A, s) : round_k_launch<CT, 2, 1, 1, 1>(st, A, s);
        case 4: return many ? round_k_launch<CT, 4, 1, 1, 4>(st, A, s) : round_k_launch<CT, 4, 1, 2, 1>(st, A, s);
        case 8: return many ? round_k_launch<CT, 8, 1, 1, 4>(st, A, s) : round_k_launch<CT, 8, 1, 4, 1>(st, A, s);
        case 16: return many ? round_k_launch<CT, 16, 1, 1, 4>(st, A, s) : round_k_launch<CT, 16, 1, 8, 1>(st, A, s);
        case 32: return round_k_launch<CT, 32, 2, 4, 1>(st, A, s);
        case 64: return round_k_launch<CT, 64, 4, 2, 1>(st, A, s);
        default: return hipErrorInvalidValue;   // n > 256: k_round_step_big
    }
}

hipError_t launch_round_k(hipStream_t st, const RoundArgs& A, int s) {
    return A.compact ? launch_round_k_t<uint16_t>(st, A, s) : launch_round_k_t<int32_t>(st, A, s);
}

void launch_round_k_gather(hipStream_t st, const RoundArgs& A, int r) {
    const int ndw = round_k_ndw(A.n);
    const int64_t work = (int64_t)A.C * ndw;
    if (work <= 0) return;
    if (A.compact)
        hipLaunchKernelGGL(k_round_k_gather<uint16_t>, dim3((unsigned)((work + 255) / 256)), dim3(256), 0, st, A, ndw, r);
    else
        hipLaunchKernelGGL(k_round_k_gather<int32_t>, dim3((unsigned)((work + 255) / 256)), dim3(256), 0, st, A, ndw, r);
}

}  // namespace hgx
