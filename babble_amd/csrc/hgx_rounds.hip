// Round assignment for n <= 256: one fused launch per round.
//
// Step r, one block per chain c, candidates W'_r = first event of every chain with
// round >= r. The chain's boundary Bm[r+1][c] is the first offset k >= Bm[r][c]
// whose event strongly sees >= SM candidates (RoundInc, hashgraph.go:285-305).
// StronglySee(x_k, w) is monotone in k (lastAncestors only grow along a chain), so
// for every candidate w the block binary-searches the first probe of a window of P
// probes that strongly sees w (log2(P+1) ballot/popcount tests instead of P); a
// histogram of those first hits gives the count per probe. Candidates are split
// over the waves, each wave keeps its candidates' firstDescendants slices in
// registers; the P probe rows (lastAncestors) are staged in LDS.
// The same step records, for the new boundary event (the candidate of round r+1),
// the bitmask of W'_r it strongly sees: DecideFame's S_{r+1} matrix for free.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

#include "hgx_device.h"
#include "hgx_kernels.h"

namespace hgx {

// Optional phase timing of the round step (build with -DHGX_STEP_PROF): thread 0 of
// every block adds clock deltas per phase into hgx_step_prof[8].
#ifdef HGX_STEP_PROF
__device__ unsigned long long hgx_step_prof[8];
#define HGX_PROF_BEGIN() long long _pt = clock64()
#define HGX_PROF(i)                                                  \
    do {                                                             \
        if (threadIdx.x == 0) {                                      \
            const long long _t = clock64();                          \
            atomicAdd(&hgx_step_prof[i], (unsigned long long)(_t - _pt)); \
            _pt = _t;                                                \
        }                                                            \
    } while (0)
#else
#define HGX_PROF_BEGIN() (void)0
#define HGX_PROF(i) (void)0
#endif

template <int CPL>
__device__ __forceinline__ bool ss_test(const int32_t* __restrict__ la_row, const int32_t (&fd)[CPL], int lane,
                                        int n, int sm) {
    int tot = 0;
#pragma unroll
    for (int q = 0; q < CPL; q++) {
        const int i = lane + 64 * q;
        // unconditional LDS read (rows are staged with CPL*64 slack, see la_s), then a
        // select: a guarded read becomes an exec branch + lgkmcnt(0) per read
        const int32_t raw = la_row[i];
        const int32_t la = (i < n) ? raw : -1;
        tot += __popcll(__ballot(la >= fd[q]));
    }
    return tot >= sm;
}

template <int CPL, int OWN, int NWAVES, int P>
__global__ void __launch_bounds__(NWAVES * 64) k_round_step2(
    int kstep, const int32_t* __restrict__ d_base, int32_t* __restrict__ Bm, const int32_t* __restrict__ c_off,
    const int32_t* __restrict__ c_len, const int32_t* __restrict__ LA, const int32_t* __restrict__ FDT,
    const int32_t* __restrict__ p_gid, const uint8_t* __restrict__ g_coin, int32_t* __restrict__ WLA,
    int32_t* __restrict__ WFD, uint8_t* __restrict__ wflag, uint8_t* __restrict__ wstat, uint8_t* __restrict__ wcoin,
    uint64_t* __restrict__ Smat, int32_t* __restrict__ p_round, int32_t* __restrict__ active, int32_t* __restrict__ lr,
    int C, int n, int nw, int sm, int64_t Pcap) {
    constexpr int NT = NWAVES * 64;
    typedef __attribute__((address_space(3))) void* lds_ptr_t;
    __shared__ int32_t cand[256];
    __shared__ int32_t kf_s[256];   // per candidate slot: first probe that strongly sees it
    __shared__ int32_t hist[P + 1];
    __shared__ int32_t s_ncand, s_first;
    __shared__ unsigned long long s_mask[4];
    // P probe rows at stride n; + 64*CPL slack so ss_test may read a full CPL*64 row
    __shared__ __attribute__((aligned(16))) int32_t la_s[P * 64 * CPL + 64 * CPL];
    HGX_PROF_BEGIN();
#ifdef HGX_STEP_PROF
    if (threadIdx.x == 0) atomicAdd(&hgx_step_prof[0], 1ull);
#endif
    const int r = *d_base + kstep;
    const int gc = blockIdx.x;
    const int g = gc / n, cl = gc % n;
    const int len = c_len[gc];
    const int off = c_off[gc];
    const int b = Bm[(size_t)r * C + gc];
    const int lane = lane_id(), wave = threadIdx.x >> 6;
    int kstar = len;
    if (b < len) {
        if (threadIdx.x == 0) s_ncand = 0;
        if (threadIdx.x < 4) s_mask[threadIdx.x] = 0;
        __syncthreads();
        for (int j = threadIdx.x; j < n; j += NT)
            if (wflag[(size_t)r * C + (size_t)g * n + j] == 1) cand[atomicAdd(&s_ncand, 1)] = j;
        __syncthreads();
        HGX_PROF(1);
        const int ncand = s_ncand;
        int32_t fd[OWN][CPL];
        int own_c[OWN];   // wave-uniform (SGPRs)
#pragma unroll
        for (int o = 0; o < OWN; o++) {
            const int wi = wave + NWAVES * o;
            own_c[o] = __builtin_amdgcn_readfirstlane((wi < ncand) ? cand[wi] : -1);
#pragma unroll
            for (int q = 0; q < CPL; q++) {
                const int i = lane + 64 * q;
                fd[o][q] = (own_c[o] >= 0 && i < n)
                               ? WFD[((size_t)r * C + (size_t)g * n + own_c[o]) * n + i] : kMaxI32;
            }
        }
        int kbase = b;
        for (;;) {
#ifdef HGX_STEP_PROF
            if (threadIdx.x == 0) atomicAdd(&hgx_step_prof[6], 1ull);
#endif
            const int np = min(P, len - kbase);
            const int nel = np * n;
            const int32_t* __restrict__ src = LA + (size_t)(off + kbase) * n;
            // stage the probe rows straight into LDS (global_load_lds): one wave
            // instruction moves 64 lanes x 16 B (or x 4 B when rows are not 16-B aligned)
            if ((n & 3) == 0) {
                for (int c0 = wave * 256; c0 < nel; c0 += NWAVES * 256) {
                    const int t = c0 + lane * 4;
                    if (t < nel)
                        __builtin_amdgcn_global_load_lds((const void*)(src + t), (lds_ptr_t)(la_s + c0), 16, 0, 0);
                }
            } else {
                for (int c0 = wave * 64; c0 < nel; c0 += NWAVES * 64) {
                    const int t = c0 + lane;
                    if (t < nel)
                        __builtin_amdgcn_global_load_lds((const void*)(src + t), (lds_ptr_t)(la_s + c0), 4, 0, 0);
                }
            }
            for (int t = threadIdx.x; t <= P; t += NT) hist[t] = 0;
            __builtin_amdgcn_s_waitcnt(0);
            __syncthreads();
            HGX_PROF(2);
            // four candidates' searches interleaved (independent LDS/ballot chains)
            static_assert(OWN % 4 == 0, "candidates are searched four at a time");
#pragma unroll
            for (int o0 = 0; o0 < OWN; o0 += 4) {
                if (own_c[o0] < 0) break;                         // wave-uniform; own_c fills in order
                int lo[4], hi[4];
#pragma unroll
                for (int u = 0; u < 4; u++) { lo[u] = 0; hi[u] = (own_c[o0 + u] >= 0) ? np : 0; }
                for (;;) {
                    bool open = false;
#pragma unroll
                    for (int u = 0; u < 4; u++) open |= lo[u] < hi[u];
                    if (!open) break;
                    int mid[4];
                    bool t[4];
#pragma unroll
                    for (int u = 0; u < 4; u++) mid[u] = min((lo[u] + hi[u]) >> 1, np - 1);
#pragma unroll
                    for (int u = 0; u < 4; u++) t[u] = ss_test<CPL>(la_s + mid[u] * n, fd[o0 + u], lane, n, sm);
#pragma unroll
                    for (int u = 0; u < 4; u++)
                        if (lo[u] < hi[u]) { if (t[u]) hi[u] = mid[u]; else lo[u] = mid[u] + 1; }
                }
#pragma unroll
                for (int u = 0; u < 4; u++) {
                    const int o = o0 + u;
                    if (own_c[o] < 0) continue;
                    int l = lo[u];
                    if (own_c[o] == cl && kbase + l == b && l < np) l++;   // x == w never counts (n == 1)
                    if (lane == 0) {
                        kf_s[wave + NWAVES * o] = l;
                        atomicAdd(&hist[l], 1);
                    }
                }
            }
            __syncthreads();
            HGX_PROF(3);
            if (threadIdx.x == 0) {
                int acc = 0, f = 0x7fffffff;
                for (int pp = 0; pp < np; pp++) {
                    acc += hist[pp];
                    if (acc >= sm) { f = pp; break; }
                }
                s_first = f;
            }
            __syncthreads();
            HGX_PROF(4);
            const int f = s_first;
            if (f != 0x7fffffff) {
                kstar = kbase + f;
                for (int j = threadIdx.x; j < ncand; j += NT)
                    if (kf_s[j] <= f) atomicOr(&s_mask[cand[j] >> 6], 1ull << (cand[j] & 63));
                break;
            }
            kbase += P;
            if (kbase >= len) { kstar = len; break; }
            __syncthreads();
        }
        __syncthreads();
        HGX_PROF(5);
        for (int k = b + (int)threadIdx.x; k < kstar; k += NT) p_round[off + k] = r;
        if (threadIdx.x == 0) {
            wstat[(size_t)r * C + gc] = (kstar > b) ? 2 : 1;
            if (kstar < len) atomicOr(&active[r], 1);
            if (kstar > b) atomicMax(&lr[g], r);
        }
        if (kstar < len && threadIdx.x < nw) Smat[((size_t)(r + 1) * C + gc) * nw + threadIdx.x] = s_mask[threadIdx.x];
    } else if (threadIdx.x == 0) {
        wstat[(size_t)r * C + gc] = 0;
    }
    if (threadIdx.x == 0) Bm[(size_t)(r + 1) * C + gc] = kstar;
    // coordinate rows of this chain's candidate for round r+1 (offset kstar)
    const size_t nrow = ((size_t)(r + 1) * C + gc) * n;
    if (kstar < len) {
        const int p = off + kstar;
        for (int i = threadIdx.x; i < n; i += NT) {
            const int32_t a = LA[(size_t)p * n + i];
            const int32_t d = FDT[(size_t)i * Pcap + p];
            WLA[nrow + i] = a;
            WFD[nrow + i] = d;
        }
        if (threadIdx.x == 0) {
            wflag[(size_t)(r + 1) * C + gc] = 1;
            wcoin[(size_t)(r + 1) * C + gc] = g_coin[p_gid[p]];
        }
    } else if (threadIdx.x == 0) {
        wflag[(size_t)(r + 1) * C + gc] = 0;
    }
    HGX_PROF(7);
}

__global__ void k_advance_round(int32_t* d_base, int by) { *d_base += by; }

bool launch_round_step(hipStream_t s, const DevArrays& a, int kstep, int C, int n, int sm, int64_t P) {
    const int nw = (n + 63) / 64;
#define STEP2(CPL, OWN, NWAVES, PP)                                                                             \
    hipLaunchKernelGGL((k_round_step2<CPL, OWN, NWAVES, PP>), dim3(C), dim3(NWAVES * 64), 0, s, kstep,         \
                       a.d_round, a.Bm, a.c_off, a.c_len, a.LA, a.FDT, a.p_gid, a.g_coin, a.WLA, a.WFD, a.wflag, \
                       a.wstat, a.wcoin, a.Smat, a.p_round, a.active, a.lr, C, n, nw, sm, P)
    if (n <= 32) STEP2(1, 8, 4, 64);
    else if (n <= 64) STEP2(1, 4, 16, 64);
    else if (n <= 128) STEP2(2, 8, 16, 64);
    else if (n <= 256) STEP2(4, 16, 16, 48);
    else return false;
#undef STEP2
    return true;
}

#ifdef HGX_STEP_PROF
void step_prof_dump() {
    unsigned long long h[8];
    if (hipMemcpyFromSymbol(h, HIP_SYMBOL(hgx_step_prof), sizeof(h)) != hipSuccess) return;
    fprintf(stderr, "[hgx] step phases (clk sums):");
    for (int i = 0; i < 8; i++) fprintf(stderr, " %d:%llu", i, h[i]);
    fprintf(stderr, "\n");
}
#else
void step_prof_dump() {}
#endif

void launch_advance_round(hipStream_t s, const DevArrays& a, int by) {
    hipLaunchKernelGGL(k_advance_round, dim3(1), dim3(1), 0, s, a.d_round, by);
}

}  // namespace hgx
