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

#include "hgx_device.h"
#include "hgx_kernels.h"

namespace hgx {

template <int CPL>
__device__ __forceinline__ bool ss_test(const int32_t* __restrict__ la_row, const int32_t (&fd)[CPL], int lane,
                                        int n, int sm) {
    int tot = 0;
#pragma unroll
    for (int q = 0; q < CPL; q++) {
        const int i = lane + 64 * q;
        const int32_t la = (i < n) ? la_row[i] : -1;
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
    __shared__ int32_t cand[256];
    __shared__ int32_t hist[P + 1];
    __shared__ int32_t s_ncand, s_first;
    __shared__ unsigned long long s_mask[4];
    __shared__ __attribute__((aligned(16))) int32_t la_s[P * 64 * CPL];
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
        const int ncand = s_ncand;
        int32_t fd[OWN][CPL];
        int own_c[OWN];
        int kfirst[OWN];
#pragma unroll
        for (int o = 0; o < OWN; o++) {
            const int wi = wave + NWAVES * o;
            own_c[o] = (wi < ncand) ? cand[wi] : -1;
            kfirst[o] = 0;
#pragma unroll
            for (int q = 0; q < CPL; q++) {
                const int i = lane + 64 * q;
                fd[o][q] = (own_c[o] >= 0 && i < n)
                               ? WFD[((size_t)r * C + (size_t)g * n + own_c[o]) * n + i] : kMaxI32;
            }
        }
        int kbase = b;
        for (;;) {
            const int np = min(P, len - kbase);
            const int nel = np * n;
            const int32_t* __restrict__ src = LA + (size_t)(off + kbase) * n;
            // stage the probe rows: 4 independent loads in flight per thread
            for (int t0 = threadIdx.x; t0 < nel; t0 += 4 * NT) {
                int32_t v[4];
#pragma unroll
                for (int u = 0; u < 4; u++) {
                    const int t = t0 + u * NT;
                    v[u] = (t < nel) ? src[t] : 0;
                }
#pragma unroll
                for (int u = 0; u < 4; u++) {
                    const int t = t0 + u * NT;
                    if (t < nel) la_s[t] = v[u];
                }
            }
            for (int t = threadIdx.x; t <= P; t += NT) hist[t] = 0;
            __syncthreads();
#pragma unroll
            for (int o = 0; o < OWN; o++) {
                if (own_c[o] < 0) continue;                       // wave-uniform
                int lo = 0, hi = np;
                while (lo < hi) {
                    const int mid = (lo + hi) >> 1;
                    if (ss_test<CPL>(la_s + mid * n, fd[o], lane, n, sm)) hi = mid; else lo = mid + 1;
                }
                if (own_c[o] == cl && kbase + lo == b && lo < np) lo++;   // x == w never counts (n == 1)
                kfirst[o] = lo;
                if (lane == 0) atomicAdd(&hist[lo], 1);
            }
            __syncthreads();
            if (threadIdx.x == 0) {
                int acc = 0, f = 0x7fffffff;
                for (int pp = 0; pp < np; pp++) {
                    acc += hist[pp];
                    if (acc >= sm) { f = pp; break; }
                }
                s_first = f;
            }
            __syncthreads();
            const int f = s_first;
            if (f != 0x7fffffff) {
                kstar = kbase + f;
#pragma unroll
                for (int o = 0; o < OWN; o++)
                    if (own_c[o] >= 0 && kfirst[o] <= f && lane == 0)
                        atomicOr(&s_mask[own_c[o] >> 6], 1ull << (own_c[o] & 63));
                break;
            }
            kbase += P;
            if (kbase >= len) { kstar = len; break; }
            __syncthreads();
        }
        __syncthreads();
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

void launch_advance_round(hipStream_t s, const DevArrays& a, int by) {
    hipLaunchKernelGGL(k_advance_round, dim3(1), dim3(1), 0, s, a.d_round, by);
}

}  // namespace hgx
