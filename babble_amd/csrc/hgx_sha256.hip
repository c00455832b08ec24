// Batched SHA-256 of event wire bodies (ingest front end).
//
// The reference hashes one event at a time on the insert path:
//   crypto.SHA256                 crypto/utils.go:11-16
//   Event.Hash  = SHA256(Marshal) hashgraph/event.go:171-180 (the event id, Hex() at :183-188)
//   EventBody.Hash                hashgraph/event.go:48-54   (the bytes Verify checks, :142-152)
//   Block.Hash                    hashgraph/block.go:44-53
// Here a whole batch of already-encoded messages is hashed in one launch: one lane per
// message, the 64-round compression fully unrolled in VGPRs (rotates are v_alignbit,
// Sigma/Ch/Maj v_bitop3). The work is VALU-bound (~1.5 k lane instructions per 64-byte
// block against ~68 bytes read), so there is no LDS staging: each lane streams its own
// message with 16-byte loads from the 16-byte-aligned address below each block (guarded:
// a 16-byte slice holding no message byte is not read), so a load may touch up to 15
// bytes before the message's first byte and up to 15 bytes past its last byte, always
// inside the 16-byte-aligned span of the message (include/hgx.h states this for the
// device entry). The Merkle-Damgard padding is built in registers.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstring>
#include <cstdio>
#include <vector>

#include "hgx.h"

namespace hgx {

__device__ __forceinline__ uint32_t rotr(uint32_t x, int n) { return __builtin_amdgcn_alignbit(x, x, n); }
// a ^ b ^ c in one v_bitop3_b32 (truth table 0x96)
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

#define HGX_SHA_R(a, b, c, d, e, f, g, h, k, w)                                        \
    do {                                                                               \
        uint32_t t1 = h + xor3(rotr(e, 6), rotr(e, 11), rotr(e, 25)) + ((e & f) ^ (~e & g)) + (k) + (w); \
        uint32_t t2 = xor3(rotr(a, 2), rotr(a, 13), rotr(a, 22)) + ((a & b) ^ (c & (a ^ b)));          \
        d += t1;                                                                       \
        h = t1 + t2;                                                                   \
    } while (0)

__device__ __forceinline__ void sha256_compress(uint32_t st[8], uint32_t w[16]) {
    constexpr uint32_t K[64] = {
        0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
        0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
        0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
        0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
        0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
        0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
        0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
        0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};
    uint32_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4], f = st[5], g = st[6], h = st[7];
#pragma unroll
    for (int i = 0; i < 64; i += 8) {
        if (i >= 16) {
            // schedule the next 8 words in place (w is a rolling 16-word window)
#pragma unroll
            for (int j = 0; j < 8; j++) {
                const int t = (i + j) & 15;
                const uint32_t x15 = w[(t + 1) & 15], x2 = w[(t + 14) & 15];
                w[t] += xor3(rotr(x15, 7), rotr(x15, 18), x15 >> 3) + w[(t + 9) & 15] +
                        xor3(rotr(x2, 17), rotr(x2, 19), x2 >> 10);
            }
        }
        HGX_SHA_R(a, b, c, d, e, f, g, h, K[i + 0], w[(i + 0) & 15]);
        HGX_SHA_R(h, a, b, c, d, e, f, g, K[i + 1], w[(i + 1) & 15]);
        HGX_SHA_R(g, h, a, b, c, d, e, f, K[i + 2], w[(i + 2) & 15]);
        HGX_SHA_R(f, g, h, a, b, c, d, e, K[i + 3], w[(i + 3) & 15]);
        HGX_SHA_R(e, f, g, h, a, b, c, d, K[i + 4], w[(i + 4) & 15]);
        HGX_SHA_R(d, e, f, g, h, a, b, c, K[i + 5], w[(i + 5) & 15]);
        HGX_SHA_R(c, d, e, f, g, h, a, b, K[i + 6], w[(i + 6) & 15]);
        HGX_SHA_R(b, c, d, e, f, g, h, a, K[i + 7], w[(i + 7) & 15]);
    }
    st[0] += a; st[1] += b; st[2] += c; st[3] += d; st[4] += e; st[5] += f; st[6] += g; st[7] += h;
}
#undef HGX_SHA_R

// One lane per message i = data[offsets[i], offsets[i+1]); digest to out + 32 i.
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4))) void k_sha256_batch(const uint8_t* __restrict__ data,
                                                      const int64_t* __restrict__ offsets, int64_t count,
                                                      uint8_t* __restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= count) return;
    const int64_t off = offsets[i];
    const int64_t len = offsets[i + 1] - off;
    uint32_t st[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a, 0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
    const int64_t nb = (len + 72) >> 6;   // ceil((len + 1 + 8) / 64)
    const uintptr_t a0 = (uintptr_t)(data + off);
    // 16-byte loads from the aligned-down address: sh16 = q*4 + sh bytes of lead-in
    const int sh16 = (int)(a0 & 15), q = sh16 >> 2, sh = sh16 & 3;
    const uint4* vp = (const uint4*)(data + (off - sh16));   // derived from data: stays a global load
    const uint64_t bits = (uint64_t)len * 8;
    // one 16-byte slice per load that holds a message byte; 5 slices cover a 64-byte block
    auto load_block = [&](int64_t b, uint4 (&E)[5]) {
        const int64_t rem = len - 64 * b;
#pragma unroll
        for (int t = 0; t < 5; t++) E[t] = (16 * t - sh16 < rem) ? vp[4 * b + t] : make_uint4(0, 0, 0, 0);
    };
    uint4 E[5];
    load_block(0, E);
    for (int64_t b = 0; b < nb; b++) {
        const int64_t rem = len - 64 * b;   // message bytes from this block's first byte on
        uint32_t D[20];
#pragma unroll
        for (int t = 0; t < 5; t++) { D[4 * t] = E[t].x; D[4 * t + 1] = E[t].y; D[4 * t + 2] = E[t].z; D[4 * t + 3] = E[t].w; }
        if (b + 1 < nb) load_block(b + 1, E);   // next block in flight during this compression
        uint32_t d[17];
#pragma unroll
        for (int j = 0; j < 17; j++) d[j] = q == 0 ? D[j] : q == 1 ? D[j + 1] : q == 2 ? D[j + 2] : D[j + 3];
        uint32_t w[16];
        const int r = (int)(rem < 64 ? rem : 64);   // valid bytes in this block, 32-bit math below
#pragma unroll
        for (int k = 0; k < 16; k++) {
            const uint32_t x = __builtin_bswap32(__builtin_amdgcn_alignbyte(d[k + 1], d[k], sh));
            const int v = r - 4 * k;   // valid bytes of word k
            uint32_t y;
            if (v >= 4) y = x;
            else if (v > 0) y = (x & (0xFFFFFFFFu << (32 - 8 * v))) | (0x80u << (24 - 8 * v));
            else y = (v == 0) ? 0x80000000u : 0u;
            w[k] = y;
        }
        if (b == nb - 1) {   // the last block (rem <= 55) carries the bit length
            w[14] = (uint32_t)(bits >> 32);
            w[15] = (uint32_t)bits;
        }
        sha256_compress(st, w);
    }
    uint32_t* o = (uint32_t*)(out + 32 * i);
#pragma unroll
    for (int k = 0; k < 8; k++) o[k] = __builtin_bswap32(st[k]);
}


__device__ __host__ __forceinline__ uint64_t splitmix64(uint64_t x) {
    uint64_t z = x + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

// synthetic message bytes for the bench leg: 8 bytes j*8.. = splitmix64(seed + j), little-endian
__global__ void k_fill_bytes(uint64_t* __restrict__ p, int64_t words, uint64_t seed) {
    for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < words; j += (int64_t)gridDim.x * blockDim.x)
        p[j] = splitmix64(seed + (uint64_t)j);
}

}  // namespace hgx

namespace {

void set_err(hgx_error* err, int32_t code, const char* msg) {
    if (!err) return;
    err->code = code;
    std::snprintf(err->msg, sizeof(err->msg), "%s", msg);
}

hipError_t launch_sha256(const uint8_t* d_data, const int64_t* d_offsets, int64_t count, uint8_t* d_out,
                         hipStream_t s) {
    if (count <= 0) return hipSuccess;
    const int64_t blocks = (count + 255) / 256;
    hipLaunchKernelGGL(hgx::k_sha256_batch, dim3((unsigned)blocks), dim3(256), 0, s, d_data, d_offsets, count, d_out);
    return hipGetLastError();
}

}  // namespace

extern "C" int32_t hgx_sha256_batch(int32_t device, const uint8_t* data, const int64_t* offsets, int64_t count,
                                    uint8_t* out32, hgx_error* err) {
    set_err(err, HGX_OK, "");
    if (count < 0 || (count > 0 && (!offsets || !out32)) || count > (int64_t)UINT32_MAX * 256) {
        set_err(err, HGX_ERR_INVALID, "hgx_sha256_batch: bad arguments");
        return HGX_ERR_INVALID;
    }
    if (count == 0) return HGX_OK;
    if (offsets[0] < 0) {
        set_err(err, HGX_ERR_INVALID, "hgx_sha256_batch: negative offset");
        return HGX_ERR_INVALID;
    }
    for (int64_t i = 0; i < count; i++)
        if (offsets[i + 1] < offsets[i]) {
            set_err(err, HGX_ERR_INVALID, "hgx_sha256_batch: offsets must be non-decreasing");
            return HGX_ERR_INVALID;
        }
    const int64_t total = offsets[count];
    if (total > 0 && !data) {
        set_err(err, HGX_ERR_INVALID, "hgx_sha256_batch: null data");
        return HGX_ERR_INVALID;
    }
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) {
        set_err(err, HGX_ERR_DEVICE, "no HIP device available (libhgx has no CPU fallback)");
        return HGX_ERR_DEVICE;
    }
    hipDeviceProp_t prop;
    if (device < 0 || device >= ndev || hipGetDeviceProperties(&prop, device) != hipSuccess ||
        std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) {
        set_err(err, HGX_ERR_DEVICE, "libhgx is built for gfx950 (MI355X) only");
        return HGX_ERR_DEVICE;
    }
    int prev = 0;
    (void)hipGetDevice(&prev);
    (void)hipSetDevice(device);
    uint8_t *d_data = nullptr, *d_out = nullptr;
    int64_t* d_off = nullptr;
    hipStream_t s = nullptr;
    hipError_t e = hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipMalloc((void**)&d_data, (size_t)total + 4);
    if (e == hipSuccess) e = hipMalloc((void**)&d_off, sizeof(int64_t) * (size_t)(count + 1));
    if (e == hipSuccess) e = hipMalloc((void**)&d_out, 32 * (size_t)count);
    if (e == hipSuccess && total > 0) e = hipMemcpyAsync(d_data, data, (size_t)total, hipMemcpyHostToDevice, s);
    if (e == hipSuccess)
        e = hipMemcpyAsync(d_off, offsets, sizeof(int64_t) * (size_t)(count + 1), hipMemcpyHostToDevice, s);
    if (e == hipSuccess) e = launch_sha256(d_data, d_off, count, d_out, s);
    if (e == hipSuccess) e = hipMemcpyAsync(out32, d_out, 32 * (size_t)count, hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    if (d_data) (void)hipFree(d_data);
    if (d_off) (void)hipFree(d_off);
    if (d_out) (void)hipFree(d_out);
    if (s) (void)hipStreamDestroy(s);
    (void)hipSetDevice(prev);
    if (e != hipSuccess) {
        set_err(err, HGX_ERR_DEVICE, hipGetErrorString(e));
        return HGX_ERR_DEVICE;
    }
    return HGX_OK;
}

extern "C" int32_t hgx_sha256_batch_device(const uint8_t* d_data, const int64_t* d_offsets, int64_t count,
                                           uint8_t* d_out32, void* stream) {
    if (count < 0 || (count > 0 && (!d_data || !d_offsets || !d_out32)) || ((uintptr_t)d_out32 & 3))
        return HGX_ERR_INVALID;
    return launch_sha256(d_data, d_offsets, count, d_out32, (hipStream_t)stream) == hipSuccess ? HGX_OK
                                                                                                : HGX_ERR_DEVICE;
}

// Measurement entry for bench.py (no torch on the device side): `count` synthetic messages,
// resident in HBM, hashed warmup + iters times; ms_per_launch from HIP events on the launch stream. Message i has length
// min_len + splitmix64(~seed + i) % (max_len - min_len + 1); the packed bytes are
// splitmix64(seed + j) for 8-byte word j. The digests of the first n_sample messages are
// copied to sample32 so the caller can check them.
extern "C" int32_t hgx_sha256_bench(int32_t device, int64_t count, int32_t min_len, int32_t max_len, uint64_t seed,
                                    int32_t warmup, int32_t iters, double* ms_per_launch, int64_t* total_bytes,
                                    int64_t* n_blocks, int64_t n_sample, uint8_t* sample32) {
    if (count <= 0 || min_len < 0 || max_len < min_len || iters <= 0 || warmup < 0 || n_sample < 0 ||
        n_sample > count || (n_sample && !sample32) || !ms_per_launch)
        return HGX_ERR_INVALID;
    std::vector<int64_t> off((size_t)count + 1);
    int64_t blocks = 0;
    off[0] = 0;
    const uint64_t span = (uint64_t)(max_len - min_len) + 1;
    for (int64_t i = 0; i < count; i++) {
        const int64_t len = min_len + (int64_t)(hgx::splitmix64(~seed + (uint64_t)i) % span);
        off[i + 1] = off[i] + len;
        blocks += (len + 72) >> 6;
    }
    const int64_t total = off[count];
    const int64_t words = (total + 7) / 8 + 1;
    int prev = 0;
    (void)hipGetDevice(&prev);
    if (hipSetDevice(device) != hipSuccess) return HGX_ERR_DEVICE;
    uint8_t *d_data = nullptr, *d_out = nullptr;
    int64_t* d_off = nullptr;
    hipStream_t s = nullptr;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    float ms = 0.f;
    hipError_t e = hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipEventCreate(&e0);
    if (e == hipSuccess) e = hipEventCreate(&e1);
    if (e == hipSuccess) e = hipMalloc((void**)&d_data, (size_t)words * 8);
    if (e == hipSuccess) e = hipMalloc((void**)&d_off, sizeof(int64_t) * (size_t)(count + 1));
    if (e == hipSuccess) e = hipMalloc((void**)&d_out, 32 * (size_t)count);
    if (e == hipSuccess)
        e = hipMemcpyAsync(d_off, off.data(), sizeof(int64_t) * (size_t)(count + 1), hipMemcpyHostToDevice, s);
    if (e == hipSuccess) {
        hipLaunchKernelGGL(hgx::k_fill_bytes, dim3(4096), dim3(256), 0, s, (uint64_t*)d_data, words, seed);
        e = hipGetLastError();
    }
    for (int32_t k = 0; e == hipSuccess && k < warmup; k++) e = launch_sha256(d_data, d_off, count, d_out, s);
    if (e == hipSuccess) e = hipEventRecord(e0, s);
    for (int32_t k = 0; e == hipSuccess && k < iters; k++) e = launch_sha256(d_data, d_off, count, d_out, s);
    if (e == hipSuccess) e = hipEventRecord(e1, s);
    if (e == hipSuccess && n_sample) e = hipMemcpyAsync(sample32, d_out, 32 * (size_t)n_sample, hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    if (e == hipSuccess) e = hipEventElapsedTime(&ms, e0, e1);
    if (d_data) (void)hipFree(d_data);
    if (d_off) (void)hipFree(d_off);
    if (d_out) (void)hipFree(d_out);
    if (e0) (void)hipEventDestroy(e0);
    if (e1) (void)hipEventDestroy(e1);
    if (s) (void)hipStreamDestroy(s);
    (void)hipSetDevice(prev);
    if (e != hipSuccess) return HGX_ERR_DEVICE;
    *ms_per_launch = (double)ms / iters;
    if (total_bytes) *total_bytes = total;
    if (n_blocks) *n_blocks = blocks;
    return HGX_OK;
}
