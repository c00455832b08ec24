// Batched ECDSA P-256 signature verification: Event.Verify (hashgraph/event.go:142-152) =
// crypto.Verify (crypto/utils.go:41-43) = Go's ecdsa.Verify on elliptic.P256() for every
// event of a sync batch, one lane per signature.
//
//   r, s in [1, N-1]; e = digest (32 bytes, big-endian; e mod N); w = s^-1 mod N;
//   u1 = e w, u2 = r w (mod N); (X : Y : Z) = u1 G + u2 Q; valid iff Z != 0 and
//   X / Z^2 == r (mod N).
//
// Arithmetic: 8 x 32-bit limbs, Montgomery multiplication (CIOS, v_mad_u64_u32) modulo p
// (field) and modulo N (scalars, s^-1 by Fermat); Jacobian points, a = -3 doubling
// (dbl-2001-b) and complete-case addition (add-2007-bl, doubling / infinity branches per
// lane). u1 G + u2 Q by fixed-base combs: for G and for every key (a context has few, each
// signing many events) a table of b * 256^j * P for the 32 byte positions j and the 255 digits b,
// affine, built once when the keys are set (512 KB per key, hgx_set_participant_keys); a verify is
// then at most 64 mixed Jacobian + affine additions (madd-2007-bl, 7M + 4S) and no doubling. The
// final compare avoids the field inversion: X == r Z^2 or, when r + N < p, X == (r + N) Z^2.
// Public keys that are not P-256 points (Go's elliptic.Unmarshal returns nil) give 2.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstring>

#include "hgx.h"
#include "hgx_kernels.h"

namespace hgx {
namespace p256 {

struct ModP {
    static constexpr uint32_t n[8] = {0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0x00000000u,
                                      0x00000000u, 0x00000000u, 0x00000001u, 0xFFFFFFFFu};
    static constexpr uint32_t n0 = 0x00000001u;   // -p^-1 mod 2^32
};
struct ModN {
    static constexpr uint32_t n[8] = {0xFC632551u, 0xF3B9CAC2u, 0xA7179E84u, 0xBCE6FAADu,
                                      0xFFFFFFFFu, 0xFFFFFFFFu, 0x00000000u, 0xFFFFFFFFu};
    static constexpr uint32_t n0 = 0xEE00BC4Fu;   // -N^-1 mod 2^32
};

// Montgomery constants (R = 2^256)
__device__ constexpr uint32_t kR2P[8] = {0x00000003u, 0x00000000u, 0xFFFFFFFFu, 0xFFFFFFFBu,
                                         0xFFFFFFFEu, 0xFFFFFFFFu, 0xFFFFFFFDu, 0x00000004u};
__device__ constexpr uint32_t kR2N[8] = {0xBE79EEA2u, 0x83244C95u, 0x49BD6FA6u, 0x4699799Cu,
                                         0x2B6BEC59u, 0x2845B239u, 0xF3D95620u, 0x66E12D94u};
__device__ constexpr uint32_t kOneP[8] = {0x00000001u, 0x00000000u, 0x00000000u, 0xFFFFFFFFu,
                                          0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFEu, 0x00000000u};
__device__ constexpr uint32_t kOneN[8] = {0x039CDAAFu, 0x0C46353Du, 0x58E8617Bu, 0x43190552u,
                                          0x00000000u, 0x00000000u, 0xFFFFFFFFu, 0x00000000u};
__device__ constexpr uint32_t kBm[8] = {0x29C4BDDFu, 0xD89CDF62u, 0x78843090u, 0xACF005CDu,
                                        0xF7212ED6u, 0xE5A220ABu, 0x04874834u, 0xDC30061Du};   // b R mod p
__device__ constexpr uint32_t kGx[8] = {0xD898C296u, 0xF4A13945u, 0x2DEB33A0u, 0x77037D81u,
                                        0x63A440F2u, 0xF8BCE6E5u, 0xE12C4247u, 0x6B17D1F2u};
__device__ constexpr uint32_t kGy[8] = {0x37BF51F5u, 0xCBB64068u, 0x6B315ECEu, 0x2BCE3357u,
                                        0x7C0F9E16u, 0x8EE7EB4Au, 0xFE1A7F9Bu, 0x4FE342E2u};
__device__ constexpr uint32_t kPm2[8] = {0xFFFFFFFDu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0x00000000u,
                                         0x00000000u, 0x00000000u, 0x00000001u, 0xFFFFFFFFu};
__device__ constexpr uint32_t kNm2[8] = {0xFC63254Fu, 0xF3B9CAC2u, 0xA7179E84u, 0xBCE6FAADu,
                                         0xFFFFFFFFu, 0xFFFFFFFFu, 0x00000000u, 0xFFFFFFFFu};

typedef uint32_t Fe[8];

__device__ __forceinline__ void cpy(Fe r, const uint32_t* a) {
#pragma unroll
    for (int i = 0; i < 8; i++) r[i] = a[i];
}

__device__ __forceinline__ bool is_zero(const Fe a) {
    uint32_t x = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) x |= a[i];
    return x == 0;
}

__device__ __forceinline__ bool eq(const Fe a, const Fe b) {
    uint32_t x = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) x |= a[i] ^ b[i];
    return x == 0;
}

// a < b as 256-bit integers
__device__ __forceinline__ bool lt(const uint32_t* a, const uint32_t* b) {
    int64_t br = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) {
        const int64_t x = (int64_t)a[i] - (int64_t)b[i] + br;
        br = x >> 32;
    }
    return br != 0;
}

// r = a b R^-1 mod M (inputs < M), CIOS
template <class M>
__device__ __forceinline__ void mmul(Fe r, const Fe a, const Fe b) {
    uint32_t t[10];
#pragma unroll
    for (int j = 0; j < 10; j++) t[j] = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) {
        uint64_t c = 0;
#pragma unroll
        for (int j = 0; j < 8; j++) {
            c += (uint64_t)a[j] * b[i] + t[j];
            t[j] = (uint32_t)c;
            c >>= 32;
        }
        c += t[8];
        t[8] = (uint32_t)c;
        t[9] = (uint32_t)(c >> 32);
        const uint32_t m = t[0] * M::n0;
        c = ((uint64_t)m * M::n[0] + t[0]) >> 32;
#pragma unroll
        for (int j = 1; j < 8; j++) {
            c += (uint64_t)m * M::n[j] + t[j];
            t[j - 1] = (uint32_t)c;
            c >>= 32;
        }
        c += t[8];
        t[7] = (uint32_t)c;
        t[8] = t[9] + (uint32_t)(c >> 32);
    }
    uint32_t d[8];
    int64_t br = 0;
#pragma unroll
    for (int j = 0; j < 8; j++) {
        const int64_t x = (int64_t)t[j] - (int64_t)M::n[j] + br;
        d[j] = (uint32_t)x;
        br = x >> 32;
    }
    const bool ge = (t[8] != 0) || (br == 0);
#pragma unroll
    for (int j = 0; j < 8; j++) r[j] = ge ? d[j] : t[j];
}

template <class M>
__device__ __forceinline__ void madd(Fe r, const Fe a, const Fe b) {
    uint32_t s[8];
    uint64_t c = 0;
#pragma unroll
    for (int j = 0; j < 8; j++) {
        c += (uint64_t)a[j] + b[j];
        s[j] = (uint32_t)c;
        c >>= 32;
    }
    uint32_t d[8];
    int64_t br = 0;
#pragma unroll
    for (int j = 0; j < 8; j++) {
        const int64_t x = (int64_t)s[j] - (int64_t)M::n[j] + br;
        d[j] = (uint32_t)x;
        br = x >> 32;
    }
    const bool ge = (c != 0) || (br == 0);
#pragma unroll
    for (int j = 0; j < 8; j++) r[j] = ge ? d[j] : s[j];
}

template <class M>
__device__ __forceinline__ void msub(Fe r, const Fe a, const Fe b) {
    uint32_t s[8];
    int64_t br = 0;
#pragma unroll
    for (int j = 0; j < 8; j++) {
        const int64_t x = (int64_t)a[j] - (int64_t)b[j] + br;
        s[j] = (uint32_t)x;
        br = x >> 32;
    }
    if (br != 0) {   // a < b: add M back
        uint64_t c = 0;
#pragma unroll
        for (int j = 0; j < 8; j++) {
            c += (uint64_t)s[j] + M::n[j];
            s[j] = (uint32_t)c;
            c >>= 32;
        }
    }
    cpy(r, s);
}

// 32 big-endian bytes -> limbs
__device__ __forceinline__ void load_be(Fe r, const uint8_t* b) {
#pragma unroll
    for (int i = 0; i < 8; i++) {
        const uint8_t* q = b + 28 - 4 * i;
        r[i] = ((uint32_t)q[0] << 24) | ((uint32_t)q[1] << 16) | ((uint32_t)q[2] << 8) | (uint32_t)q[3];
    }
}

struct Pt {
    Fe X, Y, Z;   // Montgomery form mod p; Z == 0 is the point at infinity
};

// dbl-2001-b (a = -3)
__device__ __forceinline__ void pdbl(Pt& o, const Pt& a) {
    if (is_zero(a.Z) || is_zero(a.Y)) {
#pragma unroll
        for (int i = 0; i < 8; i++) o.Z[i] = 0;
        return;
    }
    Fe delta, gamma, beta, alpha, t1, t2;
    mmul<ModP>(delta, a.Z, a.Z);
    mmul<ModP>(gamma, a.Y, a.Y);
    mmul<ModP>(beta, a.X, gamma);
    msub<ModP>(t1, a.X, delta);
    madd<ModP>(t2, a.X, delta);
    mmul<ModP>(alpha, t1, t2);
    madd<ModP>(t1, alpha, alpha);
    madd<ModP>(alpha, t1, alpha);   // 3 (X - delta)(X + delta)
    Fe b4, b8, X3;
    madd<ModP>(b4, beta, beta);
    madd<ModP>(b4, b4, b4);         // 4 beta
    madd<ModP>(b8, b4, b4);         // 8 beta
    mmul<ModP>(X3, alpha, alpha);
    msub<ModP>(X3, X3, b8);
    Fe Z3;
    madd<ModP>(t1, a.Y, a.Z);
    mmul<ModP>(Z3, t1, t1);
    msub<ModP>(Z3, Z3, gamma);
    msub<ModP>(Z3, Z3, delta);
    Fe g2;
    mmul<ModP>(g2, gamma, gamma);
    madd<ModP>(g2, g2, g2);
    madd<ModP>(g2, g2, g2);
    madd<ModP>(g2, g2, g2);         // 8 gamma^2
    msub<ModP>(t1, b4, X3);
    mmul<ModP>(t2, alpha, t1);
    msub<ModP>(o.Y, t2, g2);
    cpy(o.X, X3);
    cpy(o.Z, Z3);
}

// add-2007-bl with the equal / opposite / infinity cases
__device__ __forceinline__ void padd(Pt& o, const Pt& a, const Pt& b) {
    if (is_zero(a.Z)) { o = b; return; }
    if (is_zero(b.Z)) { o = a; return; }
    Fe z1z1, z2z2, u1, u2, s1, s2, t;
    mmul<ModP>(z1z1, a.Z, a.Z);
    mmul<ModP>(z2z2, b.Z, b.Z);
    mmul<ModP>(u1, a.X, z2z2);
    mmul<ModP>(u2, b.X, z1z1);
    mmul<ModP>(t, b.Z, z2z2);
    mmul<ModP>(s1, a.Y, t);
    mmul<ModP>(t, a.Z, z1z1);
    mmul<ModP>(s2, b.Y, t);
    Fe H, r;
    msub<ModP>(H, u2, u1);
    msub<ModP>(r, s2, s1);
    if (is_zero(H)) {
        if (is_zero(r)) {
            pdbl(o, a);
        } else {
#pragma unroll
            for (int i = 0; i < 8; i++) o.Z[i] = 0;
        }
        return;
    }
    Fe I, J, V, X3, Y3, Z3;
    madd<ModP>(t, H, H);
    mmul<ModP>(I, t, t);            // (2H)^2
    mmul<ModP>(J, H, I);
    madd<ModP>(r, r, r);            // 2 (S2 - S1)
    mmul<ModP>(V, u1, I);
    mmul<ModP>(X3, r, r);
    msub<ModP>(X3, X3, J);
    msub<ModP>(X3, X3, V);
    msub<ModP>(X3, X3, V);
    msub<ModP>(t, V, X3);
    mmul<ModP>(Y3, r, t);
    mmul<ModP>(t, s1, J);
    madd<ModP>(t, t, t);
    msub<ModP>(Y3, Y3, t);
    madd<ModP>(t, a.Z, b.Z);
    mmul<ModP>(Z3, t, t);
    msub<ModP>(Z3, Z3, z1z1);
    msub<ModP>(Z3, Z3, z2z2);
    mmul<ModP>(Z3, Z3, H);
    cpy(o.X, X3);
    cpy(o.Y, Y3);
    cpy(o.Z, Z3);
}

// madd-2007-bl: Jacobian a + affine (x2, y2) (Z2 = 1), with the infinity / doubling cases
__device__ __forceinline__ void pmadd(Pt& o, const Pt& a, const Fe x2, const Fe y2) {
    if (is_zero(a.Z)) {
        cpy(o.X, x2);
        cpy(o.Y, y2);
        cpy(o.Z, kOneP);
        return;
    }
    Fe z1z1, u2, s2, t, H, r;
    mmul<ModP>(z1z1, a.Z, a.Z);
    mmul<ModP>(u2, x2, z1z1);
    mmul<ModP>(t, a.Z, z1z1);
    mmul<ModP>(s2, y2, t);
    msub<ModP>(H, u2, a.X);
    msub<ModP>(r, s2, a.Y);
    if (is_zero(H)) {
        if (is_zero(r)) {
            pdbl(o, a);
        } else {
#pragma unroll
            for (int i = 0; i < 8; i++) o.Z[i] = 0;
        }
        return;
    }
    Fe HH, I, J, V, X3, Y3;
    mmul<ModP>(HH, H, H);
    madd<ModP>(I, HH, HH);
    madd<ModP>(I, I, I);            // 4 HH
    mmul<ModP>(J, H, I);
    madd<ModP>(r, r, r);            // 2 (S2 - Y1)
    mmul<ModP>(V, a.X, I);
    mmul<ModP>(X3, r, r);
    msub<ModP>(X3, X3, J);
    msub<ModP>(X3, X3, V);
    msub<ModP>(X3, X3, V);
    msub<ModP>(t, V, X3);
    mmul<ModP>(Y3, r, t);
    mmul<ModP>(t, a.Y, J);
    madd<ModP>(t, t, t);
    msub<ModP>(Y3, Y3, t);
    madd<ModP>(t, a.Z, H);
    mmul<ModP>(o.Z, t, t);
    msub<ModP>(o.Z, o.Z, z1z1);
    msub<ModP>(o.Z, o.Z, HH);
    cpy(o.X, X3);
    cpy(o.Y, Y3);
}

// a^(M - 2) (Montgomery form in and out), by square-and-multiply over a constant exponent
template <class M>
__device__ __forceinline__ void mpow_m2(Fe r, const Fe a, const uint32_t* e, const uint32_t* one) {
    cpy(r, one);
    for (int b = 255; b >= 0; b--) {
        mmul<M>(r, r, r);
        if ((e[b >> 5] >> (b & 31)) & 1u) mmul<M>(r, r, a);
    }
}

// comb table layout: [key][32 byte positions j][256 digits b][x | y] affine limbs (Montgomery form):
// entry (j, b) = b * 256^j * P; digit 0 unused. 512 KB per key; key nk is the base point G.
constexpr int kCombPos = 32, kCombDig = 256, kEntWords = 16;
constexpr size_t kTabWords = (size_t)kCombPos * kCombDig * kEntWords;

}  // namespace p256

using namespace p256;

// Tables, step 1: one thread per (key, byte position j): P_j = 256^j P (8 j doublings of the key's
// point), Jacobian, into base[key][j]; thread j = 0 also checks the key (0x04 prefix, X, Y < p,
// Y^2 = X^3 - 3X + b) into valid[key]. Key nk is the base point G.
__global__ void __launch_bounds__(64) k_p256_comb_base(int nk, const uint8_t* __restrict__ keys65,
                                                       uint32_t* __restrict__ base, uint8_t* __restrict__ valid) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    const int k = t / kCombPos, j = t % kCombPos;
    if (k > nk) return;
    Fe x, y;
    bool ok = true;
    if (k < nk) {
        const uint8_t* q = keys65 + 65 * (size_t)k;
        ok = q[0] == 0x04;
        load_be(x, q + 1);
        load_be(y, q + 33);
        ok = ok && lt(x, ModP::n) && lt(y, ModP::n);
    } else {
        cpy(x, kGx);
        cpy(y, kGy);
    }
    Pt P;
    mmul<ModP>(P.X, x, kR2P);
    mmul<ModP>(P.Y, y, kR2P);
    cpy(P.Z, kOneP);
    if (ok) {   // on the curve: y^2 == x^3 - 3x + b
        Fe l, r, tt;
        mmul<ModP>(l, P.Y, P.Y);
        mmul<ModP>(tt, P.X, P.X);
        mmul<ModP>(r, tt, P.X);
        msub<ModP>(r, r, P.X);
        msub<ModP>(r, r, P.X);
        msub<ModP>(r, r, P.X);
        madd<ModP>(r, r, kBm);
        ok = eq(l, r);
    }
    if (j == 0) valid[k] = ok ? 1 : 0;
    if (!ok) return;
    for (int d = 0; d < 8 * j; d++) {
        Pt t2;
        pdbl(t2, P);
        P = t2;
    }
    uint32_t* o = base + ((size_t)k * kCombPos + j) * 24;
#pragma unroll
    for (int q = 0; q < 8; q++) {
        o[q] = P.X[q];
        o[8 + q] = P.Y[q];
        o[16 + q] = P.Z[q];
    }
}

// Tables, step 2: one thread per (key, j, digit b in [1, 255]): b P_j by double-and-add over b's
// bits, to affine (Z^-1 by Fermat). A valid key's point has prime order, so no b P_j (b < 256, P_j
// != O) is the point at infinity.
__global__ void __launch_bounds__(64) k_p256_comb_fill(int nk, const uint32_t* __restrict__ base,
                                                       const uint8_t* __restrict__ valid, uint32_t* __restrict__ tab) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int b = 1 + (int)(t % 255);
    const int64_t kj = t / 255;
    const int k = (int)(kj / kCombPos), j = (int)(kj % kCombPos);
    if (k > nk || !valid[k]) return;
    Pt Pj;
    const uint32_t* bp = base + ((size_t)k * kCombPos + j) * 24;
#pragma unroll
    for (int q = 0; q < 8; q++) {
        Pj.X[q] = bp[q];
        Pj.Y[q] = bp[8 + q];
        Pj.Z[q] = bp[16 + q];
    }
    Pt acc = Pj;
    const int top = 31 - __builtin_clz((unsigned)b);
    for (int bit = top - 1; bit >= 0; bit--) {
        Pt t2;
        pdbl(t2, acc);
        acc = t2;
        if ((b >> bit) & 1) {
            padd(t2, acc, Pj);
            acc = t2;
        }
    }
    Fe zi, zi2, tt;
    mpow_m2<ModP>(zi, acc.Z, kPm2, kOneP);
    mmul<ModP>(zi2, zi, zi);
    uint32_t* e = tab + (size_t)k * kTabWords + ((size_t)j * kCombDig + b) * kEntWords;
    mmul<ModP>(tt, acc.X, zi2);
#pragma unroll
    for (int q = 0; q < 8; q++) e[q] = tt[q];
    mmul<ModP>(tt, zi2, zi);
    mmul<ModP>(zi, acc.Y, tt);
#pragma unroll
    for (int q = 0; q < 8; q++) e[8 + q] = zi[q];
}

// byte j of a 256-bit scalar (j uniform: selects, not a dynamically indexed array in scratch)
__device__ __forceinline__ uint32_t byte_at(const Fe u, int j) {
    const int li = j >> 2;
    uint32_t w = u[0];
#pragma unroll
    for (int q = 1; q < 8; q++) w = li == q ? u[q] : w;
    return (w >> (8 * (j & 3))) & 255u;
}

__device__ __forceinline__ void ent_load(Fe x, Fe y, const uint32_t* __restrict__ t) {
    const uint4* t4 = (const uint4*)t;
    const uint4 a = t4[0], b = t4[1], c = t4[2], d = t4[3];
    x[0] = a.x; x[1] = a.y; x[2] = a.z; x[3] = a.w; x[4] = b.x; x[5] = b.y; x[6] = b.z; x[7] = b.w;
    y[0] = c.x; y[1] = c.y; y[2] = c.z; y[3] = c.w; y[4] = d.x; y[5] = d.y; y[6] = d.z; y[7] = d.w;
}

__global__ void __launch_bounds__(128) k_p256_verify(int64_t count, int nk, const int32_t* __restrict__ key_idx,
                                                     const uint8_t* __restrict__ dig,
                                                     const uint8_t* __restrict__ rr, const uint8_t* __restrict__ ss,
                                                     const uint32_t* __restrict__ tab,
                                                     const uint8_t* __restrict__ valid, uint8_t* __restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= count) return;
    const int k = key_idx[i];
    if (k < 0 || k >= nk || !valid[k]) {
        out[i] = 2;
        return;
    }
    Fe r, s, e;
    load_be(r, rr + 32 * i);
    load_be(s, ss + 32 * i);
    load_be(e, dig + 32 * i);
    if (is_zero(r) || is_zero(s) || !lt(r, ModN::n) || !lt(s, ModN::n)) {
        out[i] = 0;
        return;
    }
    if (!lt(e, ModN::n)) {   // e < 2^256 < 2N: one subtraction
        Fe z = {0, 0, 0, 0, 0, 0, 0, 0};
        madd<ModN>(e, e, z);
    }
    // w = s^-1 (Montgomery form), by s^(N-2)
    Fe sm, w, u1, u2;
    mmul<ModN>(sm, s, kR2N);
    mpow_m2<ModN>(w, sm, kNm2, kOneN);
    mmul<ModN>(u1, e, w);   // e s^-1 (plain form)
    mmul<ModN>(u2, r, w);
    // fixed-base combs for G and for the key: u1 G + u2 Q = sum over the 32 byte positions j of
    // T_G[j][u1 byte j] + T_Q[j][u2 byte j], at most 64 mixed additions and no doubling; the next
    // position's two entries are loaded while the current ones are added
    const uint32_t* __restrict__ tg = tab + (size_t)nk * kTabWords;
    const uint32_t* __restrict__ tq = tab + (size_t)k * kTabWords;
    Pt acc;
#pragma unroll
    for (int q = 0; q < 8; q++) { acc.X[q] = 0; acc.Y[q] = 0; acc.Z[q] = 0; }
    Fe gx, gy, qx, qy;
    uint32_t d1 = u1[0] & 255u, d2 = u2[0] & 255u;
    ent_load(gx, gy, tg + (size_t)d1 * kEntWords);
    ent_load(qx, qy, tq + (size_t)d2 * kEntWords);
    for (int j = 0; j < kCombPos; j++) {
        Fe ngx, ngy, nqx, nqy;
        uint32_t n1 = 0, n2 = 0;
        if (j + 1 < kCombPos) {
            n1 = byte_at(u1, j + 1);
            n2 = byte_at(u2, j + 1);
            ent_load(ngx, ngy, tg + ((size_t)(j + 1) * kCombDig + n1) * kEntWords);
            ent_load(nqx, nqy, tq + ((size_t)(j + 1) * kCombDig + n2) * kEntWords);
        }
        if (d1) {
            Pt nx;
            pmadd(nx, acc, gx, gy);
            acc = nx;
        }
        if (d2) {
            Pt nx;
            pmadd(nx, acc, qx, qy);
            acc = nx;
        }
        d1 = n1;
        d2 = n2;
        cpy(gx, ngx); cpy(gy, ngy); cpy(qx, nqx); cpy(qy, nqy);
    }
    if (is_zero(acc.Z)) {
        out[i] = 0;
        return;
    }
    // X == r Z^2, or X == (r + N) Z^2 when r + N < p (x mod N == r, x in [0, p))
    Fe z2, rm, t;
    mmul<ModP>(z2, acc.Z, acc.Z);
    mmul<ModP>(rm, r, kR2P);
    mmul<ModP>(t, rm, z2);
    bool ok = eq(t, acc.X);
    if (!ok) {
        Fe rn;
        uint64_t c = 0;
#pragma unroll
        for (int q = 0; q < 8; q++) {
            c += (uint64_t)r[q] + ModN::n[q];
            rn[q] = (uint32_t)c;
            c >>= 32;
        }
        if (c == 0 && lt(rn, ModP::n)) {
            mmul<ModP>(rm, rn, kR2P);
            mmul<ModP>(t, rm, z2);
            ok = eq(t, acc.X);
        }
    }
    out[i] = ok ? 1 : 0;
}

// the comb tables plus the per-(key, position) base points of step 1 after them
size_t p256_table_bytes(int nk) { return (size_t)(nk + 1) * (kTabWords + (size_t)kCombPos * 24) * 4; }

void launch_p256_tables(hipStream_t s, int nk, const uint8_t* keys65, uint32_t* tab, uint8_t* valid) {
    uint32_t* base = tab + (size_t)(nk + 1) * kTabWords;
    hipLaunchKernelGGL(k_p256_comb_base, dim3(((nk + 1) * kCombPos + 63) / 64), dim3(64), 0, s, nk, keys65, base, valid);
    const int64_t ent = (int64_t)(nk + 1) * kCombPos * 255;
    hipLaunchKernelGGL(k_p256_comb_fill, dim3((unsigned)((ent + 63) / 64)), dim3(64), 0, s, nk, (const uint32_t*)base,
                       (const uint8_t*)valid, tab);
}

void launch_p256_verify(hipStream_t s, int64_t count, int nk, const int32_t* key_idx, const uint8_t* dig,
                        const uint8_t* r, const uint8_t* sg, const uint32_t* tab, const uint8_t* valid, uint8_t* out) {
    if (count <= 0) return;
    hipLaunchKernelGGL(k_p256_verify, dim3((unsigned)((count + 127) / 128)), dim3(128), 0, s, count, nk, key_idx, dig,
                       r, sg, tab, valid, out);
}

}  // namespace hgx

namespace {

void p256_err(hgx_error* err, int32_t code, const char* msg) {
    if (!err) return;
    err->code = code;
    std::snprintf(err->msg, sizeof(err->msg), "%s", msg);
}

bool gfx950(int32_t device) {
    int ndev = 0;
    hipDeviceProp_t prop;
    return hipGetDeviceCount(&ndev) == hipSuccess && device >= 0 && device < ndev &&
           hipGetDeviceProperties(&prop, device) == hipSuccess && std::strncmp(prop.gcnArchName, "gfx950", 6) == 0;
}

// device copies of a batch: the key tables, then verify launches (the last one's results kept)
struct P256Run {
    uint8_t *keys = nullptr, *dig = nullptr, *r = nullptr, *s = nullptr, *valid = nullptr, *out = nullptr;
    int32_t* idx = nullptr;
    uint32_t* tab = nullptr;
    hipStream_t st = nullptr;
    ~P256Run() {
        for (void* q : {(void*)keys, (void*)dig, (void*)r, (void*)s, (void*)valid, (void*)out, (void*)idx, (void*)tab})
            if (q) (void)hipFree(q);
        if (st) (void)hipStreamDestroy(st);
    }
    hipError_t upload(const uint8_t* k65, int32_t nk, const int32_t* ki, const uint8_t* d, const uint8_t* rr,
                      const uint8_t* ss, int64_t count) {
        hipError_t e = hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
        if (e == hipSuccess) e = hipMalloc((void**)&keys, 65 * (size_t)nk + 1);
        if (e == hipSuccess) e = hipMalloc((void**)&idx, 4 * (size_t)count);
        if (e == hipSuccess) e = hipMalloc((void**)&dig, 32 * (size_t)count);
        if (e == hipSuccess) e = hipMalloc((void**)&r, 32 * (size_t)count);
        if (e == hipSuccess) e = hipMalloc((void**)&s, 32 * (size_t)count);
        if (e == hipSuccess) e = hipMalloc((void**)&out, (size_t)count);
        if (e == hipSuccess) e = hipMalloc((void**)&valid, (size_t)nk + 1);
        if (e == hipSuccess) e = hipMalloc((void**)&tab, hgx::p256_table_bytes(nk));
        if (e == hipSuccess && nk) e = hipMemcpyAsync(keys, k65, 65 * (size_t)nk, hipMemcpyHostToDevice, st);
        if (e == hipSuccess) e = hipMemcpyAsync(idx, ki, 4 * (size_t)count, hipMemcpyHostToDevice, st);
        if (e == hipSuccess) e = hipMemcpyAsync(dig, d, 32 * (size_t)count, hipMemcpyHostToDevice, st);
        if (e == hipSuccess) e = hipMemcpyAsync(r, rr, 32 * (size_t)count, hipMemcpyHostToDevice, st);
        if (e == hipSuccess) e = hipMemcpyAsync(s, ss, 32 * (size_t)count, hipMemcpyHostToDevice, st);
        return e;
    }
    hipError_t tables(int32_t nk) {
        hgx::launch_p256_tables(st, nk, keys, tab, valid);
        return hipGetLastError();
    }
    hipError_t verify(int32_t nk, int64_t count) {
        hgx::launch_p256_verify(st, count, nk, idx, dig, r, s, tab, valid, out);
        return hipGetLastError();
    }
};

bool p256_args_ok(const uint8_t* keys65, int32_t n_keys, const int32_t* key_idx, const uint8_t* digest,
                  const uint8_t* r, const uint8_t* s, int64_t count, const uint8_t* out) {
    return n_keys >= 0 && count >= 0 && count <= (int64_t)UINT32_MAX * 128 &&
           (n_keys == 0 || keys65) && (count == 0 || (key_idx && digest && r && s && out));
}

}  // namespace

extern "C" int32_t hgx_p256_verify_batch(int32_t device, const uint8_t* keys65, int32_t n_keys, const int32_t* key_idx,
                                         const uint8_t* digest32, const uint8_t* r32, const uint8_t* s32, int64_t count,
                                         uint8_t* out, hgx_error* err) {
    p256_err(err, HGX_OK, "");
    if (!p256_args_ok(keys65, n_keys, key_idx, digest32, r32, s32, count, out)) {
        p256_err(err, HGX_ERR_INVALID, "hgx_p256_verify_batch: bad arguments");
        return HGX_ERR_INVALID;
    }
    if (count == 0) return HGX_OK;
    if (!gfx950(device)) {
        p256_err(err, HGX_ERR_DEVICE, "no gfx950 (MI355X) HIP device (libhgx has no CPU fallback)");
        return HGX_ERR_DEVICE;
    }
    int prev = 0;
    (void)hipGetDevice(&prev);
    (void)hipSetDevice(device);
    hipError_t e;
    {
        P256Run run;
        e = run.upload(keys65, n_keys, key_idx, digest32, r32, s32, count);
        if (e == hipSuccess) e = run.tables(n_keys);
        if (e == hipSuccess) e = run.verify(n_keys, count);
        if (e == hipSuccess) e = hipMemcpyAsync(out, run.out, (size_t)count, hipMemcpyDeviceToHost, run.st);
        if (e == hipSuccess) e = hipStreamSynchronize(run.st);
    }
    (void)hipSetDevice(prev);
    if (e != hipSuccess) {
        p256_err(err, HGX_ERR_DEVICE, hipGetErrorString(e));
        return HGX_ERR_DEVICE;
    }
    return HGX_OK;
}

extern "C" int32_t hgx_p256_verify_bench(int32_t device, const uint8_t* keys65, int32_t n_keys,
                                         const int32_t* key_idx, const uint8_t* digest32, const uint8_t* r32,
                                         const uint8_t* s32, int64_t count, int32_t warmup, int32_t iters,
                                         uint8_t* out, double* ms_per_launch) {
    if (!p256_args_ok(keys65, n_keys, key_idx, digest32, r32, s32, count, out) || count == 0 || iters <= 0 ||
        warmup < 0 || !ms_per_launch)
        return HGX_ERR_INVALID;
    if (!gfx950(device)) return HGX_ERR_DEVICE;
    int prev = 0;
    (void)hipGetDevice(&prev);
    (void)hipSetDevice(device);
    hipError_t e;
    float ms = 0.f;
    {
        P256Run run;
        hipEvent_t e0 = nullptr, e1 = nullptr;
        e = run.upload(keys65, n_keys, key_idx, digest32, r32, s32, count);
        if (e == hipSuccess) e = hipEventCreate(&e0);
        if (e == hipSuccess) e = hipEventCreate(&e1);
        // the key tables once (a context builds them when its keys are set), then verify launches
        if (e == hipSuccess) e = run.tables(n_keys);
        for (int32_t k = 0; e == hipSuccess && k < warmup; k++) e = run.verify(n_keys, count);
        if (e == hipSuccess) e = hipEventRecord(e0, run.st);
        for (int32_t k = 0; e == hipSuccess && k < iters; k++) e = run.verify(n_keys, count);
        if (e == hipSuccess) e = hipEventRecord(e1, run.st);
        if (e == hipSuccess) e = hipMemcpyAsync(out, run.out, (size_t)count, hipMemcpyDeviceToHost, run.st);
        if (e == hipSuccess) e = hipStreamSynchronize(run.st);
        if (e == hipSuccess) e = hipEventElapsedTime(&ms, e0, e1);
        if (e0) (void)hipEventDestroy(e0);
        if (e1) (void)hipEventDestroy(e1);
    }
    (void)hipSetDevice(prev);
    if (e != hipSuccess) return HGX_ERR_DEVICE;
    *ms_per_launch = (double)ms / iters;
    return HGX_OK;
}
