/*
 * TEST INFRASTRUCTURE (oracle): ECDSA P-256 known answers from the container's libcrypto
 * (OpenSSL 3.0.2), the checker for libhgx's batched verify (hgx_p256.hip).
 *
 * The reference verifies every event with Event.Verify (hashgraph/event.go:142-152):
 * crypto.ToECDSAPub(Body.Creator) (crypto/utils.go:22-28, elliptic.Unmarshal of the 65-byte
 * uncompressed point), the SHA-256 of the body (EventBody.Hash, event.go:56-62) and
 * crypto.Verify (crypto/utils.go:41-43) = Go's ecdsa.Verify on P-256: r, s in [1, N-1],
 * e = the 32-byte digest as a big-endian integer, x(u1*G + u2*Q) mod N == r. OpenSSL's
 * ECDSA_do_verify implements the same algorithm (FIPS 186-4), so its answers pin the kernel.
 *
 *   p256_ref gen  <file>   write vectors: one per line, hex fields
 *                          "pub65 digest32 r32 s32 expected key_ok tag"
 *                          expected = 1 valid / 0 invalid; key_ok = 0 when the public key is
 *                          not a P-256 point (Go's elliptic.Unmarshal returns nil)
 *   p256_ref check <file>  re-verify every line with libcrypto; exit 0 iff all agree
 *   p256_ref sign <n_keys> <in> <out>  test signatures (derived keys) for a batch of digests
 *
 * Build: gcc -O2 -o oracle/_ref/p256_ref oracle/p256_ref.c -lcrypto  (oracle/Makefile)
 */
#define OPENSSL_SUPPRESS_DEPRECATED
#include <openssl/bn.h>
#include <openssl/ec.h>
#include <openssl/ecdsa.h>
#include <openssl/obj_mac.h>
#include <openssl/sha.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static uint64_t rng = 0x9E3779B97F4A7C15ull;
static uint32_t next32(void) {
    rng ^= rng << 13;
    rng ^= rng >> 7;
    rng ^= rng << 17;
    return (uint32_t)(rng >> 16);
}

static void hexout(FILE* f, const uint8_t* b, int n) {
    for (int i = 0; i < n; i++) fprintf(f, "%02x", b[i]);
}

static int hexin(const char* s, uint8_t* b, int n) {
    for (int i = 0; i < n; i++) {
        unsigned v;
        if (sscanf(s + 2 * i, "%2x", &v) != 1) return -1;
        b[i] = (uint8_t)v;
    }
    return 0;
}

/* 1 valid, 0 invalid; *key_ok = 0 when pub65 is not a curve point */
static int verify(const EC_GROUP* grp, const uint8_t pub[65], const uint8_t dg[32], const uint8_t r[32],
                  const uint8_t s[32], int* key_ok) {
    EC_KEY* k = EC_KEY_new_by_curve_name(NID_X9_62_prime256v1);
    EC_POINT* q = EC_POINT_new(grp);
    *key_ok = EC_POINT_oct2point(grp, q, pub, 65, NULL) == 1 && EC_POINT_is_on_curve(grp, q, NULL) == 1 &&
              EC_KEY_set_public_key(k, q) == 1;
    int ok = 0;
    if (*key_ok) {
        ECDSA_SIG* sig = ECDSA_SIG_new();
        ECDSA_SIG_set0(sig, BN_bin2bn(r, 32, NULL), BN_bin2bn(s, 32, NULL));
        ok = ECDSA_do_verify(dg, 32, sig, k) == 1;
        ECDSA_SIG_free(sig);
    }
    EC_POINT_free(q);
    EC_KEY_free(k);
    return ok;
}

static void put_bn(const BIGNUM* x, uint8_t out[32]) { BN_bn2binpad(x, out, 32); }

static void emit(FILE* f, const EC_GROUP* grp, const uint8_t pub[65], const uint8_t dg[32], const uint8_t r[32],
                 const uint8_t s[32], const char* tag) {
    int key_ok = 0;
    const int ok = verify(grp, pub, dg, r, s, &key_ok);
    hexout(f, pub, 65);
    fputc(' ', f);
    hexout(f, dg, 32);
    fputc(' ', f);
    hexout(f, r, 32);
    fputc(' ', f);
    hexout(f, s, 32);
    fprintf(f, " %d %d %s\n", ok, key_ok, tag);
}

static int gen(const char* path) {
    FILE* f = fopen(path, "w");
    if (!f) return 1;
    const EC_GROUP* grp = EC_GROUP_new_by_curve_name(NID_X9_62_prime256v1);
    const BIGNUM* N = EC_GROUP_get0_order(grp);
    enum { KEYS = 6, PER_KEY = 24 };
    uint8_t pubs[KEYS][65];
    EC_KEY* keys[KEYS];
    for (int k = 0; k < KEYS; k++) {
        keys[k] = EC_KEY_new_by_curve_name(NID_X9_62_prime256v1);
        EC_KEY_generate_key(keys[k]);
        EC_POINT_point2oct(grp, EC_KEY_get0_public_key(keys[k]), POINT_CONVERSION_UNCOMPRESSED, pubs[k], 65, NULL);
    }
    uint8_t nb[32], np1[32];
    put_bn(N, nb);
    BIGNUM* t = BN_dup(N);
    BN_add_word(t, 1);
    put_bn(t, np1);
    for (int k = 0; k < KEYS; k++) {
        for (int i = 0; i < PER_KEY; i++) {
            uint8_t msg[64], dg[32], r[32], s[32];
            for (int b = 0; b < 64; b++) msg[b] = (uint8_t)next32();
            SHA256(msg, sizeof msg, dg);
            if (i == 0) memset(dg, 0, 32);          /* e = 0: u1*G is the point at infinity */
            if (i == 1) memcpy(dg, nb, 32);         /* e = N: e mod N = 0 */
            if (i == 2) memset(dg, 0xFF, 32);       /* e > N */
            ECDSA_SIG* sig = ECDSA_do_sign(dg, 32, keys[k]);
            const BIGNUM *br, *bs;
            ECDSA_SIG_get0(sig, &br, &bs);
            put_bn(br, r);
            put_bn(bs, s);
            emit(f, grp, pubs[k], dg, r, s, i < 3 ? "edge-digest" : "valid");
            /* corruptions of the same signature */
            uint8_t x[32];
            const int bit = (int)(next32() % 256);
            memcpy(x, dg, 32); x[bit / 8] ^= (uint8_t)(1u << (bit % 8));
            emit(f, grp, pubs[k], x, r, s, "digest-bit");
            memcpy(x, r, 32); x[bit / 8] ^= (uint8_t)(1u << (bit % 8));
            emit(f, grp, pubs[k], dg, x, s, "r-bit");
            memcpy(x, s, 32); x[bit / 8] ^= (uint8_t)(1u << (bit % 8));
            emit(f, grp, pubs[k], dg, r, x, "s-bit");
            emit(f, grp, pubs[(k + 1) % KEYS], dg, r, s, "other-key");
            if (i % 4 == 0) {   /* (r, N - s) is also a valid signature */
                BIGNUM* ns = BN_new();
                BN_sub(ns, N, bs);
                put_bn(ns, x);
                emit(f, grp, pubs[k], dg, r, x, "malleated-s");
                BN_free(ns);
            }
            if (i == 5) {
                uint8_t z[32] = {0};
                emit(f, grp, pubs[k], dg, z, s, "r-zero");
                emit(f, grp, pubs[k], dg, r, z, "s-zero");
                emit(f, grp, pubs[k], dg, nb, s, "r-eq-N");
                emit(f, grp, pubs[k], dg, r, nb, "s-eq-N");
                emit(f, grp, pubs[k], dg, np1, s, "r-gt-N");
                memset(x, 0xFF, 32);
                emit(f, grp, pubs[k], dg, r, x, "s-max");
            }
            if (i == 6) {   /* public keys that are not curve points */
                uint8_t bad[65];
                memcpy(bad, pubs[k], 65);
                bad[64] ^= 1;
                emit(f, grp, bad, dg, r, s, "key-off-curve");
                memcpy(bad, pubs[k], 65);
                memset(bad + 1, 0xFF, 32);
                emit(f, grp, bad, dg, r, s, "key-x-ge-p");
                memcpy(bad, pubs[k], 65);
                bad[0] = 0x05;
                emit(f, grp, bad, dg, r, s, "key-bad-prefix");
            }
            ECDSA_SIG_free(sig);
        }
    }
    BN_free(t);
    for (int k = 0; k < KEYS; k++) EC_KEY_free(keys[k]);
    fclose(f);
    return 0;
}

static int check(const char* path) {
    FILE* f = fopen(path, "r");
    if (!f) return 1;
    const EC_GROUP* grp = EC_GROUP_new_by_curve_name(NID_X9_62_prime256v1);
    char pub[140], dg[70], r[70], s[70], tag[64];
    int exp, kok, lines = 0, bad = 0;
    while (fscanf(f, "%139s %69s %69s %69s %d %d %63s", pub, dg, r, s, &exp, &kok, tag) == 7) {
        uint8_t P[65], D[32], Rb[32], Sb[32];
        if (hexin(pub, P, 65) || hexin(dg, D, 32) || hexin(r, Rb, 32) || hexin(s, Sb, 32)) return 2;
        int key_ok = 0;
        const int ok = verify(grp, P, D, Rb, Sb, &key_ok);
        if (ok != exp || key_ok != kok) {
            bad++;
            fprintf(stderr, "line %d (%s): libcrypto %d/%d, file %d/%d\n", lines + 1, tag, ok, key_ok, exp, kok);
        }
        lines++;
    }
    fclose(f);
    printf("%d vectors, %d disagree\n", lines, bad);
    return (bad || lines == 0) ? 1 : 0;
}

/* sign <n_keys> <in> <out>: test signatures for libhgx's verified insert (tests/).
 * Keys are derived, not random: private key k = SHA-256("hgx test key" | k) mod N.
 * in = records {u32 key, u8 digest[32]}; out = n_keys public keys (65 B each), then per
 * record R and S (32 B big-endian each) from ECDSA_do_sign (random nonces). */
static int sign_file(int nk, const char* in, const char* out) {
    FILE* fi = fopen(in, "rb");
    FILE* fo = fopen(out, "wb");
    if (!fi || !fo || nk <= 0) return 1;
    const EC_GROUP* grp = EC_GROUP_new_by_curve_name(NID_X9_62_prime256v1);
    const BIGNUM* N = EC_GROUP_get0_order(grp);
    EC_KEY** keys = (EC_KEY**)calloc((size_t)nk, sizeof(EC_KEY*));
    BN_CTX* ctx = BN_CTX_new();
    for (int k = 0; k < nk; k++) {
        uint8_t seed[16 + 4], h[32], pub[65];
        memcpy(seed, "hgx test key \0\0\0", 16);
        memcpy(seed + 16, &k, 4);
        SHA256(seed, sizeof seed, h);
        BIGNUM* d = BN_bin2bn(h, 32, NULL);
        BN_mod(d, d, N, ctx);
        if (BN_is_zero(d)) BN_one(d);
        keys[k] = EC_KEY_new_by_curve_name(NID_X9_62_prime256v1);
        EC_POINT* Q = EC_POINT_new(grp);
        EC_POINT_mul(grp, Q, d, NULL, NULL, ctx);
        EC_KEY_set_private_key(keys[k], d);
        EC_KEY_set_public_key(keys[k], Q);
        EC_POINT_point2oct(grp, Q, POINT_CONVERSION_UNCOMPRESSED, pub, 65, NULL);
        fwrite(pub, 1, 65, fo);
        EC_POINT_free(Q);
        BN_free(d);
    }
    uint32_t key;
    uint8_t dg[32], r[32], sg[32];
    int rc = 0;
    while (fread(&key, 4, 1, fi) == 1 && fread(dg, 1, 32, fi) == 32) {
        if ((int)key >= nk) { rc = 2; break; }
        ECDSA_SIG* sig = ECDSA_do_sign(dg, 32, keys[key]);
        const BIGNUM *br, *bs;
        ECDSA_SIG_get0(sig, &br, &bs);
        put_bn(br, r);
        put_bn(bs, sg);
        fwrite(r, 1, 32, fo);
        fwrite(sg, 1, 32, fo);
        ECDSA_SIG_free(sig);
    }
    for (int k = 0; k < nk; k++) EC_KEY_free(keys[k]);
    free(keys);
    BN_CTX_free(ctx);
    fclose(fi);
    fclose(fo);
    return rc;
}

int main(int argc, char** argv) {
    if (argc == 5 && !strcmp(argv[1], "sign")) return sign_file(atoi(argv[2]), argv[3], argv[4]);
    if (argc == 3 && !strcmp(argv[1], "gen")) return gen(argv[2]);
    if (argc == 3 && !strcmp(argv[1], "check")) return check(argv[2]);
    fprintf(stderr, "usage: p256_ref gen|check <file>\n");
    return 2;
}
