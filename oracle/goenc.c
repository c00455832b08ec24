/*
 * goenc.c -- TEST INFRASTRUCTURE (oracle side). See goenc.h for the reference
 * citations. Plain C99, no dependencies.
 */
#include "goenc.h"

#include <stdio.h>
#include <string.h>

/* ---------------- SHA-256 (FIPS 180-4) ---------------- */
static const uint32_t K256[64] = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
    0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
    0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
    0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
    0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
    0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
    0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
    0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};

#define ROR(x, n) (((x) >> (n)) | ((x) << (32 - (n))))

static void sha256_block(uint32_t h[8], const uint8_t* p) {
    uint32_t w[64];
    for (int i = 0; i < 16; i++)
        w[i] = ((uint32_t)p[4 * i] << 24) | ((uint32_t)p[4 * i + 1] << 16) |
               ((uint32_t)p[4 * i + 2] << 8) | (uint32_t)p[4 * i + 3];
    for (int i = 16; i < 64; i++) {
        uint32_t s0 = ROR(w[i - 15], 7) ^ ROR(w[i - 15], 18) ^ (w[i - 15] >> 3);
        uint32_t s1 = ROR(w[i - 2], 17) ^ ROR(w[i - 2], 19) ^ (w[i - 2] >> 10);
        w[i] = w[i - 16] + s0 + w[i - 7] + s1;
    }
    uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
    for (int i = 0; i < 64; i++) {
        uint32_t S1 = ROR(e, 6) ^ ROR(e, 11) ^ ROR(e, 25);
        uint32_t ch = (e & f) ^ (~e & g);
        uint32_t t1 = hh + S1 + ch + K256[i] + w[i];
        uint32_t S0 = ROR(a, 2) ^ ROR(a, 13) ^ ROR(a, 22);
        uint32_t mj = (a & b) ^ (a & c) ^ (b & c);
        uint32_t t2 = S0 + mj;
        hh = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
    }
    h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e; h[5] += f; h[6] += g; h[7] += hh;
}

void goenc_sha256(const uint8_t* data, size_t len, uint8_t out[32]) {
    uint32_t h[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a,
                     0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
    size_t full = len / 64;
    for (size_t i = 0; i < full; i++) sha256_block(h, data + 64 * i);
    uint8_t tail[128];
    size_t rem = len - 64 * full;
    memset(tail, 0, sizeof(tail));
    if (rem) memcpy(tail, data + 64 * full, rem);
    tail[rem] = 0x80;
    size_t tl = (rem + 9 <= 64) ? 64 : 128;
    uint64_t bits = (uint64_t)len * 8u;
    for (int i = 0; i < 8; i++) tail[tl - 1 - i] = (uint8_t)(bits >> (8 * i));
    sha256_block(h, tail);
    if (tl == 128) sha256_block(h, tail + 64);
    for (int i = 0; i < 8; i++) {
        out[4 * i] = (uint8_t)(h[i] >> 24);
        out[4 * i + 1] = (uint8_t)(h[i] >> 16);
        out[4 * i + 2] = (uint8_t)(h[i] >> 8);
        out[4 * i + 3] = (uint8_t)h[i];
    }
}

/* ---------------- base64 / hex / decimal ---------------- */
static const char B64[] = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789+/";

size_t goenc_base64(const uint8_t* in, size_t len, char* out) {
    size_t o = 0, i = 0;
    for (; i + 3 <= len; i += 3) {
        uint32_t v = ((uint32_t)in[i] << 16) | ((uint32_t)in[i + 1] << 8) | in[i + 2];
        out[o++] = B64[(v >> 18) & 63]; out[o++] = B64[(v >> 12) & 63];
        out[o++] = B64[(v >> 6) & 63];  out[o++] = B64[v & 63];
    }
    if (len - i == 1) {
        uint32_t v = (uint32_t)in[i] << 16;
        out[o++] = B64[(v >> 18) & 63]; out[o++] = B64[(v >> 12) & 63];
        out[o++] = '='; out[o++] = '=';
    } else if (len - i == 2) {
        uint32_t v = ((uint32_t)in[i] << 16) | ((uint32_t)in[i + 1] << 8);
        out[o++] = B64[(v >> 18) & 63]; out[o++] = B64[(v >> 12) & 63];
        out[o++] = B64[(v >> 6) & 63];  out[o++] = '=';
    }
    return o;
}

void goenc_hex_id(const uint8_t* in, size_t len, char* out) {
    static const char HX[] = "0123456789ABCDEF";
    out[0] = '0'; out[1] = 'x';
    for (size_t i = 0; i < len; i++) {
        out[2 + 2 * i] = HX[in[i] >> 4];
        out[3 + 2 * i] = HX[in[i] & 15];
    }
    out[2 + 2 * len] = 0;
}

size_t goenc_decimal(const uint8_t* be, size_t len, char* out) {
    uint8_t num[64];
    char rev[160];
    size_t nr = 0;
    if (len > sizeof(num)) len = sizeof(num);
    memcpy(num, be, len);
    for (;;) {
        int zero = 1;
        for (size_t i = 0; i < len; i++) if (num[i]) { zero = 0; break; }
        if (zero) break;
        uint32_t rem = 0;
        for (size_t i = 0; i < len; i++) {
            uint32_t cur = (rem << 8) | num[i];
            num[i] = (uint8_t)(cur / 10);
            rem = cur % 10;
        }
        rev[nr++] = (char)('0' + rem);
    }
    if (nr == 0) rev[nr++] = '0';
    for (size_t i = 0; i < nr; i++) out[i] = rev[nr - 1 - i];
    return nr;
}

/* ---------------- time.Time MarshalJSON (RFC3339Nano, UTC) ---------------- */
static void civil_from_days(int64_t z, int64_t* y, unsigned* m, unsigned* d) {
    z += 719468;
    const int64_t era = (z >= 0 ? z : z - 146096) / 146097;
    const unsigned doe = (unsigned)(z - era * 146097);
    const unsigned yoe = (doe - doe / 1460 + doe / 36524 - doe / 146096) / 365;
    const int64_t yy = (int64_t)yoe + era * 400;
    const unsigned doy = doe - (365 * yoe + yoe / 4 - yoe / 100);
    const unsigned mp = (5 * doy + 2) / 153;
    *d = doy - (153 * mp + 2) / 5 + 1;
    *m = mp < 10 ? mp + 3 : mp - 9;
    *y = yy + (*m <= 2);
}

size_t goenc_rfc3339nano(int64_t unix_ns, char* out) {
    int64_t secs = unix_ns / 1000000000LL;
    int64_t nsec = unix_ns % 1000000000LL;
    if (nsec < 0) { nsec += 1000000000LL; secs -= 1; }
    int64_t days = secs / 86400, sod = secs % 86400;
    if (sod < 0) { sod += 86400; days -= 1; }
    int64_t y; unsigned mo, d;
    civil_from_days(days, &y, &mo, &d);
    int n = sprintf(out, "%04lld-%02u-%02uT%02d:%02d:%02d", (long long)y, mo, d,
                    (int)(sod / 3600), (int)((sod / 60) % 60), (int)(sod % 60));
    if (nsec) {
        char frac[10];
        sprintf(frac, "%09lld", (long long)nsec);
        int l = 9;
        while (l > 0 && frac[l - 1] == '0') l--;
        out[n++] = '.';
        memcpy(out + n, frac, (size_t)l);
        n += l;
    }
    out[n++] = 'Z';
    out[n] = 0;
    return (size_t)n;
}

/* ---------------- JSON bodies ---------------- */
static size_t put(char* out, size_t o, const char* s) {
    size_t l = strlen(s);
    memcpy(out + o, s, l);
    return o + l;
}

static size_t put_txs(char* out, size_t o, int ntx, const uint8_t* const* tx,
                      const size_t* tx_len, int tx_nil) {
    if (tx_nil) return put(out, o, "null");
    out[o++] = '[';
    for (int i = 0; i < ntx; i++) {
        if (i) out[o++] = ',';
        out[o++] = '"';
        o += goenc_base64(tx[i], tx_len[i], out + o);
        out[o++] = '"';
    }
    out[o++] = ']';
    return o;
}

static size_t txs_bound(int ntx, const size_t* tx_len) {
    size_t b = 8;
    for (int i = 0; i < ntx; i++) b += 4 * (tx_len[i] / 3 + 1) + 3;
    return b;
}

size_t goenc_event_json_bound(int ntx, const size_t* tx_len, size_t creator_len) {
    return 512 + txs_bound(ntx, tx_len) + 4 * (creator_len / 3 + 1) + 2 * 200;
}

size_t goenc_event_json(int ntx, const uint8_t* const* tx, const size_t* tx_len, int tx_nil,
                        const char* sp_hex, const char* op_hex,
                        const uint8_t* creator, size_t creator_len,
                        int64_t ts_ns, int64_t index,
                        const uint8_t r_be[32], const uint8_t s_be[32], char* out) {
    char num[64];
    size_t o = 0;
    o = put(out, o, "{\"Body\":{\"Transactions\":");
    o = put_txs(out, o, ntx, tx, tx_len, tx_nil);
    o = put(out, o, ",\"Parents\":[\"");
    o = put(out, o, sp_hex);
    o = put(out, o, "\",\"");
    o = put(out, o, op_hex);
    o = put(out, o, "\"],\"Creator\":\"");
    o += goenc_base64(creator, creator_len, out + o);
    o = put(out, o, "\",\"Timestamp\":\"");
    o += goenc_rfc3339nano(ts_ns, out + o);
    o = put(out, o, "\",\"Index\":");
    sprintf(num, "%lld", (long long)index);
    o = put(out, o, num);
    o = put(out, o, "},\"R\":");
    o += goenc_decimal(r_be, 32, out + o);
    o = put(out, o, ",\"S\":");
    o += goenc_decimal(s_be, 32, out + o);
    o = put(out, o, "}\n");
    return o;
}

size_t goenc_block_json_bound(int ntx, const size_t* tx_len) {
    return 64 + txs_bound(ntx, tx_len);
}

size_t goenc_block_json(int64_t round_received, int ntx, const uint8_t* const* tx,
                        const size_t* tx_len, int tx_nil, char* out) {
    char num[32];
    size_t o = 0;
    o = put(out, o, "{\"RoundReceived\":");
    sprintf(num, "%lld", (long long)round_received);
    o = put(out, o, num);
    o = put(out, o, ",\"Transactions\":");
    o = put_txs(out, o, ntx, tx, tx_len, tx_nil);
    o = put(out, o, "}\n");
    return o;
}
