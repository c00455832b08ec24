/*
 * goenc.h -- TEST INFRASTRUCTURE (oracle side). Not part of the product path.
 *
 * Byte-exact restatement of the Go encodings the reference hashes:
 *   - crypto.SHA256                       (reference crypto/utils.go:11-16)
 *   - json.NewEncoder(&b).Encode(&Event)  (reference hashgraph/event.go:155-162,171-188)
 *   - json.NewEncoder(&b).Encode(&Block)  (reference hashgraph/block.go:26-61)
 * Go encoding/json rules used: exported fields in
 * declaration order, []byte -> std base64 with padding, nil slice -> null,
 * time.Time -> RFC3339Nano ("Z" for UTC, trailing fractional zeros trimmed),
 * big.Int (addressable value field) -> bare decimal, trailing "\n" from Encode.
 * The hash/JSON format is "parity unpinned": no reference test pins a hash value.
 */
#ifndef HG_GOENC_H
#define HG_GOENC_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

void goenc_sha256(const uint8_t* data, size_t len, uint8_t out[32]);
/* std base64 with padding; returns chars written (no NUL) */
size_t goenc_base64(const uint8_t* in, size_t len, char* out);
/* "0x" + uppercase hex (Go fmt "0x%X"); writes 2+2*len chars + NUL */
void goenc_hex_id(const uint8_t* in, size_t len, char* out);
/* big-endian unsigned magnitude -> decimal string (Go big.Int.String for x>=0) */
size_t goenc_decimal(const uint8_t* be, size_t len, char* out);
/* Unix ns -> RFC3339Nano in UTC */
size_t goenc_rfc3339nano(int64_t unix_ns, char* out);

/* Event JSON (json.Encoder output, with trailing '\n').
 * txs: ntx payloads (ptr,len); tx_nil => "Transactions":null.
 * sp_hex / op_hex: parent ids as strings ("" for none). creator: raw pubkey bytes.
 * r_be / s_be: 32-byte big-endian signature components.
 * Returns bytes written into out (caller sizes buffer; see goenc_event_json_bound). */
size_t goenc_event_json_bound(int ntx, const size_t* tx_len, size_t creator_len);
size_t goenc_event_json(int ntx, const uint8_t* const* tx, const size_t* tx_len, int tx_nil,
                        const char* sp_hex, const char* op_hex,
                        const uint8_t* creator, size_t creator_len,
                        int64_t ts_ns, int64_t index,
                        const uint8_t r_be[32], const uint8_t s_be[32], char* out);

/* Block JSON {"RoundReceived":N,"Transactions":...}\n ; tx_nil => null */
size_t goenc_block_json_bound(int ntx, const size_t* tx_len);
size_t goenc_block_json(int64_t round_received, int ntx, const uint8_t* const* tx,
                        const size_t* tx_len, int tx_nil, char* out);

#ifdef __cplusplus
}
#endif
#endif
