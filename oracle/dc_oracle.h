/*
 * oracle/dc_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * Clean-room scalar CPU restatement of the reference's hot path
 * (carycode/data_compression @ 2025-08-08). It is the *checker*: tests/, the
 * smoke() entry point and bench.py's cpu_baseline leg may call it; the product
 * (data_compression_amd/, libdc_*.so) never links or calls it.
 *
 * Parity pinning: tests/test_oracle.py checks every function here against the
 * golden vectors in tests/golden/, which tests/golden/gen_golden.py produced by
 * calling the reference C itself (oracle/_ref, compiled from /root/reference).
 * The Huffman *bitstream* (orc_huff_pack / orc_huff_unpack) has no reference
 * counterpart (n_ary_huffman.c:1661 is assert(0), :2081-2089 unimplemented):
 * its layout is build-defined (DESIGN.md "Huffman bitstream v1") and is pinned by
 * the reference-pinned code tables plus round trip -- "parity unpinned" for the
 * layout itself.
 */
#ifndef DC_ORACLE_H
#define DC_ORACLE_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- symbol statistics: n_ary_huffman.c:461-493 ---------------------------------- */
void orc_histogram_bytes(const uint8_t *x, uint64_t n, uint64_t h[256]);
/* NUL-terminated form; returns strlen(text). Bins above max_symbol_value are ignored. */
uint64_t orc_histogram_cstr(const char *text, int max_symbol_value, int *h);

/* ---- code lengths: n_ary_huffman.c:773-1208 --------------------------------------- */
/* n-ary Huffman with the reference's dummy-leaf rule (:900-903) and merge order
 * (smallest (count, node_index) first). lengths[0..max_leaf_value]. Returns the max
 * length. Counts are u64 (the reference's are int: identical results while the
 * total stays <= INT_MAX). */
int orc_huffman_lengths(int max_leaf_value, const uint64_t *freq, int n_ary, int *lengths);

/* ---- canonical n-ary codes: n_ary_huffman.c:1382-1612 ------------------------------ */
/* Writes enc_len/enc_val exactly like the reference, including leaving index
 * max_symbol_value untouched unless its length lies in [min,max] of the others. */
void orc_canonical(int max_symbol_value, const int *lengths, int n_ary,
                   int *enc_len, unsigned *enc_val);

/* ---- build-defined bitstream (DESIGN.md "Huffman bitstream v1") ------------------- */
int orc_digit_bits(int n_ary);                         /* w = ceil(log2 n) */
/* Per-byte packed codes. Returns max code bits, -1 if a code exceeds 32 bits. */
int orc_bitcodes(const int *enc_len, const unsigned *enc_val, int n_ary,
                 uint32_t code[256], uint8_t nbits[256]);
/* Pack x into MSB-first bits starting at bit `bit_base % 8` of out[0] (out must be
 * zeroed). Writes idx[c] = bit_base + bit offset of symbol c*sync_syms when idx != NULL.
 * Returns total payload bits, or UINT64_MAX if a byte has no code. */
uint64_t orc_huff_pack(const uint8_t *x, uint64_t n, const uint32_t code[256],
                       const uint8_t nbits[256], uint8_t *out, uint64_t bit_base,
                       uint32_t sync_syms, uint64_t *idx);
/* Sequential canonical decode (digit-by-digit, base-n). Returns 0 or -1 on a bad stream. */
int orc_huff_unpack(const uint8_t *in, uint64_t in_bits, uint64_t n_out,
                    int max_symbol_value, const int *enc_len, const unsigned *enc_val,
                    int n_ary, uint8_t *out);
/* base64url text of the first `bits` bits (6 per char, MSB-first, last zero-padded). */
uint64_t orc_base64url(const uint8_t *in, uint64_t bits, char *out);

/* Digit text of a bit range (intent n_ary_huffman.c:46-78, :371-455,
 * :745-753). format: 0 base64url (6 bits/char, int2digit :371-378), 1 base16 (4 bits,
 * RFC 4648 "0-9A-F"), 2 one base-n digit per char (w bits, "0-9a-f", n <= 16), 3 Z85
 * pairs (8 bits = 4 trits (n=3) or 2 base-9 digits (n=9) -> the first 81 Z85 characters,
 * :389-407), 4 five trits per byte (n=3, 10 bits -> byte 1..243, :745-748). The last
 * character's missing bits are zero. Returns the characters written, 0 on a bad format. */
uint64_t orc_text(const uint8_t *in, uint64_t bits, int format, int n_ary, char *out);
/* inverse: text -> the first `bits` bits (out zeroed by the callee, ceil(bits/8) bytes);
 * base64url also takes '+' '/' (digit2int :443-446), base16 lowercase. 0, or -1 on an
 * invalid character or a text shorter than `bits` needs. */
int orc_text_parse(const char *text, uint64_t nchar, int format, int n_ary, uint8_t *out, uint64_t bits);

/* ---- nybble codec: nybble_compression.c:517-1137 ----------------------------------- */
/* Length-based restatement of compress_bytestring(:887-1038) / decompress_bytestring
 * (:734-817). Output excludes the trailing NUL. out capacity >= n+1. */
uint64_t orc_nybble_compress(const uint8_t *x, uint64_t n, uint8_t *out, int modify);
uint64_t orc_nybble_decompress(const uint8_t *in, uint64_t m, uint8_t *out, int modify);

/* ---- small front-end: small_compression.c:507-665 ---------------------------------- */
uint64_t orc_small_compress(const uint8_t *x, uint64_t n, uint8_t *out);
/* build-defined inverse (the reference decoder, :453-505, is broken beyond ~100 B) */
uint64_t orc_small_decompress(const uint8_t *in, uint64_t m, uint8_t *out);

#ifdef __cplusplus
}
#endif
#endif
