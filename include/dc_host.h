/*
 * dc_host.h -- host-buffer convenience layer of libdc_core.so.
 *
 * Each call uploads its input to HBM, runs the device-resident stages of dc_gpu.h on a
 * per-thread context (device: $DC_DEVICE, default 0) and copies the result back. Used by
 * the drop-in shims (dc_huffman.h, dc_nybble.h, dc_small.h) and by the parity tests.
 * Host code only moves bytes and assembles headers; no compute falls back to the CPU:
 * without a usable HIP device every call returns DC_E_HIP.
 */
#ifndef DC_HOST_H
#define DC_HOST_H
#include <stdint.h>
#include "dc_gpu.h"

#ifdef __cplusplus
extern "C" {
#endif

dc_ctx *dc_host_ctx(void);
/* copy n host bytes into the per-thread 16-B aligned input buffer (device) */
int dc_host_upload(const void *h, uint64_t n, const uint8_t **d_out);
/* per-thread device scratch buffers: which = 0 out, 1 sync, 2 table, 3 hist, 4 lengths, 5 aux */
int dc_host_scratch(int which, uint64_t bytes, void **d_out);

/* ---- "DCH1" Huffman container (DESIGN.md "Container v1") -------------------------------
 * [0]  "DCH1"  [4] u8 version=1, u8 n_ary, u8 w (bits per digit), u8 flags=0
 * [8]  u64 n symbols   [16] u64 payload bits   [24] u32 sync_syms, u32 0
 * [32] u8 code length (digits) of byte 0..255
 * [288] sync index (dc_gpu.h): u64 group bases (dc_huff_sync_groups entries), then
 *       u16 chunk bit lengths (dc_huff_sync_chunks entries)
 * then the MSB-first payload, ceil(bits/8) bytes, zero-padded.
 * lengths == NULL: lengths from the input's own histogram (n_ary_huffman.c:2509-2530 flow),
 * else from lengths[0..max_symbol_value] (the caller's huffman() output).
 * sync_syms == 0: dc_huff_default_sync(n). */
uint64_t dc_huff_compress_bound(uint64_t n, uint32_t sync_syms);
int dc_huff_compress_host(const uint8_t *in, uint64_t n, int n_ary, const int32_t *lengths,
                          int max_symbol_value, uint32_t sync_syms, uint8_t *out, uint64_t cap,
                          uint64_t *out_len);
/* reads either container: "DCH1" by its magic, anything else as netstrings */
int dc_huff_decompress_host(const uint8_t *in, uint64_t m, uint8_t *out, uint64_t cap,
                            uint64_t *out_len);
int dc_huff_container_info(const uint8_t *in, uint64_t m, uint64_t *n, int *n_ary, uint64_t *bits);

/* ---- netstring container: the reference's block format (n_ary_huffman.c:1866-1943) -----
 * A sequence of netstrings "<len>:<payload>," (payload <= 32768 bytes, :1826-1827) whose
 * payload starts with a 2-byte type (:1915-1920). Written:
 *   raw    "<k+2>:\n\n<k bytes>,"   the reference compress()'s pass-through block
 *                                   (:1806-1814), byte-identical for inputs < 32767 B;
 *                                   longer inputs: consecutive blocks of <= 32766 bytes
 *   #dc1   "\n#dc1 n=<n_ary> syms=<N> bits=<payload bits> S=<sync_syms> M=<max symbol>"
 *   X      "\nX<M>:" + one character per symbol 0..M, its code length in digits
 *          ("0".."9" as the reference's "%d" (:1736-1741), then "A".."Z" for 10..35)
 *   #dcidx "\n#dcidx:" + base64url (int2digit alphabet) of the sync index bytes (dc_gpu.h:
 *          u64 group bases then u16 chunk bit lengths, little-endian), split over blocks
 *   Z      "\nZ" + base64url of the bitstream v1 (6 bits per character, MSB-first, the
 *          last character zero-padded), split over consecutive Z blocks
 * The Huffman form is written only when it is smaller than the raw form (which bounds the
 * output: dc_huff_netstring_bound). A reader skips unknown "#" blocks (:2077-2080), so the
 * reference's decompress() sees the index blocks as metadata. Decompression accepts any
 * sequence of raw blocks and Huffman segments (#dc1, X, #dcidx..., Z...), whitespace between
 * blocks, and "%i" lengths (:1825); the output is the concatenation of the segments. */
uint64_t dc_huff_netstring_bound(uint64_t n);
int dc_huff_compress_netstring(const uint8_t *in, uint64_t n, int n_ary, const int32_t *lengths,
                               int max_symbol_value, uint32_t sync_syms, uint8_t *out, uint64_t cap,
                               uint64_t *out_len);
int dc_huff_decompress_netstring(const uint8_t *in, uint64_t m, uint8_t *out, uint64_t cap,
                                 uint64_t *out_len);
/* decompressed size of a netstring container (walks the block headers on the host) */
int dc_huff_netstring_info(const uint8_t *in, uint64_t m, uint64_t *out_n);

/* ---- nybble / small byte codecs on explicit-length host buffers -------------------------- */
int dc_nyb_compress_host(const uint8_t *in, uint64_t n, int modify, uint8_t *out, uint64_t cap,
                         uint64_t *len);
int dc_nyb_decompress_host(const uint8_t *in, uint64_t m, int modify, uint8_t *out,
                           uint64_t cap, uint64_t *len);
int dc_small_compress_host(const uint8_t *in, uint64_t n, uint8_t *out, uint64_t cap,
                           uint64_t *len);
int dc_small_decompress_host(const uint8_t *in, uint64_t m, uint8_t *out, uint64_t cap,
                             uint64_t *len);

#ifdef __cplusplus
}
#endif
#endif
