/*
 * dc_gpu.h -- device-resident extended API of libdc_core.so (MI355X / gfx950).
 *
 * This is the API the drop-in shims (dc_huffman.h, dc_nybble.h), bench.py and the
 * multi-GPU driver are built on. All pointers named d_* are device pointers (HBM);
 * every call is asynchronous on the context's HIP stream unless it says otherwise.
 * Every function returns 0 (DC_OK) or a negative DC_E_* status; none of them prints.
 *
 * Reference interfaces these stages replace (file:line in carycode/data_compression):
 *   dc_huff_hist          histogram()                          n_ary_huffman.c:461-493
 *   dc_huff_table*        huffman() + convert_lengths_to_encode_table()
 *                                                              n_ary_huffman.c:1161-1208, :1382-1612
 *   dc_huff_plan/pack     represent_items_with_codes() (stub)  n_ary_huffman.c:1621-1678
 *   dc_huff_decode        decompress() data block (missing)     n_ary_huffman.c:2014-2094
 *   dc_nyb_*              compress_bytestring/decompress_bytestring
 *                                                              nybble_compression.c:734-1038
 * The Huffman bitstream layout is build-defined (DESIGN.md "Huffman bitstream v1").
 */
#ifndef DC_GPU_H
#define DC_GPU_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum {
    DC_OK = 0,
    DC_E_ARG = -1,           /* bad argument */
    DC_E_HIP = -2,           /* a HIP runtime call failed (no device, launch failure, ...) */
    DC_E_CODE_TOO_LONG = -3, /* a byte's packed code exceeds 32 bits */
    DC_E_NOCODE = -4,        /* the input holds a byte that has no code */
    DC_E_STATE = -5,         /* stage called out of order (e.g. pack before hist of that input) */
    DC_E_CAPACITY = -6,      /* output buffer too small */
    DC_E_STREAM = -7,        /* corrupt compressed stream */
    DC_E_FALLBACK = -8       /* the fused C5 path does not apply to this input: run the two stages */
};

#define DC_BLOCK_BYTES 32768u   /* encoder block: one histogram + one bit offset each */
#define DC_LUT_BITS 12          /* decoder first-level lookup table: 2^12 entries */
#define DC_MAX_SYMS 1024        /* max_symbol_value + 1 supported by the table kernel */
#define DC_MAX_DIGITS 128       /* longest code length (in base-n digits) handled */
#define DC_LUT2_CAP 7168        /* second-level decode entries (escape prefixes x 2^k) */
#define DC_LUT14_BITS 14        /* the exact redo's first level: 2^14 entries */
#define DC_LUT15_BITS 15        /* the fast decoder's first level: 2^15 entries */
#define DC_SYNC_MAX 1024        /* largest sync granularity (u16 chunk bit lengths) */

typedef struct dc_ctx dc_ctx;

/* Device-resident code table, written by the table kernels (layout is ABI). */
typedef struct dc_dtable {
    uint32_t code[256];             /* packed MSB-first code bits of byte s           */
    uint32_t nbits[256];            /* its bit length (0: byte has no code)           */
    uint32_t lut[1 << DC_LUT_BITS]; /* next 12 bits -> sym0 | bits(all)<<8 | sym1<<16 |
                                       bits(sym0)<<24 | count(1|2)<<29; 0: code > 12 b */
    uint32_t first[DC_MAX_DIGITS + 1]; /* canonical first value per digit length      */
    uint32_t count[DC_MAX_DIGITS + 1];
    uint32_t start[DC_MAX_DIGITS + 1];
    uint64_t lim[33];               /* left-justified limit per bit length (n = 2^w)  */
    uint16_t syms[DC_MAX_SYMS];     /* symbols sorted by (length, value)               */
    int32_t lengths[DC_MAX_SYMS];   /* Huffman lengths in digits (huffman())          */
    int32_t enc_len[DC_MAX_SYMS];   /* convert_lengths_to_encode_table() outputs      */
    uint32_t enc_val[DC_MAX_SYMS];
    int32_t n_ary, w, max_symbol_value, max_bits;
    int32_t min_len, max_len, status, last_written; /* last_written: index M assigned */
    /* decoder tables indexed by the LSB-first window (the stream's bits in order):
     * dlut: next 12 bits -> bits | sym << 8; bits 0: a longer code (or no code), whose
     *       12-bit prefix has escape id sym; dlut2: [id << dlut2_k | next dlut2_k bits] ->
     *       bits | sym << 8, 0: longer than 12 + dlut2_k bits or invalid (dlut2_k 0: none) */
    uint16_t dlut[1 << DC_LUT_BITS];
    uint16_t dlut2[DC_LUT2_CAP];
    int32_t dlut2_k, dec_ready;   /* dec_ready: lut/dlut/dlut2/dlut14/dlut15 are current */
    int32_t fixed8;               /* every byte's code is 8 bits (or absent): pack and decode are byte maps */
    /* fixed8 with the coded bytes one contiguous range: code = byte - fixed8_lo for the
     * fixed8_count bytes fixed8_lo.., so the maps are byte-wise subtractions (flat or random
     * bytes: n = 2 on all 256 values codes every byte as itself) */
    int32_t fixed8_affine, fixed8_lo, fixed8_count;
    /* dlut14: next 14 bits -> bits | sym << 8 for codes of <= 14 bits; bits 0: longer, sym =
     * the escape id of its 12-bit prefix (as dlut); 16-B aligned for vector copies */
    uint16_t dlut14[1 << DC_LUT14_BITS];
    /* dlut15: the same on the next 15 bits (the fast decoder's table) */
    uint16_t dlut15[1 << DC_LUT15_BITS];
} dc_dtable;

/* Node list of the n-ary Huffman tree (generate_huffman_tree's in-out list[],
 * n_ary_huffman.c:868-1005): nodes 0..M leaves, M+1.. the dummy leaves, then the internal
 * nodes in creation order. parent 0 = none (the root, or a leaf of count 0); left/right =
 * an internal node's first two children in pick order (:978-979); count = leaf frequency,
 * 1 for a dummy, the children's sum for an internal node. */
#define DC_TREE_NODES 4096
typedef struct dc_tree {
    int32_t nodes, first_internal, dummies, status;
    int32_t parent[DC_TREE_NODES];
    int32_t left[DC_TREE_NODES];
    int32_t right[DC_TREE_NODES];
    uint64_t count[DC_TREE_NODES];
} dc_tree;

/* ---- context ------------------------------------------------------------------------ */
/* stream: the hipStream_t to launch on (e.g. torch's current stream); NULL is the
 * default (legacy) stream. dc_ctx_create_owned makes a private non-blocking stream.
 * Both fail with DC_E_HIP when no HIP device is usable. */
int dc_ctx_create(dc_ctx **out, int device, void *stream);
int dc_ctx_create_owned(dc_ctx **out, int device);
void dc_ctx_destroy(dc_ctx *ctx);
int dc_ctx_sync(dc_ctx *ctx);
void *dc_ctx_stream(dc_ctx *ctx);
/* Per-stage HIP-event timing (on the stream the kernels run on). enable=1 starts
 * recording; dc_ctx_timings() synchronises and returns up to max stages. */
int dc_ctx_set_timing(dc_ctx *ctx, int enable);
int dc_ctx_timings(dc_ctx *ctx, const char **names, float *ms, int max);
/* Tuning options of a context (defaults suit MI355X; each is also read once from the
 * environment at context creation, for A/B runs: DC_HIST_GRID, DC_PACK_GRID, DC_D8_STATIC,
 * DC_DECODE_V7). Out-of-range values return DC_E_ARG and leave the option unchanged. */
enum {
    DC_OPT_HIST_GRID = 1,         /* histogram workgroups, 0 = default (512)              */
    DC_OPT_PACK_GRID = 2,         /* pack: workgroups (k_huff_pack, k_fe_pack; 0 = a block pair each)
                                     or blocks per wave (k_huff_pack_w; 0 = ~4096 waves) */
    DC_OPT_DECODE_STATIC_PCT = 3, /* fast decoder: statically dealt share of work, 0..100  */
    DC_OPT_DECODE_GENERAL = 4,    /* 1: decode with the general (any-S) decoder            */
    DC_OPT_HIST_PREFETCH = 5,     /* histogram: 32 KiB blocks in flight ahead, 1..2, 0 = 2 */
    DC_OPT_DECODE_VARIANT = 6,    /* fast decoder: 0 one code per lookup (k_huff_decode8),
                                     1 up to 3 codes per lookup (k_huff_decode9) */
    DC_OPT_NYB_ADEC_V1 = 7,       /* adaptive nybble decode: 0 tokens + control words + the
                                     SGPR-list resolve (k_nyb_resolve_c); 1 the one-pass
                                     single-wave k_nyb_adec; 2 tokens + r2's VGPR-list resolve;
                                     3 tokens + the plain-code resolve (k_nyb_resolve_s) (A/B) */
    DC_OPT_PACK_BLOCK = 8,        /* A/B builds only (-DDC_AB_KERNELS): a product build accepts 0
                                     alone. 2: the wave-per-range pack (k_huff_pack_w) instead of
                                     the workgroup-per-block one (k_huff_pack); 3: the same at 4
                                     codes a lane (0.386 vs 0.380 ms on 1 GiB C2); r6 (all slower,
                                     DESIGN.md 'Round 6'): 4 the block by LDS-DMA, 5 half-block
                                     stages, 6 one table read per byte (fold), 7 the next block's
                                     loads issued as pass B frees each piece */
    DC_OPT_NYB_WTILE_OFF = 9      /* 1: the static nybble encode and the nybble decode write each
                                     4096-element tile with a workgroup (k_fsm_write) instead of a
                                     wave (k_nyb_enc_wtile / k_nyb_dec_wtile) */
};
int dc_ctx_set_option(dc_ctx *ctx, int option, int64_t value);
const char *dc_version(void);
size_t dc_dtable_size(void);

/* ---- device memory helpers (plain hipMalloc/hipMemcpy wrappers for ctypes users) --- */
int dc_malloc(void **d_ptr, size_t bytes);
int dc_free(void *d_ptr);
int dc_memcpy_h2d(dc_ctx *ctx, void *d_dst, const void *h_src, size_t bytes);
int dc_memcpy_d2h(dc_ctx *ctx, void *h_dst, const void *d_src, size_t bytes);
int dc_memset(dc_ctx *ctx, void *d_dst, int value, size_t bytes);
/* HBM reference rate: a float4 (16-B) device-to-device copy of `bytes` (multiple of 16,
 * 16-B aligned), nt loads and stores, one uint4 per lane over the full grid (one 256-thread
 * workgroup per 4 KiB; bench.py's copy probe) */
int dc_copy_probe(dc_ctx *ctx, const void *d_src, void *d_dst, uint64_t bytes);

/* ---- Huffman, device-resident stages ------------------------------------------------- */
/* (1) byte histogram of d_in[0..n) -> d_hist[256] (u64). Keeps per-block histograms in
 *     the context for dc_huff_plan on the SAME (d_in, n). */
int dc_huff_hist(dc_ctx *ctx, const uint8_t *d_in, uint64_t n, uint64_t *d_hist);
/* (2a) table from byte histogram d_hist[256]; symbols 256..max_symbol_value count 0. */
int dc_huff_table(dc_ctx *ctx, const uint64_t *d_hist, int max_symbol_value, int n_ary,
                  dc_dtable *d_table);
/* (2b) table from an arbitrary frequency array d_freq[max_symbol_value+1] (u64). */
int dc_huff_table_freq(dc_ctx *ctx, const uint64_t *d_freq, int max_symbol_value, int n_ary,
                       dc_dtable *d_table);
/* (2c) table from given lengths d_lengths[max_symbol_value+1] (skips the merge). */
int dc_huff_table_lengths(dc_ctx *ctx, const int32_t *d_lengths, int max_symbol_value,
                          int n_ary, dc_dtable *d_table);
/* (2d) the table of (2b) plus its whole node list (generate_huffman_tree) into d_tree */
int dc_huff_tree(dc_ctx *ctx, const uint64_t *d_freq, int max_symbol_value, int n_ary, dc_dtable *d_table,
                 dc_tree *d_tree);
/* (2e) summarize_tree_with_lengths' walk for any node list: d_depth[i] (i < leaves) = parent
 *      hops from node i to the root (-1: the walk exceeds the list, a cycle) */
int dc_tree_depths(dc_ctx *ctx, const int32_t *d_parent, int list_length, int leaves, int32_t *d_depth);
/* (3) the encode plan of the input of the last dc_huff_hist under d_table: its payload bit
 *     count into *d_total_bits (device u64) and the missing-code flag (dc_huff_pack_status).
 *     The per-block bit offsets are computed at pack time by two plan kernels before the
 *     pack (k_block_local: bits per 32 KiB block and a scan per 64 blocks; k_block_final_wide:
 *     the absolute offsets, and the zeroing of the payload words two blocks share). */
int dc_huff_plan(dc_ctx *ctx, const dc_dtable *d_table, uint64_t *d_total_bits);
/* (2+3 fused) the table of d_hist (dc_huff_table) and the plan of this context's last
 *     dc_huff_hist under it (dc_huff_plan) in ONE launch: a sharded encode's step after the
 *     all-reduce of the histograms (the table of the global histogram, the bits of the shard). */
int dc_huff_table_plan(dc_ctx *ctx, const uint64_t *d_hist, int max_symbol_value, int n_ary, dc_dtable *d_table,
                       uint64_t *d_total_bits);
/* (1+2+3 fused) histogram, table and plan of d_in[0..n) in ONE launch: the histogram's last
 *     workgroup builds the table (as dc_huff_table) and the plan total (as dc_huff_plan) from
 *     the histogram it holds. The single-stream encoder's path (a sharded encode must reduce
 *     the histograms between the two, so it calls them separately). */
int dc_huff_encode_plan(dc_ctx *ctx, const uint8_t *d_in, uint64_t n, int max_symbol_value, int n_ary,
                        uint64_t *d_hist, dc_dtable *d_table, uint64_t *d_total_bits);
/* (4) pack at global bit offset bit_base into d_words (word 0 = stream word bit_base/32,
 *     MSB-first bytes; 16-B aligned). Capacity: dc_huff_words_needed().
 *     Sync index (DESIGN.md "Sync index v1"), both arrays NULL for none: chunks of
 *     sync_syms symbols (power of two, 16..DC_SYNC_MAX): d_sync_len[c] = bit length of
 *     chunk c (u16, dc_huff_sync_chunks entries); d_sync_base[g] = absolute bit offset of
 *     chunk 64g (u64, dc_huff_sync_groups entries). */
int dc_huff_pack(dc_ctx *ctx, const uint8_t *d_in, uint64_t n, const dc_dtable *d_table,
                 uint64_t bit_base, uint32_t *d_words, uint64_t words_cap,
                 uint64_t *d_sync_base, uint16_t *d_sync_len, uint32_t sync_syms);
uint64_t dc_huff_sync_chunks(uint64_t n, uint32_t sync_syms);
uint64_t dc_huff_sync_groups(uint64_t n, uint32_t sync_syms);
uint64_t dc_huff_words_needed(uint64_t bit_base, uint64_t total_bits);
/* inspection (synchronising): the exclusive per-block bit offsets of the last plan (nblocks+1
 * entries, last = total; recomputed on demand) and the per-block u16 histograms of the last
 * dc_huff_hist */
int dc_huff_plan_offsets(dc_ctx *ctx, uint64_t *h_off, uint64_t max_entries, uint64_t *h_n);
int dc_huff_block_hist(dc_ctx *ctx, uint16_t *h_bh, uint64_t max_entries);
/* (4') the same without any host round trip (graph/timing friendly): a byte without a
 *     code or words_cap too small makes the kernels write nothing; read the outcome with
 *     dc_huff_pack_status() (synchronising). */
int dc_huff_pack_async(dc_ctx *ctx, const uint8_t *d_in, uint64_t n, const dc_dtable *d_table,
                       uint64_t bit_base, uint32_t *d_words, uint64_t words_cap,
                       uint64_t *d_sync_base, uint16_t *d_sync_len, uint32_t sync_syms);
/* ... with the stream's bit offset read by the kernels from device memory (*d_bit_base, a
 * u64 written earlier on the stream, e.g. a shard's exclusive prefix of the ranks' payload
 * bits): a sharded encode then needs no host read of the gathered bit counts. */
int dc_huff_pack_async_dev(dc_ctx *ctx, const uint8_t *d_in, uint64_t n, const dc_dtable *d_table,
                           const uint64_t *d_bit_base, uint32_t *d_words, uint64_t words_cap,
                           uint64_t *d_sync_base, uint16_t *d_sync_len, uint32_t sync_syms);
int dc_huff_pack_status(dc_ctx *ctx, const dc_dtable *d_table);
/* the outcome of one particular plan + pack: gen = dc_huff_plan_gen() read right after its
 * plan (dc_huff_plan / dc_huff_encode_plan), so later encodes on the context do not answer
 * for it. DC_E_STATE when more than 30 plans have run since (its flags are recycled). */
uint32_t dc_huff_plan_gen(dc_ctx *ctx);
int dc_huff_pack_status_gen(dc_ctx *ctx, const dc_dtable *d_table, uint32_t gen);
/* C5 fused front-end encode (small_compression.c:582-665 front-end, then n-ary Huffman of its
 * output M), without M ever written to memory: the stream and sync index are exactly those of
 * dc_small_compress followed by dc_huff_encode_plan + dc_huff_pack_async on M (the same payload
 * bits, the same sync chunks of S symbols of M), from the input bytes d_in (16-B aligned, n >= 2).
 * (1-3) the histogram of M per 32 KiB block of the input, the table and the plan total in one
 *     launch (as dc_huff_encode_plan);
 * (4) two plan launches (block bit offsets, each block's first symbol index, the sync-length
 *     words of chunks spanning block boundaries zeroed) and the pack. d_sync_len (4-B aligned)
 *     and d_sync_base are required, sized for dc_small_huff_symbols() symbols: at most n + 1.
 *     Sizing: the kernels clear and add d_sync_len as whole dwords (two u16 lengths at a time),
 *     so allocate ceil(chunks / 2) * 2 + 2 u16 entries, chunks = ceil((n + 1) / S): with an odd
 *     chunk count the last dword reaches one entry past the last chunk.
 * dc_huff_pack_status then returns DC_E_FALLBACK (nothing usable written) when the front-end
 * output falls back to LITERAL (small_compression.c:655-662), when every byte value occurs in
 * M (the pack marks a pair's start with a byte value that has no code), or when a 32 KiB block
 * codes to more bits than the pack's stage holds beside its sync list; the caller then runs
 * the two stages. dc_small_huff_symbols reads the symbol count of M (synchronising). */
int dc_small_huff_plan(dc_ctx *ctx, const uint8_t *d_in, uint64_t n, int max_symbol_value, int n_ary,
                       uint64_t *d_hist, dc_dtable *d_table, uint64_t *d_total_bits);
int dc_small_huff_pack_async(dc_ctx *ctx, const uint8_t *d_in, uint64_t n, const dc_dtable *d_table,
                             uint64_t bit_base, uint32_t *d_words, uint64_t words_cap,
                             uint64_t *d_sync_base, uint16_t *d_sync_len, uint32_t sync_syms);
int dc_small_huff_symbols(dc_ctx *ctx, uint64_t *h_symbols);
/* The same fused encode for one contiguous shard of the input (dist.ShardedSmall at world > 1;
 * the front-end's only halo is one byte each side). d_shard: 4 x int64 on the
 * device, read by the kernels (no host synchronisation): {global bit of the shard's first code,
 * global index of its first symbol of M, the input byte before the shard (-1: the shard starts the
 * stream: type byte 8, raw first byte), the input byte after it (-1: none)}.
 * dc_small_huff_shard_hist: the shard's histogram of M (no table; the caller all-reduces the
 * shards' histograms and runs dc_huff_table_plan, which also plans this shard's bits).
 * dc_small_huff_shard_pack_async: the shard's codes at that global bit (d_words: word 0 = the
 * stream's word d_shard[0] / 32, the shared first and last words holding only this shard's bits,
 * OR-merged by the gather), its local sync index (chunks of S symbols from its own first symbol:
 * its own decode) and its part of the stream's sync index (d_gsync_len: u16 per global chunk c
 * at entry c - (c0 & ~1), c0 = its first chunk, the first and last entries partial: the gather adds
 * the neighbours' parts; d_gsync_base: the groups that start in the shard, from group
 * ceil(first symbol / 64 S)). Fallbacks as dc_small_huff_pack_async, except the LITERAL test,
 * which belongs to the whole stream (the caller's). Sizes: d_sync_len / d_sync_base as for
 * dc_small_huff_pack_async (n + 1 symbols, u16 lengths rounded up to whole dwords + 2 entries);
 * d_gsync_len / d_gsync_base for n + 1 + 2 S symbols (the shard's chunks counted from c0 & ~1,
 * plus the partial chunks it shares at either end), the lengths rounded the same way. */
int dc_small_huff_shard_hist(dc_ctx *ctx, const uint8_t *d_in, uint64_t n, const int64_t *d_shard,
                             uint64_t *d_hist);
int dc_small_huff_shard_pack_async(dc_ctx *ctx, const uint8_t *d_in, uint64_t n, const dc_dtable *d_table,
                                   const int64_t *d_shard, uint32_t *d_words, uint64_t words_cap,
                                   uint64_t *d_sync_base, uint16_t *d_sync_len, uint64_t *d_gsync_base,
                                   uint16_t *d_gsync_len, uint32_t sync_syms);
/* C5 decode: the Huffman decode of the m-symbol front-end stream M into d_m (16-B aligned,
 * >= m bytes), counting the symbols >= 0x80 of every group of 64 chunks on the way (S = 64), then
 * the front-end inverse (small_compression.c's decompress_bytestring, dc_small_decompress) into
 * d_out (>= 2 m bytes) from those counts, without the inverse's own counting pass over M. *h_len =
 * the decoded length (synchronising). Other sync sizes, a LITERAL stream or an unaligned d_m
 * take the two stages unchanged. */
int dc_small_huff_decode(dc_ctx *ctx, const uint32_t *d_words, uint64_t bit_base, uint64_t words,
                         const uint64_t *d_sync_base, const uint16_t *d_sync_len, uint32_t sync_syms, uint64_t m,
                         const dc_dtable *d_table, uint8_t *d_m, uint8_t *d_out, uint64_t *h_len);
/* Status word written by the table / plan kernels (host-synchronising read). */
int dc_huff_table_status(dc_ctx *ctx, const dc_dtable *d_table, int32_t *max_bits);
/* (5) decode n symbols. d_words/bit_base and the sync index as written by pack. The
 * decoder tables (dc_dtable dlut*) are rebuilt first unless this context's last pack built
 * them for d_table; a table rewritten since by other means (another context, a copy) and
 * not packed or rebuilt through this context is reported by dc_huff_decode_status as
 * DC_E_STREAM (the decoder checks dec_ready), never decoded with stale tables. */
int dc_huff_decode(dc_ctx *ctx, const uint32_t *d_words, uint64_t bit_base, uint64_t words,
                   const uint64_t *d_sync_base, const uint16_t *d_sync_len, uint32_t sync_syms,
                   uint64_t n, const dc_dtable *d_table, uint8_t *d_out);
/* ... with the bit offset in device memory (as dc_huff_pack_async_dev) */
int dc_huff_decode_dev(dc_ctx *ctx, const uint32_t *d_words, const uint64_t *d_bit_base, uint64_t words,
                       const uint64_t *d_sync_base, const uint16_t *d_sync_len, uint32_t sync_syms,
                       uint64_t n, const dc_dtable *d_table, uint8_t *d_out);
/* status of the last dc_huff_decode on this context (synchronising): 0 or DC_E_STREAM */
int dc_huff_decode_status(dc_ctx *ctx);
/* chunks of the last S = 64 dc_huff_decode on this context that took the exact redo (codes
 * longer than the 15-bit table, partial or over-long groups); synchronising, diagnostic */
int dc_huff_decode_redo_count(dc_ctx *ctx, uint64_t *count);
/* base64url text (6 bits per char, MSB-first) of bits [bit_base, bit_base+bits) */
int dc_huff_base64url(dc_ctx *ctx, const uint32_t *d_words, uint64_t bit_base, uint64_t bits,
                      char *d_text);
/* Digit text of bits [bit_base, bit_base+bits) (n_ary_huffman.c:46-78,
 * :371-455, :745-748): one character per b-bit field, MSB-first, the last zero-padded.
 *   DC_TEXT_BASE64URL  b = 6, the int2digit alphabet (:371-378)
 *   DC_TEXT_BASE16     b = 4, "0123456789ABCDEF" (RFC 4648)
 *   DC_TEXT_DIGITS     b = w, one base-n digit per character, "0123456789abcdef" (n <= 16)
 *   DC_TEXT_Z85        b = 8, 4 trits (n = 3) or 2 base-9 digits (n = 9) -> the first 81
 *                      characters of Z85 (:379-407)
 *   DC_TEXT_TRITS5     b = 10, 5 trits (n = 3) -> one byte 1..243 (:745-748)
 * d_words[0] is the word holding bit bit_base (as dc_huff_pack writes a stream).
 * A field with a digit >= n (never produced by the encoder) renders as '~' (byte 0 in
 * TRITS5). dc_huff_text_bits returns b, 0 for an unsupported (format, n). *nchar (host,
 * may be NULL) receives ceil(bits / b). */
enum { DC_TEXT_BASE64URL = 0, DC_TEXT_BASE16 = 1, DC_TEXT_DIGITS = 2, DC_TEXT_Z85 = 3, DC_TEXT_TRITS5 = 4 };
int dc_huff_text_bits(int format, int n_ary);
int dc_huff_text(dc_ctx *ctx, const uint32_t *d_words, uint64_t bit_base, uint64_t bits, int format, int n_ary,
                 char *d_text, uint64_t *nchar);
/* inverse: nchar characters -> the first `bits` bits at bit 0 of d_words (ceil(bits/32)
 * words; bits past `bits` zeroed). base64url also takes '+' '/' (digit2int :443-446),
 * base16 lowercase. An invalid character: dc_huff_text_parse_status (synchronising)
 * returns DC_E_STREAM. */
int dc_huff_text_parse(dc_ctx *ctx, const char *d_text, uint64_t nchar, int format, int n_ary, uint64_t bits,
                       uint32_t *d_words);
int dc_huff_text_parse_status(dc_ctx *ctx);
/* sync granularity (symbols per chunk): a fixed default, and the choice from the
 * planned payload (keeps a 64-chunk group within the decoder's LDS stage) */
uint32_t dc_huff_default_sync(uint64_t n);
uint32_t dc_huff_choose_sync(uint64_t n, uint64_t total_bits);

/* ---- nybble codec (nybble_compression.c), device-resident ---------------------------- */
/* Full reference byte stream (header, packed nybbles, LITERAL fallback) of d_in[0..n).
 * d_out capacity >= n + 2. *h_out_len receives the length (host, synchronising). */
int dc_nyb_compress(dc_ctx *ctx, const uint8_t *d_in, uint64_t n, int modify, uint8_t *d_out,
                    uint64_t *h_out_len);
/* Decode m compressed bytes; d_out capacity >= 2*m. *h_out_len as above. */
int dc_nyb_decompress(dc_ctx *ctx, const uint8_t *d_in, uint64_t m, int modify, uint8_t *d_out,
                      uint64_t *h_out_len);
/* Chunked container "DCNK" (build-defined; SURVEY §8(e)/(f)4: adaptive streams decode in
 * parallel only with independent chunks). Chunk k = bytes [kK, kK+K) stored as the
 * reference's own stream of that chunk (compress_bytestring on it), so each chunk decodes
 * alone. Layout: u32 'DCNK', u32 version 1, u32 modify, u32 K, u64 n, u64 nchunks,
 * u64 off[nchunks+1] (relative to the payload), payload. K >= 16; d_out / d_in 8-B aligned.
 * Decode returns DC_E_STREAM when a chunk does not decode to exactly its length (a corrupt
 * container, or input bytes >= 0x80, which the reference codec does not round-trip). */
uint64_t dc_nyb_chunked_bound(uint64_t n, uint32_t K);
int dc_nyb_compress_chunked(dc_ctx *ctx, const uint8_t *d_in, uint64_t n, int modify, uint32_t K, uint8_t *d_out,
                            uint64_t out_cap, uint64_t *h_out_len);
int dc_nyb_chunked_info(dc_ctx *ctx, const uint8_t *d_in, uint64_t m, uint64_t *h_n, int *h_modify, uint32_t *h_K);
int dc_nyb_decompress_chunked(dc_ctx *ctx, const uint8_t *d_in, uint64_t m, uint8_t *d_out, uint64_t out_cap,
                              uint64_t *h_out_len);
/* Batched decode of many independent reference streams (the throughput path for many
 * separate nybble_decompress / decompress_bytestring calls, beside the DCNK container): stream i
 * = d_in[d_in_off[i] .. d_in_off[i+1]) (device u64 offsets, count+1 entries), each a whole
 * stream as compress_bytestring writes it, decoded as decompress_bytestring(modify) does
 * (nybble_compression.c:734-817; any type byte but 0xAF / ' ' copies the stream). One lane per
 * stream (a single stream's adaptive decode is sequential). d_out_off (device, count+1) receives
 * the output offsets, *h_total the total; DC_E_CAPACITY when it exceeds out_cap (nothing
 * decoded), DC_E_STREAM when a 0xAF stream's walk leaves its bytes inconsistent, DC_E_ARG for an
 * offset range that ends before it starts. Synchronising. */
int dc_nyb_decompress_batch(dc_ctx *ctx, const uint8_t *d_in, const uint64_t *d_in_off, uint64_t count, int modify,
                            uint8_t *d_out, uint64_t out_cap, uint64_t *d_out_off, uint64_t *h_total);
/* Shard bodies (data_compression_amd/dist.py ShardedNybble). A shard buffer is
 * d_in[0 .. len): d_in[0] is the context byte (the stream's first byte on the first shard, the
 * previous shard's last byte after it) and the shard's elements are bytes 1 .. len-1, as in
 * compress_bytestring's loop (nybble_compression.c:908-996).
 * Adaptive (modify) move-to-front lists: 16 contexts x 8 bytes, most recent first.
 *   dc_nyb_mtf_summary: the lists after the shard's elements, started empty (h_cnt[c] valid
 *     entries of list c); summaries compose: lists after A then B = first 8 distinct of
 *     (B's list, A's list) per context.
 *   dc_nyb_body_plan: with the shard's entry lists h_lists (adaptive; ignored when static),
 *     h_plan[0..3] = the shard's transducer (bytes out from state 0, from state 1, exit state
 *     from 0, from 1; state 1 = the previous element's hit nybble is pending) and h_plan[4] =
 *     the rank of the shard's last element (0xFF = miss).
 *   dc_nyb_body_write: the shard's body from the entry state (pend_rank = the pending byte's
 *     rank, or -1), the odd-tail byte when is_last; no header and no LITERAL fallback (decided
 *     over the whole stream). The adaptive ranks come from the preceding dc_nyb_body_plan on
 *     the same d_in/len. d_out capacity >= 2*len. *h_state_out = exit state.
 * Static decode of a shard of the compressed stream after its 2-byte header: m bytes, plus
 * one byte of right halo (the next shard's first byte) when len = m + 1:
 *   dc_nyb_dbody_plan: h_plan[0..3] as above (state 1 = start at the low nybble);
 *   dc_nyb_dbody_write: decoded bytes from entry state s_in; d_out capacity >= 2*m. */
int dc_nyb_mtf_summary(dc_ctx *ctx, const uint8_t *d_in, uint64_t len, uint8_t *h_lists, uint8_t *h_cnt);
int dc_nyb_body_plan(dc_ctx *ctx, const uint8_t *d_in, uint64_t len, int modify, const uint8_t *h_lists,
                     uint64_t *h_plan);
int dc_nyb_body_write(dc_ctx *ctx, const uint8_t *d_in, uint64_t len, int modify, int pend_rank, int is_last,
                      uint8_t *d_out, uint64_t *h_out_len, int *h_state_out);
int dc_nyb_dbody_plan(dc_ctx *ctx, const uint8_t *d_in, uint64_t len, uint64_t m, uint64_t *h_plan);
int dc_nyb_dbody_write(dc_ctx *ctx, const uint8_t *d_in, uint64_t len, uint64_t m, int s_in, uint8_t *d_out,
                       uint64_t *h_out_len, int *h_state_out);

/* ---- small front-end (small_compression.c:507-665), device-resident ----------------- */
int dc_small_compress(dc_ctx *ctx, const uint8_t *d_in, uint64_t n, uint8_t *d_out,
                      uint64_t *h_out_len);
int dc_small_decompress(dc_ctx *ctx, const uint8_t *d_in, uint64_t m, uint8_t *d_out,
                        uint64_t *h_out_len);
/* Shard bodies (data_compression_amd/dist.py ShardedSmall): the front-end
 * output of stream bytes d_in[1 .. nelem] (no header, no LITERAL fallback), reading d_in[0]
 * as left context when left_halo (a shard after the first: d_in[0] = the previous shard's
 * last byte; else d_in[0] is the stream's raw first byte) and d_in[nelem + 1] (when
 * nelem + 1 < len) as the right halo. Pairs never overlap, so the bodies of consecutive
 * shards concatenate to the whole stream's body. d_out capacity >= nelem. */
int dc_small_compress_body(dc_ctx *ctx, const uint8_t *d_in, uint64_t len, int left_halo, uint64_t nelem,
                           uint8_t *d_out, uint64_t *h_out_len);
/* The same in two calls, so the caller can place the output once its size is known (a
 * sharded encoder aligns its re-cut segment, dist.ShardedSmall): _plan returns the body
 * length; _write, on the same input and arguments (DC_E_STATE otherwise), writes it. */
int dc_small_compress_body_plan(dc_ctx *ctx, const uint8_t *d_in, uint64_t len, int left_halo, uint64_t nelem,
                                uint64_t *h_len);
int dc_small_compress_body_write(dc_ctx *ctx, const uint8_t *d_in, uint64_t len, int left_halo, uint64_t nelem,
                                 uint8_t *d_out, uint64_t *h_len);
/* decode of a body (every byte: >= 0x80 -> ' ' + byte - 0x80); d_out capacity >= 2*m */
int dc_small_decompress_body(dc_ctx *ctx, const uint8_t *d_in, uint64_t m, uint8_t *d_out, uint64_t *h_out_len);

#ifdef __cplusplus
}
#endif
#endif
