/*
 * dc_nybble.h -- drop-in replacement for the codec entry points of nybble_compression.c
 * (carycode/data_compression @ 2025-08-08), exported by libdc_nybble.so under the
 * reference's names. Output bytes are identical to the reference's (pinned by
 * tests/golden/nybble.npz, generated from the reference itself).
 *
 * Reference interface replaced                         | reference file:line
 * ---------------------------------------------------- | ---------------------------
 * compress_bytestring(source, dest, modify)            | nybble_compression.c:887-1038
 * decompress_bytestring(source, dest, modify)          | nybble_compression.c:734-817
 * nybble_compress(source, dest)      (= modify true)   | nybble_compression.c:1134-1137
 * nybble_decompress(source, dest)    (= modify true)   | nybble_compression.c:1117-1120
 * context_table_type                                   | nybble_compression.c:540-544
 * byte_to_context / context_to_byte                    | nybble_compression.c:517-527
 * initialize_dictionary                                | nybble_compression.c:546-562
 * decompress_nybble                                    | nybble_compression.c:643-663
 * update_context                                       | nybble_compression.c:665-687
 * compress_byte_index                                  | nybble_compression.c:819-884
 *
 * The per-element helpers update ONE byte of a caller-owned host table per call (the
 * reference's loops call them per byte); they run on the host, where that table lives.
 * Their results equal the reference's (tests/golden/helpers.npz). The stream functions
 * above are the GPU path.
 *
 * C-string contract as in the reference: the input ends at its first NUL, the output is
 * NUL-terminated; dest capacity >= strlen(source)+2 (compress) / 2*strlen(source)+1
 * (decompress). No diagnostics are printed (the reference prints per byte). An empty
 * input (the reference reads past its terminator) compresses to " ".
 * libdc_nybble.so and libdc_small.so both export compress_bytestring, as the reference's
 * two programs do: link one of them, never both.
 */
#ifndef DC_NYBBLE_H
#define DC_NYBBLE_H
#include <stdbool.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DC_NYB_LETTERS 8    /* letters_per_context (:515) */
#define DC_NYB_CONTEXTS 16  /* num_contexts (:516) */

/* the reference's layout exactly (:540-544): 128 chars then 16 ints, 192 bytes */
typedef struct context_table_type {
    char letter[DC_NYB_CONTEXTS][DC_NYB_LETTERS];
    int times_used_directly[DC_NYB_CONTEXTS];
} context_table_type;

int byte_to_context(char byte);
char context_to_byte(int context);
void initialize_dictionary(context_table_type *context_table);
int decompress_nybble(context_table_type context_table, const char nybble, const char next_nybble, char *dest);
int update_context(context_table_type *context_table, const char context_byte, const char output_byte);
int compress_byte_index(context_table_type *context_table, int nybble_offset, const char *source, char *dest);

void compress_bytestring(const char *source_original, char *dest_original, bool modify);
/* Adaptive mode (modify true, and nybble_decompress below) is sequential by definition: each
 * byte's move-to-front list depends on every byte decoded before it, and the next byte's
 * context on the value a hit names, so ONE adaptive stream has no parallel decode. On the GPU
 * its token structure is found in parallel, then one wave settles the list touches (~21 MB/s,
 * slower than one host core running the reference, ~120 MB/s). The throughput
 * path for adaptive data is many independent streams: the DCNK chunk container
 * (dc_nyb_compress_chunked / dc_nyb_decompress_chunked) or dc_nyb_decompress_batch (one lane
 * per stream, dc_gpu.h). Static mode (modify false) decodes every byte independently. */
void decompress_bytestring(const char *source, char *dest_original, bool modify);
void nybble_compress(const char *source_original, char *dest_original);
void nybble_decompress(const char *source, char *dest_original);   /* adaptive: see above */

#ifdef __cplusplus
}
#endif
#endif
