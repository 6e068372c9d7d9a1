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

void compress_bytestring(const char *source_original, char *dest_original, bool modify);
void decompress_bytestring(const char *source, char *dest_original, bool modify);
void nybble_compress(const char *source_original, char *dest_original);
void nybble_decompress(const char *source, char *dest_original);

#ifdef __cplusplus
}
#endif
#endif
