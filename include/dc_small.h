/*
 * dc_small.h -- drop-in replacement for the byte front-end of small_compression.c
 * (carycode/data_compression @ 2025-08-08), exported by libdc_small.so.
 *
 * Reference interface replaced                         | reference file:line
 * ---------------------------------------------------- | ---------------------------
 * compress_bytestring(source, dest)                    | small_compression.c:582-665
 * decompress_bytestring(source, dest)                  | small_compression.c:453-505
 *
 * compress_bytestring output is byte-identical to the reference (tests/golden/small.npz).
 * decompress_bytestring is the exact inverse of that encoder (type 8: byte >= 0x80 ->
 * ' ' + (byte - 0x80)); the reference decoder is out of sync with its encoder beyond
 * ~100 bytes, so it is not reproduced. Type ' ' copies, other types give "".
 */
#ifndef DC_SMALL_H
#define DC_SMALL_H

#ifdef __cplusplus
extern "C" {
#endif

void compress_bytestring(const char *source_original, char *dest_original);
void decompress_bytestring(const char *source, char *dest_original);

#ifdef __cplusplus
}
#endif
#endif
