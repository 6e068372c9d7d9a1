// dc_nybble_abi.cpp -- libdc_nybble.so: the codec entry points of nybble_compression.c
// with the reference's signatures (include/dc_nybble.h), backed by libdc_core.so kernels.
#include <stdint.h>
#include <string.h>

#include "dc_abi_common.h"
#include "dc_nybble.h"

extern "C" {

// nybble_compression.c:887-1038
void compress_bytestring(const char *source_original, char *dest_original, bool modify)
{
    const uint64_t n = strlen(source_original);
    uint64_t len = 0;
    DC_OR_DIE("compress_bytestring",
              dc_nyb_compress_host((const uint8_t *)source_original, n, modify ? 1 : 0, (uint8_t *)dest_original,
                                   n + 2, &len));
    dest_original[len] = '\0';
}

// nybble_compression.c:734-817
void decompress_bytestring(const char *source, char *dest_original, bool modify)
{
    const uint64_t m = strlen(source);
    uint64_t len = 0;
    DC_OR_DIE("decompress_bytestring",
              dc_nyb_decompress_host((const uint8_t *)source, m, modify ? 1 : 0, (uint8_t *)dest_original,
                                     2 * m + 1, &len));
    dest_original[len] = '\0';
}

// nybble_compression.c:1134-1137, :1117-1120
void nybble_compress(const char *source_original, char *dest_original)
{
    compress_bytestring(source_original, dest_original, true);
}

void nybble_decompress(const char *source, char *dest_original)
{
    decompress_bytestring(source, dest_original, true);
}

}  // extern "C"
