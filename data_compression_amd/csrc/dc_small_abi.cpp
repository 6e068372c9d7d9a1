// dc_small_abi.cpp -- libdc_small.so: the byte front-end of small_compression.c with the
// reference's signatures (include/dc_small.h), backed by libdc_core.so kernels.
#include <stdint.h>
#include <string.h>

#include "dc_abi_common.h"
#include "dc_small.h"

extern "C" {

// small_compression.c:582-665
void compress_bytestring(const char *source_original, char *dest_original)
{
    const uint64_t n = strlen(source_original);
    uint64_t len = 0;
    DC_OR_DIE("compress_bytestring",
              dc_small_compress_host((const uint8_t *)source_original, n, (uint8_t *)dest_original, n + 2, &len));
    dest_original[len] = '\0';
}

// small_compression.c:453-505 (exact inverse of the encoder above)
void decompress_bytestring(const char *source, char *dest_original)
{
    const uint64_t m = strlen(source);
    uint64_t len = 0;
    DC_OR_DIE("decompress_bytestring",
              dc_small_decompress_host((const uint8_t *)source, m, (uint8_t *)dest_original, 2 * m + 1, &len));
    dest_original[len] = '\0';
}

}  // extern "C"
