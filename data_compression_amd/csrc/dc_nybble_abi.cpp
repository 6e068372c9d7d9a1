// dc_nybble_abi.cpp -- libdc_nybble.so: the codec entry points of nybble_compression.c
// with the reference's signatures (include/dc_nybble.h), backed by libdc_core.so kernels,
// and the reference's per-element helpers (context_table_type and its five functions).
// The helpers act on ONE byte of a caller-owned host struct per call (the reference's
// stream loops call them per byte, :909-999, :754-796): they are state updates of the
// caller's table, run where the table lives; every stream function runs on the GPU.
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

// ---- per-element helpers (nybble_compression.c:517-562, :643-687, :819-884) ----------------
// The move-to-front list of a context: letter[ctx][0] most recent. A byte's context is bits
// 3..6 of the byte before it.
int byte_to_context(char byte)   // :517-523
{
    return ((unsigned char)byte >> 3) & (DC_NYB_CONTEXTS - 1);
}

char context_to_byte(int context)   // :524-527
{
    return (char)(context << 3);
}

void initialize_dictionary(context_table_type *context_table)   // :546-562
{
    static const char kInit[DC_NYB_LETTERS + 1] = " etaoins";
    for (int c = 0; c < DC_NYB_CONTEXTS; ++c) {
        memcpy(context_table->letter[c], kInit, DC_NYB_LETTERS);
        context_table->times_used_directly[c] = 0;
    }
}

// decode one byte at dest[0] (dest[-1] = the byte before it): a nybble with its high bit
// set names letter (nybble & 7) of the context; otherwise it is the high half of a literal
// byte whose low half is next_nybble. Returns the nybbles consumed.   :643-663
int decompress_nybble(context_table_type context_table, const char nybble, const char next_nybble, char *dest)
{
    const int ctx = byte_to_context(dest[-1]);
    if (nybble & 0x08) {
        dest[0] = context_table.letter[ctx][nybble & 0x07];
        return 1;
    }
    dest[0] = (char)(((nybble & 0x07) << 4) + next_nybble);
    return 2;
}

// move output_byte to the front of the list of context_byte's context (a byte not in the
// list enters at the front and the last one drops out)   :665-687
int update_context(context_table_type *context_table, const char context_byte, const char output_byte)
{
    const int ctx = byte_to_context(context_byte);
    char *L = context_table->letter[ctx];
    int pos = 0;
    while (pos < DC_NYB_LETTERS - 1 && L[pos] != output_byte) ++pos;   // its slot, or the last one
    memmove(L + 1, L, (size_t)pos);
    L[0] = output_byte;
    context_table->times_used_directly[ctx]++;
    return 0;
}

// code source[0] (source[-1] = the byte before it) into dest at nybble_offset (0: the high
// nybble of dest[0], 1: its low nybble). In the list: one nybble 1iii, returns 1. Not in
// the list: a literal byte, byte-aligned: at offset 0 dest[0] = the byte (returns 2); at
// offset 1 the pending high nybble is rewritten as the literal source[-1] and the byte
// follows it (dest[0..1], returns 3).   :819-884
int compress_byte_index(context_table_type *context_table, int nybble_offset, const char *source, char *dest)
{
    const int ctx = byte_to_context(source[-1]);
    const char s = source[0];
    const char *L = context_table->letter[ctx];
    int i = 0;
    while (i < DC_NYB_LETTERS && L[i] != s) ++i;
    if (i == DC_NYB_LETTERS) {
        if (nybble_offset == 0) {
            dest[0] = s;
            return 2;
        }
        dest[0] = source[-1];
        dest[1] = s;
        return 3;
    }
    const int nyb = i | 0x8;
    if (nybble_offset == 0) dest[0] = (char)(nyb << 4);
    else dest[0] = (char)(dest[0] | nyb);
    return 1;
}

}  // extern "C"
