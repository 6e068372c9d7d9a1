/* A C caller of the nybble drop-in (nybble_compression.c:734, :887, :1117, :1134), in
 * the style of the reference's round-trip test (:1150-1215), plus a caller-side codec
 * loop built only from the exported per-element helpers (context_table_type,
 * initialize_dictionary, compress_byte_index, update_context, decompress_nybble,
 * byte_to_context; :517-687, :819-884) whose stream must equal the GPU stream functions'.
 * Links only libdc_nybble.so. Exit status 0 = every check passed. */
#include <stdbool.h>
#include <stdio.h>
#include <string.h>
#include "dc_nybble.h"

#define CHECK(c) do { if (!(c)) { fprintf(stderr, "FAIL %s:%d %s\n", __FILE__, __LINE__, #c); return 1; } } while (0)

/* nybble stream of src by the helpers: type byte 0xAF, the first byte raw, then per byte
 * 1 nybble (in the list), a literal byte, or 3 nybbles (pending nybble rewritten); odd tail */
static size_t helper_encode(const char *src, char *out, bool modify)
{
    context_table_type t;
    initialize_dictionary(&t);
    size_t o = 0;
    out[o++] = (char)0xAF;
    out[o++] = src[0];
    int half = 0;                               /* 1: a nybble waits in out[o]'s high half */
    for (const char *s = src + 1; *s; ++s) {
        const int k = compress_byte_index(&t, half, s, out + o);
        if (modify) update_context(&t, s[-1], s[0]);
        half += k;
        while (half >= 2) { ++o; half -= 2; }
    }
    if (half) out[o++] = src[strlen(src) - 1];  /* the last byte, as a whole literal */
    return o;
}

static size_t helper_decode(const unsigned char *in, size_t m, char *out, bool modify)
{
    context_table_type t;
    initialize_dictionary(&t);
    size_t o = 0, i = 2;
    out[o++] = (char)in[1];
    int half = 0;
    while (i < m) {
        const int hi = half ? (in[i] & 15) : (in[i] >> 4);
        const int lo = half ? (i + 1 < m ? in[i + 1] >> 4 : 0) : (in[i] & 15);
        const int k = decompress_nybble(t, (char)hi, (char)lo, out + o);
        if (modify) update_context(&t, out[o - 1], out[o]);
        ++o;
        half += k;
        while (half >= 2) { ++i; half -= 2; }
    }
    out[o] = 0;
    return o;
}

int main(void)
{
    static const char text[] =
        "Hello, world. This is a test. This is only a test. Banana banana banana banana. ";
    const int len = (int)strlen(text);
    char comp[2 * sizeof text + 8], back[4 * sizeof text + 8], mine[2 * sizeof text + 8];

    for (int modify = 0; modify <= 1; ++modify) {
        compress_bytestring(text, comp, modify);
        const int m = (int)strlen(comp);
        CHECK(m > 0 && m <= len + 1);
        decompress_bytestring(comp, back, modify);
        CHECK(strcmp(back, text) == 0);
        /* the helpers' loop gives the same 57 bytes, and decodes them back */
        const size_t hm = helper_encode(text, mine, modify);
        CHECK(hm == (size_t)m && memcmp(mine, comp, hm) == 0);
        CHECK(helper_decode((const unsigned char *)comp, (size_t)m, back, modify) == (size_t)len);
        CHECK(strcmp(back, text) == 0);
    }
    compress_bytestring(text, comp, false);
    CHECK(strlen(comp) == 57);                 /* SURVEY.md Appendix B */
    CHECK((unsigned char)comp[0] == 0xAF);
    nybble_compress(text, comp);
    nybble_decompress(comp, back);
    CHECK(strcmp(back, text) == 0);
    CHECK(byte_to_context('h') == 13 && byte_to_context(' ') == 4 && byte_to_context((char)0xC3) == 8);
    CHECK(context_to_byte(13) == 'h' - ('h' & 7));
    CHECK(sizeof(context_table_type) == 192);
    printf("dropin_nybble ok\n");
    return 0;
}
