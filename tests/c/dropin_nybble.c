/* A C caller of the nybble drop-in (nybble_compression.c:734, :887, :1117, :1134), in
 * the style of the reference's round-trip test (:1150-1215). Links only libdc_nybble.so.
 * Exit status 0 = every check passed. */
#include <stdbool.h>
#include <stdio.h>
#include <string.h>
#include "dc_nybble.h"

#define CHECK(c) do { if (!(c)) { fprintf(stderr, "FAIL %s:%d %s\n", __FILE__, __LINE__, #c); return 1; } } while (0)

int main(void)
{
    static const char text[] =
        "Hello, world. This is a test. This is only a test. Banana banana banana banana. ";
    const int len = (int)strlen(text);
    char comp[2 * sizeof text + 8], back[4 * sizeof text + 8];

    for (int modify = 0; modify <= 1; ++modify) {
        compress_bytestring(text, comp, modify);
        const int m = (int)strlen(comp);
        CHECK(m > 0 && m <= len + 1);
        decompress_bytestring(comp, back, modify);
        CHECK(strcmp(back, text) == 0);
    }
    compress_bytestring(text, comp, false);
    CHECK(strlen(comp) == 57);                 /* SURVEY.md Appendix B */
    CHECK((unsigned char)comp[0] == 0xAF);
    nybble_compress(text, comp);
    nybble_decompress(comp, back);
    CHECK(strcmp(back, text) == 0);
    printf("dropin_nybble ok\n");
    return 0;
}
