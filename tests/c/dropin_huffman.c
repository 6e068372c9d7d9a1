/* A C caller of the Huffman drop-in, written the way the reference's own driver uses
 * these functions (n_ary_huffman.c:2509-2530): histogram -> huffman ->
 * convert_lengths_to_encode_table -> represent_items_with_codes, then the container
 * round trip that replaces the static compress/decompress (:1688, :2014), and the tree
 * helpers (setup_nodes :773, generate_huffman_tree :868, summarize_tree_with_lengths
 * :1033, find_compressed_data_size :2466) on a caller-owned struct node list.
 * Links only libdc_huffman.so. Exit status 0 = every check passed. */
#include <stdbool.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include "dc_huffman.h"

#define MAXSYM 258
#define CHECK(c) do { if (!(c)) { fprintf(stderr, "FAIL %s:%d %s\n", __FILE__, __LINE__, #c); return 1; } } while (0)

static int canonical_kats(void)
{
    /* trinary known answers of the reference's test_convert_lengths_to_encode_table
     * (n_ary_huffman.c:2821-2891): lengths in, canonical values out */
    static const int len_a[21] = {0, 0, 1, 1, 1};
    static const unsigned val_a[21] = {0, 0, 0, 1, 2};
    static const int len_b[21] = {0, 0, 2, 2, 2, 2, 2, 2, 2, 2};
    static const unsigned val_b[21] = {0, 0, 0, 1, 2, 3, 4, 5, 6, 7};
    static const int len_c[21] = {0, 0, 2, 2, 2, 2, 2, 2, 2, 2, 2};
    static const unsigned val_c[21] = {0, 0, 0, 1, 2, 3, 4, 5, 6, 7, 8};
    const int *lens[3] = {len_a, len_b, len_c};
    const unsigned *vals[3] = {val_a, val_b, val_c};
    for (int k = 0; k < 3; ++k) {
        int L[21], el[21] = {0};
        unsigned ev[21] = {0};
        memcpy(L, lens[k], sizeof L);
        convert_lengths_to_encode_table(20, L, 3, el, ev);
        for (int i = 0; i < 20; ++i) {   /* index 20 = max: the reference's clear loop skips it */
            CHECK(el[i] == lens[k][i]);
            CHECK(ev[i] == vals[k][i]);
        }
    }
    return 0;
}

/* the reference's own summarize_tree_with_lengths test trees (:1112-1154), then the
 * caller-side tree path setup_nodes -> generate_huffman_tree -> summarize_tree_with_lengths,
 * which must give huffman()'s lengths (huffman() is that composition, :1161-1208) */
static int tree_helpers(const int h[])
{
    struct node list_a[6] = {{true, 9, 0, 0, 'a', 2, 0}, {true, 9, 0, 0, 'b', 2, 0}, {false, 4, 0, 1, 0, 0, 0}};
    int la['z' + 1];
    summarize_tree_with_lengths(6, list_a, 'z', la, 2);
    CHECK(la['a'] == 1 && la['b'] == 1 && la['c'] == 0);
    struct node list_b[5] = {{true, 9, 0, 0, 'a', 4, 0}, {true, 9, 0, 0, 'b', 3, 0}, {true, 8, 0, 0, 'c', 3, 0},
                             {false, 17, 1, 2, 0, 4, 0}, {false, 26, 0, 3, 0, 0, 0}};
    int lb['z' + 1];
    summarize_tree_with_lengths(5, list_b, 'z', lb, 3);
    CHECK(lb['a'] == 1 && lb['b'] == 2 && lb['c'] == 2);
    CHECK(sizeof(struct node) == 28);
    static struct node list[2 * MAXSYM];
    for (int n = 2; n <= 16; n += 7) {   /* n = 2, 9, 16 */
        int want[MAXSYM + 1], got[MAXSYM + 1];
        huffman(MAXSYM, h, n, want);
        setup_nodes(2 * MAXSYM, list, MAXSYM, h);
        CHECK(list[65].leaf && list[65].leaf_value == 65 && list[65].count == h[65] && !list[MAXSYM + 1].leaf);
        generate_huffman_tree(2 * MAXSYM, list, n, MAXSYM);
        summarize_tree_with_lengths(2 * MAXSYM, list, MAXSYM, got, MAXSYM + 1);
        int root = -1, bits = 0;
        for (int i = 0; i <= MAXSYM; ++i) {
            CHECK(got[i] == want[i]);
            bits += want[i] * h[i];
        }
        for (int i = 0; i < 2 * MAXSYM; ++i)
            if (list[i].count && !list[i].parent_index) { CHECK(root < 0); root = i; }
        CHECK(root > MAXSYM && list[root].count >= (int)strlen("Hello"));   /* one root: the last internal node */
        CHECK(find_compressed_data_size(MAXSYM, (int *)h, want, n) == bits);
    }
    return 0;
}

int main(void)
{
    static const char text[] =
        "Hello, world. This is a test. This is only a test. Banana banana banana banana. "
        "It was the best of times, it was the worst of times, it was the age of wisdom.";
    const int len = (int)strlen(text);
    int h[MAXSYM + 1], lengths[MAXSYM + 1], el[MAXSYM + 1];
    unsigned ev[MAXSYM + 1];

    if (canonical_kats()) return 1;

    histogram(text, MAXSYM, h);
    int total = 0;
    for (int i = 0; i <= MAXSYM; ++i) total += h[i];
    CHECK(total == len);
    CHECK(h['a'] > 0 && h['z'] == 0);
    if (tree_helpers(h)) return 1;

    for (int n = 2; n <= 16; n += (n < 4 ? 1 : 6)) {   /* n = 2, 3, 4, 10, 16 */
        huffman(MAXSYM, h, n, lengths);
        convert_lengths_to_encode_table(MAXSYM, lengths, n, el, ev);
        /* Kraft equality over the used symbols (+ the reference's dummy leaves) */
        double kraft = 0;
        for (int i = 0; i < MAXSYM; ++i) {
            CHECK((h[i] > 0) == (lengths[i] > 0) || (i > 255));
            if (h[i] > 0) {
                double p = 1;
                for (int d = 0; d < lengths[i]; ++d) p /= n;
                kraft += p;
            }
        }
        CHECK(kraft <= 1.0 + 1e-12);

        /* base64url text of the bitstream */
        const int bufsize = 4 * len + 64;
        char *txt = malloc(len + 1), *out = malloc(bufsize + 1);
        memcpy(txt, text, len + 1);
        memset(out, '#', bufsize + 1);
        const int w = represent_items_with_codes(MAXSYM, lengths, n, bufsize, len, txt, 3, out);
        CHECK(w > 0 && w <= bufsize - 3);
        for (int i = 0; i < w; ++i) {
            const char c = out[3 + i];
            CHECK((c >= 'A' && c <= 'Z') || (c >= 'a' && c <= 'z') || (c >= '0' && c <= '9') || c == '-' || c == '_');
        }
        CHECK(out[0] == '#' && out[1] == '#' && out[2] == '#');

        /* container round trip (the static compress/decompress replacements) */
        const int cap = 1 << 16;
        char *comp = malloc(cap), *back = malloc(len + 16);
        const int m = dc_huff_compress(MAXSYM, lengths, n, cap, len, txt, comp);
        CHECK(m > 0);
        const int got = dc_huff_decompress(m, comp, len + 16, back);
        CHECK(got == len);
        CHECK(memcmp(back, text, len) == 0);
        free(txt); free(out); free(comp); free(back);
    }
    printf("dropin_huffman ok\n");
    return 0;
}
