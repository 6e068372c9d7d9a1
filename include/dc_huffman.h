/*
 * dc_huffman.h -- drop-in replacement for the public functions of n_ary_huffman.c
 * (carycode/data_compression @ 2025-08-08), exported by libdc_huffman.so with the
 * reference's own names, argument meanings and array conventions. All compute runs in
 * gfx950 HIP kernels (libdc_core.so); see INTEGRATION.md for the one-line link change.
 *
 * Reference interface replaced                         | reference file:line
 * ---------------------------------------------------- | ---------------------------
 * histogram                                            | n_ary_huffman.c:461-493
 * huffman                                              | n_ary_huffman.c:1161-1208
 * convert_lengths_to_encode_table                      | n_ary_huffman.c:1382-1612
 * represent_items_with_codes                           | n_ary_huffman.c:1621-1678
 * dc_huff_compress  (same parameters as static compress)   | n_ary_huffman.c:1688-1815
 * dc_huff_decompress (same parameters as static decompress) | n_ary_huffman.c:2014-2094
 * struct node                                          | n_ary_huffman.c:499-531
 * setup_nodes                                          | n_ary_huffman.c:773-817
 * generate_huffman_tree     (k_huff_table's merge)     | n_ary_huffman.c:868-1005
 * summarize_tree_with_lengths (k_tree_depths)          | n_ary_huffman.c:1033-1093
 * find_compressed_data_size                            | n_ary_huffman.c:2466-2506
 *
 * Semantics and the deliberate differences (all documented in DESIGN.md §Boundary):
 *  - histogram counts bytes up to the first NUL into h[0..max_symbol_value] (bytes above
 *    max_symbol_value are ignored; the reference writes out of bounds there) and prints
 *    nothing (the reference prints one diagnostic per byte > 126, :485-487).
 *  - huffman and convert_lengths_to_encode_table reproduce the reference built with
 *    -DNDEBUG (as shipped, n=2 aborts at :908): the phantom dummy leaf, the index
 *    max_symbol_value quirks, 32-bit wrap of code values. max_symbol_value < 1024.
 *  - represent_items_with_codes (an assert(0) stub in the reference, :1661) writes the
 *    base64url rendering (6 bits per character, int2digit alphabet :371-378) of the
 *    build-defined bitstream (DESIGN.md "Huffman bitstream v1") starting at
 *    compressed_text[start] and returns the characters written, or -1 when a byte has no
 *    code, a code exceeds 32 bits, or the text would not fit in bufsize+1 bytes.
 *  - compress/decompress are `static` in the reference; the same-parameter functions
 *    are exported as dc_huff_compress/dc_huff_decompress and read/write the reference's
 *    netstring blocks (n_ary_huffman.c:1866-1943; layout in dc_host.h): the raw block is
 *    byte-identical to the reference's compress() output for inputs < 32767 bytes, and a
 *    Huffman stream is "#dc1" metadata + "X" table + "#dcidx" sync index + "Z" base64url
 *    data blocks, written when smaller than the raw form. dc_huff_decompress decodes every
 *    block and returns the decompressed length (the reference's returns the first block's
 *    netstring length and copies 2 bytes too many, :2071-2076). It also reads "DCH1".
 *  - The tree helpers work on the caller's struct node list (host memory): the merge of
 *    generate_huffman_tree and the parent walks of summarize_tree_with_lengths run on the
 *    GPU (dc_huff_tree, dc_tree_depths) and their results are written back into the list;
 *    setup_nodes (initialisation) and find_compressed_data_size (a sum over <= 1024 table
 *    entries) are host code. Results equal the reference's (tests/golden/helpers.npz).
 *    generate_huffman_tree needs max_leaf_value < 1024 and the tree to fit list_length
 *    (the reference writes past the list otherwise); `volume` is never touched.
 *  - On a HIP failure (no GPU) the void functions abort with a message, as the
 *    reference's asserts do; they never fall back to CPU compute.
 */
#ifndef DC_HUFFMAN_H
#define DC_HUFFMAN_H
#include <stdbool.h>

#ifdef __cplusplus
extern "C" {
#endif

/* the reference's node (:499-531): bool, then six ints (28 bytes) */
struct node {
    bool leaf;
    int count;
    int left_index;
    int right_index;
    int leaf_value;
    int parent_index;
    int volume;
};

void setup_nodes(const int list_length, struct node list[], const int max_leaf_value,
                 const int symbol_frequencies[]);
void generate_huffman_tree(const int list_length, struct node list[], const int compressed_symbols,
                           const int max_leaf_value);
void summarize_tree_with_lengths(const int list_length, const struct node list[], const int max_leaf_value,
                                 int lengths[], const int leaves);
int find_compressed_data_size(int max_symbol_value, int symbol_frequencies[], int canonical_lengths[],
                              int compressed_symbols);

void histogram(const char *text, const int max_symbol_value, int h[]);
void huffman(const int max_leaf_value, const int symbol_frequencies[],
             const int compressed_symbols, int lengths[]);
void convert_lengths_to_encode_table(const int max_symbol_value, const int canonical_lengths[],
                                     const int compressed_symbols, int encode_length_table[],
                                     unsigned int encode_value_table[]);
int represent_items_with_codes(const int max_symbol_value, int canonical_lengths[],
                               const int compressed_symbols, const int bufsize,
                               const int original_length, char original_text[], int start,
                               char compressed_text[]);
/* returns bytes written, or a negative DC_E_* status */
int dc_huff_compress(const int max_symbol_value, int canonical_lengths[],
                     const int compressed_symbols, const int bufsize, const int original_length,
                     char original_text[], char compressed_text[]);
/* returns the decompressed length, or a negative DC_E_* status */
int dc_huff_decompress(const int max_compressed_size, const char compressed_text[],
                       const int max_decompressed_size, char decompressed_text[]);

#ifdef __cplusplus
}
#endif
#endif
