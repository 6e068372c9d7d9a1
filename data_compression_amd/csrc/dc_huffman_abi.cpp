// dc_huffman_abi.cpp -- libdc_huffman.so: the public functions of n_ary_huffman.c with the
// reference's signatures (include/dc_huffman.h), backed by the gfx950 kernels of
// libdc_core.so. Host code marshals arrays to and from HBM; the kernels do the work.
#include <stdint.h>
#include <string.h>

#include <vector>

#include "dc_abi_common.h"
#include "dc_huffman.h"

namespace {

dc_dtable *table_buf()
{
    void *p = nullptr;
    DC_OR_DIE("dc_huffman", dc_host_scratch(2, sizeof(dc_dtable), &p));
    return (dc_dtable *)p;
}

// build the device table from caller lengths (convert_lengths_to_encode_table path)
int table_from_lengths(dc_ctx *c, int M, const int *lengths, int n, dc_dtable **out)
{
    if (M < 0 || M >= DC_MAX_SYMS || n < 2 || n > 256) return DC_E_ARG;
    void *d_len = nullptr;
    int r = dc_host_scratch(4, (size_t)(M + 1) * 4, &d_len);
    if (r) return r;
    r = dc_memcpy_h2d(c, d_len, lengths, (size_t)(M + 1) * 4);
    if (r) return r;
    dc_dtable *t = table_buf();
    r = dc_huff_table_lengths(c, (const int32_t *)d_len, M, n, t);
    if (r) return r;
    *out = t;
    return DC_OK;
}

}  // namespace

extern "C" {

// n_ary_huffman.c:461-493
void histogram(const char *text, const int max_symbol_value, int h[])
{
    dc_ctx *c = dc_host_ctx();
    if (!c) dc_die("histogram", DC_E_HIP);
    const uint64_t n = strlen(text);   // the text ends at its first NUL (:482)
    const uint8_t *d_in = nullptr;
    DC_OR_DIE("histogram", dc_host_upload(text, n, &d_in));
    void *d_hist = nullptr;
    DC_OR_DIE("histogram", dc_host_scratch(3, 256 * 8, &d_hist));
    DC_OR_DIE("histogram", dc_huff_hist(c, d_in, n, (uint64_t *)d_hist));
    uint64_t hh[256];
    DC_OR_DIE("histogram", dc_memcpy_d2h(c, hh, d_hist, sizeof(hh)));
    for (int i = 0; i <= max_symbol_value; ++i) h[i] = (i < 256) ? (int)hh[i] : 0;
}

// n_ary_huffman.c:1161-1208
void huffman(const int max_leaf_value, const int symbol_frequencies[], const int compressed_symbols, int lengths[])
{
    dc_ctx *c = dc_host_ctx();
    if (!c) dc_die("huffman", DC_E_HIP);
    const int M = max_leaf_value;
    if (M < 0 || M >= DC_MAX_SYMS || compressed_symbols < 2 || compressed_symbols > 256) dc_die("huffman", DC_E_ARG);
    std::vector<uint64_t> f(M + 1);
    for (int i = 0; i <= M; ++i) f[i] = symbol_frequencies[i] > 0 ? (uint64_t)symbol_frequencies[i] : 0;
    void *d_f = nullptr;
    DC_OR_DIE("huffman", dc_host_scratch(5, (size_t)(M + 1) * 8, &d_f));
    DC_OR_DIE("huffman", dc_memcpy_h2d(c, d_f, f.data(), (size_t)(M + 1) * 8));
    dc_dtable *t = table_buf();
    DC_OR_DIE("huffman", dc_huff_table_freq(c, (const uint64_t *)d_f, M, compressed_symbols, t));
    DC_OR_DIE("huffman", dc_memcpy_d2h(c, lengths, t->lengths, (size_t)(M + 1) * 4));
}

// n_ary_huffman.c:1382-1612
void convert_lengths_to_encode_table(const int max_symbol_value, const int canonical_lengths[],
                                     const int compressed_symbols, int encode_length_table[],
                                     unsigned int encode_value_table[])
{
    dc_ctx *c = dc_host_ctx();
    if (!c) dc_die("convert_lengths_to_encode_table", DC_E_HIP);
    const int M = max_symbol_value;
    dc_dtable *t = nullptr;
    DC_OR_DIE("convert_lengths_to_encode_table", table_from_lengths(c, M, canonical_lengths, compressed_symbols, &t));
    std::vector<int32_t> el(M + 1);
    std::vector<uint32_t> ev(M + 1);
    int32_t last = 0;
    DC_OR_DIE("convert_lengths_to_encode_table", dc_memcpy_d2h(c, el.data(), t->enc_len, (size_t)(M + 1) * 4));
    DC_OR_DIE("convert_lengths_to_encode_table", dc_memcpy_d2h(c, ev.data(), t->enc_val, (size_t)(M + 1) * 4));
    DC_OR_DIE("convert_lengths_to_encode_table", dc_memcpy_d2h(c, &last, &t->last_written, 4));
    // entries below max_symbol_value are always written (cleared or assigned, :1421-1424);
    // index max_symbol_value only when it was assigned a code
    for (int i = 0; i < M; ++i) { encode_length_table[i] = el[i]; encode_value_table[i] = ev[i]; }
    if (M >= 0 && last) { encode_length_table[M] = el[M]; encode_value_table[M] = ev[M]; }
}

// n_ary_huffman.c:1621-1678 (stub in the reference); base64url of the v1 bitstream
int represent_items_with_codes(const int max_symbol_value, int canonical_lengths[], const int compressed_symbols,
                               const int bufsize, const int original_length, char original_text[], int start,
                               char compressed_text[])
{
    dc_ctx *c = dc_host_ctx();
    if (!c) dc_die("represent_items_with_codes", DC_E_HIP);
    if (original_length < 0 || start < 0) return -1;
    dc_dtable *t = nullptr;
    if (table_from_lengths(c, max_symbol_value, canonical_lengths, compressed_symbols, &t)) return -1;
    if (dc_huff_table_status(c, t, nullptr)) return -1;
    const uint64_t n = (uint64_t)original_length;
    const uint8_t *d_in = nullptr;
    DC_OR_DIE("represent_items_with_codes", dc_host_upload(original_text, n, &d_in));
    void *d_aux = nullptr;
    DC_OR_DIE("represent_items_with_codes", dc_host_scratch(3, 256 * 8 + 64, &d_aux));
    uint64_t *d_hist = (uint64_t *)d_aux, *d_total = d_hist + 256;
    DC_OR_DIE("represent_items_with_codes", dc_huff_hist(c, d_in, n, d_hist));
    DC_OR_DIE("represent_items_with_codes", dc_huff_plan(c, t, d_total));
    uint64_t total = 0;
    DC_OR_DIE("represent_items_with_codes", dc_memcpy_d2h(c, &total, d_total, 8));
    const uint64_t words = dc_huff_words_needed(0, total);
    void *d_words = nullptr, *d_text = nullptr;
    DC_OR_DIE("represent_items_with_codes", dc_host_scratch(0, words * 4, &d_words));
    const uint64_t nchar = (total + 5) / 6;
    if ((uint64_t)start + nchar > (uint64_t)bufsize + 1) return -1;
    const int r = dc_huff_pack(c, d_in, n, t, 0, (uint32_t *)d_words, words, nullptr, nullptr, 0);
    if (r) return -1;
    DC_OR_DIE("represent_items_with_codes", dc_host_scratch(1, nchar + 16, &d_text));
    DC_OR_DIE("represent_items_with_codes", dc_huff_base64url(c, (const uint32_t *)d_words, 0, total, (char *)d_text));
    DC_OR_DIE("represent_items_with_codes", dc_memcpy_d2h(c, compressed_text + start, d_text, nchar));
    return (int)nchar;
}

// ---- the tree helpers (n_ary_huffman.c:773-1093, :2466-2506) on the caller's node list ----
// setup_nodes (:773-817): the node list's initial state (a copy of the caller's counts into
// its own struct array; no arithmetic to run anywhere else). Leaves 0..max_leaf_value, then
// internal slots; `volume` is left as the reference leaves it (untouched).
void setup_nodes(const int list_length, struct node list[], const int max_leaf_value, const int symbol_frequencies[])
{
    for (int i = 0; i < list_length; ++i) {
        const bool leaf = i <= max_leaf_value;
        list[i].leaf = leaf;
        list[i].leaf_value = leaf ? i : 0;
        list[i].count = leaf ? symbol_frequencies[i] : 0;
        list[i].parent_index = 0;
        list[i].left_index = 0;
        list[i].right_index = 0;
    }
}

// generate_huffman_tree (:868-1005): the n-ary merge of the list's leaf counts runs in
// k_huff_table (dc_huff_tree); its parents, internal counts and first two children come
// back into the caller's list, with the dummy leaves' count of 1 (:921-929).
void generate_huffman_tree(const int list_length, struct node list[], const int compressed_symbols,
                           const int max_leaf_value)
{
    dc_ctx *c = dc_host_ctx();
    if (!c) dc_die("generate_huffman_tree", DC_E_HIP);
    const int M = max_leaf_value;
    if (M < 0 || M >= DC_MAX_SYMS || M >= list_length || compressed_symbols < 2 || compressed_symbols > 256)
        dc_die("generate_huffman_tree", DC_E_ARG);
    std::vector<uint64_t> f(M + 1);
    for (int i = 0; i <= M; ++i) f[i] = list[i].count > 0 ? (uint64_t)list[i].count : 0;
    void *d_f = nullptr, *d_tree = nullptr;
    DC_OR_DIE("generate_huffman_tree", dc_host_scratch(5, (size_t)(M + 1) * 8, &d_f));
    DC_OR_DIE("generate_huffman_tree", dc_host_scratch(1, sizeof(dc_tree), &d_tree));
    DC_OR_DIE("generate_huffman_tree", dc_memcpy_h2d(c, d_f, f.data(), (size_t)(M + 1) * 8));
    DC_OR_DIE("generate_huffman_tree",
              dc_huff_tree(c, (const uint64_t *)d_f, M, compressed_symbols, table_buf(), (dc_tree *)d_tree));
    std::vector<dc_tree> h(1);
    DC_OR_DIE("generate_huffman_tree", dc_memcpy_d2h(c, h.data(), d_tree, sizeof(dc_tree)));
    const dc_tree &T = h[0];
    if (T.status) dc_die("generate_huffman_tree", T.status);
    if (T.nodes > list_length) dc_die("generate_huffman_tree", DC_E_CAPACITY);   // the reference overruns list[]
    for (int i = M + 1; i < T.first_internal; ++i) list[i].count = 1;
    for (int i = T.first_internal; i < T.nodes; ++i) {
        list[i].count = (int)(uint32_t)T.count[i];   // int, as the reference sums (:994-997)
        list[i].left_index = T.left[i];
        list[i].right_index = T.right[i];
    }
    for (int i = 0; i < T.nodes; ++i)
        if (T.parent[i]) list[i].parent_index = T.parent[i];
}

// summarize_tree_with_lengths (:1033-1093): each leaf's depth by the parent walk
// (dc_tree_depths), stored at lengths[leaf_value] in leaf order
void summarize_tree_with_lengths(const int list_length, const struct node list[], const int max_leaf_value,
                                 int lengths[], const int leaves)
{
    dc_ctx *c = dc_host_ctx();
    if (!c) dc_die("summarize_tree_with_lengths", DC_E_HIP);
    if (list_length < 1 || leaves < 0 || leaves > list_length || max_leaf_value < 0)
        dc_die("summarize_tree_with_lengths", DC_E_ARG);
    for (int i = 0; i <= max_leaf_value; ++i) lengths[i] = 0;
    if (leaves == 0) return;
    std::vector<int32_t> par(list_length), depth(leaves);
    for (int i = 0; i < list_length; ++i) par[i] = list[i].parent_index;
    void *d_par = nullptr, *d_depth = nullptr;
    DC_OR_DIE("summarize_tree_with_lengths", dc_host_scratch(5, (size_t)list_length * 4, &d_par));
    DC_OR_DIE("summarize_tree_with_lengths", dc_host_scratch(4, (size_t)leaves * 4, &d_depth));
    DC_OR_DIE("summarize_tree_with_lengths", dc_memcpy_h2d(c, d_par, par.data(), (size_t)list_length * 4));
    DC_OR_DIE("summarize_tree_with_lengths",
              dc_tree_depths(c, (const int32_t *)d_par, list_length, leaves, (int32_t *)d_depth));
    DC_OR_DIE("summarize_tree_with_lengths", dc_memcpy_d2h(c, depth.data(), d_depth, (size_t)leaves * 4));
    for (int i = 0; i < leaves; ++i) {
        const int v = list[i].leaf_value;
        if (depth[i] < 0 || v < 0 || v > max_leaf_value) dc_die("summarize_tree_with_lengths", DC_E_ARG);
        lengths[v] = depth[i];
    }
}

// find_compressed_data_size (:2466-2506): the payload in digits, sum of count x length over
// the coded symbols (the formula the encoder's plan evaluates per block, k_block_local)
int find_compressed_data_size(int max_symbol_value, int symbol_frequencies[], int canonical_lengths[],
                              int compressed_symbols)
{
    (void)compressed_symbols;
    int size = 0;
    for (int i = 0; i <= max_symbol_value; ++i)
        if (canonical_lengths[i] > 0) size += canonical_lengths[i] * symbol_frequencies[i];   // int, as :2485
    return size;
}

// same parameters as the static compress() (n_ary_huffman.c:1688-1697): the reference's
// netstring blocks (dc_host.h "netstring container"); the output is NUL-terminated when it
// fits, as the reference's sprintf leaves it (:1811)
int dc_huff_compress(const int max_symbol_value, int canonical_lengths[], const int compressed_symbols,
                     const int bufsize, const int original_length, char original_text[], char compressed_text[])
{
    if (original_length < 0 || bufsize < 0) return DC_E_ARG;
    uint64_t len = 0;
    const int r = dc_huff_compress_netstring((const uint8_t *)original_text, (uint64_t)original_length,
                                             compressed_symbols, canonical_lengths, max_symbol_value, 0,
                                             (uint8_t *)compressed_text, (uint64_t)bufsize + 1, &len);
    if (r) return r;
    if (len < (uint64_t)bufsize + 1) compressed_text[len] = 0;
    return (int)len;
}

// same parameters as the static decompress() (n_ary_huffman.c:2014-2020): every block of a
// netstring container (or a DCH1 container), not only the first; returns the decompressed
// length (the reference returns the first block's netstring length and copies two bytes too
// many of a raw block, :2071-2076)
int dc_huff_decompress(const int max_compressed_size, const char compressed_text[], const int max_decompressed_size,
                       char decompressed_text[])
{
    if (max_compressed_size < 0 || max_decompressed_size < 0) return DC_E_ARG;
    uint64_t len = 0;
    const int r = dc_huff_decompress_host((const uint8_t *)compressed_text, (uint64_t)max_compressed_size,
                                          (uint8_t *)decompressed_text, (uint64_t)max_decompressed_size, &len);
    return r ? r : (int)len;
}

}  // extern "C"
