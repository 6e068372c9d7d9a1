/*
 * oracle/dc_oracle.c -- TEST INFRASTRUCTURE ONLY: clean-room CPU restatement of the
 * reference's hot path. See dc_oracle.h for what it is allowed to be used for and how
 * it is pinned (tests/golden/, generated from the reference C itself).
 */
#include "dc_oracle.h"

#include <stdlib.h>
#include <string.h>

/* ================================================================================== */
/* histogram  (n_ary_huffman.c:461-493)                                                */
/* ================================================================================== */
void orc_histogram_bytes(const uint8_t *x, uint64_t n, uint64_t h[256])
{
    for (int i = 0; i < 256; i++) h[i] = 0;
    for (uint64_t i = 0; i < n; i++) h[x[i]]++;
}

uint64_t orc_histogram_cstr(const char *text, int max_symbol_value, int *h)
{
    /* :474-476 zero h[0..max]; :482-490 count until the terminating NUL */
    for (int i = 0; i <= max_symbol_value; i++) h[i] = 0;
    const unsigned char *c = (const unsigned char *)text;
    uint64_t n = 0;
    for (; c[n]; n++)
        if ((int)c[n] <= max_symbol_value) h[c[n]]++;
    return n;
}

/* ================================================================================== */
/* n-ary Huffman code lengths  (n_ary_huffman.c:773-1208)                              */
/*                                                                                     */
/* The reference keeps every active node in one index array, bubble-sorts it stably    */
/* by count before each merge (:672-731, :962-1002) and appends each new internal node  */
/* at the end. Induction on the merges shows the active order is always ascending      */
/* (count, node_index): leaves are nodes 0..max_leaf_value, dummy leaves                */
/* max_leaf_value+1.. (count 1, :921-929), internal nodes follow in creation order.     */
/* Internal nodes are created with non-decreasing counts and increasing indices, so the */
/* classic two-queue merge reproduces that order exactly.                               */
/* ================================================================================== */
typedef struct { uint64_t count; int index; } orc_item;

static int orc_item_less(const orc_item *a, const orc_item *b)
{
    if (a->count != b->count) return a->count < b->count;
    return a->index < b->index;
}

static int orc_item_cmp(const void *pa, const void *pb)
{
    const orc_item *a = (const orc_item *)pa, *b = (const orc_item *)pb;
    if (orc_item_less(a, b)) return -1;
    if (orc_item_less(b, a)) return 1;
    return 0;
}

int orc_huffman_lengths(int max_leaf_value, const uint64_t *freq, int n_ary, int *lengths)
{
    const int leaves = max_leaf_value + 1;
    int nonzero = 0;
    for (int i = 0; i < leaves; i++) nonzero += (freq[i] != 0);
    /* :900-903, C remainder semantics (negative when nonzero == 0 and n > 2) */
    const int dummies = (n_ary - 1) - ((nonzero - 1) % (n_ary - 1));

    const int items = nonzero + dummies;
    const int max_nodes = leaves + dummies + items + 1;
    orc_item *q1 = (orc_item *)malloc(sizeof(orc_item) * (size_t)(items + 1));
    orc_item *q2 = (orc_item *)malloc(sizeof(orc_item) * (size_t)(items + 1));
    int *parent = (int *)calloc((size_t)max_nodes, sizeof(int));
    int m = 0;
    for (int i = 0; i < leaves; i++)
        if (freq[i]) { q1[m].count = freq[i]; q1[m].index = i; m++; }
    for (int j = 0; j < dummies; j++) { q1[m].count = 1; q1[m].index = leaves + j; m++; }
    qsort(q1, (size_t)m, sizeof(orc_item), orc_item_cmp);

    int h1 = 0, h2 = 0, t2 = 0, active = m;
    int next_index = leaves + dummies;   /* first internal node, :937 + 1 */
    while (active > 1) {
        uint64_t sum = 0;
        for (int k = 0; k < n_ary; k++) {
            orc_item pick;
            int take1 = (h1 < m) && (h2 == t2 || orc_item_less(&q1[h1], &q2[h2]));
            pick = take1 ? q1[h1++] : q2[h2++];
            parent[pick.index] = next_index;
            sum += pick.count;
        }
        q2[t2].count = sum; q2[t2].index = next_index; t2++;
        next_index++;
        active -= n_ary - 1;
    }
    /* depth by walking parents to the root (:1069-1076); parent 0 means "none" */
    int max_len = 0;
    for (int i = 0; i < leaves; i++) {
        int d = 0, c = i;
        while (parent[c] != 0) { d++; c = parent[c]; }
        lengths[i] = d;
        if (d > max_len) max_len = d;
    }
    free(q1); free(q2); free(parent);
    return max_len;
}

/* ================================================================================== */
/* canonical n-ary codes  (n_ary_huffman.c:1382-1612)                                  */
/* ================================================================================== */
void orc_canonical(int max_symbol_value, const int *lengths, int n_ary,
                   int *enc_len, unsigned *enc_val)
{
    /* min/max scan and the clear loop both stop before index max_symbol_value
       (:1336, :1360, :1421) */
    int max_l = 0, min_l = 300;
    for (int i = 0; i < max_symbol_value; i++) {
        if (lengths[i] > max_l) max_l = lengths[i];
        if (lengths[i] && lengths[i] < min_l) min_l = lengths[i];
    }
    for (int i = 0; i < max_symbol_value; i++) { enc_len[i] = 0; enc_val[i] = 0; }
    uint64_t code = 0;    /* reference: int, wraps mod 2^32 -- same low 32 bits */
    for (int L = min_l; L <= max_l; L++) {
        for (int i = 0; i <= max_symbol_value; i++) {
            if (lengths[i] == L) {
                enc_len[i] = L;
                enc_val[i] = (unsigned)code;
                code++;
            }
        }
        code *= (uint64_t)n_ary;
    }
}

/* ================================================================================== */
/* build-defined bitstream v1                                                          */
/* ================================================================================== */
int orc_digit_bits(int n_ary)
{
    int w = 0;
    while ((1 << w) < n_ary) w++;
    return w;
}

int orc_bitcodes(const int *enc_len, const unsigned *enc_val, int n_ary,
                 uint32_t code[256], uint8_t nbits[256])
{
    const int w = orc_digit_bits(n_ary);
    int max_bits = 0;
    for (int s = 0; s < 256; s++) {
        const int L = enc_len[s];
        code[s] = 0; nbits[s] = 0;
        if (L <= 0) continue;
        if ((int64_t)L * w > 32) return -1;
        /* L base-n digits of the value, MSB first, each emitted as w bits */
        uint64_t v = enc_val[s], packed = 0;
        for (int d = 0; d < L; d++) {
            uint64_t digit = v % (uint64_t)n_ary;
            v /= (uint64_t)n_ary;
            packed |= digit << (w * d);
        }
        code[s] = (uint32_t)packed;
        nbits[s] = (uint8_t)(L * w);
        if (L * w > max_bits) max_bits = L * w;
    }
    return max_bits;
}

uint64_t orc_huff_pack(const uint8_t *x, uint64_t n, const uint32_t code[256],
                       const uint8_t nbits[256], uint8_t *out, uint64_t bit_base,
                       uint32_t sync_syms, uint64_t *idx)
{
    /* MSB-first: pending bits sit right-aligned in acc; whole bytes are flushed */
    uint64_t acc = 0, o = 0, total = 0;
    unsigned nacc = (unsigned)(bit_base & 7);     /* leading bits of out[0] stay zero */
    for (uint64_t i = 0; i < n; i++) {
        if (idx && sync_syms && (i % sync_syms) == 0)
            idx[i / sync_syms] = (bit_base & ~(uint64_t)7) + o * 8 + nacc;
        const unsigned nb = nbits[x[i]];
        if (nb == 0) return UINT64_MAX;
        acc = (acc << nb) | code[x[i]];
        nacc += nb;
        total += nb;
        while (nacc >= 8) {
            nacc -= 8;
            out[o++] = (uint8_t)(acc >> nacc);
        }
    }
    if (nacc) out[o] = (uint8_t)(acc << (8 - nacc));
    return total;
}

int orc_huff_unpack(const uint8_t *in, uint64_t in_bits, uint64_t n_out,
                    int max_symbol_value, const int *enc_len, const unsigned *enc_val,
                    int n_ary, uint8_t *out)
{
    /* canonical decode in the base-n digit domain: the values of one length L are a
       contiguous run starting at first[L], assigned in ascending symbol order */
    const int w = orc_digit_bits(n_ary);
    enum { MAXL = 64 };
    uint64_t first[MAXL + 1];
    int count[MAXL + 1], start[MAXL + 1];
    int syms[4096];
    int nsyms = 0;
    for (int L = 0; L <= MAXL; L++) { count[L] = 0; first[L] = UINT64_MAX; }
    for (int i = 0; i <= max_symbol_value && i < 256; i++) {
        const int L = enc_len[i];
        if (L <= 0 || L > MAXL) continue;
        if (count[L] == 0 || (uint64_t)enc_val[i] < first[L]) {
            if (count[L] == 0) first[L] = enc_val[i];
        }
        count[L]++;
    }
    for (int L = 1, acc = 0; L <= MAXL; L++) {
        start[L] = acc;
        for (int i = 0; i <= max_symbol_value && i < 256; i++)
            if (enc_len[i] == L) syms[nsyms++] = i;
        acc += count[L];
    }
    uint64_t pos = 0;
    for (uint64_t k = 0; k < n_out; k++) {
        uint64_t v = 0;
        int L = 0, found = -1;
        while (found < 0) {
            if (pos + (uint64_t)w > in_bits || L >= MAXL) return -1;
            const uint64_t byte = pos >> 3;
            const unsigned two = ((unsigned)in[byte] << 8) |
                                 ((byte + 1 < (in_bits + 7) / 8) ? in[byte + 1] : 0u);
            const uint64_t digit = (two >> (16 - (pos & 7) - (unsigned)w)) & ((1u << w) - 1u);
            pos += (uint64_t)w;
            if (digit >= (uint64_t)n_ary) return -1;
            v = v * (uint64_t)n_ary + digit;
            L++;
            if (count[L] && v >= first[L] && v - first[L] < (uint64_t)count[L])
                found = syms[start[L] + (int)(v - first[L])];
        }
        out[k] = (uint8_t)found;
    }
    return 0;
}

uint64_t orc_base64url(const uint8_t *in, uint64_t bits, char *out)
{
    /* alphabet of int2digit(), n_ary_huffman.c:371-378 */
    static const char tbl[] =
        "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789-_";
    uint64_t nchar = (bits + 5) / 6;
    for (uint64_t c = 0; c < nchar; c++) {
        unsigned v = 0;
        for (int b = 0; b < 6; b++) {
            uint64_t p = c * 6 + (uint64_t)b;
            unsigned bit = (p < bits) ? ((in[p >> 3] >> (7 - (p & 7))) & 1u) : 0u;
            v = (v << 1) | bit;
        }
        out[c] = tbl[v];
    }
    return nchar;
}

/* ---- digit text -------------------------------------------------- */
static const char orc_b64[] = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789-_";
static const char orc_hex[] = "0123456789ABCDEF";
static const char orc_dig[] = "0123456789abcdef";
/* Z85 (rfc.zeromq.org/spec/32), the table n_ary_huffman.c:389-396 names; first 81 used */
static const char orc_z85[] = "0123456789abcdefghijklmnopqrstuvwxyzABCDEFGHIJKLMNOPQRSTUVWXYZ.-:+=^!/*?&<>()[]{}@%$#";

static int orc_text_w(int n)
{
    int w = 0;
    while ((1 << w) < n) w++;
    return w;
}

/* bits per character, 0 for an unsupported (format, n) */
static int orc_text_bits(int format, int n)
{
    switch (format) {
    case 0: return 6;
    case 1: return 4;
    case 2: return (n >= 2 && n <= 16) ? orc_text_w(n) : 0;
    case 3: return (n == 3 || n == 9) ? 8 : 0;
    case 4: return n == 3 ? 10 : 0;
    default: return 0;
    }
}

/* a field of b bits (MSB-first) -> its character; a field holding a digit >= n (never
 * written by the encoder) renders as '~' (in none of the alphabets), as byte 0 in format 4 */
static int orc_text_char(unsigned f, int format, int n)
{
    switch (format) {
    case 0: return orc_b64[f];
    case 1: return orc_hex[f];
    case 2: return f < (unsigned)n ? orc_dig[f] : '~';
    case 3: {
        const int dw = n == 3 ? 2 : 4;
        unsigned v = 0;
        for (int k = 8 - dw; k >= 0; k -= dw) {
            const unsigned d = (f >> k) & ((1u << dw) - 1);
            if (d >= (unsigned)n) return '~';
            v = v * (unsigned)n + d;
        }
        return orc_z85[v];
    }
    case 4: {
        unsigned v = 0;
        for (int k = 8; k >= 0; k -= 2) {
            const unsigned d = (f >> k) & 3u;
            if (d >= 3) return 0;
            v = v * 3 + d;
        }
        return (int)(1 + v);
    }
    }
    return '~';
}

uint64_t orc_text(const uint8_t *in, uint64_t bits, int format, int n_ary, char *out)
{
    const int b = orc_text_bits(format, n_ary);
    if (b == 0) return 0;
    const uint64_t nchar = (bits + (uint64_t)b - 1) / (uint64_t)b;
    for (uint64_t c = 0; c < nchar; c++) {
        unsigned f = 0;
        for (int k = 0; k < b; k++) {
            const uint64_t p = c * (uint64_t)b + (uint64_t)k;
            f = (f << 1) | ((p < bits) ? ((in[p >> 3] >> (7 - (p & 7))) & 1u) : 0u);
        }
        out[c] = (char)orc_text_char(f, format, n_ary);
    }
    return nchar;
}

/* a character -> its field, or -1 (brute force over the fields: test infrastructure) */
static int orc_text_field(unsigned char ch, int format, int n)
{
    const int b = orc_text_bits(format, n);
    if (format == 4 ? ch == 0 : ch == '~') return -1;
    for (unsigned f = 0; f < (1u << b); f++)
        if ((unsigned char)orc_text_char(f, format, n) == ch) return (int)f;
    if (format == 0 && ch == '+') return 62;   /* digit2int, n_ary_huffman.c:443-446 */
    if (format == 0 && ch == '/') return 63;
    if (format == 1 && ch >= 'a' && ch <= 'f') return ch - 'a' + 10;
    return -1;
}

int orc_text_parse(const char *text, uint64_t nchar, int format, int n_ary, uint8_t *out, uint64_t bits)
{
    const int b = orc_text_bits(format, n_ary);
    if (b == 0 || nchar * (uint64_t)b < bits) return -1;
    memset(out, 0, (size_t)((bits + 7) / 8));
    for (uint64_t c = 0; c < nchar; c++) {
        const int f = orc_text_field((unsigned char)text[c], format, n_ary);
        if (f < 0) return -1;
        for (int k = 0; k < b; k++) {
            const uint64_t p = c * (uint64_t)b + (uint64_t)k;
            if (p < bits && ((f >> (b - 1 - k)) & 1)) out[p >> 3] |= (uint8_t)(0x80u >> (p & 7));
        }
    }
    return 0;
}

/* ================================================================================== */
/* nybble codec  (nybble_compression.c:517-1137)                                       */
/* ================================================================================== */
enum { ORC_NYBBLES = 0xAF, ORC_LITERAL = ' ' };   /* :732-733 */
static const uint8_t orc_initial_letters[8] = { ' ', 'e', 't', 'a', 'o', 'i', 'n', 's' };

static int orc_ctx(uint8_t b) { return (b >> 3) & 15; }   /* :517-523, bits 3..6 */

static void orc_mtf_init(uint8_t lists[16][8])
{
    for (int c = 0; c < 16; c++) memcpy(lists[c], orc_initial_letters, 8);
}

/* move-to-front with drop-last (:665-687) */
static void orc_mtf_touch(uint8_t list[8], uint8_t v)
{
    uint8_t carry = v;
    for (int p = 0; p < 8; p++) {
        uint8_t old = list[p];
        list[p] = carry;
        carry = old;
        if (carry == v) break;
    }
}

static int orc_rank(const uint8_t list[8], uint8_t v)
{
    for (int r = 0; r < 8; r++) if (list[r] == v) return r;
    return -1;
}

uint64_t orc_nybble_compress(const uint8_t *x, uint64_t n, uint8_t *out, int modify)
{
    if (n == 0) {   /* reference reads past the terminator here (UB); defined as LITERAL */
        out[0] = ORC_LITERAL;
        return 1;
    }
    uint8_t lists[16][8];
    orc_mtf_init(lists);
    uint64_t o = 0;
    out[o++] = ORC_NYBBLES;
    out[o++] = x[0];                      /* context seed, copied raw (:903-905) */
    int half = 0;                         /* a hit nybble is pending in out[o]'s hi half */
    for (uint64_t i = 1; i < n; i++) {
        const int c = orc_ctx(x[i - 1]);
        const int r = orc_rank(lists[c], x[i]);
        if (r < 0) {
            if (!half) {
                out[o++] = x[i];          /* byte-aligned literal (:844-846) */
            } else {
                out[o] = x[i - 1];        /* pending hit becomes a literal (:855-857) */
                out[o + 1] = x[i];
                o += 2;
                half = 0;
            }
        } else {
            const uint8_t nyb = (uint8_t)(8 | r);
            if (!half) { out[o] = (uint8_t)(nyb << 4); half = 1; }
            else { out[o] = (uint8_t)(out[o] | nyb); o++; half = 0; }
        }
        if (modify) orc_mtf_touch(lists[c], x[i]);
    }
    if (half) out[o++] = x[n - 1];        /* odd tail (:1000-1009) */
    if (o >= n) {                         /* incompressible: LITERAL (:1018-1037) */
        out[0] = ORC_LITERAL;
        memcpy(out + 1, x, (size_t)n);
        return n + 1;
    }
    return o;
}

uint64_t orc_nybble_decompress(const uint8_t *in, uint64_t m, uint8_t *out, int modify)
{
    if (m == 0) return 0;
    if (in[0] == ORC_NYBBLES) {
        if (m < 2) return 0;
        uint8_t lists[16][8];
        orc_mtf_init(lists);
        uint64_t o = 0, pos = 2;
        out[o++] = in[1];
        int off = 0;
        while (pos < m) {
            const uint8_t b = in[pos];
            int nyb, next;
            if (off == 0) { nyb = b >> 4; next = b & 15; }
            else { nyb = b & 15; next = (pos + 1 < m) ? (in[pos + 1] >> 4) : 0; }
            const int c = orc_ctx(out[o - 1]);
            int used;
            if (nyb & 8) { out[o] = lists[c][nyb & 7]; used = 1; }
            else { out[o] = (uint8_t)(((nyb & 7) << 4) + next); used = 2; }
            if (modify) orc_mtf_touch(lists[c], out[o]);
            o++;
            off += used;
            if (off >= 2) { pos++; off -= 2; }
        }
        return o;
    }
    if (in[0] == ORC_LITERAL) {
        memcpy(out, in + 1, (size_t)(m - 1));
        return m - 1;
    }
    memcpy(out, in, (size_t)m);           /* unknown type: copied with the type byte */
    return m;
}

/* ================================================================================== */
/* small front-end  (small_compression.c:507-665)                                      */
/* ================================================================================== */
enum { ORC_EIGHT_BIT_PRUNED = 8 };        /* small_compression.c:39 */

uint64_t orc_small_compress(const uint8_t *x, uint64_t n, uint8_t *out)
{
    if (n == 0) { out[0] = ORC_LITERAL; return 1; }
    uint64_t o = 0, i = 1;
    out[o++] = ORC_EIGHT_BIT_PRUNED;
    out[o++] = x[0];
    while (i < n) {
        /* ' ' followed by a lowercase letter -> one byte 0x80+letter (:524-527) */
        if (x[i] == ' ' && i + 1 < n && x[i + 1] >= 'a' && x[i + 1] <= 'z') {
            out[o++] = (uint8_t)(0x80 + x[i + 1]);
            i += 2;
        } else {
            out[o++] = x[i];
            i += 1;
        }
    }
    if (o >= n) {
        out[0] = ORC_LITERAL;
        memcpy(out + 1, x, (size_t)n);
        return n + 1;
    }
    return o;
}

uint64_t orc_small_decompress(const uint8_t *in, uint64_t m, uint8_t *out)
{
    if (m == 0) return 0;
    if (in[0] == ORC_EIGHT_BIT_PRUNED) {
        if (m < 2) return 0;
        uint64_t o = 0;
        out[o++] = in[1];
        for (uint64_t p = 2; p < m; p++) {
            if (in[p] >= 0x80) { out[o++] = ' '; out[o++] = (uint8_t)(in[p] - 0x80); }
            else out[o++] = in[p];
        }
        return o;
    }
    if (in[0] == ORC_LITERAL) {
        memcpy(out, in + 1, (size_t)(m - 1));
        return m - 1;
    }
    memcpy(out, in, (size_t)m);
    return m;
}
