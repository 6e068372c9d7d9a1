// dc_host.hip -- host-buffer entry points of libdc_core.so: a per-thread device context
// with growable scratch buffers, and the "DCH1" Huffman container built on
// the device-resident stages of dc_core.hip. Host code here only moves bytes and
// assembles headers; every byte of payload is produced and consumed by GPU kernels.

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <stdio.h>

#include <vector>

#include "dc_gpu.h"
#include "dc_host.h"

namespace {

struct Buf {
    void *p = nullptr;
    size_t cap = 0;
    int need(size_t bytes)
    {
        if (cap >= bytes && p) return DC_OK;
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
        size_t want = bytes < 4096 ? 4096 : bytes + bytes / 8;
        if (hipMalloc(&p, want) != hipSuccess) { p = nullptr; return DC_E_HIP; }
        cap = want;
        return DC_OK;
    }
};

struct HostState {
    dc_ctx *ctx = nullptr;
    Buf in, out, sync, table, hist, lens, aux, in2, aux2;
    int err = DC_OK;
};

thread_local HostState g_state;

int state(HostState **s)
{
    HostState &st = g_state;
    if (!st.ctx) {
        int dev = 0;
        const char *e = getenv("DC_DEVICE");
        if (e) dev = atoi(e);
        int r = dc_ctx_create_owned(&st.ctx, dev);
        if (r) return r;
    }
    *s = &st;
    return DC_OK;
}

#define RC(x) do { int _r = (x); if (_r) return _r; } while (0)

const uint32_t kMagic = 0x31484344u;   // "DCH1" little-endian
const size_t kHeader = 288;

inline void put32(uint8_t *p, uint32_t v) { memcpy(p, &v, 4); }
inline void put64(uint8_t *p, uint64_t v) { memcpy(p, &v, 8); }
inline uint32_t get32(const uint8_t *p) { uint32_t v; memcpy(&v, p, 4); return v; }
inline uint64_t get64(const uint8_t *p) { uint64_t v; memcpy(&v, p, 8); return v; }

}  // namespace

extern "C" {

// sync index in the container: u64 group bases, then u16 chunk bit lengths
static uint64_t index_bytes(uint64_t n, uint32_t S)
{
    return dc_huff_sync_groups(n, S) * 8 + dc_huff_sync_chunks(n, S) * 2;
}

dc_ctx *dc_host_ctx(void)
{
    HostState *s = nullptr;
    return state(&s) ? nullptr : s->ctx;
}

int dc_host_upload(const void *h, uint64_t n, const uint8_t **d_out)
{
    HostState *s;
    RC(state(&s));
    RC(s->in.need(n + 64));
    if (n) RC(dc_memcpy_h2d(s->ctx, s->in.p, h, n));
    *d_out = (const uint8_t *)s->in.p;
    return DC_OK;
}

int dc_host_scratch(int which, uint64_t bytes, void **d_out)
{
    HostState *s;
    RC(state(&s));
    Buf *b = which == 0 ? &s->out : which == 1 ? &s->sync : which == 2 ? &s->table
           : which == 3 ? &s->hist : which == 4 ? &s->lens : &s->aux;
    RC(b->need(bytes));
    *d_out = b->p;
    return DC_OK;
}

uint64_t dc_huff_compress_bound(uint64_t n, uint32_t sync_syms)
{
    if (sync_syms == 0) sync_syms = 64;   // the densest index dc_huff_choose_sync can pick
    return kHeader + index_bytes(n, sync_syms) + n * 4 + 64;   // codes are <= 32 bits per byte
}

int dc_huff_compress_host(const uint8_t *in, uint64_t n, int n_ary, const int32_t *lengths, int max_symbol_value,
                          uint32_t sync_syms, uint8_t *out, uint64_t cap, uint64_t *out_len)
{
    if ((n && !in) || !out || !out_len || n_ary < 2 || n_ary > 16) return DC_E_ARG;
    HostState *s;
    RC(state(&s));
    dc_ctx *c = s->ctx;
    if (sync_syms != 0 && (sync_syms < 16 || sync_syms > DC_SYNC_MAX || (sync_syms & (sync_syms - 1))))
        return DC_E_ARG;
    const uint8_t *d_in = nullptr;
    RC(dc_host_upload(in, n, &d_in));
    RC(s->hist.need(256 * 8 + 64));
    RC(s->table.need(sizeof(dc_dtable)));
    uint64_t *d_hist = (uint64_t *)s->hist.p;
    uint64_t *d_total = d_hist + 256;
    dc_dtable *d_tab = (dc_dtable *)s->table.p;
    RC(dc_huff_hist(c, d_in, n, d_hist));
    if (lengths) {
        const int M = max_symbol_value;
        if (M < 0 || M >= DC_MAX_SYMS) return DC_E_ARG;
        RC(s->lens.need((size_t)(M + 1) * 4));
        RC(dc_memcpy_h2d(c, s->lens.p, lengths, (size_t)(M + 1) * 4));
        RC(dc_huff_table_lengths(c, (const int32_t *)s->lens.p, M, n_ary, d_tab));
    } else {
        RC(dc_huff_table(c, d_hist, 258, n_ary, d_tab));
    }
    int32_t maxbits = 0;
    const int st = dc_huff_table_status(c, d_tab, &maxbits);
    if (st) return st;
    RC(dc_huff_plan(c, d_tab, d_total));
    uint64_t total = 0;
    RC(dc_memcpy_d2h(c, &total, d_total, 8));
    const uint64_t words = dc_huff_words_needed(0, total);
    if (sync_syms == 0) sync_syms = dc_huff_choose_sync(n, total);
    const uint64_t ng = dc_huff_sync_groups(n, sync_syms), nc = dc_huff_sync_chunks(n, sync_syms);
    const uint64_t ib = index_bytes(n, sync_syms);
    const uint64_t nbytes = (total + 7) / 8;
    const uint64_t need = kHeader + ib + nbytes;
    if (need > cap) return DC_E_CAPACITY;
    RC(s->out.need(words * 4));
    RC(s->sync.need(ib + 16));
    uint64_t *d_base = (uint64_t *)s->sync.p;
    uint16_t *d_len = (uint16_t *)(d_base + ng);
    RC(dc_huff_pack(c, d_in, n, d_tab, 0, (uint32_t *)s->out.p, words, d_base, d_len, sync_syms));
    // header: magic, version, n, w, payload bits, sync granularity, per-byte code lengths
    int32_t enc_len[256];
    RC(dc_memcpy_d2h(c, enc_len, d_tab->enc_len, sizeof(enc_len)));
    int32_t w = 0;
    RC(dc_memcpy_d2h(c, &w, &d_tab->w, 4));
    memset(out, 0, kHeader);
    put32(out, kMagic);
    out[4] = 1;
    out[5] = (uint8_t)n_ary;
    out[6] = (uint8_t)w;
    out[7] = 0;
    put64(out + 8, n);
    put64(out + 16, total);
    put32(out + 24, sync_syms);
    for (int i = 0; i < 256; ++i) out[32 + i] = (uint8_t)(enc_len[i] > 0 ? enc_len[i] : 0);
    RC(dc_memcpy_d2h(c, out + kHeader, d_base, ng * 8));
    RC(dc_memcpy_d2h(c, out + kHeader + ng * 8, d_len, nc * 2));
    RC(dc_memcpy_d2h(c, out + kHeader + ib, s->out.p, nbytes));
    *out_len = need;
    return DC_OK;
}

int dc_huff_netstring_info(const uint8_t *in, uint64_t m, uint64_t *out_n);

int dc_huff_container_info(const uint8_t *in, uint64_t m, uint64_t *n, int *n_ary, uint64_t *bits)
{
    if (in && (m < 4 || get32(in) != kMagic)) {   // netstring container: decompressed size only
        uint64_t v = 0;
        RC(dc_huff_netstring_info(in, m, &v));
        if (n) *n = v;
        if (n_ary) *n_ary = 0;
        if (bits) *bits = 0;
        return DC_OK;
    }
    if (!in || m < kHeader || get32(in) != kMagic || in[4] != 1) return DC_E_STREAM;
    if (n) *n = get64(in + 8);
    if (n_ary) *n_ary = in[5];
    if (bits) *bits = get64(in + 16);
    return DC_OK;
}

int dc_huff_decompress_netstring(const uint8_t *in, uint64_t m, uint8_t *out, uint64_t cap, uint64_t *out_len);

int dc_huff_decompress_host(const uint8_t *in, uint64_t m, uint8_t *out, uint64_t cap, uint64_t *out_len)
{
    if (!in || !out_len) return DC_E_ARG;
    if (m < 4 || get32(in) != kMagic) return dc_huff_decompress_netstring(in, m, out, cap, out_len);
    uint64_t n = 0, bits = 0;
    int nary = 0;
    RC(dc_huff_container_info(in, m, &n, &nary, &bits));
    const uint32_t S = get32(in + 24);
    if (S < 16 || S > DC_SYNC_MAX || (S & (S - 1)) || nary < 2) return DC_E_STREAM;
    const uint64_t ng = dc_huff_sync_groups(n, S), nc = dc_huff_sync_chunks(n, S);
    const uint64_t ib = index_bytes(n, S);
    const uint64_t nbytes = (bits + 7) / 8;
    if (kHeader + ib + nbytes > m) return DC_E_STREAM;
    if (n > cap) return DC_E_CAPACITY;
    if (n && !out) return DC_E_ARG;
    HostState *s;
    RC(state(&s));
    dc_ctx *c = s->ctx;
    int32_t lens[259];
    for (int i = 0; i < 256; ++i) lens[i] = in[32 + i];
    lens[256] = lens[257] = lens[258] = 0;
    RC(s->lens.need(sizeof(lens)));
    RC(s->table.need(sizeof(dc_dtable)));
    RC(dc_memcpy_h2d(c, s->lens.p, lens, sizeof(lens)));
    dc_dtable *d_tab = (dc_dtable *)s->table.p;
    RC(dc_huff_table_lengths(c, (const int32_t *)s->lens.p, 258, nary, d_tab));
    const int st = dc_huff_table_status(c, d_tab, nullptr);
    if (st) return st;
    const uint64_t words = dc_huff_words_needed(0, bits);
    RC(s->in.need(words * 4 + 64));
    RC(s->sync.need(ib + 16));
    RC(s->out.need(n + 64));
    uint64_t *d_base = (uint64_t *)s->sync.p;
    uint16_t *d_len = (uint16_t *)(d_base + ng);
    RC(dc_memset(c, s->in.p, 0, words * 4));
    RC(dc_memcpy_h2d(c, d_base, in + kHeader, ng * 8));
    RC(dc_memcpy_h2d(c, d_len, in + kHeader + ng * 8, nc * 2));
    RC(dc_memcpy_h2d(c, s->in.p, in + kHeader + ib, nbytes));
    RC(dc_huff_decode(c, (const uint32_t *)s->in.p, 0, words, d_base, d_len, S, n, d_tab, (uint8_t *)s->out.p));
    RC(dc_huff_decode_status(c));
    RC(dc_memcpy_d2h(c, out, s->out.p, n));
    *out_len = n;
    return DC_OK;
}

// ---- netstring container: the reference's block format -----------------------------
// n_ary_huffman.c:1866-1943 ("netstring" blocks of <= 2^15 payload bytes, 2-byte type:
// "\n\n" raw, "\n#" metadata, "\nX" table, "\nZ" data), written by compress() (:1688-1815)
// and read by decompress() (:2014-2094). DESIGN.md §2 "Netstring container v1" gives the
// exact layout of each block this build writes; the raw block is byte-identical to the
// reference's pass-through block (:1806-1814), and the X block to its table block
// (:1710-1747) whenever every length is < 10.
#define NS_MAX_PAYLOAD 32768u   // get_compressed_block_length: length <= 32768 (:1826-1827)

static const char kLenDigits[] = "0123456789ABCDEFGHIJKLMNOPQRSTUVWXYZ";   // length L -> one char

// framed copy of a text: blocks of C characters, each "<hdr><C chars>," (the last block
// with its own header); one byte per thread (the text is ~1/8 of the input's bytes)
struct NsHdr { uint8_t b[16]; uint32_t len; };
__global__ void k_ns_frame(const uint8_t *__restrict__ text, uint64_t nchar, uint32_t C, NsHdr full, NsHdr last,
                           uint8_t *__restrict__ out)
{
    const uint64_t nb = (nchar + C - 1) / C;
    const uint64_t stride = (uint64_t)full.len + C + 1;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nchar; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t b = i / C, j = i - b * C;
        const bool lastb = b + 1 == nb;
        const NsHdr &h = lastb ? last : full;
        uint8_t *blk = out + b * stride;
        blk[h.len + j] = text[i];
        if (j == 0)
            for (uint32_t k = 0; k < h.len; ++k) blk[k] = h.b[k];
        const uint64_t cnt = lastb ? nchar - b * C : C;
        if (j + 1 == cnt) blk[h.len + cnt] = ',';
    }
}

// gather of byte ranges: range r = src[off[r] .. off[r] + len[r]) -> dst[dst_off[r] ..);
// one workgroup per range (grid-stride over ranges)
__global__ void k_ns_gather(const uint8_t *__restrict__ src, const uint64_t *__restrict__ ranges, uint64_t nranges,
                            uint8_t *__restrict__ dst)
{
    for (uint64_t r = blockIdx.x; r < nranges; r += gridDim.x) {
        const uint64_t so = ranges[3 * r], len = ranges[3 * r + 1], d = ranges[3 * r + 2];
        for (uint64_t i = threadIdx.x; i < len; i += blockDim.x) dst[d + i] = src[so + i];
    }
}

namespace {

size_t ns_put_header(uint8_t *o, uint64_t payload_len, const char *type_and_prefix, size_t tl)
{
    const int k = snprintf((char *)o, 8, "%llu:", (unsigned long long)payload_len);   // <= 32768
    memcpy(o + k, type_and_prefix, tl);
    return (size_t)k + tl;
}

uint64_t ns_digits(uint64_t v)
{
    uint64_t d = 1;
    while (v >= 10) { v /= 10; ++d; }
    return d;
}

// total bytes of `nchar` characters framed in blocks whose payload is prefix (tl bytes) +
// up to C characters
uint64_t ns_framed_size(uint64_t nchar, uint64_t tl, uint64_t C)
{
    if (nchar == 0) return 0;
    const uint64_t nb = (nchar + C - 1) / C, lastc = nchar - (nb - 1) * C;
    return (nb - 1) * (ns_digits(C + tl) + 1 + tl + C + 1) + ns_digits(lastc + tl) + 1 + tl + lastc + 1;
}

NsHdr ns_hdr(uint64_t cnt, const char *prefix, size_t tl)
{
    NsHdr h;
    memset(&h, 0, sizeof(h));
    h.len = (uint32_t)ns_put_header(h.b, cnt + tl, prefix, tl);
    return h;
}

// frame nchar device characters into d_out (device); returns bytes written
int ns_frame(dc_ctx *c, const uint8_t *d_text, uint64_t nchar, const char *prefix, size_t tl, uint8_t *d_out,
             uint64_t *written)
{
    *written = 0;
    if (nchar == 0) return DC_OK;
    const uint32_t C = (uint32_t)(NS_MAX_PAYLOAD - tl);
    const uint64_t nb = (nchar + C - 1) / C;
    const NsHdr full = ns_hdr(C, prefix, tl), last = ns_hdr(nchar - (nb - 1) * C, prefix, tl);
    const uint64_t threads = nchar < (1ull << 26) ? nchar : (1ull << 26);
    hipLaunchKernelGGL(k_ns_frame, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, (hipStream_t)dc_ctx_stream(c),
                       d_text, nchar, C, full, last, d_out);
    if (hipGetLastError() != hipSuccess) return DC_E_HIP;
    *written = ns_framed_size(nchar, tl, C);
    return DC_OK;
}

// the raw pass-through container of in[0..n) (n_ary_huffman.c:1806-1814), into host out
int ns_write_raw(const uint8_t *in, uint64_t n, uint8_t *out, uint64_t cap, uint64_t *out_len)
{
    const uint64_t C = NS_MAX_PAYLOAD - 2;
    const uint64_t need = n ? ns_framed_size(n, 2, C) : 5;   // empty input: "2:\n\n,"
    if (need > cap) return DC_E_CAPACITY;
    uint8_t *o = out;
    uint64_t i = 0;
    do {
        const uint64_t k = n - i < C ? n - i : C;
        o += ns_put_header(o, k + 2, "\n\n", 2);
        if (k) memcpy(o, in + i, k);
        o += k;
        *o++ = ',';
        i += k;
    } while (i < n);
    *out_len = (uint64_t)(o - out);
    return DC_OK;
}

struct NsBlock { uint64_t off, len; char type; };

// parse one netstring block at p (leading whitespace skipped, as sscanf("%i") does in
// get_compressed_block_length, :1825); false at the end of the input or on a malformed block
bool ns_next(const uint8_t *in, uint64_t m, uint64_t *p, NsBlock *b, bool *bad)
{
    uint64_t q = *p;
    while (q < m && (in[q] == ' ' || in[q] == '\n' || in[q] == '\t' || in[q] == '\r')) ++q;
    if (q >= m || in[q] == 0) { *p = q; return false; }
    char num[32];
    uint64_t k = 0;
    while (q + k < m && k < 31 && in[q + k] != ':') { num[k] = (char)in[q + k]; ++k; }
    if (q + k >= m || in[q + k] != ':' || k == 0) { *bad = true; return false; }
    num[k] = 0;
    char *end = nullptr;
    const long long len = strtoll(num, &end, 0);   // "%i": decimal, 0x hex, 0 octal
    if (end == num || len < 2 || len > (long long)NS_MAX_PAYLOAD) { *bad = true; return false; }
    const uint64_t d = q + k + 1;
    if (d + (uint64_t)len >= m || in[d + len] != ',' || in[d] != '\n') { *bad = true; return false; }
    b->type = (char)in[d + 1];
    b->off = d + 2;
    b->len = (uint64_t)len - 2;
    *p = d + len + 1;
    return true;
}

// key=value of a "#dc1" metadata block
bool ns_meta_get(const uint8_t *s, uint64_t len, const char *key, uint64_t *v)
{
    const size_t kl = strlen(key);
    for (uint64_t i = 0; i + kl + 1 < len; ++i) {
        if ((i == 0 || s[i - 1] == ' ') && memcmp(s + i, key, kl) == 0 && s[i + kl] == '=') {
            *v = strtoull((const char *)s + i + kl + 1, nullptr, 10);
            return true;
        }
    }
    return false;
}

// One Huffman segment of a netstring stream: its metadata, table and the text ranges of its
// index and data blocks.
struct NsSeg {
    uint64_t nary = 0, syms = 0, bits = 0, S = 0, M = 258;
    bool have_meta = false, have_table = false;
    int32_t lengths[DC_MAX_SYMS];
    uint64_t zchars = 0, ichars = 0;
};

}  // namespace

uint64_t dc_huff_netstring_bound(uint64_t n)
{
    return (n ? ns_framed_size(n, 2, NS_MAX_PAYLOAD - 2) : 5) + 16;   // the raw form: never exceeded
}

int dc_huff_compress_netstring(const uint8_t *in, uint64_t n, int n_ary, const int32_t *lengths, int max_symbol_value,
                               uint32_t sync_syms, uint8_t *out, uint64_t cap, uint64_t *out_len)
{
    if ((n && !in) || !out || !out_len || n_ary < 2 || n_ary > 16) return DC_E_ARG;
    if (lengths && (max_symbol_value < 0 || max_symbol_value >= DC_MAX_SYMS)) return DC_E_ARG;
    if (sync_syms != 0 && (sync_syms < 16 || sync_syms > DC_SYNC_MAX || (sync_syms & (sync_syms - 1))))
        return DC_E_ARG;
    const uint64_t raw_size = n ? ns_framed_size(n, 2, NS_MAX_PAYLOAD - 2) : 5;
    if (n == 0) return ns_write_raw(in, n, out, cap, out_len);
    HostState *s;
    RC(state(&s));
    dc_ctx *c = s->ctx;
    const uint8_t *d_in = nullptr;
    RC(dc_host_upload(in, n, &d_in));
    RC(s->hist.need(256 * 8 + 64));
    RC(s->table.need(sizeof(dc_dtable)));
    uint64_t *d_hist = (uint64_t *)s->hist.p, *d_total = d_hist + 256;
    dc_dtable *d_tab = (dc_dtable *)s->table.p;
    RC(dc_huff_hist(c, d_in, n, d_hist));
    const int M = lengths ? max_symbol_value : 258;
    if (lengths) {
        RC(s->lens.need((size_t)(M + 1) * 4));
        RC(dc_memcpy_h2d(c, s->lens.p, lengths, (size_t)(M + 1) * 4));
        RC(dc_huff_table_lengths(c, (const int32_t *)s->lens.p, M, n_ary, d_tab));
    } else {
        RC(dc_huff_table(c, d_hist, M, n_ary, d_tab));
    }
    int32_t maxbits = 0;
    if (dc_huff_table_status(c, d_tab, &maxbits) != DC_OK || maxbits <= 0 || maxbits > 32)
        return ns_write_raw(in, n, out, cap, out_len);   // no v1 stream for this table: raw block
    RC(dc_huff_plan(c, d_tab, d_total));
    uint64_t total = 0;
    RC(dc_memcpy_d2h(c, &total, d_total, 8));
    if (sync_syms == 0) sync_syms = dc_huff_choose_sync(n, total);
    const uint64_t ng = dc_huff_sync_groups(n, sync_syms), nc = dc_huff_sync_chunks(n, sync_syms);
    const uint64_t ib = ng * 8 + nc * 2;
    std::vector<int32_t> len_h(M + 1);
    RC(dc_memcpy_d2h(c, len_h.data(), d_tab->lengths, (size_t)(M + 1) * 4));   // as :1736-1741 writes them
    // metadata + table blocks (host), then index and data text (device, framed)
    char meta[160];
    const int ml = snprintf(meta, sizeof(meta), "\n#dc1 n=%d syms=%llu bits=%llu S=%u M=%d", n_ary,
                            (unsigned long long)n, (unsigned long long)total, sync_syms, M);
    std::vector<uint8_t> head(64 + ml + M + 1 + 16);
    uint8_t *h = head.data();
    h += ns_put_header(h, (uint64_t)ml, meta, (size_t)ml);
    *h++ = ',';
    char xp[16];
    const int xl = snprintf(xp, sizeof(xp), "\nX%d:", M);
    h += ns_put_header(h, (uint64_t)xl + M + 1, xp, (size_t)xl);
    for (int i = 0; i <= M; ++i) {
        const int L = len_h[i] > 0 ? len_h[i] : 0;
        if (L > 35) return ns_write_raw(in, n, out, cap, out_len);
        *h++ = (uint8_t)kLenDigits[L];
    }
    *h++ = ',';
    const uint64_t head_len = (uint64_t)(h - head.data());
    const char *ip = "\n#dcidx:";
    const char *zp = "\nZ";
    const uint64_t ichars = (ib * 8 + 5) / 6, zchars = (total + 5) / 6;
    const uint64_t need = head_len + ns_framed_size(ichars, 8, NS_MAX_PAYLOAD - 8) + ns_framed_size(zchars, 2, NS_MAX_PAYLOAD - 2);
    if (need >= raw_size) return ns_write_raw(in, n, out, cap, out_len);   // Huffman saves nothing
    if (need > cap) return DC_E_CAPACITY;
    const uint64_t words = dc_huff_words_needed(0, total);
    RC(s->out.need(words * 4));
    RC(s->sync.need(ib + 64));
    uint64_t *d_base = (uint64_t *)s->sync.p;
    uint16_t *d_len = (uint16_t *)(d_base + ng);
    RC(dc_memset(c, (uint8_t *)s->sync.p + ib, 0, 64));
    {   // a byte without a code (caller lengths that miss a byte of the input): raw block
        const int r = dc_huff_pack(c, d_in, n, d_tab, 0, (uint32_t *)s->out.p, words, d_base, d_len, sync_syms);
        if (r == DC_E_NOCODE) return ns_write_raw(in, n, out, cap, out_len);
        RC(r);
    }
    // text of index and payload, then the framed container, in one device buffer
    RC(s->aux.need(ichars + zchars + need + 64));
    uint8_t *d_itext = (uint8_t *)s->aux.p, *d_ztext = d_itext + ichars, *d_cont = d_ztext + zchars;
    uint64_t nci = 0, ncz = 0, wi = 0, wz = 0;
    RC(dc_huff_text(c, (const uint32_t *)s->sync.p, 0, ib * 8, DC_TEXT_BASE64URL, 2, (char *)d_itext, &nci));
    RC(dc_huff_text(c, (const uint32_t *)s->out.p, 0, total, DC_TEXT_BASE64URL, 2, (char *)d_ztext, &ncz));
    RC(ns_frame(c, d_itext, nci, ip, 8, d_cont + head_len, &wi));
    RC(ns_frame(c, d_ztext, ncz, zp, 2, d_cont + head_len + wi, &wz));
    if (head_len + wi + wz != need) return DC_E_STATE;
    memcpy(out, head.data(), head_len);
    RC(dc_memcpy_d2h(c, out + head_len, d_cont + head_len, wi + wz));
    *out_len = need;
    return DC_OK;
}

// Walk the blocks: out_n = decompressed size (raw bytes + symbols of every Huffman segment)
int dc_huff_netstring_info(const uint8_t *in, uint64_t m, uint64_t *out_n)
{
    if (!in || !out_n) return DC_E_ARG;
    uint64_t p = 0, tot = 0, v = 0;
    NsBlock b;
    bool bad = false;
    while (ns_next(in, m, &p, &b, &bad)) {
        if (b.type != '\n' && b.type != '#' && b.type != 'X' && b.type != 'Z') return DC_E_STREAM;   // :2067-2070
        if (b.type == '\n') tot += b.len;
        else if (b.type == '#' && b.len >= 4 && memcmp(in + b.off, "dc1 ", 4) == 0 &&
                 ns_meta_get(in + b.off, b.len, "syms", &v))
            tot += v;
    }
    if (bad) return DC_E_STREAM;
    *out_n = tot;
    return DC_OK;
}

int dc_huff_decompress_netstring(const uint8_t *in, uint64_t m, uint8_t *out, uint64_t cap, uint64_t *out_len)
{
    if (!in || !out_len) return DC_E_ARG;
    uint64_t n = 0;
    RC(dc_huff_netstring_info(in, m, &n));
    if (n > cap) return DC_E_CAPACITY;
    if (n && !out) return DC_E_ARG;
    *out_len = 0;
    if (n == 0) return DC_OK;
    HostState *s;
    RC(state(&s));
    dc_ctx *c = s->ctx;
    hipStream_t st = (hipStream_t)dc_ctx_stream(c);
    const uint8_t *d_src = nullptr;
    RC(dc_host_upload(in, m, &d_src));
    RC(s->out.need(n + 64));
    uint8_t *d_dst = (uint8_t *)s->out.p;
    std::vector<uint64_t> raw;            // (src, len, dst) triples of raw blocks
    uint64_t dpos = 0;                    // output position
    NsSeg seg;
    std::vector<uint64_t> zr, ir;         // text ranges of the current segment's Z / index blocks
    auto gather = [&](const std::vector<uint64_t> &r, uint8_t *dst) -> int {
        const uint64_t k = r.size() / 3;
        if (!k) return DC_OK;
        RC(s->lens.need(r.size() * 8));
        RC(dc_memcpy_h2d(c, s->lens.p, r.data(), r.size() * 8));
        hipLaunchKernelGGL(k_ns_gather, dim3((unsigned)(k < 65535 ? k : 65535)), dim3(256), 0, st, d_src,
                           (const uint64_t *)s->lens.p, k, dst);
        if (hipGetLastError() != hipSuccess) return DC_E_HIP;
        return dc_ctx_sync(c);
    };
    auto flush = [&]() -> int {   // decode the finished Huffman segment into d_dst + dpos
        if (!seg.have_meta && !seg.zchars) return DC_OK;
        if (!seg.have_meta || !seg.have_table || seg.nary < 2 || seg.nary > 16) return DC_E_STREAM;
        const uint32_t S = (uint32_t)seg.S;
        if (S < 16 || S > DC_SYNC_MAX || (S & (S - 1)) || seg.zchars != (seg.bits + 5) / 6) return DC_E_STREAM;
        const uint64_t ng = dc_huff_sync_groups(seg.syms, S), nc = dc_huff_sync_chunks(seg.syms, S);
        const uint64_t ib = ng * 8 + nc * 2;
        if (seg.ichars != (ib * 8 + 5) / 6 || dpos + seg.syms > n) return DC_E_STREAM;
        // index and data text -> contiguous device text -> bits
        RC(s->aux.need(seg.ichars + seg.zchars + 64));
        uint8_t *d_it = (uint8_t *)s->aux.p, *d_zt = d_it + seg.ichars;
        std::vector<uint64_t> r2;
        uint64_t o = 0;
        for (size_t i = 0; i < ir.size(); i += 2) { r2.push_back(ir[i]); r2.push_back(ir[i + 1]); r2.push_back(o); o += ir[i + 1]; }
        for (size_t i = 0; i < zr.size(); i += 2) { r2.push_back(zr[i]); r2.push_back(zr[i + 1]); r2.push_back(o); o += zr[i + 1]; }
        RC(gather(r2, d_it));
        const uint64_t words = dc_huff_words_needed(0, seg.bits);
        RC(s->in2.need(words * 4 + 64));
        RC(s->sync.need(ib + 64));
        RC(dc_memset(c, s->in2.p, 0, words * 4 + 64));
        RC(dc_huff_text_parse(c, (const char *)d_it, seg.ichars, DC_TEXT_BASE64URL, 2, ib * 8, (uint32_t *)s->sync.p));
        RC(dc_huff_text_parse_status(c));
        RC(dc_huff_text_parse(c, (const char *)d_zt, seg.zchars, DC_TEXT_BASE64URL, 2, seg.bits, (uint32_t *)s->in2.p));
        RC(dc_huff_text_parse_status(c));
        const int M = (int)seg.M;
        RC(s->table.need(sizeof(dc_dtable)));
        RC(s->hist.need((size_t)(M + 1) * 4));
        RC(dc_memcpy_h2d(c, s->hist.p, seg.lengths, (size_t)(M + 1) * 4));
        dc_dtable *d_tab = (dc_dtable *)s->table.p;
        RC(dc_huff_table_lengths(c, (const int32_t *)s->hist.p, M, (int)seg.nary, d_tab));
        int32_t mb = 0;
        if (dc_huff_table_status(c, d_tab, &mb) != DC_OK || mb > 32) return DC_E_STREAM;
        // decode into a 16-B aligned scratch when the segment does not start aligned
        uint8_t *dst = d_dst + dpos;
        const bool aligned = (((uintptr_t)dst) & 15) == 0;
        if (!aligned) RC(s->aux2.need(seg.syms + 64));
        uint64_t *d_base = (uint64_t *)s->sync.p;
        RC(dc_huff_decode(c, (const uint32_t *)s->in2.p, 0, words, d_base, (const uint16_t *)(d_base + ng), S,
                          seg.syms, d_tab, aligned ? dst : (uint8_t *)s->aux2.p));
        RC(dc_huff_decode_status(c));
        if (!aligned && hipMemcpyAsync(dst, s->aux2.p, seg.syms, hipMemcpyDeviceToDevice, st) != hipSuccess)
            return DC_E_HIP;
        dpos += seg.syms;
        seg = NsSeg();
        zr.clear();
        ir.clear();
        return DC_OK;
    };
    uint64_t p = 0;
    NsBlock b;
    bool bad = false;
    while (ns_next(in, m, &p, &b, &bad)) {
        const uint8_t *d = in + b.off;
        switch (b.type) {
        case '\n':   // raw pass-through (:2071-2076): the payload after the type bytes
            RC(flush());
            raw.push_back(b.off); raw.push_back(b.len); raw.push_back(dpos);
            dpos += b.len;
            break;
        case '#':
            if (b.len >= 4 && memcmp(d, "dc1 ", 4) == 0) {   // starts a Huffman segment
                RC(flush());
                uint64_t v = 0;
                seg.have_meta = ns_meta_get(d, b.len, "n", &seg.nary) && ns_meta_get(d, b.len, "syms", &seg.syms) &&
                                ns_meta_get(d, b.len, "bits", &seg.bits) && ns_meta_get(d, b.len, "S", &seg.S);
                if (ns_meta_get(d, b.len, "M", &v)) seg.M = v;
                if (!seg.have_meta || seg.M >= DC_MAX_SYMS) return DC_E_STREAM;
            } else if (b.len >= 6 && memcmp(d, "dcidx:", 6) == 0) {
                ir.push_back(b.off + 6); ir.push_back(b.len - 6);
                seg.ichars += b.len - 6;
            }   // other metadata: skipped (:2077-2080)
            break;
        case 'X': {   // "<M>:" then one length character per symbol 0..M (:1710-1747)
            char *e = nullptr;
            char num[16] = {0};
            memcpy(num, d, b.len < 15 ? b.len : 15);
            const long Mx = strtol(num, &e, 10);
            if (e == num || *e != ':' || Mx < 0 || Mx >= DC_MAX_SYMS) return DC_E_STREAM;
            const uint64_t h0 = (uint64_t)(e - num) + 1;
            if (b.len != h0 + (uint64_t)Mx + 1) return DC_E_STREAM;
            for (long i = 0; i <= Mx; ++i) {
                const char *q = strchr(kLenDigits, d[h0 + i]);
                if (!q || !d[h0 + i]) return DC_E_STREAM;
                seg.lengths[i] = (int32_t)(q - kLenDigits);
            }
            seg.M = (uint64_t)Mx;
            seg.have_table = true;
            break;
        }
        case 'Z':
            zr.push_back(b.off); zr.push_back(b.len);
            seg.zchars += b.len;
            break;
        default:
            return DC_E_STREAM;   // unknown block type (:2067-2070)
        }
    }
    if (bad) return DC_E_STREAM;
    RC(flush());
    if (dpos != n) return DC_E_STREAM;
    RC(gather(raw, d_dst));
    RC(dc_memcpy_d2h(c, out, d_dst, n));
    *out_len = n;
    return DC_OK;
}

// ---- host-buffer nybble / small wrappers (byte arrays, explicit lengths) --------------
static int run_bytes(int which, const uint8_t *in, uint64_t n, int modify, uint8_t *out, uint64_t cap,
                     uint64_t *out_len)
{
    HostState *s;
    RC(state(&s));
    const uint8_t *d_in = nullptr;
    RC(dc_host_upload(in, n, &d_in));
    const uint64_t outcap = 2 * n + 64;
    RC(s->out.need(outcap));
    uint64_t len = 0;
    uint8_t *d_out = (uint8_t *)s->out.p;
    switch (which) {
    case 0: RC(dc_nyb_compress(s->ctx, d_in, n, modify, d_out, &len)); break;
    case 1: RC(dc_nyb_decompress(s->ctx, d_in, n, modify, d_out, &len)); break;
    case 2: RC(dc_small_compress(s->ctx, d_in, n, d_out, &len)); break;
    default: RC(dc_small_decompress(s->ctx, d_in, n, d_out, &len)); break;
    }
    if (len > cap) return DC_E_CAPACITY;
    RC(dc_memcpy_d2h(s->ctx, out, d_out, len));
    *out_len = len;
    return DC_OK;
}

int dc_nyb_compress_host(const uint8_t *in, uint64_t n, int modify, uint8_t *out, uint64_t cap, uint64_t *len)
{ return run_bytes(0, in, n, modify, out, cap, len); }
int dc_nyb_decompress_host(const uint8_t *in, uint64_t m, int modify, uint8_t *out, uint64_t cap, uint64_t *len)
{ return run_bytes(1, in, m, modify, out, cap, len); }
int dc_small_compress_host(const uint8_t *in, uint64_t n, uint8_t *out, uint64_t cap, uint64_t *len)
{ return run_bytes(2, in, n, 0, out, cap, len); }
int dc_small_decompress_host(const uint8_t *in, uint64_t m, uint8_t *out, uint64_t cap, uint64_t *len)
{ return run_bytes(3, in, m, 0, out, cap, len); }

}  // extern "C"
