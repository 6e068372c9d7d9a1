// dc_host.hip -- host-buffer entry points of libdc_core.so: a per-thread device context
// with growable scratch buffers, and the "DCH1" Huffman container built on
// the device-resident stages of dc_core.hip. Host code here only moves bytes and
// assembles headers; every byte of payload is produced and consumed by GPU kernels.

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

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
    Buf in, out, sync, table, hist, lens, aux;
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

int dc_huff_container_info(const uint8_t *in, uint64_t m, uint64_t *n, int *n_ary, uint64_t *bits)
{
    if (!in || m < kHeader || get32(in) != kMagic || in[4] != 1) return DC_E_STREAM;
    if (n) *n = get64(in + 8);
    if (n_ary) *n_ary = in[5];
    if (bits) *bits = get64(in + 16);
    return DC_OK;
}

int dc_huff_decompress_host(const uint8_t *in, uint64_t m, uint8_t *out, uint64_t cap, uint64_t *out_len)
{
    if (!in || !out_len) return DC_E_ARG;
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
