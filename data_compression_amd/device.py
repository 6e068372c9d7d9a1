"""Device-resident pipelines on torch tensors (HBM) over libdc_core.so.

`Codec` owns one dc_ctx bound to a HIP stream (torch's current stream by default, so
torch.cuda events and synchronisation see the kernels). Stages map 1:1 onto dc_gpu.h:

    hist = c.hist(x)                      # H1  histogram()             n_ary_huffman.c:461
    tab  = c.table(hist, n_ary)           # H2-H6 huffman()+convert()   :1161, :1382
    bits = c.plan(tab)                    # per-block bit counts + scan (:2485 formula)
    c.pack(x, tab, bit_base, words, sync, S)          # H7 encode (build-defined v1)
    c.decode(words, bit_base, sync, S, n, tab, out)   # H8 decode
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from ._lib import DcError, check, core

try:
    import torch
except Exception:  # pragma: no cover
    torch = None


def _ptr(t) -> int:
    if t is None:
        return None
    if isinstance(t, int):
        return t
    return t.data_ptr()


class Codec:
    _host_default = None

    def __init__(self, device: int = 0, stream=None, own_stream: bool = False):
        self.L = core()
        self.ctx = C.c_void_p()
        if own_stream:
            check("dc_ctx_create_owned", self.L.dc_ctx_create_owned(C.byref(self.ctx), device))
        else:
            # torch's current stream (its default stream has handle 0 = the HIP NULL stream)
            if stream is not None:
                handle = stream if isinstance(stream, int) else stream.cuda_stream
            elif torch is not None and torch.cuda.is_available():
                handle = torch.cuda.current_stream(device).cuda_stream
            else:
                handle = 0
            check("dc_ctx_create", self.L.dc_ctx_create(C.byref(self.ctx), device, handle or None))
        self.device = device
        self.table_bytes = int(self.L.dc_dtable_size())

    @classmethod
    def host_default(cls):
        if cls._host_default is None:
            cls._host_default = cls(own_stream=True)
        return cls._host_default

    def close(self):
        if self.ctx:
            self.L.dc_ctx_destroy(self.ctx)
            self.ctx = C.c_void_p()

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass

    # ---- helpers --------------------------------------------------------------------
    def sync(self):
        check("dc_ctx_sync", self.L.dc_ctx_sync(self.ctx))

    def timing(self, enable: bool):
        check("dc_ctx_set_timing", self.L.dc_ctx_set_timing(self.ctx, int(enable)))

    OPTIONS = {"hist_grid": 1, "pack_grid": 2, "decode_static_pct": 3, "decode_general": 4, "hist_prefetch": 5,
               "decode_variant": 6, "nyb_adec_v1": 7, "pack_block": 8, "nyb_wtile_off": 9}

    def set_option(self, name, value: int):
        """dc_ctx_set_option (dc_gpu.h DC_OPT_*): tuning knobs of this context."""
        check("dc_ctx_set_option", self.L.dc_ctx_set_option(self.ctx, self.OPTIONS.get(name, name), int(value)))

    def timings(self, max_n: int = 1024):
        names = (C.c_char_p * max_n)()
        ms = (C.c_float * max_n)()
        n = self.L.dc_ctx_timings(self.ctx, names, ms, max_n)
        if n < 0:
            raise DcError("dc_ctx_timings", n)
        return [(names[i].decode(), float(ms[i])) for i in range(n)]

    def _t(self, nbytes, dtype=None):
        return torch.empty(nbytes, dtype=dtype or torch.uint8, device=f"cuda:{self.device}")

    # ---- Huffman stages ---------------------------------------------------------------
    def hist(self, x, out=None):
        out = out if out is not None else self._t(256, torch.int64)
        check("dc_huff_hist", self.L.dc_huff_hist(self.ctx, _ptr(x), x.numel(), _ptr(out)))
        return out

    def table(self, hist, n_ary: int, max_symbol_value: int = 258, out=None):
        out = out if out is not None else self._t(self.table_bytes)
        check("dc_huff_table", self.L.dc_huff_table(self.ctx, _ptr(hist), max_symbol_value, n_ary, _ptr(out)))
        return out

    def alloc_table(self):
        """An uninitialised device table (dc_dtable bytes), e.g. a broadcast target."""
        return self._t(self.table_bytes)

    def table_freq(self, freq, n_ary: int, max_symbol_value: int, out=None):
        out = out if out is not None else self._t(self.table_bytes)
        check("dc_huff_table_freq",
              self.L.dc_huff_table_freq(self.ctx, _ptr(freq), max_symbol_value, n_ary, _ptr(out)))
        return out

    def table_lengths(self, lengths, n_ary: int, max_symbol_value: int = 258, out=None):
        out = out if out is not None else self._t(self.table_bytes)
        check("dc_huff_table_lengths",
              self.L.dc_huff_table_lengths(self.ctx, _ptr(lengths), max_symbol_value, n_ary, _ptr(out)))
        return out

    def table_status(self, tab):
        mb = C.c_int32(0)
        st = self.L.dc_huff_table_status(self.ctx, _ptr(tab), C.byref(mb))
        return st, mb.value

    def plan(self, tab, total=None):
        total = total if total is not None else self._t(1, torch.int64)
        check("dc_huff_plan", self.L.dc_huff_plan(self.ctx, _ptr(tab), _ptr(total)))
        self._last_total = total
        return total

    @property
    def fused_plan(self) -> bool:
        """Whether the library has dc_huff_encode_plan (hist + table + plan in one launch)."""
        return hasattr(self.L, "dc_huff_encode_plan")

    def encode_plan(self, x, n_ary: int, max_symbol_value: int = 258, hist=None, table=None, total=None):
        """hist -> table -> plan in one launch (dc_huff_encode_plan): the histogram kernel's
        last workgroup builds the table and the payload bit count. Returns (hist, table, total)."""
        hist = hist if hist is not None else self._t(256, torch.int64)
        table = table if table is not None else self._t(self.table_bytes)
        total = total if total is not None else self._t(1, torch.int64)
        check("dc_huff_encode_plan", self.L.dc_huff_encode_plan(self.ctx, _ptr(x), x.numel(), max_symbol_value, n_ary,
                                                                _ptr(hist), _ptr(table), _ptr(total)))
        self._last_total = total
        return hist, table, total

    def table_plan(self, hist, n_ary: int, max_symbol_value: int = 258, out=None, total=None):
        """table of `hist` + the plan of this context's last hist() under it, one launch
        (dc_huff_table_plan: a shard's encode after the all-reduce). Returns (table, total)."""
        table = out if out is not None else self._t(self.table_bytes)
        total = total if total is not None else self._t(1, torch.int64)
        check("dc_huff_table_plan", self.L.dc_huff_table_plan(self.ctx, _ptr(hist), max_symbol_value, n_ary,
                                                              _ptr(table), _ptr(total)))
        self._last_total = total
        return table, total

    def plan_total(self) -> int:
        return int(self._last_total.item())

    def words_needed(self, bit_base: int, total_bits: int) -> int:
        return int(self.L.dc_huff_words_needed(bit_base, total_bits))

    def sync_sizes(self, n: int, sync_syms: int):
        """(groups, chunks) of the sync index for n symbols."""
        return (int(self.L.dc_huff_sync_groups(n, sync_syms)), int(self.L.dc_huff_sync_chunks(n, sync_syms)))

    def alloc_sync(self, n: int, sync_syms: int):
        g, c = self.sync_sizes(n, sync_syms)   # (2 lengths of slack past the view: the kernels add into whole dwords)
        return (self._t(max(g, 1), torch.int64), self._t(max(c, 1) + 2, torch.int16)[: max(c, 1)])

    def pack(self, x, tab, bit_base, words, sync, sync_syms):
        base, lens = sync if sync is not None else (None, None)
        check("dc_huff_pack", self.L.dc_huff_pack(self.ctx, _ptr(x), x.numel(), _ptr(tab), bit_base, _ptr(words),
                                                  words.numel(), _ptr(base), _ptr(lens),
                                                  sync_syms if sync is not None else 0))

    def pack_async(self, x, tab, bit_base, words, sync, sync_syms):
        """bit_base: an int, or a one-element int64 device tensor read by the kernels
        (dc_huff_pack_async_dev: no host read of a gathered offset)."""
        base, lens = sync if sync is not None else (None, None)
        S = sync_syms if sync is not None else 0
        if hasattr(bit_base, "data_ptr"):
            check("dc_huff_pack_async_dev",
                  self.L.dc_huff_pack_async_dev(self.ctx, _ptr(x), x.numel(), _ptr(tab), _ptr(bit_base), _ptr(words),
                                                words.numel(), _ptr(base), _ptr(lens), S))
            return
        check("dc_huff_pack_async",
              self.L.dc_huff_pack_async(self.ctx, _ptr(x), x.numel(), _ptr(tab), bit_base, _ptr(words),
                                        words.numel(), _ptr(base), _ptr(lens), S))

    def pack_status(self, tab, gen=None):
        """Outcome of the last plan + pack (gen=None), or of the plan whose plan_gen() was gen."""
        if gen is None:
            return int(self.L.dc_huff_pack_status(self.ctx, _ptr(tab)))
        return int(self.L.dc_huff_pack_status_gen(self.ctx, _ptr(tab), gen))

    def plan_gen(self) -> int:
        """Identity of the last plan on this context (dc_huff_plan_gen), for pack_status(gen=)."""
        return int(self.L.dc_huff_plan_gen(self.ctx))

    def decode(self, words, bit_base, sync, sync_syms, n, tab, out):
        """bit_base: an int, or a one-element int64 device tensor (dc_huff_decode_dev)."""
        base, lens = sync
        if hasattr(bit_base, "data_ptr"):
            check("dc_huff_decode_dev", self.L.dc_huff_decode_dev(self.ctx, _ptr(words), _ptr(bit_base), words.numel(),
                                                                  _ptr(base), _ptr(lens), sync_syms, n, _ptr(tab),
                                                                  _ptr(out)))
            return
        check("dc_huff_decode", self.L.dc_huff_decode(self.ctx, _ptr(words), bit_base, words.numel(), _ptr(base),
                                                      _ptr(lens), sync_syms, n, _ptr(tab), _ptr(out)))

    def copy_probe(self, src, dst):
        """dc_copy_probe: a float4 device-to-device copy (the HBM reference rate of bench.py)."""
        check("dc_copy_probe", self.L.dc_copy_probe(self.ctx, _ptr(src), _ptr(dst), min(src.numel() * src.element_size(),
                                                                                       dst.numel() * dst.element_size())))

    def decode_status(self):
        return int(self.L.dc_huff_decode_status(self.ctx))

    def decode_redo_count(self) -> int:
        """Chunks of the last S = 64 decode that took the exact redo (diagnostic)."""
        v = C.c_uint64(0)
        check("dc_huff_decode_redo_count", self.L.dc_huff_decode_redo_count(self.ctx, C.byref(v)))
        return int(v.value)

    # ---- small front-end shard bodies (dist.ShardedSmall) --------------------
    def small_body(self, y, left_halo: bool, nelem: int, head: bytes = b"", out=None):
        """Front-end body of stream bytes y[1..nelem] (y[0]: left context; y[nelem+1], when
        present, the right halo) -> uint8 device tensor, after the bytes `head` (written in
        place, no copy of the body). out: optional buffer of >= nelem + len(head) bytes."""
        h = len(head)
        if out is None:
            out = self._t(max(nelem + h, 1))
        elif out.numel() < nelem + h or out.dtype != torch.uint8 or not out.is_contiguous():
            raise ValueError("small_body output: contiguous uint8 of >= nelem + len(head) bytes")
        if h:
            out[:h] = torch.tensor(list(head), dtype=torch.uint8, device=out.device)
        n = C.c_uint64(0)
        check("dc_small_compress_body", self.L.dc_small_compress_body(self.ctx, _ptr(y), y.numel(), int(left_halo),
                                                                      nelem, _ptr(out) + h, C.byref(n)))
        return out[: h + n.value]

    def small_body_plan(self, y, left_halo: bool, nelem: int) -> int:
        """Length of small_body(y, left_halo, nelem) without writing it (dc_small_compress_body_plan);
        small_body_write then writes it wherever the caller places it."""
        n = C.c_uint64(0)
        check("dc_small_compress_body_plan", self.L.dc_small_compress_body_plan(self.ctx, _ptr(y), y.numel(),
                                                                                int(left_halo), nelem, C.byref(n)))
        return n.value

    def small_body_write(self, y, left_halo: bool, nelem: int, out, head: bytes = b""):
        """The planned body after `head`, into out (>= len(head) + planned bytes) -> view of out."""
        h = len(head)
        if out.dtype != torch.uint8 or not out.is_contiguous() or out.numel() < h:
            raise ValueError("small_body_write output: contiguous uint8")
        if h:
            out[:h] = torch.tensor(list(head), dtype=torch.uint8, device=out.device)
        n = C.c_uint64(0)
        check("dc_small_compress_body_write", self.L.dc_small_compress_body_write(
            self.ctx, _ptr(y), y.numel(), int(left_halo), nelem, _ptr(out) + h, C.byref(n)))
        return out[: h + n.value]

    def _dec_out(self, seg, out):
        if out is None:
            return self._t(max(2 * seg.numel(), 1))
        if out.numel() < 2 * seg.numel() or out.dtype != torch.uint8 or not out.is_contiguous():
            raise ValueError("front-end decode output: contiguous uint8 of >= 2 * input bytes")
        return out

    def small_decompress(self, seg, out=None):
        """A front-end stream that starts with its type byte (rank 0's segment). out: an
        optional preallocated buffer of >= 2 * seg.numel() bytes (the result is a view)."""
        out = self._dec_out(seg, out)
        n = C.c_uint64(0)
        check("dc_small_decompress", self.L.dc_small_decompress(self.ctx, _ptr(seg), seg.numel(), _ptr(out),
                                                                C.byref(n)))
        return out[: n.value]

    def small_decompress_body(self, seg, out=None):
        out = self._dec_out(seg, out)
        n = C.c_uint64(0)
        check("dc_small_decompress_body", self.L.dc_small_decompress_body(self.ctx, _ptr(seg), seg.numel(),
                                                                          _ptr(out), C.byref(n)))
        return out[: n.value]

    # ---- nybble codec, whole streams and shard bodies (dist.ShardedNybble) -----
    def nyb_compress(self, x, modify: bool, out=None):
        """compress_bytestring (nybble_compression.c:887-1038) of device bytes x (into `out`
        when given: at least x.numel() + 2 bytes)."""
        if out is None:
            out = self._t(x.numel() + 2)
        elif out.numel() < x.numel() + 2 or out.dtype != torch.uint8 or not out.is_contiguous():
            raise ValueError("nyb_compress output: contiguous uint8 of >= n + 2 bytes")
        n = C.c_uint64(0)
        check("dc_nyb_compress", self.L.dc_nyb_compress(self.ctx, _ptr(x), x.numel(), int(modify), _ptr(out),
                                                        C.byref(n)))
        return out[: n.value]

    def nyb_decompress(self, comp, modify: bool, out=None):
        """decompress_bytestring (nybble_compression.c:734-817) of device bytes comp (into
        `out`, any alignment, when given: at least 2 * comp.numel() bytes)."""
        if out is None:
            out = self._t(max(2 * comp.numel(), 1))
        elif out.numel() < 2 * comp.numel():
            raise ValueError("out holds fewer than 2 * comp.numel() bytes")
        n = C.c_uint64(0)
        check("dc_nyb_decompress", self.L.dc_nyb_decompress(self.ctx, _ptr(comp), comp.numel(), int(modify),
                                                            _ptr(out), C.byref(n)))
        return out[: n.value]

    def nyb_compress_chunked(self, x, modify: bool, chunk: int = 1 << 16):
        """DCNK container: chunks of `chunk` bytes, each the reference stream of that chunk."""
        cap = int(self.L.dc_nyb_chunked_bound(x.numel(), chunk))
        out = self._t(cap)
        n = C.c_uint64(0)
        check("dc_nyb_compress_chunked", self.L.dc_nyb_compress_chunked(self.ctx, _ptr(x), x.numel(), int(modify),
                                                                        chunk, _ptr(out), cap, C.byref(n)))
        return out[: n.value]

    def nyb_decompress_chunked(self, comp):
        n, mod, K = C.c_uint64(0), C.c_int32(0), C.c_uint32(0)
        check("dc_nyb_chunked_info", self.L.dc_nyb_chunked_info(self.ctx, _ptr(comp), comp.numel(), C.byref(n),
                                                                C.byref(mod), C.byref(K)))
        out = self._t(max(n.value, 1))
        got = C.c_uint64(0)
        check("dc_nyb_decompress_chunked", self.L.dc_nyb_decompress_chunked(self.ctx, _ptr(comp), comp.numel(),
                                                                            _ptr(out), n.value, C.byref(got)))
        return out[: got.value]

    def nyb_decompress_batch(self, data, offsets, modify: bool, out_cap: int | None = None):
        """dc_nyb_decompress_batch: streams data[offsets[i]:offsets[i+1]] (device uint8 data,
        device int64 offsets, count + 1 entries) decoded one lane per stream. Returns
        (output bytes, output offsets), both device tensors."""
        count = offsets.numel() - 1
        out_off = self._t(count + 1, torch.int64)
        cap = out_cap if out_cap is not None else 2 * data.numel() + 16
        out = self._t(max(cap, 1))
        tot = C.c_uint64(0)
        check("dc_nyb_decompress_batch", self.L.dc_nyb_decompress_batch(self.ctx, _ptr(data), _ptr(offsets), count,
                                                                        int(modify), _ptr(out), cap, _ptr(out_off),
                                                                        C.byref(tot)))
        return out[: tot.value], out_off

    def nyb_mtf_summary(self, y):
        """Move-to-front lists after elements y[1..] from empty lists: (lists[16][8], cnt[16])."""
        lists = np.zeros(128, np.uint8)
        cnt = np.zeros(16, np.uint8)
        check("dc_nyb_mtf_summary", self.L.dc_nyb_mtf_summary(self.ctx, _ptr(y), y.numel(), lists.ctypes.data,
                                                              cnt.ctypes.data))
        return lists.reshape(16, 8), cnt

    def nyb_body_plan(self, y, modify: bool, lists=None):
        """(c0, c1, s0, s1, last_rank) of the shard's elements y[1..] (dc_nyb_body_plan)."""
        plan = np.zeros(5, np.uint64)
        la = np.ascontiguousarray(lists, dtype=np.uint8) if modify else None
        check("dc_nyb_body_plan", self.L.dc_nyb_body_plan(self.ctx, _ptr(y), y.numel(), int(modify),
                                                          la.ctypes.data if modify else None, plan.ctypes.data))
        return [int(v) for v in plan]

    def _headed(self, cap, head):
        out = self._t(max(cap + len(head), 1))
        if head:
            out[: len(head)] = torch.tensor(list(head), dtype=torch.uint8, device=out.device)
        return out

    def nyb_body_write(self, y, modify: bool, pend_rank: int, is_last: bool, head: bytes = b""):
        """Body of the shard's elements y[1..] after the bytes `head` (written in place)."""
        h = len(head)
        out = self._headed(2 * y.numel(), head)
        n = C.c_uint64(0)
        st = C.c_int32(0)
        check("dc_nyb_body_write", self.L.dc_nyb_body_write(self.ctx, _ptr(y), y.numel(), int(modify), pend_rank,
                                                            int(is_last), _ptr(out) + h, C.byref(n), C.byref(st)))
        return out[: h + n.value]

    def nyb_dbody_plan(self, y, m: int):
        plan = np.zeros(4, np.uint64)
        check("dc_nyb_dbody_plan", self.L.dc_nyb_dbody_plan(self.ctx, _ptr(y), y.numel(), m, plan.ctypes.data))
        return [int(v) for v in plan]

    def nyb_dbody_write(self, y, m: int, s_in: int, head: bytes = b""):
        h = len(head)
        out = self._headed(2 * m, head)
        n = C.c_uint64(0)
        st = C.c_int32(0)
        check("dc_nyb_dbody_write", self.L.dc_nyb_dbody_write(self.ctx, _ptr(y), y.numel(), m, s_in, _ptr(out) + h,
                                                              C.byref(n), C.byref(st)))
        return out[: h + n.value]

    # ---- digit text: formats as dc_gpu.h DC_TEXT_* ------------------------
    TEXT_FORMATS = {"base64url": 0, "base16": 1, "digits": 2, "z85": 3, "trits5": 4}

    def text_bits(self, fmt, n_ary: int) -> int:
        """Bits per character of a text format (0: unsupported for this n)."""
        return int(self.L.dc_huff_text_bits(self.TEXT_FORMATS.get(fmt, fmt), n_ary))

    def text(self, words, bit_base: int, bits: int, fmt, n_ary: int):
        """Digit text of bits [bit_base, bit_base+bits) of `words` -> uint8 device tensor."""
        f = self.TEXT_FORMATS.get(fmt, fmt)
        b = self.text_bits(f, n_ary)
        if b == 0:
            raise ValueError(f"text format {fmt} does not support n={n_ary}")
        out = self._t(max((bits + b - 1) // b, 1))
        nc = C.c_uint64(0)
        check("dc_huff_text", self.L.dc_huff_text(self.ctx, _ptr(words), bit_base, bits, f, n_ary, _ptr(out),
                                                  C.byref(nc)))
        return out[: nc.value]

    def text_parse(self, text, fmt, n_ary: int, bits: int):
        """Inverse of text(): uint8 device tensor of characters -> int32 words holding the
        first `bits` bits. Raises DcError on an invalid character."""
        f = self.TEXT_FORMATS.get(fmt, fmt)
        words = self._t(max((bits + 31) // 32, 1), torch.int32)
        check("dc_huff_text_parse", self.L.dc_huff_text_parse(self.ctx, _ptr(text), text.numel(), f, n_ary, bits,
                                                              _ptr(words)))
        check("dc_huff_text_parse_status", self.L.dc_huff_text_parse_status(self.ctx))
        return words

    def default_sync(self, n: int) -> int:
        return int(self.L.dc_huff_default_sync(n))

    def choose_sync(self, n: int, total_bits: int) -> int:
        return int(self.L.dc_huff_choose_sync(n, total_bits))

    def encode(self, x, n_ary: int = 2, sync_syms: int | None = None, bit_base: int = 0):
        """hist -> table -> plan -> pack on one device. Returns dict of device tensors."""
        n = x.numel()
        if hasattr(self.L, "dc_huff_encode_plan"):
            hist, tab, total = self.encode_plan(x, n_ary)
        else:   # an older diagnostic library (tools/, DC_CORE_LIB): the three launches
            hist = self.hist(x)
            tab = self.table(hist, n_ary)
            total = self.plan(tab)
        bits = int(total.item())
        S = sync_syms or self.choose_sync(n, bits)
        words = self._t(self.words_needed(bit_base, bits), torch.int32)
        sync = self.alloc_sync(n, S)
        self.pack(x, tab, bit_base, words, sync, S)
        return {"hist": hist, "table": tab, "bits": bits, "words": words, "sync": sync, "S": S,
                "bit_base": bit_base, "n": n}

    def decode_into(self, enc, out):
        self.decode(enc["words"], enc["bit_base"], enc["sync"], enc["S"], enc["n"], enc["table"], out)

    # ---- C5 fused front-end encode (small_compression.c front-end, then Huffman; one pass) -----
    def small_huff_plan(self, x, n_ary: int = 16, max_symbol_value: int = 258, hist=None, table=None, total=None):
        """dc_small_huff_plan: histogram of the front-end output of x (never written), table and
        plan total in one launch. Returns (hist, table, total); DcError DC_E_FALLBACK for n < 2."""
        hist = hist if hist is not None else self._t(256, torch.int64)
        table = table if table is not None else self._t(self.table_bytes)
        total = total if total is not None else self._t(1, torch.int64)
        check("dc_small_huff_plan", self.L.dc_small_huff_plan(self.ctx, _ptr(x), x.numel(), max_symbol_value, n_ary,
                                                              _ptr(hist), _ptr(table), _ptr(total)))
        self._last_total = total
        return hist, table, total

    def small_huff_pack_async(self, x, tab, bit_base, words, sync, sync_syms):
        base, lens = sync
        check("dc_small_huff_pack_async",
              self.L.dc_small_huff_pack_async(self.ctx, _ptr(x), x.numel(), _ptr(tab), bit_base, _ptr(words),
                                              words.numel(), _ptr(base), _ptr(lens), sync_syms))

    # ---- the same for one shard of the stream (dist.ShardedSmall at world > 1) -------------
    def small_shard_hist(self, x, shard, hist=None):
        """dc_small_huff_shard_hist: the histogram of the shard's front-end output; shard = the
        4 int64 of FeShard on the device (global bit, first symbol, byte before, byte after)."""
        hist = hist if hist is not None else self._t(256, torch.int64)
        check("dc_small_huff_shard_hist", self.L.dc_small_huff_shard_hist(self.ctx, _ptr(x), x.numel(), _ptr(shard),
                                                                          _ptr(hist)))
        return hist

    def small_shard_pack_async(self, x, tab, shard, words, sync, gsync, sync_syms):
        """dc_small_huff_shard_pack_async: codes at the global bit shard[0], the local sync index
        into sync, this shard's part of the stream's sync index into gsync."""
        base, lens = sync
        gbase, glens = gsync
        check("dc_small_huff_shard_pack_async",
              self.L.dc_small_huff_shard_pack_async(self.ctx, _ptr(x), x.numel(), _ptr(tab), _ptr(shard), _ptr(words),
                                                    words.numel(), _ptr(base), _ptr(lens), _ptr(gbase), _ptr(glens),
                                                    sync_syms))

    def small_huff_symbols(self) -> int:
        v = C.c_uint64(0)
        check("dc_small_huff_symbols", self.L.dc_small_huff_symbols(self.ctx, C.byref(v)))
        return int(v.value)

    def small_huff_encode(self, x, n_ary: int = 16, sync_syms: int = 64, bit_base: int = 0, words=None, sync=None):
        """The C5 encode of device bytes x: the front-end (small_compression.c:582-665) and the
        n-ary Huffman code of its output M in one pass over x, M never written. Returns the
        dict of encode() for M ("n" = symbols of M) with "fused": True, bit-identical to
        small_compress + encode. When the fused path does not apply (DC_E_FALLBACK: LITERAL
        output, every byte value present in M, an over-long block) the two stages run and
        "fused" is False. words / sync: optional preallocated buffers (sync for n + 1 symbols)."""
        n = x.numel()
        try:
            hist, tab, total = self.small_huff_plan(x, n_ary)
        except DcError as e:
            if e.rc != -8:
                raise
            return self._small_huff_two_stage(x, n_ary, sync_syms, bit_base)
        bits = int(total.item())
        need = self.words_needed(bit_base, bits)
        if words is None or words.numel() < need:
            words = self._t(need, torch.int32)
        sync = sync if sync is not None else self.alloc_sync(n + 1, sync_syms)
        self.small_huff_pack_async(x, tab, bit_base, words, sync, sync_syms)
        st = self.pack_status(tab)
        if st == -8:
            return self._small_huff_two_stage(x, n_ary, sync_syms, bit_base)
        check("dc_small_huff_pack_async", st)
        m = self.small_huff_symbols()
        ng, nch = self.sync_sizes(m, sync_syms)   # the index of m symbols (the buffers hold n + 1)
        return {"hist": hist, "table": tab, "bits": bits, "words": words, "S": sync_syms, "bit_base": bit_base,
                "sync": (sync[0][: max(ng, 1)], sync[1][: max(nch, 1)]), "n": m, "fused": True}

    def _small_huff_two_stage(self, x, n_ary, sync_syms, bit_base):
        fe = self._t(x.numel() + 64)
        m = C.c_uint64(0)
        check("dc_small_compress", self.L.dc_small_compress(self.ctx, _ptr(x), x.numel(), _ptr(fe), C.byref(m)))
        enc = self.encode(fe[: m.value], n_ary=n_ary, sync_syms=sync_syms, bit_base=bit_base)
        enc["fused"] = False
        return enc

    def small_huff_decode(self, enc, out=None, mbuf=None):
        """Huffman decode of M, then the front-end inverse (dc_small_huff_decode: the inverse
        takes the decoder's per-group counts instead of a counting pass of its own): the input
        bytes, a view of out (>= 2 * enc["n"] bytes) when given. mbuf: optional buffer for M."""
        m = enc["n"]
        mbuf = mbuf if mbuf is not None else self._t(max(m, 1) + 16)
        out = self._dec_out(mbuf[: m], out)
        n = C.c_uint64(0)
        base, lens = enc["sync"]
        bb = enc["bit_base"]
        if hasattr(bb, "data_ptr"):   # (device-resident offset: the two stages)
            self.decode(enc["words"], bb, enc["sync"], enc["S"], m, enc["table"], mbuf)
            return self.small_decompress(mbuf[: m], out=out)
        check("dc_small_huff_decode", self.L.dc_small_huff_decode(
            self.ctx, _ptr(enc["words"]), bb, enc["words"].numel(), _ptr(base), _ptr(lens), enc["S"], m,
            _ptr(enc["table"]), _ptr(mbuf), _ptr(out), C.byref(n)))
        return out[: n.value]

    # ---- allocation helpers (the engine interface used by dist.ShardedHuffman) -----------
    def alloc_words(self, bit_base: int, bits: int):
        return self._t(self.words_needed(bit_base, bits), torch.int32)

    def alloc_bytes(self, n: int):
        return self._t(max(n, 1))

    # ---- host helpers -------------------------------------------------------------------
    def histogram_host(self, x: np.ndarray, max_symbol_value: int = 258) -> np.ndarray:
        from ._lib import vp
        n = x.size
        d_in = C.c_void_p()
        d_h = C.c_void_p()
        check("dc_malloc", self.L.dc_malloc(C.byref(d_in), n + 64))
        check("dc_malloc", self.L.dc_malloc(C.byref(d_h), 256 * 8))
        try:
            if n:
                check("h2d", self.L.dc_memcpy_h2d(self.ctx, d_in, x.ctypes.data_as(vp), n))
            check("dc_huff_hist", self.L.dc_huff_hist(self.ctx, d_in, n, d_h))
            h = np.zeros(256, dtype=np.uint64)
            check("d2h", self.L.dc_memcpy_d2h(self.ctx, h.ctypes.data_as(vp), d_h, 256 * 8))
        finally:
            self.L.dc_free(d_in)
            self.L.dc_free(d_h)
        out = np.zeros(max_symbol_value + 1, dtype=np.int64)
        k = min(256, max_symbol_value + 1)
        out[:k] = h[:k].astype(np.int64)
        return out
