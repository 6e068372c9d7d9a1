"""CPU engine for the multi-rank orchestration tests (TEST INFRASTRUCTURE).

Implements the engine interface of data_compression_amd.device.Codec on CPU tensors with
the oracle, so data_compression_amd.dist.ShardedHuffman can be exercised with gloo
process groups in a container without a GPU. The product engine is device.Codec.
"""
import numpy as np
import torch

from oracle import oracle as orc


class CpuEngine:
    def __init__(self):
        self._hist_in = None

    def hist(self, x, out=None):
        self._hist_in = x
        return torch.from_numpy(orc.histogram(x.numpy()).astype(np.int64))

    # the table travels as one int64 tensor (dist broadcast): n_ary, lengths[259],
    # enc_len[259], enc_val[259], code[256], nbits[256]
    _TAB_LEN = 1 + 3 * 259 + 2 * 256

    def table(self, hist, n_ary, out=None):
        h = hist.numpy().astype(np.uint64)
        L = orc.huffman_lengths(h, n_ary)
        el, ev = orc.canonical(L, n_ary)
        code, nb, mx = orc.bitcodes(el, ev, n_ary)
        assert 0 < mx <= 32
        t = np.concatenate([[n_ary], L, el, ev, code, nb]).astype(np.int64)
        assert t.size == self._TAB_LEN
        return torch.from_numpy(t)

    def alloc_table(self):
        return torch.zeros(self._TAB_LEN, dtype=torch.int64)

    @staticmethod
    def _tab(t):
        a = t.numpy()
        L, el, ev = a[1:260].astype(np.int32), a[260:519].astype(np.int32), a[519:778].astype(np.uint32)
        return {"n_ary": int(a[0]), "L": L, "el": el, "ev": ev, "code": a[778:1034].astype(np.uint32),
                "nb": a[1034:1290].astype(np.uint8)}

    def plan(self, tab, total=None):
        tab = self._tab(tab)
        h = orc.histogram(self._hist_in.numpy()).astype(np.int64)
        self._total = int((h * tab["nb"].astype(np.int64)).sum())
        return torch.tensor([self._total], dtype=torch.int64)

    def table_plan(self, hist, n_ary, out=None, total=None):
        """dc_huff_table_plan: the table of hist and this engine's last hist() planned under it."""
        tab = self.table(hist, n_ary, out=out)
        return tab, self.plan(tab, total=total)

    def plan_total(self):
        return self._total

    def alloc_words(self, bit_base, bits):
        return torch.zeros(((bit_base & 31) + bits + 31) // 32 + 24, dtype=torch.int32)

    def alloc_sync(self, n, S):
        c = (n + S - 1) // S
        return (torch.zeros(max((c + 63) // 64, 1), dtype=torch.int64), torch.zeros(max(c, 1) + 2, dtype=torch.int16)[: max(c, 1)])

    def sync_sizes(self, n, S):
        c = (n + S - 1) // S
        return (c + 63) // 64, c

    def alloc_bytes(self, n):
        return torch.zeros(max(n, 1), dtype=torch.uint8)

    def pack_async(self, x, tab, bit_base, words, sync, S):
        bit_base = int(bit_base)   # an int, or a one-element tensor (device engine: read by the kernels)
        tab = self._tab(tab)
        xs = x.numpy()
        payload, bits, idx = orc.huff_pack(xs, tab["code"], tab["nb"], bit_base=bit_base, sync_syms=S)
        w = words.numpy().view(np.uint8)
        off = (bit_base >> 3) - ((bit_base >> 5) << 2)
        w[:] = 0
        w[off: off + len(payload)] = payload
        base, lens = orc.sync_compact(idx, bit_base, bits)
        sync[0][: len(base)] = torch.from_numpy(base.astype(np.int64))
        sync[1][: len(lens)] = torch.from_numpy(lens.view(np.int16))

    def pack_status(self, tab, gen=None):
        return 0   # the oracle pack above either writes the whole stream or raises

    def plan_gen(self):
        return 0

    def decode(self, words, bit_base, sync, S, n, tab, out):
        bit_base = int(bit_base)
        tab = self._tab(tab)
        bits_all = np.unpackbits(words.numpy().view(np.uint8))
        stream = np.packbits(bits_all[bit_base & 31:])
        total = int(sync[1][: (n + S - 1) // S].numpy().view(np.uint16).astype(np.int64).sum())
        y = orc.huff_unpack(stream, total, n, tab["el"], tab["ev"], tab["n_ary"])
        out[:n] = torch.from_numpy(y)

    # ---- the fused C5 encode of a shard (dist.ShardedSmall at world > 1), restated ----------
    @staticmethod
    def _shard_syms(x, shard):
        """The front-end output M of a shard (small_compression.c:582-665; shard = (global bit,
        first symbol, byte before or -1, byte after or -1)): a pair ' ' + lowercase letter is
        the symbol letter | 0x80 at its second byte, nothing at its first; the stream's first
        shard begins with the type byte 8 and a raw first byte."""
        a = x.numpy().astype(np.int64)
        left, right = int(shard[2]), int(shard[3])
        first = left < 0
        low = (a >= ord("a")) & (a <= ord("z"))
        prev = np.concatenate([[max(left, 0)], a[:-1]])
        nxt = np.concatenate([a[1:], [max(right, 0)]])
        nlow = (nxt >= ord("a")) & (nxt <= ord("z"))
        i = np.arange(a.size)
        sec = (prev == ord(" ")) & low & ((i >= 2) | (not first))
        start = (a == ord(" ")) & nlow & ((i >= 1) | (not first))
        sym = np.where(sec, a | 0x80, a)[~start]
        return np.concatenate([[8] if first else [], sym]).astype(np.uint8)

    @staticmethod
    def _check_granules(x):
        # the HIP kernels read a shard as 16-B granules: dc_small_huff_shard_hist returns
        # DC_E_ARG for a misaligned one (device.Codec raises), and so does this restatement
        if x.data_ptr() % 16:
            raise RuntimeError("dc_small_huff_shard_hist: status -1 (shard not 16-B aligned)")

    def small_shard_hist(self, x, shard, hist=None):
        self._check_granules(x)
        y = self._shard_syms(x, shard)
        self._hist_in = torch.from_numpy(y)
        return torch.from_numpy(orc.histogram(y).astype(np.int64))

    def small_shard_pack_async(self, x, tab, shard, words, sync, gsync, S):
        self._check_granules(x)
        y = self._shard_syms(x, shard)
        B, M = int(shard[0]), int(shard[1])
        self.pack_async(torch.from_numpy(y), tab, B, words, sync, S)   # codes + the local index
        t = self._tab(tab)
        L = t["nb"][y].astype(np.int64)
        pos = B + np.concatenate([[0], np.cumsum(L)])   # global bit of each symbol (and the end)
        m = y.size
        c = (M + np.arange(m)) // S
        c0e = (M // S) & ~1
        gl = np.bincount(c - c0e, weights=L).astype(np.int64)
        gsync[1][: gl.size] = torch.from_numpy(gl.astype(np.uint16).view(np.int16))
        G = 64 * S
        g0, g1 = -(-M // G), -(-(M + m) // G)
        gb = pos[np.arange(g0, g1) * G - M]
        gsync[0][: gb.size] = torch.from_numpy(gb.astype(np.int64))

    # ---- small front-end shard bodies (dist.ShardedSmall), restated with numpy ------------
    def small_body(self, y, left_halo, nelem, head=b"", out=None):
        """small_compression.c:582-665 body of y[1..nelem] (dc_small_compress_body), after `head`."""
        a = y.numpy()
        i = np.arange(1, nelem + 1)
        low = (a >= ord("a")) & (a <= ord("z"))
        sp = a == ord(" ")
        second = sp[i - 1] & low[i] & ((i >= 2) | bool(left_halo))
        nxt_low = np.zeros(nelem, bool)
        has = i + 1 < a.size
        nxt_low[has] = low[i[has] + 1]
        start = sp[i] & nxt_low
        vals = np.where(start, 0x80 + a[np.minimum(i + 1, a.size - 1)].astype(np.int64), a[i]).astype(np.uint8)
        res = torch.from_numpy(np.concatenate([np.frombuffer(head, np.uint8), vals[~second]]))
        if out is None:
            return res
        out[: res.numel()] = res
        return out[: res.numel()]

    def small_body_plan(self, y, left_halo, nelem):
        return self.small_body(y, left_halo, nelem).numel()

    def small_body_write(self, y, left_halo, nelem, out, head=b""):
        return self.small_body(y, left_halo, nelem, head=head, out=out)

    def small_decompress(self, seg):
        return torch.from_numpy(np.frombuffer(orc.small_decompress(seg.numpy().tobytes()), np.uint8).copy())

    def small_decompress_body(self, seg):
        a = seg.numpy()
        pair = a >= 0x80
        out = np.empty(a.size + int(pair.sum()), np.uint8)
        pos = np.arange(a.size) + np.concatenate([[0], np.cumsum(pair)[:-1]])
        out[pos] = np.where(pair, ord(" "), a)
        out[pos[pair] + 1] = a[pair] - 0x80
        return torch.from_numpy(out)

    # ---- nybble shard bodies (dist.ShardedNybble), restated in plain Python ----------------
    # nybble_compression.c: context byte_to_context :517-523, compress_byte_index :819-884,
    # update_context :665-687, compress_bytestring :887-1038, decompress_nybble :643-663.
    _STATIC = b" etaoins"

    @staticmethod
    def _touch(lst, v):
        if v in lst:
            lst.remove(v)
        lst.insert(0, v)
        del lst[8:]

    def _ranks(self, a, modify, lists):
        L = [list(r) for r in lists] if modify else None
        rk = []
        for i in range(1, len(a)):
            x = a[i]
            if modify:
                c = (a[i - 1] >> 3) & 15
                rk.append(L[c].index(x) if x in L[c] else 0xFF)
                self._touch(L[c], x)
            else:
                rk.append(self._STATIC.index(x) if x in self._STATIC else 0xFF)
        return rk

    def nyb_mtf_summary(self, y):
        a = bytes(y.numpy())
        L = [[] for _ in range(16)]
        for i in range(1, len(a)):
            self._touch(L[(a[i - 1] >> 3) & 15], a[i])
        lists = np.zeros((16, 8), np.uint8)
        cnt = np.zeros(16, np.uint8)
        for c in range(16):
            lists[c, : len(L[c])] = L[c]
            cnt[c] = len(L[c])
        return lists, cnt

    @staticmethod
    def _walk(a, rk, s, pend, is_last):
        out = bytearray()
        for j, r in enumerate(rk):
            i = j + 1
            if r != 0xFF:
                if s:
                    rp = rk[j - 1] if j else pend
                    out.append(((8 | rp) << 4) | (8 | r))
                    s = 0
                else:
                    s = 1
            else:
                out += bytes([a[i - 1], a[i]]) if s else bytes([a[i]])
                s = 0
        if is_last and s:
            out.append(a[-1])
        return bytes(out), s

    def nyb_body_plan(self, y, modify, lists=None):
        a = bytes(y.numpy())
        rk = self._ranks(a, modify, lists)
        self._plan = (a, rk)
        o0, s0 = self._walk(a, rk, 0, 0, False)
        o1, s1 = self._walk(a, rk, 1, 0, False)
        return [len(o0), len(o1), s0, s1, rk[-1] if rk else 0xFF]

    def nyb_body_write(self, y, modify, pend_rank, is_last, head=b""):
        a, rk = self._plan
        assert a == bytes(y.numpy())
        out, _ = self._walk(a, rk, 1 if pend_rank >= 0 else 0, pend_rank, is_last)
        return torch.from_numpy(np.frombuffer(bytes(head) + out, np.uint8).copy())

    def _dwalk(self, a, m, s):
        out = bytearray()
        for k in range(m):
            b = a[k]
            h, l = b >> 4, b & 15
            nxt = a[k + 1] >> 4 if k + 1 < len(a) else 0
            if s == 0 and not (h & 8):
                out.append(b)
                continue
            if s == 0:
                out.append(self._STATIC[h & 7])
            if l & 8:
                out.append(self._STATIC[l & 7])
                s = 0
            else:
                out.append(((l & 7) << 4) + nxt)
                s = 1
        return bytes(out), s

    def nyb_dbody_plan(self, y, m):
        a = bytes(y.numpy())
        o0, s0 = self._dwalk(a, m, 0)
        o1, s1 = self._dwalk(a, m, 1)
        return [len(o0), len(o1), s0, s1]

    def nyb_dbody_write(self, y, m, s_in, head=b""):
        out, _ = self._dwalk(bytes(y.numpy()), m, s_in)
        return torch.from_numpy(np.frombuffer(bytes(head) + out, np.uint8).copy())

    def nyb_decompress(self, comp, modify):
        return torch.from_numpy(np.frombuffer(orc.nybble_decompress(bytes(comp.numpy()), modify), np.uint8).copy())
