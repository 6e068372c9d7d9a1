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

    def table(self, hist, n_ary, out=None):
        h = hist.numpy().astype(np.uint64)
        L = orc.huffman_lengths(h, n_ary)
        el, ev = orc.canonical(L, n_ary)
        code, nb, mx = orc.bitcodes(el, ev, n_ary)
        assert 0 < mx <= 32
        return {"L": L, "el": el, "ev": ev, "code": code, "nb": nb, "n_ary": n_ary}

    def plan(self, tab, total=None):
        h = orc.histogram(self._hist_in.numpy()).astype(np.int64)
        self._total = int((h * tab["nb"].astype(np.int64)).sum())
        return torch.tensor([self._total], dtype=torch.int64)

    def plan_total(self):
        return self._total

    def alloc_words(self, bit_base, bits):
        return torch.zeros(((bit_base & 31) + bits + 31) // 32 + 24, dtype=torch.int32)

    def alloc_sync(self, n, S):
        c = (n + S - 1) // S
        return (torch.zeros(max((c + 63) // 64, 1), dtype=torch.int64), torch.zeros(max(c, 1), dtype=torch.int16))

    def alloc_bytes(self, n):
        return torch.zeros(max(n, 1), dtype=torch.uint8)

    def pack_async(self, x, tab, bit_base, words, sync, S):
        xs = x.numpy()
        payload, bits, idx = orc.huff_pack(xs, tab["code"], tab["nb"], bit_base=bit_base, sync_syms=S)
        w = words.numpy().view(np.uint8)
        off = (bit_base >> 3) - ((bit_base >> 5) << 2)
        w[:] = 0
        w[off: off + len(payload)] = payload
        base, lens = orc.sync_compact(idx, bit_base, bits)
        sync[0][: len(base)] = torch.from_numpy(base.astype(np.int64))
        sync[1][: len(lens)] = torch.from_numpy(lens.view(np.int16))

    def decode(self, words, bit_base, sync, S, n, tab, out):
        bits_all = np.unpackbits(words.numpy().view(np.uint8))
        stream = np.packbits(bits_all[bit_base & 31:])
        total = int(sync[1][: (n + S - 1) // S].numpy().view(np.uint16).astype(np.int64).sum())
        y = orc.huff_unpack(stream, total, n, tab["el"], tab["ev"], tab["n_ary"])
        out[:n] = torch.from_numpy(y)

    # ---- small front-end shard bodies (dist.ShardedSmall), restated with numpy ------------
    def small_body(self, y, left_halo, nelem):
        """small_compression.c:582-665 body of y[1..nelem] (dc_small_compress_body)."""
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
        return torch.from_numpy(vals[~second].copy())

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
