"""The code table built from a global histogram whose total exceeds 2^32 (C4 is
8 GiB = 8 shards x 1 GiB, whose all-reduced histogram sums to 2^33). The reference counts in
`int` (n_ary_huffman.c:868-1005: parent sums overflow past 2^31), so above INT_MAX the oracle is
the build's u64 restatement (orc_huffman_lengths / orc_canonical), compared here with
the GPU table kernel (dc_huff_table: k_huff_table's keys are count << 11 | index in u64) on
histograms of ~2^33 total with heavy ties, for n = 2 and n = 16; then a small stream is packed
with that table and compared with orc_huff_pack (n_ary_huffman.c:1382-1612 codes)."""
import ctypes as C

import numpy as np
import pytest

from oracle import oracle as orc

pytestmark = pytest.mark.gpu

MAX_SYMS, MAX_DIGITS = 1024, 128


class DTable(C.Structure):   # include/dc_gpu.h dc_dtable, up to the fields read here
    _fields_ = [("code", C.c_uint32 * 256), ("nbits", C.c_uint32 * 256), ("lut", C.c_uint32 * (1 << 12)),
                ("first", C.c_uint32 * (MAX_DIGITS + 1)), ("count", C.c_uint32 * (MAX_DIGITS + 1)),
                ("start", C.c_uint32 * (MAX_DIGITS + 1)), ("lim", C.c_uint64 * 33),
                ("syms", C.c_uint16 * MAX_SYMS), ("lengths", C.c_int32 * MAX_SYMS),
                ("enc_len", C.c_int32 * MAX_SYMS), ("enc_val", C.c_uint32 * MAX_SYMS),
                ("n_ary", C.c_int32), ("w", C.c_int32), ("max_symbol_value", C.c_int32), ("max_bits", C.c_int32),
                ("min_len", C.c_int32), ("max_len", C.c_int32), ("status", C.c_int32)]


@pytest.fixture(scope="module")
def torch_cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch


@pytest.fixture(scope="module")
def codec(torch_cuda):
    from data_compression_amd.device import Codec
    return Codec(0)


def _fields(tab):
    b = tab.cpu().numpy()
    return DTable.from_buffer_copy(b[: C.sizeof(DTable)].tobytes())


def _hists():
    """u64 histograms of total >= 2^32: C4-like Zipf over 255 byte values scaled to 8 GiB (as
    the 8-rank all_reduce of 1 GiB shards would give), the same with heavy ties (counts rounded
    to a few distinct values), a uniform 2^33 total (every count tied), and counts near 2^33
    each beside small ones (the sums of merged nodes pass 2^36)."""
    rng = np.random.default_rng(0xC4)
    out = []
    ranks = np.arange(1, 256, dtype=np.float64)
    z = 1.0 / ranks
    perm = rng.permutation(255) + 1
    h = np.zeros(256, np.uint64)
    h[perm] = np.floor(z / z.sum() * float(8 << 30)).astype(np.uint64)
    out.append(("zipf-8GiB", h))
    ht = h.copy()
    ht[perm] = (np.round(ht[perm].astype(np.float64) / 2**27) * 2**27).astype(np.uint64) + (1 << 20)
    out.append(("zipf-ties", ht))
    out.append(("uniform-2^33", np.full(256, (1 << 33) // 256, np.uint64)))
    hb = np.zeros(256, np.uint64)
    hb[1:40] = np.uint64(1 << 33)
    hb[40:80] = rng.integers(1, 1 << 20, 40).astype(np.uint64)
    hb[80:90] = np.uint64(3)
    out.append(("huge-and-small", hb))
    return out


@pytest.mark.parametrize("n_ary", [2, 16])
def test_table_from_u64_histogram_past_2_32(torch_cuda, codec, n_ary):
    torch = torch_cuda
    for name, h in _hists():
        assert int(h.sum()) > (1 << 32), name
        ht = torch.from_numpy(h.astype(np.int64)).cuda()
        tab = codec.table(ht, n_ary)
        f = _fields(tab)
        hh = np.zeros(259, np.uint64)
        hh[:256] = h
        L = np.asarray(orc.huffman_lengths(hh, n_ary))[:259]
        el, ev = orc.canonical(L, n_ary)
        got_L = np.frombuffer(bytes(f.lengths), np.int32)[:259]
        code, nb, mx = orc.bitcodes(el, ev, n_ary)
        # a code past 32 bits (n = 2 beside counts 2^31 times smaller) is DC_E_CODE_TOO_LONG (-3)
        assert f.status == (0 if 0 < mx <= 32 else -3), (name, f.status, mx)
        assert np.array_equal(got_L, L), (name, np.nonzero(got_L != L)[0][:8])
        assert np.array_equal(np.frombuffer(bytes(f.enc_len), np.int32)[:258], np.asarray(el)[:258]), name
        assert np.array_equal(np.frombuffer(bytes(f.enc_val), np.uint32)[:258], np.asarray(ev)[:258]), name
        assert np.array_equal(np.frombuffer(bytes(f.nbits), np.uint32), np.asarray(nb)[:256].astype(np.uint32)), name
        if not 0 < mx <= 32:
            continue
        # a small stream coded with the big table: the GPU pack against orc_huff_pack
        present = np.nonzero(h)[0].astype(np.uint8)
        x = present[np.random.default_rng(len(name)).integers(0, present.size, 200_003)]
        payload, bits, _ = orc.huff_pack(x, code, nb, sync_syms=64)
        xt = torch.from_numpy(x).cuda()
        codec.hist(xt)
        total = codec.plan(tab)
        assert int(total.item()) == bits, name
        words = codec.alloc_words(0, bits)
        sync = codec.alloc_sync(x.size, 64)
        codec.pack(xt, tab, 0, words, sync, 64)
        assert codec.pack_status(tab) == 0, name
        got = words.cpu().numpy().view(np.uint8)[: len(payload)]
        assert np.array_equal(got, payload), name
        out = torch.empty(x.size, dtype=torch.uint8, device="cuda")
        codec.decode(words, 0, sync, 64, x.size, tab, out)
        assert codec.decode_status() == 0 and np.array_equal(out.cpu().numpy(), x), name
