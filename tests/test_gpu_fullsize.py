"""Bit-exactness at the benchmarked sizes (GPU): the streams bench.py times are compared
with the CPU oracle bit for bit, not only by round trip.

  * C2 / C3 at 1 GiB: the bench's own rank-0 input (synth.device_text, the same generator
    and seed as bench.py); payload and sync index against oracle/dc_oracle.c's
    orc_huff_pack of the same bytes. C2 is ~4.6e9 bits and C3 ~8.6e9: past 2^32, so a
    32-bit offset error anywhere in pack would show here.
  * C4, 8 shards of 128 MiB (one per thread rank, each its own context on the one GPU)
    through dist.ShardedHuffman: the OR-merged shard streams equal the oracle's encoding of
    the concatenated 1 GiB (~6.7e9 bits): u64 histogram all-reduce, global bit offsets past
    2^32, boundary words shared by two ranks.

Each test needs ~3 GB of host memory and ~10-30 s (the oracle encodes at ~0.2 GB/s).
"""
import threading

import numpy as np
import pytest

from oracle import oracle as orc

pytestmark = pytest.mark.gpu

GiB = 1 << 30


@pytest.fixture(scope="module")
def torch_cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch


def _oracle_stream(xh, n_ary, S):
    h = orc.histogram(xh)
    L = orc.huffman_lengths(h, n_ary)
    el, ev = orc.canonical(L, n_ary)
    code, nb, mx = orc.bitcodes(el, ev, n_ary)
    assert 0 < mx <= 32
    payload, bits, idx = orc.huff_pack(xh, code, nb, sync_syms=S)
    base, lens = orc.sync_compact(idx, 0, bits)
    return h, payload, bits, base, lens


def _words_bytes(words, nbytes):
    return words.view(-1).cpu().numpy().view(np.uint8)[:nbytes]


@pytest.mark.parametrize("cfg,n_ary", [("C2", 2), ("C3", 16)])
def test_benchmarked_stream_bit_exact_vs_oracle(torch_cuda, cfg, n_ary):
    torch = torch_cuda
    from data_compression_amd import synth
    from data_compression_amd.device import Codec
    c = Codec(0)
    x = synth.device_text(cfg, GiB, seed=0xC2, device=torch.device("cuda", 0))   # bench.py rank 0
    enc = c.encode(x, n_ary=n_ary)
    S = enc["S"]
    xh = x.cpu().numpy()
    h, payload, bits, base, lens = _oracle_stream(xh, n_ary, S)
    assert np.array_equal(enc["hist"].cpu().numpy().astype(np.uint64), h)
    assert enc["bits"] == bits and bits > (1 << 32)
    assert np.array_equal(_words_bytes(enc["words"], len(payload)), payload)
    assert np.array_equal(enc["sync"][0].cpu().numpy().astype(np.uint64), base)
    assert np.array_equal(enc["sync"][1].cpu().numpy().view(np.uint16), lens)
    del payload, base, lens
    out = torch.empty_like(x)
    c.decode_into(enc, out)
    assert c.decode_status() == 0 and torch.equal(out, x)
    del enc, out, x
    torch.cuda.empty_cache()


class _ThreadRanks:
    def __init__(self, world):
        self.world, self.bar, self.slots = world, threading.Barrier(world), [None] * world

    def gather(self, rank, vals):
        self.slots[rank] = vals
        self.bar.wait()
        out = list(self.slots)
        self.bar.wait()
        return out


def run_thread_ranks(torch, shards, n_ary, S, table_mode="replicate"):
    """dist.ShardedHuffman over world = len(shards) thread ranks on one GPU, collectives by a
    barrier. Returns per rank (bit_base, bits, words (host u32), decoded == shard)."""
    from data_compression_amd.device import Codec
    from data_compression_amd.dist import ShardedHuffman
    world = len(shards)
    tr = _ThreadRanks(world)
    res, errs = [None] * world, []

    def run(r):
        try:
            torch.cuda.set_device(0)
            sh = ShardedHuffman(Codec(0), table_mode=table_mode)
            sh.world, sh.rank = world, r
            sh.table_src = world - 1

            def all_reduce(t):
                tot = np.sum(np.array(tr.gather(r, t.cpu().tolist()), dtype=np.uint64), axis=0)
                t.copy_(torch.from_numpy(tot.astype(np.int64)).to(t.device))

            def all_gather_scalar(t):
                v = tr.gather(r, int(t.item()))
                return torch.tensor(v, dtype=t.dtype, device=t.device)

            def broadcast_table(t):
                v = tr.gather(r, t.cpu().numpy().tobytes())[world - 1]
                t.copy_(torch.from_numpy(np.frombuffer(v, dtype=np.uint8).copy()).to(t.device))
            sh._all_reduce, sh._all_gather_scalar = all_reduce, all_gather_scalar
            sh._reduce_to_src, sh._broadcast_table = all_reduce, broadcast_table
            xs = shards[r]
            s = sh.finalize(sh.encode(xs, n_ary=n_ary, sync_syms=S))
            y = sh.decode(s)
            nw = (s.bit_base % 32 + s.bits + 31) // 32
            res[r] = (s.bit_base, s.bits, s.words[:nw].cpu().numpy().view(np.uint32).copy(),
                      bool(torch.equal(y[: xs.numel()], xs)))
        except Exception as e:   # noqa: BLE001
            errs.append(repr(e))
            tr.bar.abort()

    ths = [threading.Thread(target=run, args=(r,)) for r in range(world)]
    for t in ths:
        t.start()
    for t in ths:
        t.join(timeout=300)
    assert not errs, errs
    return res


def merge_words(res):
    total = res[-1][0] + res[-1][1]
    merged = np.zeros((total + 31) // 32, np.uint32)
    for base, bits, w, _ in res:
        w0 = base // 32
        k = min(w.size, merged.size - w0)
        merged[w0: w0 + k] |= w[:k]
    return merged, total


def test_c4_eight_shards_merge_bit_exact_vs_oracle(torch_cuda):
    """BASELINE configs[3] layout on one GPU: 8 ranks x 128 MiB of Zipf bytes (seed
    0xC4 + rank, as bench.py --cfg C4 draws them), n = 2."""
    torch = torch_cuda
    from data_compression_amd import synth
    dev = torch.device("cuda", 0)
    world, per, S = 8, 128 << 20, 64
    shards = [synth.device_text("C4", per, seed=0xC4 + r, device=dev) for r in range(world)]
    res = run_thread_ranks(torch, shards, 2, S)
    assert all(r[3] for r in res)
    merged, total = merge_words(res)
    assert total > (1 << 32)
    xh = torch.cat(shards).cpu().numpy()
    del shards
    torch.cuda.empty_cache()
    _, payload, bits, _, _ = _oracle_stream(xh, 2, S)
    assert bits == total
    assert np.array_equal(merged.view(np.uint8)[: len(payload)], payload)


def test_c5_frontend_pipeline_1gib_bit_exact_vs_oracle(torch_cuda):
    """BASELINE configs[4] on one GPU at the benchmarked size: the 1 GiB syslog-like stream
    bench.py --cfg C5 --frontend draws on rank 0 (same generator and seed), through
    dist.ShardedSmall (world 1: small front-end body + n = 16 Huffman with the sync index)
    equals the oracle's small_compress (small_compression.c:582-665) followed by its
    huff_pack of that front-end output, payload and sync index bit for bit; and it decodes
    back to the input."""
    torch = torch_cuda
    import bench
    from data_compression_amd import synth
    from data_compression_amd.device import Codec
    from data_compression_amd.dist import ShardedSmall
    c = Codec(0)
    x = synth.device_text("C5", GiB, seed=bench.input_seed("C5", 0), device=torch.device("cuda", 0))
    S = 64
    sm = ShardedSmall(c)
    s = sm.h.finalize(sm.encode(x, n_ary=16, sync_syms=S))
    assert not s.literal
    xh = x.cpu().numpy()
    fe = np.frombuffer(orc.small_compress(xh.tobytes()), np.uint8)
    assert s.n == fe.size
    _, payload, bits, base, lens = _oracle_stream(fe, 16, S)
    assert s.bits == bits
    assert np.array_equal(_words_bytes(s.words, len(payload)), payload)
    assert np.array_equal(s.sync[0].cpu().numpy().astype(np.uint64), base)
    assert np.array_equal(s.sync[1][: lens.size].cpu().numpy().view(np.uint16), lens)
    del payload, base, lens, fe
    out = torch.empty(2 * s.n + 64, dtype=torch.uint8, device=x.device)
    y = sm.decode(s, out=out)
    assert c.decode_status() == 0 and torch.equal(y, x)
    del s, out, x
    torch.cuda.empty_cache()


@pytest.mark.parametrize("modify", [False, True])
def test_nybble_256mib_vs_oracle(torch_cuda, modify):
    """nybble_compression.c compress_bytestring (static) / nybble_compress (adaptive,
    :887-1038) at 256 MiB of English-like text: the device stream is byte-identical to the
    oracle's, and the decode (static: parallel transducer; adaptive: tokens + resolve) gives
    the input back."""
    torch = torch_cuda
    from data_compression_amd import synth
    from data_compression_amd.device import Codec
    c = Codec(0)
    x = synth.device_text("C1", 256 << 20, seed=0xC1, device=torch.device("cuda", 0))
    comp = c.nyb_compress(x, modify)
    want = orc.nybble_compress(x.cpu().numpy().tobytes(), modify)
    assert comp.numel() == len(want)
    assert np.array_equal(comp.cpu().numpy(), np.frombuffer(want, np.uint8))
    del want
    if modify:   # the sequential resolve runs ~12 MB/s: its 256 MiB would take ~20 s, check 16 MiB
        x16 = x[: 16 << 20]
        comp16 = c.nyb_compress(x16, True)
        y = c.nyb_decompress(comp16, True)
        assert torch.equal(y, x16)
    else:
        y = c.nyb_decompress(comp, False)
        assert torch.equal(y, x)
    torch.cuda.empty_cache()
