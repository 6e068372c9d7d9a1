"""Multi-rank orchestration (data_compression_amd.dist) on CPU with gloo, world size 2 and 3.

Every rank encodes its contiguous shard at its global bit offset; the gathered stream
must be bit-identical to the single-stream encoding of the concatenated input, and each
rank must decode its own shard back. The per-rank engine is the oracle (tests/cpu_engine);
on GPUs the same dist code runs with device.Codec over RCCL (bench.py --gpus N).
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n_ary, S, shard, total, q, table_mode="replicate"):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from data_compression_amd import synth
    from data_compression_amd.dist import ShardedHuffman
    from tests.cpu_engine import CpuEngine
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        x = synth.enwik_like(total, seed=21)
        lo = rank * shard
        hi = total if rank == world - 1 else lo + shard
        xs = torch.from_numpy(x[lo:hi].copy())
        sh = ShardedHuffman(CpuEngine(), table_mode=table_mode, table_src=world - 1)
        s = sh.encode(xs, n_ary=n_ary, sync_syms=S)
        y = sh.decode(s)
        ok = bool(torch.equal(y[: xs.numel()], xs))
        g = sh.gather(s, dst=0)
        if rank == 0:
            words, bits, bases, lens = g
            q.put(("merged", words.numpy().copy(), bits, bases.numpy().copy(), lens.numpy().copy()))
        q.put(("ok", rank, ok))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,n_ary,table_mode", [(2, 2, "replicate"), (3, 16, "replicate"), (2, 3, "replicate"),
                                                    (2, 2, "broadcast"), (3, 16, "broadcast")])
def test_sharded_stream_is_bit_identical(world, n_ary, table_mode):
    from data_compression_amd import synth
    from oracle import oracle as orc
    S = 64
    shard = 64 * S * 5
    total = shard * (world - 1) + 12_345
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n_ary, S, shard, total, q, table_mode)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world + 1)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    oks = [r for r in res if r[0] == "ok"]
    assert len(oks) == world and all(r[2] for r in oks)
    _, words, bits, bases, lens = next(r for r in res if r[0] == "merged")
    # single-stream reference encoding of the whole input
    x = synth.enwik_like(total, seed=21)
    h = orc.histogram(x)
    L = orc.huffman_lengths(h, n_ary)
    el, ev = orc.canonical(L, n_ary)
    code, nb, _ = orc.bitcodes(el, ev, n_ary)
    payload, rbits, idx = orc.huff_pack(x, code, nb, sync_syms=S)
    rbase, rlens = orc.sync_compact(idx, 0, rbits)
    assert bits == rbits
    got = words.view(np.uint8)[: len(payload)]
    assert np.array_equal(got, payload)
    assert np.array_equal(bases.astype(np.uint64), rbase)
    assert np.array_equal(lens.view(np.uint16), rlens)


def _small_worker(rank, world, port, cuts, kind, n_ary, S, q, fused=False, misalign=-1):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from data_compression_amd.dist import ShardedSmall
    from tests.cpu_engine import CpuEngine
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        x = _small_input(kind, cuts[-1])
        xs = torch.from_numpy(x[cuts[rank]: cuts[rank + 1]].copy())
        if rank == misalign:   # a slice one byte into a buffer: not 16-B aligned
            buf = torch.empty(xs.numel() + 1, dtype=torch.uint8)
            buf[1:] = xs
            xs = buf[1:]
            assert xs.data_ptr() % 16
        sm = ShardedSmall(CpuEngine(), fused=fused)
        s = sm.encode(xs, n_ary=n_ary, sync_syms=S)
        y = sm.decode(s)   # (finalize: a LITERAL stream falls back to the two stages here)
        path = "fused" if getattr(s, "shard_fused", None) is not None else "two-stage"
        g = sm.gather(s, dst=0)
        q.put(("dec", rank, y.numpy().copy(), s.literal, path))
        if rank == 0:
            words, bits, bases, lens = g
            q.put(("merged", words.numpy().copy(), bits, bases.numpy().copy(), lens.numpy().copy()))
    finally:
        dist.destroy_process_group()


def _small_input(kind, n):
    from data_compression_amd import synth
    if kind == "log":
        return synth.log_like(n, seed=33)
    rng = np.random.default_rng(4)
    return rng.integers(ord("A"), ord("Z") + 1, size=n, dtype=np.uint8)   # no pairs: LITERAL


@pytest.mark.parametrize("world,kind,fused,cut,misalign", [(2, "log", False, "pair", -1), (3, "log", False, "pair", -1),
                                                           (2, "upper", False, "pair", -1), (2, "log", True, "pair", -1),
                                                           (3, "log", True, "pair", -1), (3, "log", True, "space_end", -1),
                                                           (3, "log", True, "space_start", -1),
                                                           (2, "upper", True, "pair", -1), (3, "log", True, "pair", 1)])
def test_sharded_small_frontend_huffman(world, kind, fused, cut, misalign):
    """C5 orchestration (dist.ShardedSmall). Two stages: halo exchange, body per rank, global
    LITERAL decision, re-cut at 64*S, sharded Huffman. Fused (world > 1): each shard's one-pass
    encode at its global bit and symbol offsets, no re-cut (a LITERAL stream falls back to the
    two stages). Either way the gathered stream AND its sync index equal the oracle's
    single-stream Huffman encoding of the single-stream front-end output, and the ranks'
    decoded segments concatenate to the input. Cuts: on a pair's halves (' ' | letter), after a
    ' ' that starts no pair, or on a ' ' that starts one (' ' + letter | ...). misalign: that
    rank's shard is a view one byte into a buffer (the fused kernels need 16-B granules: the rank
    encodes an aligned copy and stays in step with the others' collectives)."""
    from oracle import oracle as orc
    S, n_ary = 64, 16
    total = 64 * S * 4 * world + 777
    x = _small_input(kind, total)
    low = lambda v: ord("a") <= v <= ord("z")   # noqa: E731
    cuts = [0]
    for r in range(1, world):
        c = r * total // world + 13 * r
        if kind == "log":
            want = {"pair": lambda c: x[c - 1] == ord(" ") and low(x[c]),
                    "space_end": lambda c: x[c - 1] == ord(" ") and not low(x[c]),
                    "space_start": lambda c: x[c] == ord(" ") and low(x[c + 1])}[cut]
            while not want(c):
                c += 1
        cuts.append(c)
    cuts.append(total)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_small_worker, args=(r, world, port, cuts, kind, n_ary, S, q, fused, misalign))
             for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=180) for _ in range(world + 1)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    decs = sorted((r for r in res if r[0] == "dec"), key=lambda r: r[1])
    assert np.array_equal(np.concatenate([d[2] for d in decs]), x)
    fe = np.frombuffer(orc.small_compress(x.tobytes()), np.uint8)
    assert all(d[3] == (fe[0] == ord(" ")) for d in decs)
    assert all(d[4] == ("fused" if fused and kind == "log" else "two-stage") for d in decs)
    _, words, bits, bases, lens = next(r for r in res if r[0] == "merged")
    h = orc.histogram(fe)
    L = orc.huffman_lengths(h, n_ary)
    el, ev = orc.canonical(L, n_ary)
    code, nb, _ = orc.bitcodes(el, ev, n_ary)
    payload, rbits, idx = orc.huff_pack(fe, code, nb, sync_syms=S)
    assert bits == rbits
    assert np.array_equal(words.view(np.uint8)[: len(payload)], payload)
    rbase, rlens = orc.sync_compact(idx, 0, rbits)
    assert np.array_equal(bases.astype(np.uint64), rbase)
    assert np.array_equal(lens.view(np.uint16), rlens)


def _nyb_worker(rank, world, port, cuts, kind, modify, dcuts, q):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from data_compression_amd.dist import ShardedNybble
    from tests.cpu_engine import CpuEngine
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        x = _nyb_input(kind, cuts[-1])
        xs = torch.from_numpy(x[cuts[rank]: cuts[rank + 1]].copy())
        sn = ShardedNybble(CpuEngine())
        seg, literal = sn.compress(xs, modify)
        sizes = [cuts[r + 1] - cuts[r] for r in range(world)]
        if modify:
            y = sn.decode_replica(seg, sizes, True)
            yd = None
        else:
            y = sn.decompress(seg)
            # the same stream re-cut at arbitrary byte positions (dcuts), decoded again
            from oracle import oracle as orc
            whole = np.frombuffer(orc.nybble_compress(x.tobytes(), False), np.uint8)
            lo, hi = int(dcuts[rank] * whole.size), int(dcuts[rank + 1] * whole.size)
            yd = sn.decompress(torch.from_numpy(whole[lo:hi].copy())).numpy().copy()
        q.put(("r", rank, seg.numpy().copy(), literal, y.numpy().copy(), yd))
    finally:
        dist.destroy_process_group()


def _nyb_input(kind, n):
    from data_compression_amd import synth
    if kind == "text":
        return synth.english_like(n, seed=12)
    rng = np.random.default_rng(5)
    return rng.integers(ord("A"), ord("Z") + 1, size=n, dtype=np.uint8)   # all misses: LITERAL


@pytest.mark.parametrize("world,kind,modify,tiny", [(2, "text", False, False), (3, "text", False, False),
                                                    (4, "text", True, False), (2, "text", True, False),
                                                    (2, "upper", False, False), (3, "upper", True, False),
                                                    (4, "text", False, True), (4, "text", True, True)])
def test_sharded_nybble(world, kind, modify, tiny):
    """SURVEY §8(e) nybble rows (dist.ShardedNybble): 1-byte halos, carried run parity (and,
    adaptive, the composed move-to-front lists). The ranks' segments concatenate to the
    reference's single-stream compress_bytestring output; decoding gives the input back,
    also when the compressed stream is cut at arbitrary bytes (static)."""
    from oracle import oracle as orc
    total = 3000 * world + 123
    x = _nyb_input(kind, total)
    rng = np.random.default_rng(world * 7 + modify)
    cuts = [0] + sorted(int(v) for v in rng.choice(np.arange(2, total - 1), world - 1, replace=False)) + [total]
    if tiny:   # 1-byte shards (a rank whose only element is its halo-context element), one of them last
        cuts = [0, 1500, 1501] + [total - 1][: world - 3] + [total]
    dcuts = [0.0] + sorted(float(v) for v in rng.uniform(0.05, 0.95, world - 1)) + [1.0]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_nyb_worker, args=(r, world, port, cuts, kind, modify, dcuts, q))
             for r in range(world)]
    for p in procs:
        p.start()
    res = sorted((q.get(timeout=180) for _ in range(world)), key=lambda r: r[1])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    ref = orc.nybble_compress(x.tobytes(), modify)
    assert b"".join(r[2].tobytes() for r in res) == ref
    assert all(r[3] == (ref[:1] == b" ") for r in res)
    assert np.array_equal(np.concatenate([r[4] for r in res]), x)
    if not modify:
        assert np.array_equal(np.concatenate([r[5] for r in res]), x)
