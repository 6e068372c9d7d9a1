"""GPU parity of the fused C5 encode of shards (dc_small_huff_shard_hist / _shard_pack_async,
dist.ShardedSmall at world > 1), the kernels driven in one process: one codec context per
simulated rank, the collectives replaced by sums and prefix sums on the device (the gloo tests in
test_dist.py run the orchestration itself with the CPU restatement). The shards' words OR-merged
at their global bit offsets and their parts of the stream's sync index added must equal the
oracle's single-stream Huffman encoding of the single-stream front-end output
(small_compression.c:582-665 then n_ary_huffman.c), bit for bit, and each shard's local index
must decode its own symbols.
"""
import numpy as np
import pytest

from oracle import oracle as orc

pytestmark = pytest.mark.gpu

LOW = range(ord("a"), ord("z") + 1)


@pytest.fixture(scope="module")
def torch_cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch


def _cuts(x, world, cut):
    total = x.size
    cuts = [0]
    for r in range(1, world):
        c = r * total // world + 29 * r
        want = {"pair": lambda c: x[c - 1] == 32 and x[c] in LOW,
                "space_end": lambda c: x[c - 1] == 32 and x[c] not in LOW,
                "space_start": lambda c: x[c] == 32 and x[c + 1] in LOW,
                "any": lambda c: True}[cut]
        while not want(c):
            c += 1
        cuts.append(c)
    return cuts + [total]


def _shards_encode(torch, x, cuts, n_ary, S):
    from data_compression_amd.device import Codec
    world = len(cuts) - 1
    dev = torch.device("cuda", 0)
    xs = [torch.from_numpy(x[cuts[r]: cuts[r + 1]].copy()).to(dev) for r in range(world)]
    cs = [Codec(0) for _ in range(world)]
    sh = []
    for r in range(world):
        left = int(x[cuts[r] - 1]) if r > 0 else -1
        right = int(x[cuts[r + 1]]) if r < world - 1 else -1
        sh.append(torch.tensor([0, 0, left, right], dtype=torch.int64, device=dev))
    hists = [cs[r].small_shard_hist(xs[r], sh[r]) for r in range(world)]
    hg = torch.stack(hists).sum(0)                                    # the all_reduce
    plans = [cs[r].table_plan(hg, n_ary) for r in range(world)]
    bits = torch.stack([p[1].reshape(()) for p in plans])
    syms = torch.stack([h.sum() for h in hists])
    for r in range(world):                                            # the all_gather + prefix
        sh[r][0] = bits[:r].sum()
        sh[r][1] = syms[:r].sum()
    out = []
    for r in range(world):
        tab = plans[r][0]
        nb_r = int(bits[r].item())
        words = cs[r].alloc_words(0, nb_r + 32)
        sync = cs[r].alloc_sync(xs[r].numel() + 1, S)
        gsync = cs[r].alloc_sync(xs[r].numel() + 1 + 2 * S, S)
        cs[r].small_shard_pack_async(xs[r], tab, sh[r], words, sync, gsync, S)
        assert cs[r].pack_status(tab) == 0
        out.append({"c": cs[r], "tab": tab, "words": words, "sync": sync, "gsync": gsync,
                    "B": int(sh[r][0].item()), "M": int(sh[r][1].item()), "bits": nb_r, "m": int(syms[r].item())})
    return out


@pytest.mark.parametrize("world,cut,n_ary,size", [(2, "pair", 16, 3 << 20), (3, "space_start", 16, 3 << 20),
                                                  (3, "space_end", 2, 3 << 20), (4, "any", 16, 5 << 20),
                                                  (3, "pair", 9, 200_000)])
def test_c5_fused_shards_bit_exact_vs_oracle(torch_cuda, world, cut, n_ary, size):
    torch = torch_cuda
    from data_compression_amd import synth
    S = 64
    x = synth.log_like(size, seed=0xC5 + world)
    cuts = _cuts(x, world, cut)
    parts = _shards_encode(torch, x, cuts, n_ary, S)
    fe = np.frombuffer(orc.small_compress(x.tobytes()), np.uint8)
    assert fe[0] == 8   # (not LITERAL: the fused path applies)
    h = orc.histogram(fe)
    L = orc.huffman_lengths(h, n_ary)
    el, ev = orc.canonical(L, n_ary)
    code, nb, _ = orc.bitcodes(el, ev, n_ary)
    payload, rbits, idx = orc.huff_pack(fe, code, nb, sync_syms=S)
    rbase, rlens = orc.sync_compact(idx, 0, rbits)
    assert sum(p["bits"] for p in parts) == rbits
    assert sum(p["m"] for p in parts) == fe.size
    # words: each shard's at its global word, OR-merged where two shards share one
    merged = np.zeros((rbits + 31) // 32 + 2, np.uint32)
    for p in parts:
        nw = (p["B"] % 32 + p["bits"] + 31) // 32
        w0 = p["B"] // 32
        merged[w0: w0 + nw] |= p["words"][:nw].cpu().numpy().view(np.uint32)
    assert np.array_equal(merged.view(np.uint8)[: len(payload)], payload)
    # the stream's sync index from the shards' parts
    lens = np.zeros(rlens.size, np.int64)
    base = np.zeros(rbase.size, np.uint64)
    for p in parts:
        M, m = p["M"], p["m"]
        c0 = M // S
        c0e = c0 & ~1
        nl = (M + m - 1) // S - c0 + 1
        gl = p["gsync"][1].cpu().numpy().view(np.uint16)[c0 - c0e: c0 - c0e + nl]
        lens[c0: c0 + nl] += gl
        g0, g1 = -(-M // (64 * S)), -(-(M + m) // (64 * S))
        base[g0: g1] = p["gsync"][0][: g1 - g0].cpu().numpy().astype(np.uint64)
    assert np.array_equal(lens, rlens.astype(np.int64))
    assert np.array_equal(base, rbase)
    # each shard decodes its own symbols from its own words and local index
    for p in parts:
        m = p["m"]
        y = torch.empty(m + 64, dtype=torch.uint8, device="cuda")
        ng, nch = p["c"].sync_sizes(m, S)
        p["c"].decode(p["words"], p["B"], (p["sync"][0][:ng], p["sync"][1][:nch]), S, m, p["tab"], y)
        assert p["c"].decode_status() == 0
        assert np.array_equal(y[:m].cpu().numpy(), fe[p["M"]: p["M"] + m])
