"""Table kernels against the oracle on large-count histograms (C4 Zipf shards, C2, C3): the
lengths and bit lengths of k_huff_table (dc_huff_table), of the fused histogram + table
(dc_huff_encode_plan) and of the table + plan (dc_huff_table_plan), per symbol.

    python tools/dbg_table.py
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from data_compression_amd import synth  # noqa: E402
from data_compression_amd.device import Codec  # noqa: E402
from oracle import oracle as orc  # noqa: E402

OFF_NBITS, OFF_LEN, OFF_STATUS = 1024, 22296, 34608
dev = torch.device("cuda", 0)
c = Codec(0)


def fields(tab):
    b = tab.cpu().numpy()
    return (b[OFF_LEN: OFF_LEN + 4 * 259].view(np.int32).copy(), b[OFF_NBITS: OFF_NBITS + 1024].view(np.uint32).copy(),
            int(b[OFF_STATUS: OFF_STATUS + 4].view(np.int32)[0]))


def check(name, hist_np, tab):
    L, nb, st = fields(tab)
    ref = np.asarray(orc.huffman_lengths(hist_np.astype(np.uint64), 2))[:259]
    bad = np.nonzero(L != ref)[0]
    miss = np.nonzero((hist_np[:256] != 0) & (nb == 0))[0]
    print(f"{name}: status {st} length mismatches {bad.size} {list(bad[:8])} (got {list(L[bad[:8]])} want "
          f"{list(ref[bad[:8]])}); coded-but-missing {list(miss[:8])}", flush=True)


for cfg, size, seeds in (("C4", 128 << 20, [0xC4 + r for r in range(8)]), ("C2", 256 << 20, [0xC2]),
                         ("C3", 256 << 20, [0xC3])):
    hs = []
    x = None
    for s in seeds:
        x = synth.device_text(cfg, size, seed=s, device=dev)
        hs.append(c.hist(x).cpu().numpy().astype(np.uint64))
    H = np.sum(hs, axis=0)
    ht = torch.from_numpy(H.astype(np.int64)).to(dev)
    check(f"{cfg} k_huff_table (all shards)", H, c.table(ht, 2))
    tab, tot = c.table_plan(ht, 2)
    check(f"{cfg} k_huff_table + plan", H, tab)
    h1, tab1, tot1 = c.encode_plan(x, 2)
    check(f"{cfg} fused (last shard)", hs[-1], tab1)
    check(f"{cfg} k_huff_table (last shard)", hs[-1], c.table(torch.from_numpy(hs[-1].astype(np.int64)).to(dev), 2))
