"""Decode time (huff_decode + huff_decode_fix launches) of the core library in DC_CORE_LIB
(default: the in-tree one) on C2 and C3 streams. usage: [DC_CORE_LIB=...] python tools/cmp_decode.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from data_compression_amd import synth  # noqa: E402
from data_compression_amd.device import Codec  # noqa: E402

c = Codec(0)
for cfg, nary in (("C2", 2), ("C3", 16), ("C4", 2), ("C5", 16)):
    x = synth.device_text(cfg, 1 << 30, seed=0xC2, device=torch.device("cuda", 0))
    enc = c.encode(x, n_ary=nary, sync_syms=64)
    out = torch.empty_like(x)
    for _ in range(3):
        c.decode_into(enc, out)
    torch.cuda.synchronize()
    ok = c.decode_status() == 0 and torch.equal(out, x)
    c.timing(True)
    for _ in range(10):
        c.decode_into(enc, out)
    kt = c.timings()
    c.timing(False)
    tot = {}
    for name, ms in kt:
        tot.setdefault(name, []).append(ms)
    d = {k: round(float(np.mean(v)), 4) for k, v in tot.items()}
    print(f"{os.environ.get('DC_CORE_LIB', 'tree')[-30:]} {cfg} n={nary} bits/sym {enc['bits'] / x.numel():.2f} ok={ok} {d} "
          f"sum {sum(d.values()):.4f}", flush=True)
    del x, out, enc
    torch.cuda.empty_cache()
