"""A/B timing of decode kernels on one encoded stream (same process, interleaved rounds).

    python tools/dec_ab.py [--cfg C2] [--size BYTES] [--nary 2] [--rounds 5] [--iters 10]
Prints per-variant HIP-event mean ms of the huff_decode launch (fast default "v8" vs the
general decoder "v7"; "sNN": the fast decoder with a static share of NN %).
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from data_compression_amd import synth  # noqa: E402
from data_compression_amd.device import Codec  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--cfg", default="C2")
ap.add_argument("--size", type=int, default=1 << 30)
ap.add_argument("--nary", type=int, default=2)
ap.add_argument("--rounds", type=int, default=5)
ap.add_argument("--iters", type=int, default=10)
ap.add_argument("--variants", default="v8,v7")
ap.add_argument("--nocheck", action="store_true", help="ablation builds: skip the output check")
a = ap.parse_args()
dev = torch.device("cuda", 0)
x = synth.device_text(a.cfg, a.size, seed=0xC2, device=dev)
c = Codec(0)
enc = c.encode(x, n_ary=a.nary, sync_syms=64)
out = torch.empty_like(x)
res = {v: [] for v in a.variants.split(",")}
fix = {}
for r in range(a.rounds):
    for v in res:
        c.set_option("decode_general", 1 if v == "v7" else 0)
        c.set_option("decode_static_pct", int(v[1:]) if v.startswith("s") else 60)
        c.decode_into(enc, out)
        torch.cuda.synchronize()
        c.timing(True)
        for _ in range(a.iters):
            c.decode_into(enc, out)
        kt = c.timings()
        c.timing(False)
        ms = [m for name, m in kt if name == "huff_decode"]
        fx = [m for name, m in kt if name == "huff_decode_fix"]
        res[v].append(float(np.mean(ms)) + (float(np.mean(fx)) if fx else 0.0))
        fix.setdefault(v, []).append(float(np.mean(fx)) if fx else 0.0)
        assert a.nocheck or (c.decode_status() == 0 and torch.equal(out, x)), v
for v, l in res.items():
    print(f"{v}: median {np.median(l):.4f} ms  min {np.min(l):.4f}  (fixup {np.median(fix[v]):.4f}; {a.cfg} "
          f"{a.size >> 20} MiB n={a.nary}; redo chunks {c.decode_redo_count()})", flush=True)
