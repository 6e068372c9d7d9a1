"""A/B of context options on one stage's HIP-event time (same process, interleaved rounds).

    python tools/kern_ab.py --stage hist --option hist_prefetch --values 1,2,3 [--cfg C2]
stages: hist (k_hist_blocks), encode (hist+table+plan+pack), decode, step (encode+decode)
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from data_compression_amd import synth  # noqa: E402
from data_compression_amd.device import Codec  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--cfg", default="C2")
ap.add_argument("--size", type=int, default=1 << 30)
ap.add_argument("--nary", type=int, default=2)
ap.add_argument("--stage", default="hist")
ap.add_argument("--option", default="hist_prefetch")
ap.add_argument("--values", default="1,2")
ap.add_argument("--rounds", type=int, default=5)
ap.add_argument("--iters", type=int, default=10)
ap.add_argument("--no-check", action="store_true", help="ablation builds with garbage output")
a = ap.parse_args()
dev = torch.device("cuda", 0)
x = synth.device_text(a.cfg, a.size, seed=0xC2, device=dev)
c = Codec(0)
enc = c.encode(x, n_ary=a.nary, sync_syms=64)
out = torch.empty_like(x)
ref_hist = torch.bincount(x.to(torch.int64), minlength=256)
vals = [int(v) for v in a.values.split(",")]
res = {v: {} for v in vals}


def run():
    if a.stage == "hist":
        c.hist(x)
    elif a.stage == "decode":
        c.decode_into(enc, out)
    else:
        e = c.encode(x, n_ary=a.nary, sync_syms=64)
        if a.stage == "step":
            c.decode_into(e, out)


for r in range(a.rounds):
    for v in vals:
        c.set_option(a.option, v)
        run()
        torch.cuda.synchronize()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.iters):
            run()
        torch.cuda.synchronize()
        res[v].setdefault("wall", []).append((time.perf_counter() - t0) / a.iters * 1e3)
        c.timing(True)
        for _ in range(a.iters):
            run()
        kt = c.timings()
        c.timing(False)
        for name, ms in kt:
            res[v].setdefault(name, []).append(ms)
        if a.stage == "hist":
            assert torch.equal(c.hist(x), ref_hist), v
        if a.stage in ("decode", "step") and not a.no_check:
            assert c.decode_status() == 0 and torch.equal(out, x), v
for v in vals:
    print(f"{a.option}={v}: " + ", ".join(f"{k} {np.median(m):.4f}" for k, m in res[v].items()), flush=True)
