"""Adaptive nybble decode diagnostics (run under gpurun): for the bench text (C1 device text)
and the numpy english_like text, whether the fast resolve's re-encode check accepts the result
(the resolve launched once) or the exact step ran again, the per-launch times, and whether the
round trip gives back the input."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from data_compression_amd import synth
from data_compression_amd.device import Codec

c = Codec(0)
dev = torch.device("cuda", 0)
cases = [("C1 device", synth.device_text("C1", 16 << 20, seed=0xC2, device=dev)),
         ("english_like", torch.from_numpy(synth.english_like(4 << 20, seed=5)).to(dev))]
for name, x in cases:
    comp = c.nyb_compress(x, True)
    y = c.nyb_decompress(comp, True)
    torch.cuda.synchronize()
    c.timing(True)
    t = time.perf_counter()
    y = c.nyb_decompress(comp, True)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t) * 1e3
    tl = c.timings()
    c.timing(False)
    names = [n for n, _ in tl]
    agg = {}
    for n_, v in tl:
        agg.setdefault(n_, [0, 0.0]); agg[n_][0] += 1; agg[n_][1] += v
    hi = int((x >= 128).sum().item())
    print(f"{name}: {x.numel()} B, bytes >= 0x80: {hi}, wall {ms:.1f} ms, "
          f"resolve launches {names.count('nyb_resolve')}, roundtrip {torch.equal(y, x)}", flush=True)
    print("   ", {k: (v[0], round(v[1], 3)) for k, v in agg.items()}, flush=True)
