"""Per-kernel HIP-event times of one codec stage on the 1 GiB bench input, for ablation
libraries (DC_CORE_LIB=tools/_ablX/libdc_core.so) against the in-tree one.

    python tools/abl_time.py [--stage decode|encode|step] [--cfg C2] [--iters 20] [--tag NAME]

Prints one JSON line: {"tag", "stage", "kernels": {name: mean ms}}. Ablation builds produce
garbage output: nothing is checked.
"""
import argparse
import json
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
ap.add_argument("--stage", default="decode")
ap.add_argument("--iters", type=int, default=20)
ap.add_argument("--warm", type=int, default=30)
ap.add_argument("--opt", action="append", default=[], help="context option name=value (repeatable)")
ap.add_argument("--tag", default=os.path.basename(os.path.dirname(os.environ.get("DC_CORE_LIB", "base/x"))))
a = ap.parse_args()
dev = torch.device("cuda", 0)
x = synth.device_text(a.cfg, a.size, seed=0xC2, device=dev)
c = Codec(0)
for o in a.opt:
    k, v = o.split("=")
    c.set_option(k, int(v))
if a.stage in ("nyb_adaptive", "nyb_static"):   # the whole-stream nybble encoders on 1 GiB
    pass
elif a.stage == "nyb_static_step":   # the static encode and the decode of its output
    ybuf = torch.empty(2 * x.numel() + 16, dtype=torch.uint8, device=dev)
elif a.stage in ("c5_enc", "c5_step"):   # the fused C5 encode (and the counted decode)
    enc = c.small_huff_encode(x, a.nary, 64)
elif a.stage in ("batch", "chunk_enc"):   # the one-lane-per-stream nybble paths on 4 KiB streams
    x = x[: 256 << 20]
    cont = c.nyb_compress_chunked(x, True, 4096)
    nch = (x.numel() + 4095) // 4096
    offs = cont[32: 32 + 8 * (nch + 1)].view(torch.int64).clone()
    pay = cont[32 + 8 * (nch + 1):]
else:
    enc = c.encode(x, n_ary=a.nary, sync_syms=64)
out = torch.empty_like(x)
out2 = torch.empty(2 * x.numel() + 64, dtype=torch.uint8, device=dev) if a.stage == "c5_step" else None


def run():
    if a.stage == "decode":
        c.decode_into(enc, out)
    elif a.stage in ("c5_enc", "c5_step"):
        e = c.small_huff_encode(x, a.nary, 64)
        if a.stage == "c5_step":
            c.small_huff_decode(e, out=out2)
    elif a.stage in ("nyb_adaptive", "nyb_static"):
        c.nyb_compress(x, a.stage == "nyb_adaptive")
    elif a.stage == "nyb_static_step":
        c.nyb_decompress(c.nyb_compress(x, False), False, out=ybuf)
    elif a.stage == "batch":
        c.nyb_decompress_batch(pay, offs, True, out_cap=x.numel())
    elif a.stage == "chunk_enc":
        c.nyb_compress_chunked(x, True, 4096)
    elif a.stage == "hist":
        c.hist(x)
    else:
        e = c.encode(x, n_ary=a.nary, sync_syms=64)
        if a.stage == "step":
            c.decode_into(e, out)


for _ in range(a.warm):
    run()
torch.cuda.synchronize()
c.timing(True)
for _ in range(a.iters):
    run()
kt = c.timings()
c.timing(False)
per = {}
for name, ms in kt:
    per.setdefault(name, []).append(ms)
print(json.dumps({"tag": a.tag, "opts": a.opt, "stage": a.stage, "cfg": a.cfg,
                  "kernels": {k: round(float(np.mean(v)), 4) for k, v in per.items()}}), flush=True)
