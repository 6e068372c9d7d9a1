"""A/B-build check of a context option's kernel variant: the stream it writes on the 1 GiB bench
input equals the default kernels' word for word (same table, same plan), and decodes back.

    DC_CORE_LIB=tools/_ab/libdc_core.so python tools/variant_check.py --opt pack_block=4 [--cfg C2 --nary 2]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from data_compression_amd import synth  # noqa: E402
from data_compression_amd.device import Codec  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--cfg", default="C2")
ap.add_argument("--nary", type=int, default=2)
ap.add_argument("--size", type=int, default=1 << 30)
ap.add_argument("--opt", action="append", default=[])
a = ap.parse_args()
dev = torch.device("cuda", 0)
x = synth.device_text(a.cfg, a.size, seed=0xC2, device=dev)
ref = Codec(0)
e0 = ref.encode(x, n_ary=a.nary, sync_syms=64)
c = Codec(0)
for o in a.opt:
    k, v = o.split("=")
    c.set_option(k, int(v))
e1 = c.encode(x, n_ary=a.nary, sync_syms=64)
st = c.pack_status(e1["table"])
nw = (e0["bits"] + 31) // 32
same = e1["bits"] == e0["bits"] and torch.equal(e1["words"][:nw], e0["words"][:nw])
same_sync = all(torch.equal(p, q) for p, q in zip(e0["sync"], e1["sync"]))
out = torch.empty_like(x)
ref.decode_into(e1, out)
rt = ref.decode_status() == 0 and torch.equal(out, x)
print(f"variant {a.opt} {a.cfg}: pack_status {st} words_equal {same} sync_equal {same_sync} roundtrip {rt}", flush=True)
sys.exit(0 if (st == 0 and same and same_sync and rt) else 1)
