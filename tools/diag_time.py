"""Decode timing of an ablation build (tools/diag_build.sh OUT FLAGS): mean ms of the
huff_decode launch on 1 GiB C2, output not checked. usage: python tools/diag_time.py OUT"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if len(sys.argv) > 1 and sys.argv[1] != "base":
    os.environ["DC_CORE_LIB"] = os.path.join(REPO, "tools", sys.argv[1], "libdc_core.so")
sys.path.insert(0, REPO)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from data_compression_amd import synth  # noqa: E402
from data_compression_amd.device import Codec  # noqa: E402

x = synth.device_text("C2", 1 << 30, seed=0xC2, device=torch.device("cuda", 0))
c = Codec(0)
enc = c.encode(x, n_ary=2, sync_syms=64)
out = torch.empty_like(x)
for _ in range(3):
    c.decode_into(enc, out)
torch.cuda.synchronize()
c.timing(True)
for _ in range(10):
    c.decode_into(enc, out)
kt = c.timings()
ms = [m for name, m in kt if name == "huff_decode"]
print(f"{sys.argv[1] if len(sys.argv) > 1 else 'base'}: decode {np.mean(ms):.4f} ms", flush=True)
