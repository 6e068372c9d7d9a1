"""Per-wave time split of k_huff_decode8 from the -DDC_DIAG build (tools/diag_build.sh)."""
import ctypes as C
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["DC_CORE_LIB"] = os.path.join(REPO, "tools", "_diag", "libdc_core.so")
sys.path.insert(0, REPO)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from data_compression_amd import _lib, synth  # noqa: E402
from data_compression_amd.device import Codec  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "C2"
nary = int(sys.argv[2]) if len(sys.argv) > 2 else 2
x = synth.device_text(cfg, 1 << 30, seed=0xC2, device=torch.device("cuda", 0))
c = Codec(0)
enc = c.encode(x, n_ary=nary, sync_syms=64)
out = torch.empty_like(x)
for _ in range(3):
    c.decode_into(enc, out)
torch.cuda.synchronize()
L = _lib.load("libdc_core.so")
buf = np.zeros(256 * 16 * 4, np.uint64)
assert L.dc_diag_read(buf.ctypes.data_as(C.c_void_p), C.c_size_t(buf.nbytes)) == 0
d = buf.reshape(-1, 4).astype(np.float64)
tot, st, de, _ = d.T
sl = (buf.reshape(-1, 4)[:, 3] & np.uint64(0xffffffffff)).astype(np.float64)   # loop bottom: geometry, scheduling, issue
print(f"{cfg} n={nary}: per wave cycles total {tot.mean():.0f}  stage {st.mean():.0f} ({st.sum()/tot.sum():.1%})  "
      f"decode {de.mean():.0f} ({de.sum()/tot.sum():.1%})  bottom {sl.mean():.0f} ({sl.sum()/tot.sum():.1%})  "
      f"max total {tot.max():.0f} min {tot.min():.0f}")
assert torch.equal(out, x)
meta = buf.reshape(-1, 4)[:, 3]
xcc = (meta >> np.uint64(56)).astype(np.int64)
hwid = ((meta >> np.uint64(40)) & np.uint64(0xffff)).astype(np.int64)
cu = (hwid >> 8) & 15
sh = (hwid >> 12) & 1
se = (hwid >> 13) & 7
for x in range(8):
    m = xcc == x
    if m.any():
        print(f"xcc {x}: waves {m.sum():4d} total mean {tot[m].mean():.0f} max {tot[m].max():.0f} min {tot[m].min():.0f}")
wg = tot.reshape(-1, 16 if tot.size == 4096 else 8)
spread = wg.max(1) / wg.min(1)
print("within-workgroup max/min: mean %.3f max %.3f" % (spread.mean(), spread.max()))
print("workgroup means: min %.0f max %.0f" % (wg.mean(1).min(), wg.mean(1).max()))
