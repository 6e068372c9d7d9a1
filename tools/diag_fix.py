"""Per-wave time split of k_huff_decode8_fix from the -DDC_DIAG build (tools/diag_build.sh _diag -DDC_DIAG)."""
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

x = synth.device_text("C2", 1 << 30, seed=0xC2, device=torch.device("cuda", 0))
c = Codec(0)
enc = c.encode(x, n_ary=2, sync_syms=64)
out = torch.empty_like(x)
for _ in range(3):
    c.decode_into(enc, out)
torch.cuda.synchronize()
L = _lib.load("libdc_core.so")
buf = np.zeros(256 * 16 * 4, np.uint64)
assert L.dc_diag_read(buf.ctypes.data_as(C.c_void_p), C.c_size_t(buf.nbytes)) == 0
raw = buf.reshape(-1, 4)[: 256 * 16]
d = raw.astype(np.float64)
tot, _, dec, _ = d.T
tab = (raw[:, 1] & 0xffffffff).astype(np.float64)
pos = (raw[:, 1] >> 32).astype(np.float64)
rounds = (raw[:, 3] & 255).astype(np.float64)
wait = ((raw[:, 3] >> 8) & ((1 << 28) - 1)).astype(np.float64)
first = (raw[:, 3] >> 36).astype(np.float64)
act = rounds > 0
print(f"fix waves {len(tot)} (with a round: {act.sum()}): total {tot.mean():.0f} cyc (max {tot.max():.0f})  list ready at {tab.mean():.0f} "
      f"(max {tab.max():.0f})  decode {dec[act].mean():.0f} per active wave (max {dec.max():.0f})  rounds {rounds.mean():.2f} (max {rounds.max():.0f})  "
      f"row waits {wait[act].mean():.0f}  first row at {pos[act].mean():.0f} (max {pos.max():.0f})  [s_memtime: shader clock cycles]")
