"""Phase split of k_huff_table from the -DDC_DIAG build (tools/diag_build.sh _diag -DDC_DIAG)."""
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

x = synth.device_text("C2", 64 << 20, seed=0xC2, device=torch.device("cuda", 0))
c = Codec(0)
h = c.hist(x)
for _ in range(3):
    tab = c.table(h, 2)
torch.cuda.synchronize()
L = _lib.load("libdc_core.so")
buf = np.zeros(16, np.uint64)
assert L.dc_diag_tbl_read(buf.ctypes.data_as(C.c_void_p)) == 0
names = ["keys", "sort", "merge", "depth", "canonical"]
d = np.diff(buf[:5].astype(np.int64))
print("table phases (cycles):", {n: int(v) for n, v in zip(names[1:], d)}, "total", int(buf[4] - buf[0]),
      "| sort", int(buf[8] - buf[1]), "merge", int(buf[2] - buf[8]),
      "| canonical: counts", int(buf[9] - buf[3]), "prefix", int(buf[10] - buf[9]), "ranks", int(buf[11] - buf[10]),
      "tail", int(buf[4] - buf[11]))
