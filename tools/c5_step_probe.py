"""Host wall time of each step of the fused C5 bench step (encode + counted decode, world 1), to
find where the timed loop loses time against the HIP-event split (run under gpurun)."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from data_compression_amd.device import Codec  # noqa: E402
from data_compression_amd.dist import ShardedSmall  # noqa: E402

n = 1 << 30
dev = torch.device("cuda", 0)
x = bench.bench_input("C5", n, bench.input_seed("C5", 0), dev)
c = Codec(0)
S = 64
ss = ShardedSmall(c)
tab = torch.empty(c.table_bytes, dtype=torch.uint8, device=dev)
total = torch.empty(1, dtype=torch.int64, device=dev)
words = torch.empty(c.words_needed(2**40, 32 * n) + 8, dtype=torch.int32, device=dev)
sync_fe = c.alloc_sync(n + 1, S)
fe_out = torch.empty(2 * n + 64, dtype=torch.uint8, device=dev)
st = {}


def step():
    st["s"] = ss.encode(x, 16, S, words=words, sync=sync_fe, table=tab, total=total)
    st["d"] = ss.decode(st["s"], out=fe_out)


for _ in range(45):
    step()
torch.cuda.synchronize()
ts = []
t0 = time.perf_counter()
for _ in range(50):
    a = time.perf_counter()
    step()
    ts.append((time.perf_counter() - a) * 1e3)
torch.cuda.synchronize()
el = (time.perf_counter() - t0) * 1e3
print("total ms per step", round(el / 50, 4), "steps (host ms):", [round(v, 3) for v in ts])
# host syncs inside one step
import ctypes  # noqa: E402,F401
t = time.perf_counter()
s = ss.encode(x, 16, S, words=words, sync=sync_fe, table=tab, total=total)
t1 = time.perf_counter()
ss.decode(s, out=fe_out)
t2 = time.perf_counter()
torch.cuda.synchronize()
print("encode host ms", round((t1 - t) * 1e3, 3), "decode host ms", round((t2 - t1) * 1e3, 3))
