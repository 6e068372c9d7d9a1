"""Where the bench's fixed ~0.8 ms per timed region goes (run under gpurun): the C2 step of
bench.py, 20 steps after a synchronize, a HIP event between steps (torch's stream, which the
codec launches on); per-step GPU times and host time of the region."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from data_compression_amd.device import Codec  # noqa: E402
from data_compression_amd.dist import ShardedHuffman  # noqa: E402

n = 1 << 30
dev = torch.device("cuda", 0)
x = bench.bench_input("C2", n, bench.input_seed("C2", 0), dev)
c = Codec(0)
S = 64
sh = ShardedHuffman(c, table_mode="replicate")
hist = torch.empty(256, dtype=torch.int64, device=dev)
tab = torch.empty(c.table_bytes, dtype=torch.uint8, device=dev)
total = torch.empty(1, dtype=torch.int64, device=dev)
words = torch.empty(c.words_needed(2**40, 32 * n) + 8, dtype=torch.int32, device=dev)
sync = c.alloc_sync(n, S)
out = torch.empty(n, dtype=torch.uint8, device=dev)
st = {}


def step():
    st["s"] = sh.encode(x, 2, S, words=words, sync=sync, hist=hist, table=tab, total=total)
    sh.decode(st["s"], out=out)


for _ in range(5):
    step()
torch.cuda.synchronize()
for trial in range(3):
    K = 20
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(K + 1)]
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ev[0].record()
    th = []
    for k in range(K):
        step()
        ev[k + 1].record()
        th.append(time.perf_counter() - t0)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    per = [ev[k].elapsed_time(ev[k + 1]) for k in range(K)]
    print("trial %d host %.3f ms (%.4f/step) events sum %.3f; per step %s; host enqueue ms %s" % (
        trial, el * 1e3, el * 1e3 / K, sum(per), " ".join("%.3f" % p for p in per),
        " ".join("%.2f" % (t * 1e3) for t in th[:6])), flush=True)
