"""Host enqueue time of the bench step (C2, 1 GiB) against its GPU time: if the enqueue of a
step approaches the step, the loop is host-bound. Same objects and calls as bench.py."""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

import torch

from data_compression_amd import synth
from data_compression_amd.device import Codec
from data_compression_amd.dist import ShardedHuffman

n = 1 << 30
dev = torch.device("cuda", 0)
x = synth.device_text("C2", n, seed=0xC2, device=dev)
c = Codec(0)
S = 64
sh = ShardedHuffman(c)
hist = torch.empty(256, dtype=torch.int64, device=dev)
tab = torch.empty(c.table_bytes, dtype=torch.uint8, device=dev)
total = torch.empty(1, dtype=torch.int64, device=dev)
words = torch.empty(c.words_needed(2**40, 32 * n) + 8, dtype=torch.int32, device=dev)
sync = c.alloc_sync(n, S)
out = torch.empty(n, dtype=torch.uint8, device=dev)


def step():
    s = sh.encode(x, 2, S, words=words, sync=sync, hist=hist, table=tab, total=total)
    sh.decode(s, out=out)


for _ in range(5):
    step()
torch.cuda.synchronize()
K = 50
t0 = time.perf_counter()
for _ in range(K):
    step()
t1 = time.perf_counter()
torch.cuda.synchronize()
t2 = time.perf_counter()
print(f"enqueue {1e3 * (t1 - t0) / K:.4f} ms/step, total {1e3 * (t2 - t0) / K:.4f} ms/step")
