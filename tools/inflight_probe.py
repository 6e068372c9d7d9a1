"""Steps in flight: the bench step (encode + decode of the 1 GiB input, world 1) issued on one
codec context, against two contexts on two HIP streams taking alternate steps (each with its own
buffers), so one step's serial tail (table build, plan, redo, host reads) overlaps the next
step's kernels. Prints ms per step of each arrangement, interleaved rounds (run under gpurun).
usage: python tools/inflight_probe.py [cfg] [nary] [--frontend] [--rounds R] [--steps K]"""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from data_compression_amd.device import Codec  # noqa: E402
from data_compression_amd.dist import ShardedHuffman, ShardedSmall  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("cfg", nargs="?", default="C2")
ap.add_argument("nary", nargs="?", type=int, default=2)
ap.add_argument("--frontend", action="store_true")
ap.add_argument("--rounds", type=int, default=3)
ap.add_argument("--steps", type=int, default=50)
a = ap.parse_args()
n = 1 << 30
dev = torch.device("cuda", 0)
x = bench.bench_input(a.cfg, n, bench.input_seed(a.cfg, 0), dev)
S = 64


class Lane:
    def __init__(self, stream):
        self.stream = stream
        with torch.cuda.stream(stream):
            self.c = Codec(0, stream=stream)
            c = self.c
            self.tab = torch.empty(c.table_bytes, dtype=torch.uint8, device=dev)
            self.total = torch.empty(1, dtype=torch.int64, device=dev)
            self.words = torch.empty(c.words_needed(2**40, 32 * n) + 8, dtype=torch.int32, device=dev)
            if a.frontend:
                self.ss = ShardedSmall(c)
                self.sync = c.alloc_sync(n + 1, S)
                self.out = torch.empty(2 * n + 64, dtype=torch.uint8, device=dev)
            else:
                self.sh = ShardedHuffman(c)
                self.hist = torch.empty(256, dtype=torch.int64, device=dev)
                self.sync = c.alloc_sync(n, S)
                self.out = torch.empty(n, dtype=torch.uint8, device=dev)
        self.st = {}

    def step(self):
        with torch.cuda.stream(self.stream):
            if a.frontend:
                s = self.ss.encode(x, a.nary, S, words=self.words, sync=self.sync, table=self.tab, total=self.total)
                self.st["d"] = self.ss.decode(s, out=self.out)
            else:
                s = self.sh.encode(x, a.nary, S, words=self.words, sync=self.sync, hist=self.hist, table=self.tab,
                                   total=self.total)
                self.sh.decode(s, out=self.out)
                self.st["d"] = self.out
            self.st["s"] = s

    def ok(self):
        return bool(torch.equal(self.st["d"][:n], x))


def run(k, nl, threaded=False):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    bench.run_steps(lanes[:nl], k, threaded)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / k * 1e3


def split():   # bench.split_timed on lane 0 (HIP events on its stream)
    ln = lanes[0]
    with torch.cuda.stream(ln.stream):
        e, d, st = bench.split_timed(lambda: ln.step(), lambda: None, 20)
    return round(st, 4)


lanes = [Lane(torch.cuda.Stream(dev))]
run(45, 1)
print({"cfg": a.cfg, "nary": a.nary, "frontend": a.frontend}, flush=True)
print({"one_lane": {"serial_ms": round(run(a.steps, 1), 4), "split_ms": split()}}, flush=True)
lanes.append(Lane(torch.cuda.Stream(dev)))
run(10, 2)
print({"two_lanes_idle": {"serial_ms": round(run(a.steps, 1), 4), "split_ms": split()}}, flush=True)
for r in range(a.rounds):
    print({"round": r, "serial_ms": round(run(a.steps, 1), 4), "split_ms": split(),
           "two_ms_one_thread": round(run(a.steps, 2), 4), "split_ms_after": split(),
           "two_ms_threads": round(run(a.steps, 2, True), 4), "split_ms_after_threads": split()}, flush=True)
print({"ok": [ln.ok() for ln in lanes]})
