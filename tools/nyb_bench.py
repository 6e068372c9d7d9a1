"""Nybble codec throughput on the GPU beside the CPU oracle (one pinned host core), SURVEY
§8 rows N1-N4 / BASELINE configs[0]: static and adaptive (modify) compress_bytestring /
decompress_bytestring on a 4 KiB ASCII buffer (C1) and a 64 MiB english-like text.
GPU times are HIP-event-free wall times of the device calls with inputs resident in HBM
(each call ends in a host read of the output length, as the C ABI does).
    python tools/nyb_bench.py [--big MiB] [--reps N]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from data_compression_amd import synth  # noqa: E402
from data_compression_amd.device import Codec  # noqa: E402
from oracle import oracle as orc  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--big", type=int, default=64)
ap.add_argument("--reps", type=int, default=5)
a = ap.parse_args()
c = Codec(0)


def wall(fn, reps):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps


def cpu_wall(fn, budget=10.0):
    old = os.sched_getaffinity(0)
    os.sched_setaffinity(0, {min(old)})
    try:
        t = time.perf_counter()
        k = 0
        while True:
            fn()
            k += 1
            el = time.perf_counter() - t
            if el > budget / 4 or k >= 1000:
                return el / k
    finally:
        os.sched_setaffinity(0, old)


rows = []
for name, n in (("C1 4 KiB ascii", 4096), (f"{a.big} MiB english-like", a.big << 20)):
    x = synth.english_like(n, seed=1)
    xt = torch.from_numpy(x).cuda()
    xb = x.tobytes()
    for modify in (False, True):
        comp = c.nyb_compress(xt, modify)
        cb = comp.cpu().numpy().tobytes()
        assert cb == orc.nybble_compress(xb, modify)
        back = c.nyb_decompress(comp, modify)
        assert np.array_equal(back.cpu().numpy(), x)
        reps = a.reps if n > 1 << 20 else 50
        te = wall(lambda: c.nyb_compress(xt, modify), reps)
        td = wall(lambda: c.nyb_decompress(comp, modify), 1 if (modify and n > 1 << 20) else reps)
        ce = cpu_wall(lambda: orc.nybble_compress(xb, modify))
        cd = cpu_wall(lambda: orc.nybble_decompress(cb, modify))
        rows.append({"input": name, "mode": "adaptive" if modify else "static", "bytes": n,
                     "gpu_enc_MBps": round(n / te / 1e6, 1), "gpu_dec_MBps": round(n / td / 1e6, 1),
                     "cpu_enc_MBps": round(n / ce / 1e6, 1), "cpu_dec_MBps": round(n / cd / 1e6, 1),
                     "ratio": round(len(cb) / n, 4)})
        print(json.dumps(rows[-1]), flush=True)
