"""C5 fused encode on the GPU (dc_small_huff_plan + dc_small_huff_pack_async): per-kernel
HIP-event times and the host time per encode on the bench's 1 GiB syslog-like input (the
two-stage kernels are in the C5 bench line's "kernels"). Prints one JSON line.
usage: python tools/fe_time.py [reps]"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402
from data_compression_amd import synth  # noqa: E402
from data_compression_amd.device import Codec  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    dev = torch.device("cuda", 0)
    c = Codec(0)
    n = 1 << 30
    x = synth.device_text("C5", n, seed=bench.input_seed("C5", 0), device=dev)
    S = 64
    enc = c.small_huff_encode(x, 16, S)          # buffers, first touch, and the fused check
    assert enc["fused"]
    words, sync = enc["words"], enc["sync"]
    hist, tab, total = c._t(256, torch.int64), c.alloc_table(), c._t(1, torch.int64)

    def fused():
        c.small_huff_plan(x, 16, hist=hist, table=tab, total=total)
        c.small_huff_pack_async(x, tab, 0, words, sync, S)

    for _ in range(5):
        fused()
    c.sync()
    c.timing(True)
    t0 = time.perf_counter()
    for _ in range(reps):
        fused()
    c.sync()
    t1 = time.perf_counter()
    ks = {}
    for k, ms in c.timings(4096):
        ks.setdefault(k, []).append(ms)
    c.timing(False)
    out = {"host_ms_per_encode": round((t1 - t0) * 1e3 / reps, 4),
           "kernels": {k: round(sum(v) / len(v), 4) for k, v in ks.items()},
           "status": c.pack_status(tab), "M": enc["n"], "bits": int(total.item()),
           "same_bits": int(total.item()) == enc["bits"]}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
