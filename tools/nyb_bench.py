"""Nybble codec throughput on device (secondary path; not the bench.py headline).

python tools/nyb_bench.py [--mib 1024] -> one JSON line: GB/s (input bytes / time) of the
static transducer encode/decode, the parallel adaptive encode, and the chunked (DCNK)
adaptive encode/decode, on english-like text resident in HBM (HIP events on the codec's
stream = torch's current stream)."""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from data_compression_amd import synth  # noqa: E402
from data_compression_amd.device import Codec  # noqa: E402


def timed(fn, reps=3):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        out = fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps, out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mib", type=int, default=1024)
    ap.add_argument("--chunk", type=int, default=4096)
    a = ap.parse_args()
    n = a.mib << 20
    base = torch.from_numpy(synth.english_like(64 << 20, seed=11)).cuda()
    x = base.repeat((n + base.numel() - 1) // base.numel())[:n].contiguous()
    c = Codec(0)
    res = {"input": "english-like text (64 MiB generator tiled)", "bytes": n}
    for modify in (False, True):
        tag = "adaptive" if modify else "static"
        ms, comp = timed(lambda: c.nyb_compress(x, modify))
        res[f"{tag}_encode_GBps"] = round(n / ms / 1e6, 2)
        res[f"{tag}_ratio"] = round(comp.numel() / n, 4)
        if not modify:
            ms, back = timed(lambda: c.nyb_decompress(comp, False))
            assert torch.equal(back, x)
            res["static_decode_GBps"] = round(n / ms / 1e6, 2)
        ms, kc = timed(lambda: c.nyb_compress_chunked(x, modify, a.chunk))
        res[f"{tag}_chunked_encode_GBps"] = round(n / ms / 1e6, 2)
        ms, back = timed(lambda: c.nyb_decompress_chunked(kc))
        assert torch.equal(back, x)
        res[f"{tag}_chunked_decode_GBps"] = round(n / ms / 1e6, 2)
        res[f"{tag}_chunked_ratio"] = round(kc.numel() / n, 4)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
