"""bench.py with the HIP-event split (split_timed) also measured on lane 0 before and after each
timed loop, and three times in a row where bench.py takes it: where does the split lose time
when lanes are in flight? Prints to stderr; bench.py's line on stdout. (run under gpurun)"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

_split, _timed = bench.split_timed, bench.timed_steps


def probe(tag, ln):
    with torch.cuda.stream(ln.stream):
        e, d, st = _split(ln.encode, ln.decode, 20)
    print(f"[diag] {tag}: split {e:.4f} + {d:.4f} = step {st:.4f}", file=sys.stderr, flush=True)


def timed(lanes, k, threaded, world, dev):
    probe(f"before timed_steps(L={len(lanes)}, threaded={threaded})", lanes[0])
    r = _timed(lanes, k, threaded, world, dev)
    print(f"[diag] timed_steps(L={len(lanes)}) = {r:.4f} ms", file=sys.stderr, flush=True)
    probe(f"after timed_steps(L={len(lanes)})", lanes[0])
    return r


def split(enc, dec, k):
    out = None
    for i in range(3):
        r = _split(enc, dec, k)
        print(f"[diag] bench split #{i}: {r[0]:.4f} + {r[1]:.4f} = step {r[2]:.4f}", file=sys.stderr, flush=True)
        out = out or r
    return out


bench.split_timed, bench.timed_steps = split, timed
sys.argv = ["bench.py"] + sys.argv[1:]
bench.main()
