"""RCCL on the device (the "nccl" calls of dist.py and bench.py had never run).

A one-GPU box cannot host two RCCL ranks (RCCL refuses two ranks on one device; the
multi-rank paths are rehearsed with gloo, tools/gpu_rehearse.sh), so this runs the RCCL
backend at world size 1 in a child process: init_process_group("nccl", device_id=...) as
bench.py does it, every collective dist.ShardedHuffman issues (all_reduce, reduce,
broadcast, all_gather_into_tensor, all_gather, batch_isend_irecv as a self-exchange), and a
sharded encode/decode round trip through the same process group.
"""
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import os, sys
sys.path.insert(0, os.environ["DC_REPO"])
import torch, torch.distributed as dist
dev = torch.device("cuda", 0)
torch.cuda.set_device(0)
dist.init_process_group("nccl", device_id=dev)
assert dist.get_backend() == "nccl" and dist.get_world_size() == 1
h = torch.arange(256, dtype=torch.int64, device=dev)
dist.all_reduce(h)
dist.reduce(h, dst=0)
dist.broadcast(h, src=0)
assert torch.equal(h, torch.arange(256, dtype=torch.int64, device=dev))
out = torch.empty(1, dtype=torch.int64, device=dev)
dist.all_gather_into_tensor(out, torch.tensor([7], dtype=torch.int64, device=dev))
assert int(out.item()) == 7
lst = [torch.empty(5, dtype=torch.int64, device=dev)]
dist.all_gather(lst, torch.arange(5, dtype=torch.int64, device=dev))
assert torch.equal(lst[0], torch.arange(5, dtype=torch.int64, device=dev))
src = torch.arange(1000, dtype=torch.int32, device=dev)
dst = torch.zeros_like(src)
ops = [dist.P2POp(dist.isend, src, 0), dist.P2POp(dist.irecv, dst, 0)]
for w in dist.batch_isend_irecv(ops):
    w.wait()
assert torch.equal(src, dst)
from data_compression_amd import synth
from data_compression_amd.device import Codec
from data_compression_amd.dist import ShardedHuffman
c = Codec(0)
x = synth.device_text("C2", 3 << 20, seed=0xC2, device=dev)
for mode in ("replicate", "broadcast"):
    sh = ShardedHuffman(c, table_mode=mode)
    s = sh.encode(x, 2, 64)
    y = sh.decode(s)
    sh.finalize(s)
    g = sh.gather(s)
    assert torch.equal(y, x) and g[1] == s.bits > 0, mode
torch.cuda.synchronize()
dist.destroy_process_group()
print("rccl ok")
"""


@pytest.mark.gpu
def test_rccl_world1_collectives_and_sharded_roundtrip():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import socket
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    env = dict(os.environ, DC_REPO=REPO, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE="1", RANK="0",
               LOCAL_RANK="0")
    r = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True, text=True, timeout=180)
    assert r.returncode == 0 and "rccl ok" in r.stdout, r.stdout[-2000:] + r.stderr[-4000:]
