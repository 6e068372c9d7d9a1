import sys, os
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
import torch
from data_compression_amd import synth
from data_compression_amd.device import Codec
x = synth.device_text("C2", 1 << 30, seed=0xC2, device=torch.device("cuda", 0))
c = Codec(0)
enc = c.encode(x, n_ary=2, sync_syms=64)
out = torch.empty_like(x)
c.decode_into(enc, out)
print("redo chunks", c.decode_redo_count(), "of", (1<<30)//64)
