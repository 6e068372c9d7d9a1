"""Adaptive nybble decode check (run under gpurun): sizes up to 1 MiB, first mismatch."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from data_compression_amd import synth
from data_compression_amd.device import Codec
from oracle import oracle as orc
c = Codec(0)
if len(sys.argv) > 1:
    c.set_option("nyb_adec_v1", int(sys.argv[1]))
x = synth.english_like(1 << 20, seed=5)
for n in [16, 100, 65536]:
    s = x[:n].tobytes()
    comp = orc.nybble_compress(s, True)
    ct = torch.from_numpy(np.frombuffer(comp, np.uint8).copy()).cuda()
    y = c.nyb_decompress(ct, True).cpu().numpy()
    ok = y.tobytes() == s
    if not ok:
        m = min(len(y), n)
        d = np.nonzero(y[:m] != x[:m])[0]
        print(n, "FAIL len", len(y), "first diff", d[:5].tolist() if d.size else None,
              "got", bytes(y[:20]), "want", s[:20], flush=True)
    else:
        print(n, "ok", flush=True)
