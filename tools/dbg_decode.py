import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from data_compression_amd import synth
from data_compression_amd.device import Codec
from oracle import oracle as orc
c = Codec(0)
for n, S in ((32767, 64), (32767, 128), (4095, 64), (40000, 64), (200000, 256)):
    x = synth.english_like(n, seed=n + 2)
    h = orc.histogram(x); L = orc.huffman_lengths(h, 2); el, ev = orc.canonical(L, 2); code, nb, mx = orc.bitcodes(el, ev, 2)
    xt = torch.from_numpy(x).cuda()
    enc = c.encode(xt, n_ary=2, sync_syms=S)
    out = torch.zeros(n + 16, dtype=torch.uint8, device="cuda")
    c.decode_into(enc, out)
    y = out[:n].cpu().numpy()
    bad = np.nonzero(y != x)[0]
    print("n", n, "S", S, "maxbits", mx, "nbad", bad.size, "status", c.decode_status())
    if bad.size:
        i = bad[0]; ch = i // S
        sync = enc["sync"].cpu().numpy()
        print("  first bad", i, "chunk", ch, "pos in chunk", i % S, "sync", sync[ch], "w0&3", (sync[ch] >> 5) & 3, "sh", sync[ch] & 31,
              "exp", x[i], "got", y[i], "nb exp", nb[x[i]], "prev ok syms nb", [int(nb[v]) for v in x[i-4:i]])
        bc = np.unique(bad // S)
        print("  bad chunks", bc[:20], "count", bc.size, "of", (n + S - 1) // S)
        # bits consumed before the first bad symbol within chunk
        st = ch * S
        print("  bits before bad within chunk", int(nb[x[st:i]].sum()), "(words", int((sync[ch] & 31) + nb[x[st:i]].sum()) // 32, ")")
