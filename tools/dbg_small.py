import sys, os, ctypes as C
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from data_compression_amd import synth
from data_compression_amd.device import Codec
from oracle import oracle as orc
c = Codec(0)
for n in (15, 16, 100, 40000):
    x = synth.english_like(n, seed=n + 2)
    h = orc.histogram(x); L = orc.huffman_lengths(h, 2); el, ev = orc.canonical(L, 2); code, nb, mx = orc.bitcodes(el, ev, 2)
    xt = torch.from_numpy(x).cuda()
    hist = c.hist(xt); tab = c.table(hist, 2); tot = c.plan(tab)
    nbk = (n + 32767) // 32768
    bh = np.zeros(nbk * 256, np.uint16)
    c.L.dc_huff_block_hist(c.ctx, bh.ctypes.data_as(C.c_void_p), bh.size)
    off = np.zeros(nbk + 1, np.uint64); k = C.c_uint64(0)
    c.L.dc_huff_plan_offsets(c.ctx, off.ctypes.data_as(C.c_void_p), off.size, C.byref(k))
    bhr = bh.reshape(nbk, 256).astype(np.int64)
    print(n, "total", int(tot.item()), "orc", int((h * nb).sum()), "off", off, "host dot", (bhr * nb.astype(np.int64)).sum(1), "bh==h", np.array_equal(bhr.sum(0), h.astype(np.int64)))
