"""Summarise tools/pmc.sh output: per kernel, mean counter value per dispatch."""
import csv
import glob
import os
import sys
from collections import defaultdict

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
want = ("k_hist_blocks", "k_huff_pack", "k_huff_decode", "k_huff_table", "k_hist_reduce", "k_block_scan")
vals = defaultdict(lambda: defaultdict(list))
for f in sorted(glob.glob(os.path.join(root, "p*", "run_counter_collection.csv"))):
    per = defaultdict(float)
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0]
        if k not in want:
            continue
        key = (k, r["Dispatch_Id"], r["Counter_Name"])
        per[key] += float(r["Counter_Value"])
    for (k, d, c), v in per.items():
        vals[k][c].append(v)
for k in want:
    if k not in vals:
        continue
    print(k)
    for c, v in sorted(vals[k].items()):
        print("   %-22s %16.0f" % (c, sum(v) / len(v)))
