"""Summarise a rocprofv3 --stats kernel table for bench.py: per kernel of ours, the mean
launch duration (ms), tagged with the bench workload, so bench.py can report the
dominant kernel's roofline fraction from rocprof beside its own HIP-event figure.

    python tools/rocprof_report.py <kernel_stats.csv> <out.json> [cfg size n_ary]
"""
import csv
import json
import sys

src, dst = sys.argv[1], sys.argv[2]
wl = sys.argv[3:6] if len(sys.argv) > 5 else ["C2", str(1 << 30), "2"]   # bench.py defaults
out = {}
for r in csv.DictReader(open(src)):
    k = r["Name"].split("(")[0].replace("void ", "").split("<")[0].strip()
    if not k.startswith("k_"):
        continue
    if k == "k_huff_decode8_fix":
        k = "k_huff_decode_fix"
    elif k.startswith("k_huff_decode"):   # k_huff_decode8<NW, NC> is the decode launch
        k = "k_huff_decode"
    calls, avg = int(r["Calls"]), float(r["AverageNs"])
    mx = float(r["MaxNs"]) / 1e6
    prev = out.get(k)
    if prev:   # several template instances under one name: call-weighted mean
        tot = prev["calls"] + calls
        avg = (prev["mean_ms"] * 1e6 * prev["calls"] + avg * calls) / tot
        calls, mx = tot, max(mx, prev["max_ms"])
    out[k] = {"calls": calls, "mean_ms": avg / 1e6, "max_ms": mx}
json.dump({"source": src, "workload": {"cfg": wl[0], "size": int(wl[1]), "n_ary": int(wl[2])}, "kernels": out},
          open(dst, "w"), indent=1)
print(json.dumps(out, indent=1))
