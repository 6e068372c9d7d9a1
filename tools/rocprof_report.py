"""Summarise a rocprofv3 --stats kernel table for bench.py: per kernel of ours, the mean
launch duration (ms), tagged with the bench workload, so bench.py can report the
dominant kernel's roofline fraction from rocprof beside its own HIP-event figure.

    python tools/rocprof_report.py <kernel_stats.csv> <out.json> [cfg size n_ary]

With the kernel trace beside the stats (run_kernel_trace.csv, --kernel-trace) it also reports
mean_ms_isolated: the mean over the dispatches no other dispatch overlapped in time. bench.py
runs its timed loop with steps in flight (two codec contexts on two streams, whose kernels
overlap and each run longer), and its HIP-event kernel times on one context alone afterwards;
the isolated dispatches are the ones comparable with those.
"""
import csv
import json
import os
import sys

src, dst = sys.argv[1], sys.argv[2]
wl = sys.argv[3:6] if len(sys.argv) > 5 else ["C2", str(1 << 30), "2"]   # bench.py defaults


def short(name):
    k = name.split("(")[0].replace("void ", "").split("<")[0].strip()
    if k == "k_huff_decode8_fix":
        return "k_huff_decode_fix"
    if k.startswith("k_huff_decode"):   # k_huff_decode8<NW, NC> is the decode launch
        return "k_huff_decode"
    return k


out = {}
for r in csv.DictReader(open(src)):
    k = short(r["Name"])
    if not k.startswith("k_"):
        continue
    calls, avg = int(r["Calls"]), float(r["AverageNs"])
    mx = float(r["MaxNs"]) / 1e6
    prev = out.get(k)
    if prev:   # several template instances under one name: call-weighted mean
        tot = prev["calls"] + calls
        avg = (prev["mean_ms"] * 1e6 * prev["calls"] + avg * calls) / tot
        calls, mx = tot, max(mx, prev["max_ms"])
    out[k] = {"calls": calls, "mean_ms": avg / 1e6, "max_ms": mx}
trace = os.path.join(os.path.dirname(src), os.path.basename(src).replace("kernel_stats", "kernel_trace"))
if os.path.exists(trace):
    ds = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]))
                for r in csv.DictReader(open(trace)))
    iso = {}
    end_before = 0   # latest end of the dispatches starting earlier
    for i, (b, e, k) in enumerate(ds):
        nxt = ds[i + 1][0] if i + 1 < len(ds) else None
        if b >= end_before and (nxt is None or nxt >= e):
            iso.setdefault(k, []).append((e - b) / 1e6)
        end_before = max(end_before, e)
    for k, v in iso.items():
        if k in out:
            out[k]["isolated_calls"] = len(v)
            out[k]["mean_ms_isolated"] = sum(v) / len(v)
json.dump({"source": src, "workload": {"cfg": wl[0], "size": int(wl[1]), "n_ary": int(wl[2])}, "kernels": out},
          open(dst, "w"), indent=1)
print(json.dumps(out, indent=1))
