"""tools/rocprof_report.py: the per-kernel means bench.py prices its rocprof roofline by, and the
mean over the dispatches no other kernel overlapped (bench.py's timed loop keeps two steps in
flight, so overlapped dispatches run longer than the one-context HIP-event times beside them)."""
import csv
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_isolated_means(tmp_path):
    stats = tmp_path / "run_kernel_stats.csv"
    trace = tmp_path / "run_kernel_trace.csv"
    with open(stats, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Name", "Calls", "AverageNs", "MaxNs"])
        w.writerow(["k_huff_pack(unsigned char const*)", 3, 300000, 500000])
        w.writerow(["void k_huff_decode8<11, 2, false>(unsigned int const*)", 2, 400000, 400000])
        w.writerow(["__amd_rocclr_copyBuffer", 1, 1000, 1000])
    # pack 0-200 (alone), decode 300-700 overlaps pack 600-1100, pack 1200-1400 (alone),
    # decode 1500-1900 (alone)
    rows = [("k_huff_pack(x)", 0, 200), ("void k_huff_decode8<11, 2, false>(x)", 300, 700),
            ("k_huff_pack(x)", 600, 1100), ("k_huff_pack(x)", 1200, 1400),
            ("void k_huff_decode8<11, 2, false>(x)", 1500, 1900)]
    with open(trace, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Kernel_Name", "Start_Timestamp", "End_Timestamp"])
        for r in rows:
            w.writerow(r)
    out = tmp_path / "r.json"
    subprocess.run([sys.executable, os.path.join(REPO, "tools", "rocprof_report.py"), str(stats), str(out), "C2",
                    str(1 << 30), "2"], check=True, capture_output=True)
    d = json.load(open(out))
    assert d["workload"] == {"cfg": "C2", "size": 1 << 30, "n_ary": 2}
    k = d["kernels"]
    assert set(k) == {"k_huff_pack", "k_huff_decode"}
    assert abs(k["k_huff_pack"]["mean_ms"] - 0.3) < 1e-9
    assert k["k_huff_pack"]["isolated_calls"] == 2 and abs(k["k_huff_pack"]["mean_ms_isolated"] - 200e-6) < 1e-12
    assert k["k_huff_decode"]["isolated_calls"] == 1 and abs(k["k_huff_decode"]["mean_ms_isolated"] - 400e-6) < 1e-12
