"""One-line summary of a bench.py JSON line on stdin."""
import json
import sys

d = json.loads(sys.stdin.read())
r = d["roofline"]
k = {n: v["ms"] for n, v in d.get("kernels", {}).items()}
print("value", d["value"], "ms", d["ms_per_step"], "in_flight", d.get("in_flight"), "serial", d.get("ms_per_step_serial"), "split", r.get("encode_ms"), r.get("decode_ms"),
      r.get("split_step_ms"), "frac", r["frac"], "enc", r.get("encode_frac"), "dec", r.get("decode_frac"),
      "copy", r.get("copy_probe_GBps"), "ok", d["roundtrip_ok"], "cpu", d.get("cpu_baseline", {}).get("value"))
print("kernels", k)
