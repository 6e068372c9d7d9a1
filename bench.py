"""Headline benchmark: GB/s encode+decode on a 1 GiB byte stream per MI355X, % HBM roofline.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--cfg C2] [--nary 2] [--size BYTES]
    torchrun --nproc-per-node N bench.py --gpus N ...          (driver launches N>1 so)

Workload (BASELINE.json metric / configs[1] generator at the metric's 1 GiB): a 1 GiB
enwik-like synthetic byte stream per GPU, binary (n=2) Huffman. One step = the whole
codec on that stream, inputs resident in HBM:
    encode = histogram -> [RCCL all-reduce of the 256-bin histogram] -> code table ->
             per-block bit plan -> [RCCL all-gather of per-rank bit counts] -> pack at the
             rank's global bit offset (+ sync index)
    decode = parallel decode of the rank's shard back to bytes
value = total uncompressed bytes of all ranks / step time (GB/s, 1e9), "scaling": "weak".
The round trip is verified (decoded == input) after the timed region.

roofline: dominant kernel, algorithmic bytes per launch / its mean HIP-event duration on
the codec's stream, against 8.0 TB/s. cpu_baseline: the oracle (single-threaded C
restatement) on a bounded sample of the same stream, rank 0, N=1 only.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

HBM_PEAK = 8.0e12          # MI355X HBM3E spec, bytes/s (MI355X_MICROARCH.md)
METRIC = "GB/s encode+decode on 1 GiB byte stream at 1/2/4/8 MI355X; % HBM roofline"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)   # ~1 ms each: amortises the bracketing syncs
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--prewarm", type=int, default=40,
                    help="untimed steps before the W warmup steps: the GPU reaches its steady clocks "
                         "only after ~20-30 ms of load (tools/step_probe.py, profiles/r3w_step_probe.log: "
                         "after 5 warmup steps the first timed steps ran 1.15 -> 1.03 ms, steady 1.02)")
    ap.add_argument("--cfg", default="C2")
    ap.add_argument("--frontend", action="store_true",
                    help="C5 pipeline: small_compression.c front-end, then n-ary Huffman (dist.ShardedSmall)")
    ap.add_argument("--two-stage", action="store_true",
                    help="C5 at one GPU: the front-end and the Huffman code as two passes (default: the fused "
                         "one-pass encode and the counted decode, dc_small_huff_*)")
    ap.add_argument("--nary", type=int, default=2)
    ap.add_argument("--size", type=int, default=1 << 30, help="bytes per GPU")
    ap.add_argument("--sync", type=int, default=0, help="sync-index granularity (0 = default)")
    ap.add_argument("--cpu-sample", type=int, default=256 << 20)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--table-mode", default=None, choices=["replicate", "broadcast"],
                    help="multi-GPU code table: built on rank 0 and broadcast over RCCL (the default at "
                         "N > 1, north_star's 'RCCL broadcast of the shared code table'), or built on every rank")
    ap.add_argument("--gather-reps", type=int, default=5,
                    help="N > 1: timed gathers of the whole stream to rank 0 after the timed region")
    ap.add_argument("--profile-steps", type=int, default=20)
    ap.add_argument("--in-flight", type=int, default=2,
                    help="steps in flight: L codec contexts, each on its own HIP stream with its own buffers, "
                         "take steps i = j mod L (at one GPU each from its own host thread), so one step's "
                         "serial tail (table build, plan, redo, host reads) overlaps the next step's kernels. "
                         "Every step still codes the whole input; ms_per_step_serial beside it is one context")
    ap.add_argument("--codec", default="huffman", choices=["huffman", "nybble"],
                    help="nybble: nybble_compression.c's codec on 1 GiB of English-like text (--mode)")
    ap.add_argument("--mode", default="static", choices=["static", "adaptive"],
                    help="nybble: static (compress_bytestring modify=false: encode + decode per step) or adaptive "
                         "(nybble_compress: encode per step; the sequential decode timed on a sample)")
    return ap.parse_args()


def main():
    a = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if a.table_mode is None:
        a.table_mode = "broadcast" if world > 1 else "replicate"
    _trace_setup(rank)
    _phase(rank, "start")
    # ranks beyond the visible GPUs share them (a rehearsal of the multi-rank path on a
    # smaller box; one rank per GPU otherwise)
    local = int(os.environ.get("LOCAL_RANK", "0")) % max(torch.cuda.device_count(), 1)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        # RCCL; DC_BENCH_BACKEND=gloo rehearses the multi-rank path with ranks sharing a GPU
        # (RCCL refuses two ranks on one device)
        backend = os.environ.get("DC_BENCH_BACKEND", "nccl")
        dist.init_process_group(backend, **({"device_id": dev} if backend == "nccl" else {}))

    from data_compression_amd import synth
    from data_compression_amd.device import Codec

    if a.codec == "nybble":
        return main_nybble(a, dev, rank, world)
    n = a.size
    _phase(rank, "device up")
    x = bench_input(a.cfg, n, input_seed(a.cfg, rank), dev)
    torch.cuda.synchronize()
    _phase(rank, "input generated")
    c = Codec(local)   # launches on torch's current stream
    # sync granularity: chosen once from this stream's planned payload (outside the timed
    # region), as the encoder would for a stream of these statistics (dc_huff_choose_sync)
    probe_tab = c.table(c.hist(x), a.nary)
    S = a.sync or c.choose_sync(n, int(c.plan(probe_tab).item()))
    if world > 1:   # one granularity for the whole stream
        st = torch.tensor([S], dtype=torch.int64, device=dev)
        dist.all_reduce(st, op=dist.ReduceOp.MIN)
        S = int(st.item())
    ngroups, nchunks = c.sync_sizes(n, S)

    # each lane codes its own copy of the input (lanes in flight never stream the same addresses,
    # so neither can hit lines the other just pulled into the 256 MiB Infinity Cache)
    lanes = [Lane(a, dev, local, x if i == 0 else x.clone(), S, n, world) for i in range(max(1, a.in_flight))]
    lane0 = lanes[0]
    c, state = lane0.c, lane0.state
    threaded = world == 1   # (at N > 1 one host thread keeps every rank's collectives in one order)
    _phase(rank, "buffers ready")
    run_steps(lanes, a.prewarm + a.warmup, threaded)   # the same count on every rank (steps hold collectives)
    torch.cuda.synchronize()
    _phase(rank, "warmup done")
    ms_step = timed_steps(lanes, a.steps, threaded, world, dev)
    _phase(rank, "timed steps done")
    ms_serial = timed_steps(lanes[:1], a.steps, False, world, dev) if len(lanes) > 1 else ms_step
    _phase(rank, "serial steps done")
    torch.cuda.set_stream(lane0.stream)   # the rest runs on lane 0 (its codec's stream)
    encode, decode, step = lane0.encode, lane0.decode, lane0.step
    sh = lane0.sh
    # encode / decode split: HIP events on the codec's stream (torch's current stream) inside
    # back-to-back steps run right after the timed region (clocks still at their steady
    # state): before the histogram, between the pack and the decode, after the redo, so
    # encode_ms + decode_ms is the step (split_step_ms beside ms_per_step shows it). The
    # per-kernel HIP-event durations follow, then the copy probe: all before the round-trip
    # checks (the first steps after a 1 GiB torch.equal ran ~2 ms slower in all, which moved
    # whichever timing came next, tools/bench_split_diag.py)
    enc_ms, dec_ms, split_step_ms = split_timed(encode, decode, a.profile_steps)
    c.timing(True)
    for _ in range(a.profile_steps):
        step()
    kt = c.timings()
    c.timing(False)
    copy_gbps = copy_probe(c, x, a.profile_steps)

    # ---- correctness of the measured configuration (outside the timed region) ----------
    st = c.pack_status(state["s"].table)
    ok = st == 0 and all([ln.roundtrip_ok() for ln in lanes])   # (each lane's last step)
    bits = state["s"].bits if a.frontend else int(lane0.total.item())   # this rank's payload bits
    if world > 1:
        okt = torch.tensor([1 if ok else 0], device=dev)
        dist.all_reduce(okt, op=dist.ReduceOp.MIN)
        ok = bool(okt.item())

    # ---- N > 1: the gather of the whole stream to rank 0 (end-to-end GB/s
    # beside the codec-only value), timed separately, outside the codec's timed region --------
    gather = None
    if world > 1 and not a.frontend and a.gather_reps > 0:
        s_enc = state["s"]
        sh.gather(s_enc)   # untimed first call: host finalize, buffer allocation
        torch.cuda.synchronize()
        dist.barrier()
        torch.cuda.synchronize()
        tg = time.perf_counter()
        for _ in range(a.gather_reps):
            g = sh.gather(s_enc)
        torch.cuda.synchronize()
        dist.barrier()
        gel = time.perf_counter() - tg
        gt = torch.tensor([gel], dtype=torch.float64, device=dev)
        dist.all_reduce(gt, op=dist.ReduceOp.MAX)
        gather_ms = float(gt.item()) / a.gather_reps * 1e3
        # the merged stream holds every rank's payload bits (after finalize, s_enc.bits is this rank's)
        allbits = torch.tensor([s_enc.bits], dtype=torch.int64, device=dev)
        dist.all_reduce(allbits)
        ok_g = g is not None and int(g[1]) == int(allbits.item()) if rank == 0 else g is None
        okg = torch.tensor([1 if ok_g else 0], device=dev)
        dist.all_reduce(okg, op=dist.ReduceOp.MIN)
        gather = {"gather_ms": round(gather_ms, 4), "reps": a.gather_reps,
                  "e2e_GBps": round(world * n / ((ms_step + gather_ms) * 1e-3) / 1e9, 2),
                  "bytes_to_rank0": None, "ok": bool(okg.item())}
        if rank == 0 and g is not None:
            gather["bytes_to_rank0"] = int(g[0].numel() * 4 + g[2].numel() * 8 + g[3].numel() * 2)
        _phase(rank, "gather timed")

    per = {}
    for name, ms in kt:
        per.setdefault(name, []).append(ms)
    payload = (bits + 7) // 8
    nh = state["s"].n if a.frontend else n   # symbols the Huffman stage codes (front-end output in C5)
    if a.frontend:
        ngroups, nchunks = c.sync_sizes(nh, S)
    sync_bytes = ngroups * 8 + nchunks * 2
    alg = {"hist_blocks": nh, "huff_pack": nh + payload + sync_bytes, "huff_decode": payload + sync_bytes + nh}
    if a.frontend:   # SURVEY §8(d), as for nybble: the front-end moves N + its output each way
        alg.update({"small_write": n + nh, "small_dec_write": nh + n, "small_body_tiles": n, "small_dec_tiles": nh,
                    # the fused encode (world 1): the input read twice, the payload and index written
                    "fe_hist_blocks": n, "fe_pack": n + payload + sync_bytes})
    kernels = {}
    for name, v in per.items():
        m = float(np.mean(v))
        e = {"ms": round(m, 4), "launches_per_step": len(v) // a.profile_steps}
        if name in alg:
            e["GBps"] = round(alg[name] / (m * 1e-3) / 1e9, 1)
        kernels[name] = e
    dom = max(per, key=lambda k: float(np.sum(per[k])))
    dom_ms = float(np.mean(per[dom]))
    dom_bytes = alg.get(dom, n)
    achieved = dom_bytes / (dom_ms * 1e-3) / 1e9
    traffic, traffic_src = pmc_traffic("k_" + dom, a, n)
    rp_ms, rp_src = rocprof_mean("k_" + dom, a, n)

    # whole-pipeline rooflines (SURVEY §8(d) bytes over the whole encode / whole decode time:
    # extra passes such as the histogram's read of the input count against them)
    enc_alg = n + payload + sync_bytes   # the pipeline's input (C5: before the front-end) + its output
    enc_frac = enc_alg / (enc_ms * 1e-3) / HBM_PEAK
    dec_frac = enc_alg / (dec_ms * 1e-3) / HBM_PEAK
    value = world * n / (ms_step * 1e-3) / 1e9
    res = {
        "metric": METRIC,
        "value": round(value, 2),
        "unit": "GB/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "prewarm": a.prewarm,
        "ms_per_step": round(ms_step, 4),
        "in_flight": len(lanes),
        "in_flight_inputs": "distinct",
        "ms_per_step_serial": round(ms_serial, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic",
        "config": {"workload": f"{a.cfg} {CFG_TEXT.get(a.cfg, a.cfg)}, {n >> 20} MiB per GPU, "
                               + ("small front-end + " if a.frontend else "")
                               + f"n={a.nary} Huffman encode+decode"
                               + (" (configs[1] generator at the metric's 1 GiB)" if a.cfg == "C2" else ""),
                   "frontend": bool(a.frontend), "fused": bool(a.frontend and getattr(state["s"], "fused", False)),
                   "bytes_per_gpu": n, "n_ary": a.nary, "sync_syms": S,
                   "parallelism": f"shard{world}" if world > 1 else "single"},
        "roofline": {"bound": "hbm", "kernel": dom, "achieved": round(achieved, 1), "peak": HBM_PEAK / 1e9,
                     "unit": "GB/s", "frac": round(achieved * 1e9 / HBM_PEAK, 4), "traffic": traffic,
                     "traffic_source": traffic_src,
                     "alg_bytes_per_launch": dom_bytes, "mean_ms": round(dom_ms, 4),
                     "frac_rocprof": round(dom_bytes / (rp_ms * 1e-3) / HBM_PEAK, 4) if rp_ms else None,
                     "rocprof_mean_ms": round(rp_ms, 4) if rp_ms else None, "rocprof_source": rp_src,
                     "frac_headline": "frac: HIP events around each launch in this run (they include the "
                                      "launch's own dispatch gap, so they read a few % above rocprof); "
                                      "frac_rocprof: the committed rocprofv3 kernel-trace mean of this command "
                                      "over the dispatches no other kernel overlapped",
                     "copy_probe_GBps": _r(copy_gbps, 1),
                     "frac_vs_copy": _r(copy_gbps and achieved / copy_gbps, 4),
                     "encode_frac": round(enc_frac, 4), "decode_frac": round(dec_frac, 4),
                     "encode_frac_vs_copy": _r(copy_gbps and enc_frac * HBM_PEAK / 1e9 / copy_gbps, 4),
                     "decode_frac_vs_copy": _r(copy_gbps and dec_frac * HBM_PEAK / 1e9 / copy_gbps, 4),
                     "encode_ms": round(enc_ms, 4), "decode_ms": round(dec_ms, 4),
                     "split_step_ms": round(split_step_ms, 4),
                     "split_source": f"HIP events inside {a.profile_steps} back-to-back steps after the timed region",
                     "pipeline_alg_bytes": enc_alg},
        "encode_GBps": round(n / (enc_ms * 1e-3) / 1e9, 2),
        "decode_GBps": round(n / (dec_ms * 1e-3) / 1e9, 2),
        "ratio": round(payload / n, 4),
        "kernels": kernels,
        "roundtrip_ok": ok,
    }
    if world > 1:
        res["table_mode"] = a.table_mode
        if gather is not None:
            res["gather"] = gather
    if rank == 0 and world == 1 and not a.no_cpu:
        res["cpu_baseline"] = cpu_baseline(x, a)
    if rank == 0:
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()


NYB_METRIC = "GB/s nybble encode+decode on 1 GiB byte stream per MI355X; % HBM roofline"


def main_nybble(a, dev, rank, world):
    """nybble_compression.c's codec as a bench line: 1 GiB of the C1
    English-like text generator per GPU, device-resident. A step = the whole codec call(s),
    each ending in its host read of the output length (the reference API returns the length):
      static   compress_bytestring(modify=false) + decompress_bytestring of its output
      adaptive nybble_compress (modify=true); its decode is sequential by definition (each
               byte's list depends on every byte before it), timed once on a 16 MiB sample
    N > 1: every rank codes its own 1 GiB stream (independent objects, no collective)."""
    n = a.size
    modify = a.mode == "adaptive"
    x = bench_input("C1", n, 0xC1 + 7919 * rank, dev)
    torch.cuda.synchronize()
    lanes = [NybLane(dev, x if i == 0 else x.clone(), modify) for i in range(max(1, a.in_flight))]   # distinct inputs
    lane0 = lanes[0]
    c, st, encode, decode, step = lane0.c, lane0.st, lane0.encode, lane0.decode, lane0.step
    # (no collective in a step: every lane has a host thread of its own at any N)
    run_steps(lanes, a.prewarm + a.warmup, True)
    torch.cuda.synchronize()
    ms_step = timed_steps(lanes, a.steps, True, world, dev)
    ms_serial = timed_steps(lanes[:1], a.steps, False, world, dev) if len(lanes) > 1 else ms_step
    torch.cuda.set_stream(lane0.stream)   # the rest runs on lane 0 (its codec's stream)
    m = st["comp"].numel()

    def timed(fn, k):
        fn()
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(k):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t) / k * 1e3

    enc_ms = timed(encode, a.profile_steps)
    if modify:   # the sequential whole-stream decode, on a sample; the round trip of that sample
        xs = x[: 16 << 20]
        cs = c.nyb_compress(xs, True)
        ys = c.nyb_decompress(cs, True)
        torch.cuda.synchronize()
        t = time.perf_counter()
        ys = c.nyb_decompress(cs, True)
        torch.cuda.synchronize()
        dec_sample_ms = (time.perf_counter() - t) * 1e3
        ok = bool(torch.equal(ys, xs))
        dec_ms = None
        # the many-stream throughput path (dc_nyb_decompress_batch, one lane per stream): the
        # first 256 MiB as independent 4 KiB streams (each the reference's nybble_compress of its
        # bytes, as the DCNK container holds them), decoded from their concatenation + offsets
        KB = 4096
        xb = x[: min(n, 256 << 20)]
        cont = c.nyb_compress_chunked(xb, True, KB)
        nch = (xb.numel() + KB - 1) // KB
        offs = cont[32: 32 + 8 * (nch + 1)].view(torch.int64).clone()
        pay = cont[32 + 8 * (nch + 1):]
        yb, _ = c.nyb_decompress_batch(pay, offs, True, out_cap=xb.numel())
        torch.cuda.synchronize()
        t = time.perf_counter()
        reps = 5
        for _ in range(reps):
            yb, _ = c.nyb_decompress_batch(pay, offs, True, out_cap=xb.numel())
        torch.cuda.synchronize()
        bt = (time.perf_counter() - t) / reps
        ok = ok and bool(torch.equal(yb, xb))
        dec_batch = {"streams": int(nch), "stream_bytes": KB, "bytes": int(xb.numel()), "ms": round(bt * 1e3, 3),
                     "GBps": round(xb.numel() / bt / 1e9, 2),
                     "path": "dc_nyb_decompress_batch: one lane per independent stream (lengths, scan, decode)"}
    else:
        dec_ms = timed(decode, a.profile_steps)
        ok = True
    c.timing(True)
    for _ in range(a.profile_steps):
        step()
    kt = c.timings()
    c.timing(False)
    # round trips after the timings (bench.py main: a 1 GiB compare slows the steps after it);
    # adaptive: every lane's stream equals lane 0's, whose round trip the sample checked
    ok = ok and all([ln.roundtrip_ok() if not modify else bool(torch.equal(ln.st["comp"], st["comp"]))
                     for ln in lanes])
    per = {}
    for name, ms in kt:
        per.setdefault(name, []).append(ms)
    # SURVEY §8(d), nybble: N + N_comp each way; the plan (tiles) passes read one side
    # (adaptive: the MTF walk reads the input and writes a rank per element; the resolve pass
    # reads only the first-touch step records, not priced here)
    alg = {"nyb_enc_tiles": n, "nyb_enca_tiles": n, "nyb_enc_write": n + m, "nyb_dec_tiles": m,
           "nyb_dec_write": m + n, "mtf_tiles": 2 * n if modify else n}
    kernels = {}
    for name, v in per.items():
        mm = float(np.mean(v))
        e = {"ms": round(mm, 4), "launches_per_step": len(v) // a.profile_steps}
        if name in alg:
            e["GBps"] = round(alg[name] / (mm * 1e-3) / 1e9, 1)
        kernels[name] = e
    dom = max(per, key=lambda k: float(np.sum(per[k])))
    dom_ms = float(np.mean(per[dom]))
    dom_bytes = alg.get(dom, n)
    achieved = dom_bytes / (dom_ms * 1e-3) / 1e9
    wl = f"C1-nyb-{a.mode}"
    # the timed stage's kernel as the PMC summary names it (template argument = the transducer mode)
    # (the writers: a wave per tile for the static encode and the decode, k_fsm_write for the
    # adaptive encode's ranks; DC_OPT_NYB_WTILE_OFF, dc_gpu.h)
    kname = {"nyb_enc_tiles": "k_nyb_tiles<0>", "nyb_enca_tiles": "k_fsm_tiles<0>",
             "nyb_enc_write": "k_nyb_enc_wtile<true>" if modify else "k_nyb_enc_wtile<false>",
             "nyb_dec_tiles": "k_nyb_tiles<1>", "nyb_dec_write": "k_nyb_dec_wtile",
             "mtf_tiles": "k_mtf_walk<2>" if modify else "k_mtf_walk<0>", "mtf_ranks": "k_mtf_resolve"}.get(dom, "k_" + dom)
    traffic, traffic_src = pmc_traffic(kname, argparse.Namespace(cfg=wl, nary=0), n)
    if traffic is None and "<" in kname:   # (a summary from before the kernel was a template)
        traffic, traffic_src = pmc_traffic(kname.split("<")[0], argparse.Namespace(cfg=wl, nary=0), n)
    kern_sum = sum(float(np.sum(v)) for v in per.values()) / a.profile_steps
    enc_frac = (n + m) / (enc_ms * 1e-3) / HBM_PEAK
    res = {
        "metric": NYB_METRIC if not modify else NYB_METRIC.replace("encode+decode", "encode"),
        "value": round(world * n / (ms_step * 1e-3) / 1e9, 2),
        "unit": "GB/s", "n_gpus": world, "steps": a.steps, "warmup": a.warmup, "prewarm": a.prewarm,
        "ms_per_step": round(ms_step, 4),
        "in_flight": len(lanes),
        "in_flight_inputs": "distinct",
        "ms_per_step_serial": round(ms_serial, 4), "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "dtype": "u8", "data": "synthetic",
        "config": {"workload": f"nybble {'adaptive (nybble_compress)' if modify else 'static (compress_bytestring)'}"
                               f" on {n >> 20} MiB of C1 English-like text per GPU"
                               + ("; encode per step (decode: sequential, decode_sample)" if modify else
                                  "; encode + decode per step"),
                   "codec": "nybble", "mode": a.mode, "bytes_per_gpu": n,
                   "parallelism": f"replica{world}" if world > 1 else "single"},
        "roofline": {"bound": "hbm", "kernel": dom, "achieved": round(achieved, 1), "peak": HBM_PEAK / 1e9,
                     "unit": "GB/s", "frac": round(achieved * 1e9 / HBM_PEAK, 4), "traffic": traffic,
                     "traffic_source": traffic_src, "alg_bytes_per_launch": dom_bytes, "mean_ms": round(dom_ms, 4),
                     "encode_frac": round(enc_frac, 4), "encode_ms": round(enc_ms, 4),
                     "kernel_sum_ms_per_step": round(kern_sum, 4), "pipeline_alg_bytes": n + m},
        "encode_GBps": round(n / (enc_ms * 1e-3) / 1e9, 2),
        "ratio": round(m / n, 4),
        "kernels": kernels,
        "roundtrip_ok": ok,
    }
    if dec_ms is not None:
        res["roofline"].update({"decode_frac": round((m + n) / (dec_ms * 1e-3) / HBM_PEAK, 4),
                                "decode_ms": round(dec_ms, 4)})
        res["decode_GBps"] = round(n / (dec_ms * 1e-3) / 1e9, 2)
    else:
        res["decode_sample"] = {"bytes": 16 << 20, "ms": round(dec_sample_ms, 2),
                                "MBps": round((16 << 20) / (dec_sample_ms * 1e-3) / 1e6, 1),
                                "path": "tokens (parallel transducer) + control words + k_nyb_resolve_c (one wave)"}
        res["decode_batch"] = dec_batch
    if rank == 0 and world == 1 and not a.no_cpu:
        res["cpu_baseline"] = cpu_baseline_nybble(x, a, modify)
    if rank == 0:
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()


class NybLane:
    """bench.py's nybble step (main_nybble) on a codec context of its own, on its own HIP stream
    with its own buffers (steps in flight, as Lane)."""

    def __init__(self, dev, x, modify):
        from data_compression_amd.device import Codec
        n = x.numel()
        self.stream = torch.cuda.Stream(dev)
        self.x, self.modify, self.st = x, modify, {}
        with torch.cuda.stream(self.stream):
            self.c = Codec(dev.index or 0, stream=self.stream)
            self.comp_buf = torch.empty(n + 2, dtype=torch.uint8, device=dev)
            self.out = torch.empty(2 * n + 16, dtype=torch.uint8, device=dev)

    def encode(self):
        self.st["comp"] = self.c.nyb_compress(self.x, self.modify, out=self.comp_buf)

    def decode(self):
        self.st["y"] = self.c.nyb_decompress(self.st["comp"], self.modify, out=self.out)

    def step(self):
        with torch.cuda.stream(self.stream):
            self.encode()
            if not self.modify:
                self.decode()

    def roundtrip_ok(self):   # (adaptive: main_nybble checks a sample's round trip)
        with torch.cuda.stream(self.stream):
            return self.modify or bool(torch.equal(self.st["y"], self.x))


def cpu_baseline_nybble(x, a, modify):
    """The oracle's nybble codec (oracle/dc_oracle.c, nybble_compression.c restated) on one
    pinned host core: a bounded sample of the same stream, encode + decode."""
    from oracle import oracle as orc
    m = min(a.cpu_sample, x.numel()) if not modify else min(a.cpu_sample, 64 << 20, x.numel())
    s = x[:m].cpu().numpy().tobytes()
    old = os.sched_getaffinity(0)
    core = min(old)
    os.sched_setaffinity(0, {core})
    reps = []
    try:
        for _ in range(CPU_REPS):
            t0 = time.perf_counter()
            comp = orc.nybble_compress(s, modify)
            t1 = time.perf_counter()
            back = orc.nybble_decompress(comp, modify)
            t2 = time.perf_counter()
            assert back == s
            r = _cpu_report(m, t0, t1, t2, core, f"nybble {'adaptive' if modify else 'static'}, ")
            r["encode_GBps"] = round(m / (t1 - t0) / 1e9, 4)
            r["decode_GBps"] = round(m / (t2 - t1) / 1e9, 4)
            reps.append(r)
    finally:
        os.sched_setaffinity(0, old)
    return _cpu_median(reps)


def bench_input(cfg, n, seed, dev):
    """The synthetic input, generated on the device (synth.device_text). DC_BENCH_SYNTH=host
    generates it with the numpy generator instead and copies it over: for rehearsals whose
    ranks share one GPU, where several processes' torch generation at once stalled inside
    torch (tools/synth_stall.py)."""
    from data_compression_amd import synth
    if os.environ.get("DC_BENCH_SYNTH") == "host":
        return torch.from_numpy(synth.GENERATORS[cfg](n, seed=seed)).to(dev)
    return synth.device_text(cfg, n, seed=seed, device=dev)


def input_seed(cfg, rank):
    """Seed of rank r's synthetic shard (C4 is seeded 0xC4 + rank; the other
    configs keep the r2 seeds, 0xC2 + 7919 r, which the committed profiles were measured on)."""
    return 0xC4 + rank if cfg == "C4" else 0xC2 + 7919 * rank


_T0 = time.perf_counter()


def _phase(rank, what):
    """DC_BENCH_PHASES=1: a timestamped progress line per rank on stderr (multi-rank
    rehearsals: where each rank is when one stalls)."""
    if os.environ.get("DC_BENCH_PHASES"):
        sys.stderr.write(f"[rank {rank}] {time.perf_counter() - _T0:8.2f} s  {what}\n")
        sys.stderr.flush()


def _trace_setup(rank):
    """DC_BENCH_TRACE_AFTER=T: every rank writes its Python stacks every T seconds to
    gpurun_out/trace_rank<r>.log and keeps running (none exits first, so a stall leaves
    the stacks of all ranks, not just of the one whose timer fired)."""
    t = os.environ.get("DC_BENCH_TRACE_AFTER")
    if not t:
        return
    import faulthandler
    os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
    f = open(os.path.join(REPO, "gpurun_out", f"trace_rank{rank}.log"), "w")
    _trace_setup.f = f   # keep the file open for the process's lifetime
    faulthandler.dump_traceback_later(float(t), repeat=True, file=f, exit=False)


def _pos_checksum(t, off):
    """sum over i of (t[i] + 1) * w(off + i) mod 2^64, w a 32-bit multiplicative hash of the
    global position (int64 arithmetic wraps)."""
    h = torch.zeros((), dtype=torch.int64, device=t.device)
    step = 1 << 26
    for a in range(0, t.numel(), step):
        v = t[a: a + step].to(torch.int64) + 1
        idx = torch.arange(off + a, off + a + v.numel(), dtype=torch.int64, device=t.device)
        h += (v * ((idx * 0x9E3779B1) & 0xFFFFFFFF)).sum()
    return h


def _concat_equal(y, x, world, dev):
    """Whether the ranks' y segments, concatenated in rank order, equal the ranks' x shards
    concatenated (lengths and position-weighted checksums, summed over ranks)."""
    n = torch.tensor([y.numel(), x.numel()], dtype=torch.int64, device=dev)
    alln = [torch.empty_like(n) for _ in range(world)]
    dist.all_gather(alln, n)
    alln = [v.tolist() for v in alln]
    r = dist.get_rank()
    oy, ox = sum(v[0] for v in alln[:r]), sum(v[1] for v in alln[:r])
    hs = torch.stack([_pos_checksum(y, oy), _pos_checksum(x, ox)])
    dist.all_reduce(hs)
    return sum(v[0] for v in alln) == sum(v[1] for v in alln) and bool(hs[0] == hs[1])


CFG_TEXT = {"C2": "enwik-like text", "C3": "uniform random bytes", "C4": "Zipf s=1 bytes",
            "C5": "syslog-like text"}


def profile_files(kind):
    """The committed summaries of one kind ("pmc_traffic" or "rocprof"), newest first, in the
    order profiles/INDEX.json lists them (by when the profile was taken: the file names' round
    tags are not in time order, r4f was taken after r4q). Files the index does not list are
    never cited."""
    try:
        idx = json.load(open(os.path.join(REPO, "profiles", "INDEX.json")))
    except (OSError, ValueError):
        return []
    return [os.path.join(REPO, "profiles", f) for f in idx.get(kind, [])]


def pmc_traffic(kernel, a, n):
    """HBM bytes per launch of `kernel` from the newest committed PMC summary
    (profiles/*_pmc_traffic.json, written by tools/pmc.sh + tools/pmc_report.py from separate
    --pmc passes of this same bench command; FETCH_SIZE x2 per MI355X_MICROARCH.md). PMC
    counters cannot be read inside the timed run, so the figure is the profiled run's,
    reported only when that run's workload matches this one."""
    for f in profile_files("pmc_traffic"):
        try:
            d = json.load(open(f))
        except (OSError, ValueError):
            continue
        w = d.get("workload", {})
        if (w.get("cfg"), w.get("size"), w.get("n_ary")) != (a.cfg, n, a.nary):
            continue
        k = d.get("kernels", {}).get(kernel)
        if k:
            return k["traffic_bytes"], os.path.relpath(f, REPO)
    return None, None


def rocprof_mean(kernel, a, n):
    """Mean launch duration (ms) of `kernel` from the newest committed rocprofv3 --stats summary
    of this bench command (profiles/*_rocprof.json, tools/rocprof_report.py), when its workload
    matches: the roofline fraction by rocprof beside the HIP-event one."""
    for f in profile_files("rocprof"):
        try:
            d = json.load(open(f))
        except (OSError, ValueError):
            continue
        w = d.get("workload", {})
        if (w.get("cfg"), w.get("size"), w.get("n_ary")) != (a.cfg, n, a.nary):
            continue
        k = d.get("kernels", {}).get(kernel)
        if k:
            # the dispatches no other kernel overlapped (the timed loop runs steps in flight,
            # whose kernels overlap; the HIP-event times beside it come from one context alone)
            return k.get("mean_ms_isolated", k["mean_ms"]), os.path.relpath(f, REPO)
    return None, None


def _r(v, nd):
    return None if v is None else round(v, nd)


class Lane:
    """One codec context on its own HIP stream with its own buffers: the bench step (encode +
    decode of the whole input x, world ranks) as lane.step(). Steps in flight (--in-flight)
    are lanes taking alternate steps; a lane's state holds its last step's stream and output."""

    def __init__(self, a, dev, local, x, S, n, world):
        from data_compression_amd.device import Codec
        from data_compression_amd.dist import ShardedHuffman, ShardedSmall
        self.stream = torch.cuda.Stream(dev)
        self.x, self.n, self.world, self.dev, self.frontend = x, n, world, dev, a.frontend
        self.state = st = {}
        with torch.cuda.stream(self.stream):
            self.c = c = Codec(local, stream=self.stream)
            self.sh = sh = ShardedHuffman(c, table_mode=a.table_mode)
            hist = torch.empty(256, dtype=torch.int64, device=dev)
            self.tab = tab = torch.empty(c.table_bytes, dtype=torch.uint8, device=dev)
            self.total = total = torch.empty(1, dtype=torch.int64, device=dev)
            words = torch.empty(c.words_needed(2**40, 32 * n) + 8, dtype=torch.int32, device=dev)
            if not a.frontend:
                sync = c.alloc_sync(n, S)
                self.out = out = torch.empty(n, dtype=torch.uint8, device=dev)

                def encode():   # hist -> [all_reduce] -> table -> plan -> [all_gather] -> pack
                    st["s"] = sh.encode(x, a.nary, S, words=words, sync=sync, hist=hist, table=tab, total=total)

                def decode():
                    sh.decode(st["s"], out=out)
                    st["dec"] = out
            else:   # C5: front-end bodies + halo/LITERAL/re-cut exchanges, then sharded Huffman
                ss = ShardedSmall(c, table_mode=a.table_mode, fused=not a.two_stage)
                sync_fe = c.alloc_sync(n + 1, S)   # the front-end stream holds up to n + 1 symbols
                gsync_fe = c.alloc_sync(n + 1 + 2 * S, S) if world > 1 else None   # (a shard's part of the stream's index)
                fe_out = torch.empty(2 * n + 64, dtype=torch.uint8, device=dev)   # dc_small_decompress: >= 2 * m

                def encode():
                    st["s"] = ss.encode(x, a.nary, S, words=words, sync=sync_fe, table=tab, total=total, gsync=gsync_fe)

                def decode():
                    st["dec"] = ss.decode(st["s"], out=fe_out)
        self.encode, self.decode = encode, decode

    def step(self):
        with torch.cuda.stream(self.stream):
            self.encode()
            self.decode()

    def roundtrip_ok(self):
        with torch.cuda.stream(self.stream):
            y = self.state["dec"]
            if self.frontend and self.world > 1:
                # a rank's decoded front-end segment covers a different byte range than its input
                # shard (the re-cut moves bytes between ranks): compare the concatenations through
                # a position-weighted checksum over global offsets
                ok = _concat_equal(y, self.x, self.world, self.dev)
            else:
                ok = bool(torch.equal(y, self.x))
            return self.c.decode_status() == 0 and ok


def run_steps(lanes, k, threaded):
    """k steps, step i on lane i mod L. threaded: one host thread per lane (a codec call that
    ends in a host read then blocks only its own lane); otherwise issued in order by this
    thread (at N > 1: every rank's collectives in the same order)."""
    nl = len(lanes)
    if nl == 1 or not threaded:
        for i in range(k):
            lanes[i % nl].step()
        return
    import threading
    dev = torch.cuda.current_device() if torch.cuda.is_available() else None
    errs = []

    def work(j):
        try:
            if dev is not None:   # (the current device is per thread)
                torch.cuda.set_device(dev)
            for _ in range(j, k, nl):
                lanes[j].step()
        except BaseException as e:   # re-raised on the calling thread
            errs.append(e)

    ts = [threading.Thread(target=work, args=(j,)) for j in range(1, nl)]
    for t in ts:
        t.start()
    work(0)
    for t in ts:
        t.join()
    if errs:
        raise errs[0]


def timed_steps(lanes, k, threaded, world, dev):
    """ms per step of k steps over the lanes, bracketed by a barrier and a device-wide
    synchronize on both sides; the max over ranks."""
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    run_steps(lanes, k, threaded)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    if world > 1:
        tt = torch.tensor([el], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        el = float(tt.item())
    return el / k * 1e3


def split_timed(encode, decode, k):
    """Encode and decode time per step from HIP events recorded inside K back-to-back steps:
    e0 before the encode, e1 between encode and decode, e2 after the decode. Returns
    (encode ms, decode ms, step ms), means over the K steps; the step time spans e0 of the
    first step to e2 of the last, divided by K."""
    ev = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(k)]
    for e in ev:
        e[0].record()
        encode()
        e[1].record()
        decode()
        e[2].record()
    torch.cuda.synchronize()
    enc = float(np.mean([e[0].elapsed_time(e[1]) for e in ev]))
    dec = float(np.mean([e[1].elapsed_time(e[2]) for e in ev]))
    return enc, dec, ev[0][0].elapsed_time(ev[-1][2]) / k


def copy_probe(c, x, reps):
    """The chip's achievable HBM rate on this box, the reference for the fractions: a
    hand-written float4 copy of the input (dc_copy_probe: 16-B loads and stores), read +
    write bytes over its mean HIP-event time on the codec's stream. Probes the 16-B aligned
    prefix; None when the probe cannot run (the codec's line is printed either way)."""
    m = x.numel() & ~15
    if m < (1 << 20):
        return None
    try:
        y = torch.empty(m, dtype=torch.uint8, device=x.device)
        c.copy_probe(x[:m], y)
        c.timing(True)
        for _ in range(reps):
            c.copy_probe(x[:m], y)
        ms = float(np.mean([t for name, t in c.timings() if name == "copy_probe"]))
        c.timing(False)
        del y
    except Exception:   # e.g. no room for the second buffer: report no reference rate
        c.timing(False)
        return None
    return 2 * m / (ms * 1e-3) / 1e9


CPU_REPS = 3   # the CPU baseline is the median of this many timings (the spread is reported)


def cpu_baseline(x, a):
    """Oracle (single-threaded C restatement, oracle/dc_oracle.c) on a bounded sample, pinned
    to one host core (taskset -c 0 equivalent) for the timed part; the median of
    CPU_REPS timings, with their spread."""
    from oracle import oracle as orc
    m = min(a.cpu_sample, x.numel())
    s = x[:m].cpu().numpy()
    old = os.sched_getaffinity(0)
    core = min(old)
    os.sched_setaffinity(0, {core})
    try:
        return _cpu_median([_cpu_timed(orc, s, m, a, core) for _ in range(CPU_REPS)])
    finally:
        os.sched_setaffinity(0, old)


def _cpu_median(reps):
    """The median run of the CPU baseline, with every run's value and the spread."""
    vals = [r["value"] for r in reps]
    med = dict(sorted(reps, key=lambda r: r["value"])[len(reps) // 2])
    med["reps"] = vals
    med["spread"] = round((max(vals) - min(vals)) / med["value"], 4) if med["value"] else None
    med["sample"] += f"; median of {len(reps)} timings"
    return med


def _cpu_timed(orc, s, m, a, core):
    if a.frontend:   # C5 leg: the reference front-end, then the Huffman codec on its output
        t0 = time.perf_counter()
        fe = np.frombuffer(orc.small_compress(s.tobytes()), np.uint8)
        h = orc.histogram(fe)
        L = orc.huffman_lengths(h, a.nary)
        el, ev = orc.canonical(L, a.nary)
        code, nb, _ = orc.bitcodes(el, ev, a.nary)
        payload, bits, _ = orc.huff_pack(fe, code, nb, sync_syms=4096)
        t1 = time.perf_counter()
        back_fe = orc.huff_unpack(payload, bits, fe.size, el, ev, a.nary)
        back = np.frombuffer(orc.small_decompress(back_fe.tobytes()), np.uint8)
        t2 = time.perf_counter()
        assert np.array_equal(back, s)
        return _cpu_report(m, t0, t1, t2, core, "small front-end + n-ary Huffman, ")
    t0 = time.perf_counter()
    h = orc.histogram(s)
    L = orc.huffman_lengths(h, a.nary)
    el, ev = orc.canonical(L, a.nary)
    code, nb, _ = orc.bitcodes(el, ev, a.nary)
    payload, bits, _ = orc.huff_pack(s, code, nb, sync_syms=4096)
    t1 = time.perf_counter()
    back = orc.huff_unpack(payload, bits, m, el, ev, a.nary)
    t2 = time.perf_counter()
    assert np.array_equal(back, s)
    return _cpu_report(m, t0, t1, t2, core, "")


def _cpu_report(m, t0, t1, t2, core, what):
    try:
        cpu = open("/proc/cpuinfo").read().split("model name")[1].split("\n")[0].strip(": \t")
    except Exception:
        cpu = "unknown"
    return {"value": round(m / (t2 - t0) / 1e9, 4), "unit": "GB/s", "cores": 1, "kind": "port",
            "sample": f"{what}first {m >> 20} MiB of the rank-0 stream; encode {t1 - t0:.2f} s + decode "
                      f"{t2 - t1:.2f} s; pinned to cpu {core}; {cpu}; nproc={os.cpu_count()}"}


if __name__ == "__main__":
    main()
