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
    ap.add_argument("--cfg", default="C2")
    ap.add_argument("--frontend", action="store_true",
                    help="C5 pipeline: small_compression.c front-end, then n-ary Huffman (dist.ShardedSmall)")
    ap.add_argument("--nary", type=int, default=2)
    ap.add_argument("--size", type=int, default=1 << 30, help="bytes per GPU")
    ap.add_argument("--sync", type=int, default=0, help="sync-index granularity (0 = default)")
    ap.add_argument("--cpu-sample", type=int, default=256 << 20)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--table-mode", default="replicate", choices=["replicate", "broadcast"],
                    help="multi-GPU code table: built on every rank, or on rank 0 and broadcast")
    ap.add_argument("--profile-steps", type=int, default=20)
    return ap.parse_args()


def main():
    a = parse()
    if os.environ.get("DC_BENCH_TRACE_AFTER"):   # diagnosis of a stuck rank: Python stacks, then exit
        import faulthandler
        faulthandler.dump_traceback_later(float(os.environ["DC_BENCH_TRACE_AFTER"]), exit=True)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
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

    n = a.size
    x = synth.device_text(a.cfg, n, seed=0xC2 + 7919 * rank, device=dev)
    torch.cuda.synchronize()
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

    from data_compression_amd.dist import ShardedHuffman
    sh = ShardedHuffman(c, table_mode=a.table_mode)
    hist = torch.empty(256, dtype=torch.int64, device=dev)
    tab = torch.empty(c.table_bytes, dtype=torch.uint8, device=dev)
    total = torch.empty(1, dtype=torch.int64, device=dev)
    words = torch.empty(c.words_needed(2**40, 32 * n) + 8, dtype=torch.int32, device=dev)
    sync = c.alloc_sync(n, S)
    out = torch.empty(n, dtype=torch.uint8, device=dev)
    state = {}

    def encode():   # hist -> [all_reduce] -> table -> plan -> [all_gather] -> pack
        state["s"] = sh.encode(x, a.nary, S, words=words, sync=sync, hist=hist, table=tab, total=total)

    def decode():
        sh.decode(state["s"], out=out)

    if a.frontend:   # C5: front-end bodies + halo/LITERAL/re-cut exchanges, then sharded Huffman
        from data_compression_amd.dist import ShardedSmall
        ss = ShardedSmall(c, table_mode=a.table_mode)

        def encode():   # noqa: F811
            state["s"] = ss.encode(x, a.nary, S)

        fe_out = torch.empty(2 * n + 64, dtype=torch.uint8, device=dev)   # dc_small_decompress: >= 2 * m

        def decode():   # noqa: F811
            state["dec"] = ss.decode(state["s"], out=fe_out)

    def step():
        encode()
        decode()

    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    if world > 1:
        tt = torch.tensor([el], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        el = float(tt.item())
    ms_step = el / a.steps * 1e3

    # ---- correctness of the measured configuration (outside the timed region) ----------
    st = c.pack_status(state["s"].table if a.frontend else tab)
    y = state["dec"] if a.frontend else out
    if a.frontend and world > 1:
        # a rank's decoded front-end segment covers a different byte range than its input
        # shard (the re-cut moves bytes between ranks): compare the concatenations through a
        # position-weighted checksum over global offsets
        ok = st == 0 and c.decode_status() == 0 and _concat_equal(y, x, world, dev)
    else:
        ok = st == 0 and c.decode_status() == 0 and bool(torch.equal(y, x))
    bits = state["s"].bits if a.frontend else int(total.item())   # this rank's payload bits
    if world > 1:
        okt = torch.tensor([1 if ok else 0], device=dev)
        dist.all_reduce(okt, op=dist.ReduceOp.MIN)
        ok = bool(okt.item())

    # ---- encode / decode split and per-kernel HIP-event durations ------------------------
    def timed(fn, k):   # host-timed calls, one untimed call first (the stage switch)
        fn()
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(k):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t) / k * 1e3

    enc_ms = timed(encode, a.profile_steps)
    dec_ms = timed(decode, a.profile_steps)
    c.timing(True)
    for _ in range(a.profile_steps):
        step()
    kt = c.timings()
    c.timing(False)
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
        alg.update({"small_write": n + nh, "small_dec_write": nh + n, "small_body_tiles": n, "small_dec_tiles": nh})
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
        "ms_per_step": round(ms_step, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic",
        "config": {"workload": f"{a.cfg} {CFG_TEXT.get(a.cfg, a.cfg)}, {n >> 20} MiB per GPU, "
                               + ("small front-end + " if a.frontend else "")
                               + f"n={a.nary} Huffman encode+decode"
                               + (" (configs[1] generator at the metric's 1 GiB)" if a.cfg == "C2" else ""),
                   "frontend": bool(a.frontend),
                   "bytes_per_gpu": n, "n_ary": a.nary, "sync_syms": S,
                   "parallelism": f"shard{world}" if world > 1 else "single"},
        "roofline": {"bound": "hbm", "kernel": dom, "achieved": round(achieved, 1), "peak": HBM_PEAK / 1e9,
                     "unit": "GB/s", "frac": round(achieved * 1e9 / HBM_PEAK, 4), "traffic": traffic,
                     "traffic_source": traffic_src,
                     "alg_bytes_per_launch": dom_bytes, "mean_ms": round(dom_ms, 4),
                     "encode_frac": round(enc_frac, 4), "decode_frac": round(dec_frac, 4),
                     "encode_ms": round(enc_ms, 4), "decode_ms": round(dec_ms, 4),
                     "pipeline_alg_bytes": enc_alg},
        "encode_GBps": round(n / (enc_ms * 1e-3) / 1e9, 2),
        "decode_GBps": round(n / (dec_ms * 1e-3) / 1e9, 2),
        "ratio": round(payload / n, 4),
        "kernels": kernels,
        "roundtrip_ok": ok,
    }
    if rank == 0 and world == 1 and not a.no_cpu:
        res["cpu_baseline"] = cpu_baseline(x, a)
    if rank == 0:
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()


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


def pmc_traffic(kernel, a, n):
    """HBM bytes per launch of `kernel` from the newest committed PMC summary
    (profiles/*_pmc_traffic.json, written by tools/pmc.sh + tools/pmc_report.py from separate
    --pmc passes of this same bench command; FETCH_SIZE x2 per MI355X_MICROARCH.md). PMC
    counters cannot be read inside the timed run, so the figure is the profiled run's,
    reported only when that run's workload matches this one."""
    import glob
    files = sorted(glob.glob(os.path.join(REPO, "profiles", "*_pmc_traffic.json")))   # rNN_ prefix: newest last
    for f in reversed(files):
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


def cpu_baseline(x, a):
    """Oracle (single-threaded C restatement, oracle/dc_oracle.c) on a bounded sample, pinned
    to one host core (taskset -c 0 equivalent) for the timed part."""
    from oracle import oracle as orc
    m = min(a.cpu_sample, x.numel())
    s = x[:m].cpu().numpy()
    old = os.sched_getaffinity(0)
    core = min(old)
    os.sched_setaffinity(0, {core})
    try:
        return _cpu_timed(orc, s, m, a, core)
    finally:
        os.sched_setaffinity(0, old)


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
