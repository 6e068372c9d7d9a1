"""Build recipe for the native libraries (in-tree, so they travel with the repo snapshot).

    python -m data_compression_amd.build          # or __graft_entry__.build()

  lib/libdc_core.so     gfx950 HIP kernels + dc_gpu.h / dc_host.h API   (hipcc)
  lib/libdc_huffman.so  drop-in for n_ary_huffman.c public functions    (g++, links core)
  lib/libdc_nybble.so   drop-in for nybble_compression.c codec          (g++, links core)
  lib/libdc_small.so    drop-in for small_compression.c front-end       (g++, links core)

Only gfx950 code objects are produced (no CUDA, no multi-arch fat binary).
"""
from __future__ import annotations

import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

PKG = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
LIB = os.path.join(PKG, "lib")
INC = os.path.join(REPO, "include")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("DC_OFFLOAD_ARCH", "gfx950")

CORE_SRC = ["dc_core.hip", "dc_host.hip"]
SHIMS = {
    "libdc_huffman.so": "dc_huffman_abi.cpp",
    "libdc_nybble.so": "dc_nybble_abi.cpp",
    "libdc_small.so": "dc_small_abi.cpp",
}


def _run(cmd):
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        sys.stderr.write(" ".join(cmd) + "\n" + r.stdout + r.stderr)
        raise RuntimeError(f"build step failed: {cmd[-1]}")
    return r


def _stale(target, deps):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def build(force: bool = False, verbose: bool = False) -> None:
    os.makedirs(LIB, exist_ok=True)
    headers = [os.path.join(INC, h) for h in os.listdir(INC) if h.endswith(".h")]
    hdr_local = [os.path.join(CSRC, h) for h in os.listdir(CSRC) if h.endswith(".h")]
    core = os.path.join(LIB, "libdc_core.so")
    core_deps = [os.path.join(CSRC, s) for s in CORE_SRC] + headers + hdr_local
    objs = []
    jobs = []
    for s in CORE_SRC:
        src = os.path.join(CSRC, s)
        obj = os.path.join(LIB, s.replace(".hip", ".o"))
        objs.append(obj)
        if force or _stale(obj, [src] + headers + hdr_local):
            jobs.append([HIPCC, f"--offload-arch={ARCH}", "-O3", "-fPIC", "-std=c++17", "-Wall",
                         "-I" + INC, "-I" + CSRC, "-c", src, "-o", obj])
    with ThreadPoolExecutor(max_workers=4) as ex:
        list(ex.map(_run, jobs))
    if force or jobs or _stale(core, core_deps + objs):
        _run([HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", core] + objs)
    shim_jobs = []
    for lib, src in SHIMS.items():
        target = os.path.join(LIB, lib)
        srcp = os.path.join(CSRC, src)
        if force or _stale(target, [srcp, core] + headers + hdr_local):
            shim_jobs.append(["g++", "-O2", "-fPIC", "-shared", "-std=c++17", "-Wall", "-Wextra",
                              "-I" + INC, "-I" + CSRC, srcp, "-o", target, "-L" + LIB, "-ldc_core",
                              "-Wl,-rpath,$ORIGIN"])
    with ThreadPoolExecutor(max_workers=4) as ex:
        list(ex.map(_run, shim_jobs))
    if verbose:
        print("built:", sorted(os.listdir(LIB)))


if __name__ == "__main__":
    build(force="--force" in sys.argv, verbose=True)
