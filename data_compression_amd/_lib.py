"""Loading of the in-tree native libraries (data_compression_amd/lib/*.so).

The libraries link the HIP runtime by soname (libamdhip64.so.7). PyTorch-ROCm ships its
own copy; importing torch first makes every later dlopen resolve to that one copy, so
the kernels and torch share one runtime (device memory, streams, RCCL). Nothing here
falls back to Python or CPU compute: a missing library raises.
"""
from __future__ import annotations

import ctypes as C
import os

try:  # one HIP runtime per process: torch's, when torch is present
    import torch  # noqa: F401
except Exception:  # pragma: no cover - torch is optional for the C-ABI itself
    torch = None

PKG = os.path.dirname(os.path.abspath(__file__))
LIBDIR = os.path.join(PKG, "lib")

_cache: dict[str, C.CDLL] = {}

vp = C.c_void_p
u8p = C.POINTER(C.c_uint8)
u64 = C.c_uint64
u32 = C.c_uint32
i32 = C.c_int


class DcError(RuntimeError):
    NAMES = {-1: "DC_E_ARG", -2: "DC_E_HIP", -3: "DC_E_CODE_TOO_LONG", -4: "DC_E_NOCODE",
             -5: "DC_E_STATE", -6: "DC_E_CAPACITY", -7: "DC_E_STREAM", -8: "DC_E_FALLBACK"}

    def __init__(self, fn, rc):
        super().__init__(f"{fn} failed: {self.NAMES.get(rc, rc)}")
        self.rc = rc


def check(fn, rc):
    if rc != 0:
        raise DcError(fn, rc)
    return rc


def lib_path(name: str) -> str:
    if name == "libdc_core.so" and os.environ.get("DC_CORE_LIB"):   # diagnostic builds (tools/)
        return os.environ["DC_CORE_LIB"]
    return os.path.join(LIBDIR, name)


def load(name: str) -> C.CDLL:
    if name in _cache:
        return _cache[name]
    path = lib_path(name)
    if not os.path.exists(path):
        raise RuntimeError(f"{path} is missing: run `python -m data_compression_amd.build` "
                           "(hipcc --offload-arch=gfx950); there is no CPU fallback")
    lib = C.CDLL(path)
    if name == "libdc_core.so":
        _declare_core(lib)
    _cache[name] = lib
    return lib


def core() -> C.CDLL:
    return load("libdc_core.so")


def _declare_core(L):
    P = vp
    sig = {
        "dc_ctx_create": ([C.POINTER(vp), i32, vp], i32),
        "dc_ctx_create_owned": ([C.POINTER(vp), i32], i32),
        "dc_ctx_destroy": ([vp], None),
        "dc_ctx_sync": ([vp], i32),
        "dc_ctx_stream": ([vp], vp),
        "dc_ctx_set_timing": ([vp, i32], i32),
        "dc_ctx_set_option": ([vp, i32, C.c_int64], i32),
        "dc_ctx_timings": ([vp, C.POINTER(C.c_char_p), C.POINTER(C.c_float), i32], i32),
        "dc_version": ([], C.c_char_p),
        "dc_dtable_size": ([], C.c_size_t),
        "dc_malloc": ([C.POINTER(vp), C.c_size_t], i32),
        "dc_free": ([vp], i32),
        "dc_memcpy_h2d": ([vp, vp, vp, C.c_size_t], i32),
        "dc_memcpy_d2h": ([vp, vp, vp, C.c_size_t], i32),
        "dc_memset": ([vp, vp, i32, C.c_size_t], i32),
        "dc_huff_hist": ([vp, P, u64, P], i32),
        "dc_huff_table": ([vp, P, i32, i32, P], i32),
        "dc_huff_table_freq": ([vp, P, i32, i32, P], i32),
        "dc_huff_table_lengths": ([vp, P, i32, i32, P], i32),
        "dc_huff_table_status": ([vp, P, C.POINTER(C.c_int32)], i32),
        "dc_huff_plan": ([vp, P, P], i32),
        "dc_huff_encode_plan": ([vp, P, u64, i32, i32, P, P, P], i32),
        "dc_huff_table_plan": ([vp, P, i32, i32, P, P], i32),
        "dc_small_huff_plan": ([vp, P, u64, i32, i32, P, P, P], i32),
        "dc_small_huff_pack_async": ([vp, P, u64, P, u64, P, u64, P, P, u32], i32),
        "dc_small_huff_symbols": ([vp, C.POINTER(u64)], i32),
        "dc_small_huff_shard_hist": ([vp, P, u64, P, P], i32),
        "dc_small_huff_shard_pack_async": ([vp, P, u64, P, P, P, u64, P, P, P, P, u32], i32),
        "dc_small_huff_decode": ([vp, P, u64, u64, P, P, u32, u64, P, P, P, C.POINTER(u64)], i32),
        "dc_copy_probe": ([vp, P, P, u64], i32),
        "dc_huff_pack": ([vp, P, u64, P, u64, P, u64, P, P, u32], i32),
        "dc_huff_sync_chunks": ([u64, u32], u64),
        "dc_huff_sync_groups": ([u64, u32], u64),
        "dc_huff_words_needed": ([u64, u64], u64),
        "dc_huff_pack_async": ([vp, P, u64, P, u64, P, u64, P, P, u32], i32),
        "dc_huff_pack_async_dev": ([vp, P, u64, P, P, P, u64, P, P, u32], i32),
        "dc_huff_pack_status": ([vp, P], i32),
        "dc_huff_plan_gen": ([vp], u32),
        "dc_huff_pack_status_gen": ([vp, P, u32], i32),
        "dc_huff_plan_offsets": ([vp, P, u64, C.POINTER(u64)], i32),
        "dc_huff_block_hist": ([vp, P, u64], i32),
        "dc_huff_decode": ([vp, P, u64, u64, P, P, u32, u64, P, P], i32),
        "dc_huff_decode_dev": ([vp, P, P, u64, P, P, u32, u64, P, P], i32),
        "dc_huff_decode_status": ([vp], i32),
        "dc_huff_decode_redo_count": ([vp, C.POINTER(u64)], i32),
        "dc_huff_base64url": ([vp, P, u64, u64, P], i32),
        "dc_huff_text_bits": ([i32, i32], i32),
        "dc_huff_text": ([vp, P, u64, u64, i32, i32, P, C.POINTER(u64)], i32),
        "dc_huff_text_parse": ([vp, P, u64, i32, i32, u64, P], i32),
        "dc_huff_text_parse_status": ([vp], i32),
        "dc_huff_default_sync": ([u64], u32),
        "dc_huff_choose_sync": ([u64, u64], u32),
        "dc_nyb_compress": ([vp, P, u64, i32, P, C.POINTER(u64)], i32),
        "dc_nyb_decompress": ([vp, P, u64, i32, P, C.POINTER(u64)], i32),
        "dc_nyb_chunked_bound": ([u64, u32], u64),
        "dc_nyb_compress_chunked": ([vp, P, u64, i32, u32, P, u64, C.POINTER(u64)], i32),
        "dc_nyb_chunked_info": ([vp, P, u64, C.POINTER(u64), C.POINTER(i32), C.POINTER(u32)], i32),
        "dc_nyb_decompress_chunked": ([vp, P, u64, P, u64, C.POINTER(u64)], i32),
        "dc_nyb_decompress_batch": ([vp, P, P, u64, i32, P, u64, P, C.POINTER(u64)], i32),
        "dc_nyb_mtf_summary": ([vp, P, u64, P, P], i32),
        "dc_nyb_body_plan": ([vp, P, u64, i32, P, P], i32),
        "dc_nyb_body_write": ([vp, P, u64, i32, i32, i32, P, C.POINTER(u64), C.POINTER(i32)], i32),
        "dc_nyb_dbody_plan": ([vp, P, u64, u64, P], i32),
        "dc_nyb_dbody_write": ([vp, P, u64, u64, i32, P, C.POINTER(u64), C.POINTER(i32)], i32),
        "dc_small_compress": ([vp, P, u64, P, C.POINTER(u64)], i32),
        "dc_small_decompress": ([vp, P, u64, P, C.POINTER(u64)], i32),
        "dc_small_compress_body": ([vp, P, u64, i32, u64, P, C.POINTER(u64)], i32),
        "dc_small_compress_body_plan": ([vp, P, u64, i32, u64, C.POINTER(u64)], i32),
        "dc_small_compress_body_write": ([vp, P, u64, i32, u64, P, C.POINTER(u64)], i32),
        "dc_small_decompress_body": ([vp, P, u64, P, C.POINTER(u64)], i32),
        "dc_host_ctx": ([], vp),
        "dc_huff_compress_bound": ([u64, u32], u64),
        "dc_huff_compress_host": ([u8p, u64, i32, C.POINTER(C.c_int32), i32, u32, u8p, u64, C.POINTER(u64)], i32),
        "dc_huff_decompress_host": ([u8p, u64, u8p, u64, C.POINTER(u64)], i32),
        "dc_huff_netstring_bound": ([u64], u64),
        "dc_huff_compress_netstring": ([u8p, u64, i32, C.POINTER(C.c_int32), i32, u32, u8p, u64, C.POINTER(u64)], i32),
        "dc_huff_decompress_netstring": ([u8p, u64, u8p, u64, C.POINTER(u64)], i32),
        "dc_huff_netstring_info": ([u8p, u64, C.POINTER(u64)], i32),
        "dc_huff_container_info": ([u8p, u64, C.POINTER(u64), C.POINTER(i32), C.POINTER(u64)], i32),
        "dc_nyb_compress_host": ([u8p, u64, i32, u8p, u64, C.POINTER(u64)], i32),
        "dc_nyb_decompress_host": ([u8p, u64, i32, u8p, u64, C.POINTER(u64)], i32),
        "dc_small_compress_host": ([u8p, u64, u8p, u64, C.POINTER(u64)], i32),
        "dc_small_decompress_host": ([u8p, u64, u8p, u64, C.POINTER(u64)], i32),
    }
    for name, (args, res) in sig.items():
        if os.environ.get("DC_CORE_LIB") and not hasattr(L, name):   # older diagnostic build
            continue
        f = getattr(L, name)
        f.argtypes = args
        f.restype = res
