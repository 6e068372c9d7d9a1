"""Python mirror of small_compression.c's byte front-end (small_compression.c:453-665),
calling libdc_small.so -- the drop-in C-ABI with the reference's own names."""
from __future__ import annotations

import ctypes as C

from ._lib import load

_L = None


def lib():
    global _L
    if _L is None:
        _L = load("libdc_small.so")
        for f in ("compress_bytestring", "decompress_bytestring"):
            getattr(_L, f).argtypes = [C.c_char_p, C.c_char_p]
            getattr(_L, f).restype = None
    return _L


def compress_bytestring(source: bytes) -> bytes:
    dst = C.create_string_buffer(len(source) + 2)
    lib().compress_bytestring(bytes(source), dst)
    return dst.value


def decompress_bytestring(source: bytes) -> bytes:
    dst = C.create_string_buffer(2 * len(source) + 1)
    lib().decompress_bytestring(bytes(source), dst)
    return dst.value
