"""Python mirror of nybble_compression.c's codec interface (nybble_compression.c:734-1137),
calling libdc_nybble.so -- the drop-in C-ABI with the reference's own names."""
from __future__ import annotations

import ctypes as C

from ._lib import load

_L = None


def lib():
    global _L
    if _L is None:
        _L = load("libdc_nybble.so")
        for f in ("compress_bytestring", "decompress_bytestring"):
            getattr(_L, f).argtypes = [C.c_char_p, C.c_char_p, C.c_bool]
            getattr(_L, f).restype = None
        for f in ("nybble_compress", "nybble_decompress"):
            getattr(_L, f).argtypes = [C.c_char_p, C.c_char_p]
            getattr(_L, f).restype = None
    return _L


def compress_bytestring(source: bytes, modify: bool) -> bytes:
    dst = C.create_string_buffer(len(source) + 2)
    lib().compress_bytestring(bytes(source), dst, modify)
    return dst.value


def decompress_bytestring(source: bytes, modify: bool) -> bytes:
    """C-string result, as a reference caller sees it (stops at the first NUL)."""
    dst = C.create_string_buffer(2 * len(source) + 1)
    lib().decompress_bytestring(bytes(source), dst, modify)
    return dst.value


def decompress_raw(source: bytes, modify: bool) -> bytes:
    """Every byte the decoder writes (decoded NULs included), via the same kernels."""
    from ._lib import DcError, core
    m = len(source)
    a = (C.c_uint8 * max(m, 1)).from_buffer_copy(bytes(source) or b"\0")
    cap = 2 * m + 1
    out = (C.c_uint8 * cap)()
    n = C.c_uint64(0)
    rc = core().dc_nyb_decompress_host(a, m, 1 if modify else 0, out, cap, C.byref(n))
    if rc:
        raise DcError("dc_nyb_decompress_host", rc)
    return bytes(out[: n.value])


def nybble_compress(source: bytes) -> bytes:
    dst = C.create_string_buffer(len(source) + 2)
    lib().nybble_compress(bytes(source), dst)
    return dst.value


def nybble_decompress(source: bytes) -> bytes:
    dst = C.create_string_buffer(2 * len(source) + 1)
    lib().nybble_decompress(bytes(source), dst)
    return dst.value
