"""Python mirror of n_ary_huffman.c's public interface, calling libdc_huffman.so (the
drop-in C-ABI) -- same names, argument meaning and array conventions as the reference
(n_ary_huffman.c:461-493, :1161-1208, :1382-1612, :1621-1678), so the parity tests read
like the reference's own tests. Every call runs the gfx950 kernels of libdc_core.so.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from ._lib import DcError, core, load

_L = None


def lib():
    global _L
    if _L is None:
        _L = load("libdc_huffman.so")
        ip = C.POINTER(C.c_int)
        _L.histogram.argtypes = [C.c_char_p, C.c_int, ip]
        _L.histogram.restype = None
        _L.huffman.argtypes = [C.c_int, ip, C.c_int, ip]
        _L.huffman.restype = None
        _L.convert_lengths_to_encode_table.argtypes = [C.c_int, ip, C.c_int, ip, C.POINTER(C.c_uint)]
        _L.convert_lengths_to_encode_table.restype = None
        _L.represent_items_with_codes.argtypes = [C.c_int, ip, C.c_int, C.c_int, C.c_int, C.c_char_p,
                                                  C.c_int, C.c_char_p]
        _L.represent_items_with_codes.restype = C.c_int
        _L.dc_huff_compress.argtypes = [C.c_int, ip, C.c_int, C.c_int, C.c_int, C.c_char_p, C.c_char_p]
        _L.dc_huff_compress.restype = C.c_int
        _L.dc_huff_decompress.argtypes = [C.c_int, C.c_char_p, C.c_int, C.c_char_p]
        _L.dc_huff_decompress.restype = C.c_int
    return _L


def _ip(a):
    return a.ctypes.data_as(C.POINTER(C.c_int))


def histogram(text: bytes, max_symbol_value: int = 258) -> np.ndarray:
    """histogram(text, max_symbol_value, h) -- counts up to the first NUL."""
    h = np.zeros(max_symbol_value + 1, dtype=np.int32)
    lib().histogram(bytes(text), max_symbol_value, _ip(h))
    return h


def huffman(max_leaf_value: int, symbol_frequencies, compressed_symbols: int) -> np.ndarray:
    f = np.zeros(max_leaf_value + 1, dtype=np.int32)
    src = np.asarray(symbol_frequencies, dtype=np.int64)[: max_leaf_value + 1]
    f[: len(src)] = src
    out = np.zeros(max_leaf_value + 1, dtype=np.int32)
    lib().huffman(max_leaf_value, _ip(f), compressed_symbols, _ip(out))
    return out


def convert_lengths_to_encode_table(max_symbol_value: int, canonical_lengths, compressed_symbols: int,
                                    encode_length_table=None, encode_value_table=None, size=None):
    """Returns (encode_length_table, encode_value_table). Pass pre-filled arrays to see
    which entries the function leaves untouched (index max_symbol_value, :1421)."""
    size = size or (max_symbol_value + 1)
    L = np.zeros(size, dtype=np.int32)
    src = np.asarray(canonical_lengths, dtype=np.int32)
    L[: len(src)] = src
    el = np.zeros(size, np.int32) if encode_length_table is None else np.array(encode_length_table, np.int32)
    ev = np.zeros(size, np.uint32) if encode_value_table is None else np.array(encode_value_table, np.uint32)
    lib().convert_lengths_to_encode_table(max_symbol_value, _ip(L), compressed_symbols, _ip(el),
                                          ev.ctypes.data_as(C.POINTER(C.c_uint)))
    return el, ev


def represent_items_with_codes(max_symbol_value: int, canonical_lengths, compressed_symbols: int,
                               original_text: bytes, start: int = 0, bufsize: int | None = None):
    """Returns (count, compressed_text bytes [start:start+count]) or (-1, b"")."""
    L = np.zeros(max_symbol_value + 1, dtype=np.int32)
    src = np.asarray(canonical_lengths, dtype=np.int32)
    L[: len(src)] = src
    n = len(original_text)
    if bufsize is None:
        bufsize = start + (n * 32 + 5) // 6 + 8
    out = C.create_string_buffer(bufsize + 1)
    txt = C.create_string_buffer(bytes(original_text), n + 1)
    r = lib().represent_items_with_codes(max_symbol_value, _ip(L), compressed_symbols, bufsize, n, txt,
                                         start, out)
    if r < 0:
        return r, b""
    return r, out.raw[start : start + r]


def compress(data: bytes, n_ary: int = 2, lengths=None, max_symbol_value: int = 258) -> bytes:
    """dc_huff_compress (same parameters as the reference's static compress,
    n_ary_huffman.c:1688) -> netstring blocks (raw, or #dc1 + X + #dcidx + Z).
    lengths None: the input's own Huffman lengths (histogram -> huffman on the GPU)."""
    data = bytes(data)
    n = len(data)
    if lengths is None:
        lengths = huffman(max_symbol_value, histogram_bytes(data, max_symbol_value), n_ary)
    L = np.zeros(max_symbol_value + 1, dtype=np.int32)
    L[: len(lengths)] = np.asarray(lengths, dtype=np.int32)
    cap = int(core().dc_huff_netstring_bound(n)) + 1
    out = C.create_string_buffer(cap)
    r = lib().dc_huff_compress(max_symbol_value, _ip(L), n_ary, cap - 1, n, C.create_string_buffer(data, n + 1), out)
    if r < 0:
        raise DcError("dc_huff_compress", r)
    return out.raw[:r]


def compress_dch1(data: bytes, n_ary: int = 2, sync_syms: int = 0) -> bytes:
    """The binary "DCH1" container (dc_huff_compress_host; dc_host.h)."""
    data = bytes(data)
    n = len(data)
    cap = int(core().dc_huff_compress_bound(n, sync_syms))
    out = (C.c_uint8 * cap)()
    got = C.c_uint64(0)
    src = (C.c_uint8 * max(n, 1)).from_buffer_copy(data + b"\0")
    rc = core().dc_huff_compress_host(src, n, n_ary, None, 258, sync_syms, out, cap, C.byref(got))
    if rc:
        raise DcError("dc_huff_compress_host", rc)
    return bytes(out[: got.value])


def decompress(blob: bytes, max_decompressed_size: int | None = None) -> bytes:
    """dc_huff_decompress: a netstring container (this build's or the reference compress()'s
    raw blocks) or a DCH1 container."""
    blob = bytes(blob)
    if max_decompressed_size is None:
        nn = C.c_uint64(0)
        buf = (C.c_uint8 * len(blob)).from_buffer_copy(blob)
        rc = core().dc_huff_container_info(buf, len(blob), C.byref(nn), None, None)
        if rc:
            raise DcError("dc_huff_container_info", rc)
        max_decompressed_size = int(nn.value)
    out = C.create_string_buffer(max_decompressed_size + 1)
    r = lib().dc_huff_decompress(len(blob), blob, max_decompressed_size, out)
    if r < 0:
        raise DcError("dc_huff_decompress", r)
    return out.raw[:r]


def histogram_bytes(data: bytes, max_symbol_value: int = 258) -> np.ndarray:
    """Histogram of an arbitrary byte string (NULs included), via the device API."""
    from .device import Codec
    c = Codec.host_default()
    return c.histogram_host(np.frombuffer(bytes(data), dtype=np.uint8), max_symbol_value)
