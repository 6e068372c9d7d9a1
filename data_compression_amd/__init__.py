"""data_compression_amd -- MI355X-native (gfx950) n-ary Huffman + nybble-packing codec.

A drop-in for the hot path of carycode/data_compression: the C-ABI shims
(lib/libdc_huffman.so, libdc_nybble.so, libdc_small.so) export the reference's own
function names; libdc_core.so holds the HIP kernels and the device-resident API.

    from data_compression_amd import huffman, nybble, small   # reference-named mirrors
    from data_compression_amd.device import Codec             # device-resident stages
    from data_compression_amd import dist                     # multi-GPU (RCCL) driver
"""
from . import _lib  # noqa: F401  (imports torch first: one HIP runtime per process)

__all__ = ["huffman", "nybble", "small", "device", "dist", "synth", "build"]
__version__ = "0.1.0"
