"""CPU-side checks of the drop-in boundary: every function declared in include/*.h is
exported by the library that implements it, the libraries load, and the product never
routes through the oracle. No compute call is made here (no GPU in this container)."""
import os
import re
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(REPO, "data_compression_amd", "lib")
INC = os.path.join(REPO, "include")

HEADER_LIB = {
    "dc_gpu.h": "libdc_core.so",
    "dc_host.h": "libdc_core.so",
    "dc_huffman.h": "libdc_huffman.so",
    "dc_nybble.h": "libdc_nybble.so",
    "dc_small.h": "libdc_small.so",
}


@pytest.fixture(scope="module", autouse=True)
def built():
    from data_compression_amd import build
    build.build()


def declared(header):
    text = open(os.path.join(INC, header)).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    text = re.sub(r"//.*", "", text)
    names = re.findall(r"^\s*(?:[A-Za-z_][\w\s\*]*?[\s\*])([A-Za-z_]\w*)\s*\(", text, flags=re.M)
    return sorted({n for n in names if n not in ("if", "while", "for", "return", "sizeof")})


def exported(lib):
    out = subprocess.run(["nm", "-D", "--defined-only", os.path.join(LIB, lib)], capture_output=True,
                         text=True, check=True).stdout
    return {line.split()[-1] for line in out.splitlines() if " T " in line}


@pytest.mark.parametrize("header", sorted(HEADER_LIB))
def test_header_symbols_exported(header):
    names = declared(header)
    assert names, header
    missing = [n for n in names if n not in exported(HEADER_LIB[header])]
    assert not missing, (header, missing)


def test_reference_names_present():
    # the reference's own entry points
    assert {"histogram", "huffman", "convert_lengths_to_encode_table",
            "represent_items_with_codes"} <= exported("libdc_huffman.so")
    assert {"compress_bytestring", "decompress_bytestring", "nybble_compress",
            "nybble_decompress"} <= exported("libdc_nybble.so")
    assert {"compress_bytestring", "decompress_bytestring"} <= exported("libdc_small.so")


def test_libraries_load_and_report_gfx950():
    from data_compression_amd import _lib, huffman, nybble, small
    assert b"gfx950" in _lib.core().dc_version()
    huffman.lib(); nybble.lib(); small.lib()


def test_code_objects_are_gfx950_only():
    blob = open(os.path.join(LIB, "libdc_core.so"), "rb").read()
    targets = set(re.findall(rb"amdgcn-amd-amdhsa-[-a-z0-9:+]*", blob))
    assert targets == {b"amdgcn-amd-amdhsa--gfx950"}, targets


def test_product_never_imports_oracle():
    pkg = os.path.join(REPO, "data_compression_amd")
    pat = re.compile(r"^\s*(from\s+oracle|import\s+oracle|#\s*include\s+[\"<].*oracle)", re.M)
    for root, _, files in os.walk(pkg):
        for f in files:
            if f.endswith((".py", ".cpp", ".hip", ".h")):
                src = open(os.path.join(root, f)).read()
                assert not pat.search(src), f
                assert "liboracle" not in src, f


def test_no_device_fails_loudly():
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    from data_compression_amd.device import Codec
    from data_compression_amd._lib import DcError
    with pytest.raises(DcError):
        Codec()


# ---- C callers of the drop-in (tests/c/): the headers compile as C and every symbol a
# reference-style caller uses resolves against its one library ------------------------
C_DRIVERS = ("huffman", "nybble")


def build_c_driver(name, outdir):
    import subprocess
    lib = os.path.join(REPO, "data_compression_amd", "lib")
    exe = os.path.join(str(outdir), f"dropin_{name}")
    subprocess.run(["gcc", "-std=c11", "-O2", "-Wall", "-Werror", "-I", os.path.join(REPO, "include"),
                    os.path.join(REPO, "tests", "c", f"dropin_{name}.c"), "-L", lib, f"-ldc_{name}",
                    f"-Wl,-rpath,{lib}", "-o", exe], check=True)
    return exe


@pytest.mark.parametrize("name", C_DRIVERS)
def test_c_driver_links(name, tmp_path):
    exe = build_c_driver(name, tmp_path)
    assert os.path.exists(exe)
