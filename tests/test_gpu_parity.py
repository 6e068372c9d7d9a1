"""GPU parity tests: the HIP path (through the C-ABI) against the reference's golden
vectors and the CPU oracle, on the same inputs. Bit-exact everywhere (integer/byte work).

Run on an MI355X:  python -m pytest tests -m gpu -x -q
"""
import os

import numpy as np
import pytest

from oracle import oracle as orc

pytestmark = pytest.mark.gpu

G = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
NARY = (2, 3, 4, 5, 9, 10, 16)


def _load(name):
    return np.load(os.path.join(G, name), allow_pickle=False)


@pytest.fixture(scope="module")
def torch_cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch


@pytest.fixture(scope="module")
def codec(torch_cuda):
    from data_compression_amd.device import Codec
    return Codec(0)


# ---------------------------------------------------------------- reference golden vectors
def test_histogram_matches_reference(torch_cuda):
    from data_compression_amd import huffman as H
    d = _load("histogram.npz")
    for x, h in zip(d["inputs"], d["counts"]):
        assert np.array_equal(H.histogram(x.tobytes(), 258), h.astype(np.int32))


def test_huffman_lengths_match_reference(torch_cuda):
    from data_compression_amd import huffman as H
    d = _load("huffman_tables.npz")
    bad = []
    for i in range(len(d["n"])):
        L = H.huffman(258, d["freq"][i], int(d["n"][i]))
        if not np.array_equal(L, d["lengths"][i]):
            bad.append((str(d["names"][i]), int(d["n"][i])))
    assert not bad, bad[:10]


def test_canonical_codes_match_reference(torch_cuda):
    from data_compression_amd import huffman as H
    d = _load("huffman_tables.npz")
    for i in range(len(d["n"])):
        el, ev = H.convert_lengths_to_encode_table(258, d["lengths"][i], int(d["n"][i]))
        assert np.array_equal(el, d["enc_len"][i]), i
        assert np.array_equal(ev, d["enc_val"][i]), i


def test_canonical_known_answers_and_untouched_last_index(torch_cuda):
    from data_compression_amd import huffman as H
    d = _load("canonical_kat.npz")
    for L, el_ref, ev_ref in zip(d["lengths"], d["enc_len"], d["enc_val"]):
        el, ev = H.convert_lengths_to_encode_table(20, L, 3, size=80)
        assert np.array_equal(el, el_ref) and np.array_equal(ev, ev_ref)
    # index max_symbol_value is not cleared by the reference (n_ary_huffman.c:1421)
    L = np.zeros(21, np.int32); L[2:6] = 2
    el, ev = H.convert_lengths_to_encode_table(20, L, 2, np.full(21, 77, np.int32), np.full(21, 99, np.uint32))
    assert el[20] == 77 and ev[20] == 99 and el[19] == 0 and ev[19] == 0
    L[20] = 2
    el, ev = H.convert_lengths_to_encode_table(20, L, 2, np.full(21, 77, np.int32), np.full(21, 99, np.uint32))
    assert el[20] == 2 and ev[20] == 4


def _nyb():
    d = _load("nybble.npz")
    return d, int(d["n_inputs"][0]), int(d["n_dec_only"][0])


@pytest.mark.parametrize("modify", [False, True])
def test_nybble_compress_matches_reference(torch_cuda, modify):
    from data_compression_amd import nybble as N
    d, n, _ = _nyb()
    for i in range(n):
        x = d[f"in_{i}"].tobytes()
        assert N.compress_bytestring(x, modify) == d[f"comp_{i}_{int(modify)}"].tobytes(), i


@pytest.mark.parametrize("modify", [False, True])
def test_nybble_decompress_matches_reference(torch_cuda, modify):
    from data_compression_amd import nybble as N
    d, n, nd = _nyb()
    for i in range(n):
        c = d[f"comp_{i}_{int(modify)}"].tobytes()
        assert N.decompress_raw(c, modify) == d[f"back_{i}_{int(modify)}"].tobytes(), i
    for j in range(nd):
        c = d[f"dec_in_{j}"].tobytes()
        assert N.decompress_raw(c, modify) == d[f"dec_out_{j}_{int(modify)}"].tobytes(), j


def test_nybble_appendix_b_and_wrappers(torch_cuda):
    from data_compression_amd import nybble as N
    text = (b"Hello, world. This is a test. This is only a test. "
            b"Banana banana banana banana. ")
    s = N.compress_bytestring(text, False)
    t = N.nybble_compress(text)
    assert len(s) == 57 and len(t) == 57
    assert t.hex().startswith("af48656c6c6f2c20776f726c642e2054686973af88eaeb73")
    assert N.decompress_bytestring(s, False) == text
    assert N.nybble_decompress(t) == text
    assert N.compress_bytestring(b"", True) == b" "


def test_small_frontend_matches_reference(torch_cuda):
    from data_compression_amd import small as S
    d = _load("small.npz")
    for i in range(int(d["n_inputs"][0])):
        x = d[f"in_{i}"].tobytes()
        c = S.compress_bytestring(x)
        assert c == d[f"comp_{i}"].tobytes(), i
        assert S.decompress_bytestring(c) == x, i


# ---------------------------------------------------------------- bitstream vs the oracle
def _inputs():
    from data_compression_amd import synth
    out = []
    for cfg, gen in synth.GENERATORS.items():
        for n in (1, 15, 16, 17, 4095, 32767, 32768, 32769, 100_003):
            out.append((f"{cfg}-{n}", gen(n, seed=n + len(cfg))))
    out.append(("C2-1M", synth.enwik_like(1 << 20, seed=99)))
    out.append(("same-byte", np.full(70_000, 65, np.uint8)))
    out.append(("two-bytes", np.tile(np.array([1, 255], np.uint8), 40_000)))
    out.append(("with-nul", synth.uniform_bytes(50_000, seed=5, lo=0, hi=255)))
    return out


def _oracle_encode(x, n):
    h = orc.histogram(x)
    L = orc.huffman_lengths(h, n)
    el, ev = orc.canonical(L, n)
    code, nb, mx = orc.bitcodes(el, ev, n)
    return L, el, ev, code, nb, mx


@pytest.mark.parametrize("n_ary", NARY)
def test_pack_bit_exact_vs_oracle(torch_cuda, codec, n_ary):
    torch = torch_cuda
    for name, x in _inputs():
        L, el, ev, code, nb, mx = _oracle_encode(x, n_ary)
        if mx > 32 or mx <= 0:
            continue
        S = 64
        payload, bits, idx = orc.huff_pack(x, code, nb, sync_syms=S)
        xt = torch.from_numpy(x).cuda()
        enc = codec.encode(xt, n_ary=n_ary, sync_syms=S)
        hist = enc["hist"].cpu().numpy().astype(np.uint64)
        assert np.array_equal(hist, orc.histogram(x)), name
        assert enc["bits"] == bits, name
        got = enc["words"].cpu().numpy().view(np.uint8)[: len(payload)]
        assert np.array_equal(got, payload), name
        base, lens = orc.sync_compact(idx, 0, bits)
        assert np.array_equal(enc["sync"][0].cpu().numpy().astype(np.uint64)[: len(base)], base), name
        assert np.array_equal(enc["sync"][1].cpu().numpy().view(np.uint16)[: len(lens)], lens), name
        out = torch.empty(x.size + 16, dtype=torch.uint8, device="cuda")
        codec.decode_into(enc, out)
        assert codec.decode_status() == 0
        assert np.array_equal(out[: x.size].cpu().numpy(), x), name


@pytest.mark.parametrize("bit_base", [0, 1, 13, 31, 32, 77, (1 << 33) + 5])
def test_pack_at_bit_offset(torch_cuda, codec, bit_base):
    """The multi-GPU shard path: a shard encoded at a global bit offset."""
    torch = torch_cuda
    from data_compression_amd import synth
    x = synth.enwik_like(300_000, seed=3)
    L, el, ev, code, nb, mx = _oracle_encode(x, 2)
    S = 256
    payload, bits, idx = orc.huff_pack(x, code, nb, bit_base=bit_base, sync_syms=S)
    xt = torch.from_numpy(x).cuda()
    enc = codec.encode(xt, n_ary=2, sync_syms=S, bit_base=bit_base)
    got = enc["words"].cpu().numpy().view(np.uint8)
    off = (bit_base >> 3) - ((bit_base >> 5) << 2)   # words start at stream word bit_base/32
    assert np.array_equal(got[off: off + len(payload)], payload)
    assert not got[:off].any()
    base, lens = orc.sync_compact(idx, bit_base, bits)
    assert np.array_equal(enc["sync"][0].cpu().numpy().astype(np.uint64), base)
    assert np.array_equal(enc["sync"][1].cpu().numpy().view(np.uint16), lens)
    out = torch.empty(x.size, dtype=torch.uint8, device="cuda")
    codec.decode_into(enc, out)
    assert np.array_equal(out.cpu().numpy(), x)


@pytest.mark.parametrize("bit_base", [0, 5, 31, 32, 1000, 128 * 3])
@pytest.mark.parametrize("kind", ["text", "flat16", "tail"])
def test_pack_into_dirty_words(torch_cuda, codec, bit_base, kind):
    """No zeroing launch precedes the pack: blocks that share a word clear and set only their
    own bits (the first block also the bits before bit_base, the last the pad). Into a words
    buffer full of ones, every word the stream touches must match the oracle's bit for bit,
    zero bits before bit_base and after the last code included; words outside stay ones."""
    torch = torch_cuda
    from data_compression_amd import synth
    if kind == "text":
        x, n_ary = synth.enwik_like(200_003, seed=51), 2          # fast path, ragged last block
    elif kind == "flat16":
        x, n_ary = synth.uniform_bytes((3 << 15) + 13, seed=52), 16   # 8-bit codes: byte map at bit_base % 128 == 0
    else:
        x, n_ary = synth.enwik_like((2 << 15) + 1, seed=53), 2        # a 1-byte last block (slow path)
    L, el, ev, code, nb, mx = _oracle_encode(x, n_ary)
    payload, bits, _ = orc.huff_pack(x, code, nb, bit_base=bit_base)
    xt = torch.from_numpy(x).cuda()
    hist = codec.hist(xt)
    tab = codec.table(hist, n_ary)
    total = codec.plan(tab)
    assert int(total.item()) == bits
    nw = codec.words_needed(bit_base, bits)
    words = torch.full((nw,), -1, dtype=torch.int32, device="cuda")
    codec.pack(xt, tab, bit_base, words, None, 0)
    got = words.cpu().numpy().view(np.uint8)
    off = (bit_base >> 3) - ((bit_base >> 5) << 2)
    end = ((bit_base & 31) + bits + 31) // 32 * 4   # bytes of the words the stream touches
    want = np.zeros(end, np.uint8)
    want[off: off + len(payload)] = payload
    assert np.array_equal(got[:end], want), (kind, bit_base)
    assert (got[end:] == 0xFF).all(), (kind, bit_base)


# alphabets whose codes are all 8 bits (flat counts): C3's bytes 1..255 (255 symbols + 1 dummy
# fill a depth-2 16-ary tree), a run 10..250 (241 + 15 dummies), 241 bytes with gaps (no run:
# the LDS byte map), and bytes 0..254 at n = 2 (+ the one dummy of n = 2: every byte coded as
# itself; all 256 would give 257 leaves and 9-bit codes)
FIXED8_ALPHABETS = {"c3": (np.arange(1, 256), 16, 1), "run": (np.arange(10, 251), 16, 10),
                    "gaps": (np.setdiff1d(np.arange(256), np.arange(3, 256, 17)), 16, None),
                    "n2": (np.arange(0, 255), 2, 0)}


@pytest.mark.parametrize("alpha", list(FIXED8_ALPHABETS))
@pytest.mark.parametrize("bit_base", [0, 128 * 3, 8, 32])
def test_fixed8_byte_map_paths(torch_cuda, codec, bit_base, alpha):
    """Every code 8 bits (dc_dtable.fixed8): pack and decode run as byte maps when the stream
    starts on a 128-bit boundary (bit_base 0, 384), and the general kernels otherwise (8, 32);
    both bit-exact vs the oracle, ragged ends included. When the coded bytes are one run
    (fixed8_affine) the maps are byte-wise subtractions, and a code past the run in the stream
    (a dummy leaf's) is reported as a stream error like the LDS map's missing entry."""
    torch = torch_cuda
    syms, n_ary, lo = FIXED8_ALPHABETS[alpha]
    rng = np.random.default_rng(bit_base + 7)
    for n in (1 << 20, (1 << 20) + 12_345, 100_003):
        x = rng.permutation(np.resize(syms.astype(np.uint8), n))
        L, el, ev, code, nb, mx = _oracle_encode(x, n_ary)
        assert set(np.unique(nb[:256])) == {0, 8}
        if lo is not None:   # the codes are byte - lo (what the affine map computes)
            assert all(int(code[s]) == int(s) - lo for s in syms)
        S = 64
        payload, bits, idx = orc.huff_pack(x, code, nb, bit_base=bit_base, sync_syms=S)
        xt = torch.from_numpy(x).cuda()
        enc = codec.encode(xt, n_ary=n_ary, sync_syms=S, bit_base=bit_base)
        assert enc["bits"] == bits == 8 * n
        got = enc["words"].cpu().numpy().view(np.uint8)
        off = (bit_base >> 3) - ((bit_base >> 5) << 2)
        assert np.array_equal(got[off: off + len(payload)], payload), (n, bit_base)
        base, lens = orc.sync_compact(idx, bit_base, bits)
        assert np.array_equal(enc["sync"][0].cpu().numpy().astype(np.uint64), base), (n, bit_base)
        assert np.array_equal(enc["sync"][1].cpu().numpy().view(np.uint16), lens), (n, bit_base)
        out = torch.empty(n, dtype=torch.uint8, device="cuda")
        codec.decode_into(enc, out)
        assert codec.decode_status() == 0 and np.array_equal(out.cpu().numpy(), x), (n, bit_base)
        if bit_base % 128 == 0:   # the byte map redoes nothing (the general decoder redoes the ragged tail)
            assert codec.decode_redo_count() == 0
        if alpha == "c3" and bit_base == 0 and n == 100_003:
            # code 255 (the dummy leaf's) in the middle of the stream: an error, not a byte
            wb = enc["words"].view(torch.uint8)
            wb[n // 2] = 255
            codec.decode_into(enc, out)
            assert codec.decode_status() != 0


@pytest.mark.parametrize("case", ["unaligned-out", "long-halves"])
def test_pack_store_paths(torch_cuda, codec, case):
    """k_huff_pack fast path: word stores when the output is not 16-B aligned, and the
    per-code flush fallback for 8-code halves of more than 64 bits."""
    torch = torch_cuda
    from data_compression_amd import synth
    if case == "unaligned-out":
        x = synth.enwik_like(200_000, seed=21)
    else:
        x = _chain_stream(20, 3)   # codes up to 20 bits: many halves above 64 bits
    L, el, ev, code, nb, mx = _oracle_encode(x, 2)
    payload, bits, idx = orc.huff_pack(x, code, nb, sync_syms=64)
    xt = torch.from_numpy(x).cuda()
    tab = codec.table(codec.hist(xt), 2)
    assert int(codec.plan(tab).item()) == bits
    nw = codec.words_needed(0, bits)
    shift = 1 if case == "unaligned-out" else 0
    buf = torch.zeros(nw + 8, dtype=torch.int32, device="cuda")
    words = buf[shift: shift + nw]
    sync = codec.alloc_sync(x.size, 64)
    codec.pack(xt, tab, 0, words, sync, 64)
    assert codec.pack_status(tab) == 0
    got = words.cpu().numpy().view(np.uint8)[: len(payload)]
    assert np.array_equal(got, payload), case
    assert not buf[:shift].any() and not buf[shift + nw:].any()


@pytest.mark.parametrize("S", [16, 128, 1024])   # 1024: spans exceed the LDS stage -> HBM path
def test_decode_of_oracle_stream(torch_cuda, codec, S):
    torch = torch_cuda
    from data_compression_amd import synth
    for n_ary in (2, 3, 16):
        x = synth.log_like(200_000, seed=n_ary)
        L, el, ev, code, nb, mx = _oracle_encode(x, n_ary)
        payload, bits, idx = orc.huff_pack(x, code, nb, sync_syms=S)
        words = np.zeros((len(payload) + 3) // 4 + 32, np.uint32)
        words.view(np.uint8)[: len(payload)] = payload
        lens = torch.from_numpy(L.astype(np.int32)).cuda()
        tab = codec.table_lengths(lens, n_ary)
        out = torch.empty(x.size, dtype=torch.uint8, device="cuda")
        base, lens = orc.sync_compact(idx, 0, bits)
        sync = (torch.from_numpy(base.astype(np.int64)).cuda(), torch.from_numpy(lens.view(np.int16)).cuda())
        codec.decode(torch.from_numpy(words.view(np.int32)).cuda(), 0, sync, S, x.size, tab, out)
        assert codec.decode_status() == 0
        assert np.array_equal(out.cpu().numpy(), x)


def test_represent_items_with_codes_base64url(torch_cuda):
    from data_compression_amd import huffman as H
    from data_compression_amd import synth
    x = synth.english_like(5000, seed=8)
    h = H.histogram(x.tobytes(), 258)
    for n_ary in (2, 3, 16):
        L = H.huffman(258, h, n_ary)
        el, ev = orc.canonical(L, n_ary)
        code, nb, mx = orc.bitcodes(el, ev, n_ary)
        payload, bits, _ = orc.huff_pack(x, code, nb)
        want = orc.base64url(payload, bits)
        cnt, text = H.represent_items_with_codes(258, L, n_ary, x.tobytes(), start=3)
        assert cnt == len(want) and text == want
    # a byte without a code -> -1 (the reference asserts, :1658)
    L = np.zeros(259, np.int32); L[ord("a")] = 1; L[ord("b")] = 1
    assert H.represent_items_with_codes(258, L, 2, b"abc")[0] == -1


def test_container_roundtrip_and_edges(torch_cuda):
    from data_compression_amd import huffman as H
    from data_compression_amd import synth
    cases = [b"", b"a", b"aaaa", bytes(range(256)) * 3, synth.enwik_like(123_457, seed=1).tobytes(),
             synth.uniform_bytes(70_000, seed=2, lo=0, hi=255).tobytes()]
    for data in cases:
        for n_ary in (2, 3, 16):
            blob = H.compress(data, n_ary)
            assert H.decompress(blob) == data


# ---------------------------------------------------------------- full-size properties
@pytest.mark.parametrize("cfg,n_ary,size", [("C2", 2, 1 << 30), ("C3", 16, 1 << 30), ("C4", 2, 256 << 20),
                                            ("C5", 16, 256 << 20)])
def test_full_size_roundtrip(torch_cuda, codec, cfg, n_ary, size):
    torch = torch_cuda
    x = _device_input(torch, cfg, size)
    enc = codec.encode(x, n_ary=n_ary)
    hist = enc["hist"]
    assert torch.equal(hist, torch.bincount(x.to(torch.int64), minlength=256))
    nbits = torch.from_numpy(_nbits_of(codec, enc["table"])).cuda()
    assert enc["bits"] == int((hist * nbits).sum().item())
    out = torch.empty_like(x)
    codec.decode_into(enc, out)
    assert codec.decode_status() == 0
    assert torch.equal(out, x)
    # encoding is deterministic: a second encode is bit-identical
    enc2 = codec.encode(x, n_ary=n_ary)
    nw = (enc["bits"] + 31) // 32
    assert torch.equal(enc2["words"][:nw], enc["words"][:nw])
    del enc, enc2, out, x
    torch.cuda.empty_cache()


def _nbits_of(codec, tab):
    import ctypes as C
    raw = tab.cpu().numpy()
    return raw[1024:2048].view(np.uint32).astype(np.int64)


def _device_input(torch, cfg, size):
    from data_compression_amd import synth
    piece = 64 << 20
    parts = []
    gen = synth.GENERATORS[cfg]
    for k in range(0, size, piece):
        m = min(piece, size - k)
        if cfg == "C3":
            arr = synth.uniform_bytes(m, seed=0xC3 + k, lo=1, hi=255)
        else:
            arr = gen(m, seed=0xC0 + k)
        parts.append(torch.from_numpy(arr).cuda())
    return torch.cat(parts)


def test_nybble_static_large_vs_oracle(torch_cuda):
    from data_compression_amd import nybble as N
    from data_compression_amd import synth
    x = synth.english_like(1 << 20, seed=4).tobytes()
    c = N.compress_bytestring(x, False)
    assert c == orc.nybble_compress(x, False)
    assert N.decompress_bytestring(c, False) == x
    y = synth.log_like(300_000, seed=5).tobytes()
    c = N.compress_bytestring(y, True)
    assert c == orc.nybble_compress(y, True)
    assert N.decompress_bytestring(c, True) == y


# ---------------------------------------------------------------- C callers of the drop-in
@pytest.mark.parametrize("name", ["huffman", "nybble"])
def test_c_driver_runs(torch_cuda, name, tmp_path):
    import subprocess
    from tests.test_abi import build_c_driver
    exe = build_c_driver(name, tmp_path)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert f"dropin_{name} ok" in r.stdout


# ---------------------------------------------------------------- decoder paths (S = 64)
def _chain_stream(nsym, seed):
    """Symbol counts 2^0 .. 2^(nsym-1): the Huffman tree is a chain, so binary code lengths
    reach about nsym bits and codes longer than the decoder's 12 + 8 bit two-level table occur."""
    f = [1 << i for i in range(nsym)]
    syms = np.repeat(np.arange(1, nsym + 1, dtype=np.uint8), f)
    rng = np.random.default_rng(seed)
    rng.shuffle(syms)
    return syms


@pytest.mark.parametrize("case", ["chain16", "chain23", "enwik", "two-long-per-batch"])
def test_decode_fast_path_rare_codes(torch_cuda, codec, case):
    """k_huff_decode8: codes of 13..20 bits (second-level table), > 20 bits (the wave's
    exact redo), several long codes inside one 4-symbol batch (window overflow)."""
    torch = torch_cuda
    from data_compression_amd import synth
    if case == "chain16":
        x = _chain_stream(16, 1)
    elif case == "chain23":
        x = _chain_stream(23, 2)
    elif case == "enwik":
        x = synth.enwik_like(3 << 20, seed=11)
    else:
        # mostly one frequent byte, with runs of rare bytes (long codes back to back)
        rng = np.random.default_rng(4)
        x = np.full(1 << 20, 32, np.uint8)
        rare = rng.integers(0, x.size - 8, 3000)
        for r in rare:
            x[r:r + 4] = rng.integers(128, 256, 4)
    L, el, ev, code, nb, mx = _oracle_encode(x, 2)
    assert 0 < mx <= 32
    payload, bits, idx = orc.huff_pack(x, code, nb, sync_syms=64)
    xt = torch.from_numpy(x).cuda()
    enc = codec.encode(xt, n_ary=2, sync_syms=64)
    assert enc["bits"] == bits
    out = torch.empty_like(xt)
    codec.decode_into(enc, out)
    assert codec.decode_status() == 0
    assert np.array_equal(out.cpu().numpy(), x), case


@pytest.mark.parametrize("n_ary", [2, 3, 16])
def test_decode_v8_equals_v7(torch_cuda, codec, n_ary):
    """The S = 64 fast decoder and the general decoder give identical bytes."""
    torch = torch_cuda
    from data_compression_amd import synth
    x = synth.log_like((2 << 20) + 12345, seed=n_ary)
    xt = torch.from_numpy(x).cuda()
    enc = codec.encode(xt, n_ary=n_ary, sync_syms=64)
    a = torch.empty_like(xt)
    codec.decode_into(enc, a)
    assert codec.decode_status() == 0
    codec.set_option("decode_general", 1)
    try:
        b = torch.empty_like(xt)
        codec.decode_into(enc, b)
        assert codec.decode_status() == 0
    finally:
        codec.set_option("decode_general", 0)
    assert torch.equal(a, b) and torch.equal(a, xt)


def test_decode_corrupt_stream_reports(torch_cuda, codec):
    """Garbage payload under a valid index: the decoder stays in bounds and flags it or
    decodes garbage; it never faults."""
    torch = torch_cuda
    from data_compression_amd import synth
    x = synth.enwik_like(1 << 20, seed=12)
    xt = torch.from_numpy(x).cuda()
    enc = codec.encode(xt, n_ary=3, sync_syms=64)
    g = torch.Generator(device="cpu").manual_seed(1)
    enc["words"].copy_(torch.randint(-2**31, 2**31 - 1, enc["words"].shape, generator=g, dtype=torch.int32).cuda())
    out = torch.empty_like(xt)
    codec.decode_into(enc, out)
    codec.decode_status()   # 0 or DC_E_STREAM; it must return
    torch.cuda.synchronize()


def test_decode_error_slots_and_stale_tables(torch_cuda, codec):
    """Error flags live in per-call rotating slots (no clearing launch): an error stays with
    its own call. A decode right after this context's pack skips the decoder-table launch; a
    table whose bytes were replaced since (not through the library) reads dec_ready 0 in the
    decoder: reported as a stream error, never silent garbage. Every later call is clean again."""
    torch = torch_cuda
    from data_compression_amd import synth
    from data_compression_amd.device import Codec
    other = Codec(0)
    x = synth.enwik_like(300_000, seed=31)
    xt = torch.from_numpy(x).cuda()
    out = torch.empty_like(xt)
    for _ in range(40):   # > 32 slots: the rotation wraps
        enc = codec.encode(xt, n_ary=2, sync_syms=64)
        codec.decode_into(enc, out)
        assert codec.decode_status() == 0 and torch.equal(out, xt)
    # a table rewritten behind the library's back (plain bytes of another context's table,
    # built BEFORE the encode, so no table write follows the pack): the decoder sees its
    # dec_ready 0 and reports it (a table written through the library since the pack makes
    # the decode rebuild the decoder tables instead: test_decode_table_rewritten_at_same_address)
    stale = other.table(other.hist(torch.from_numpy(synth.uniform_bytes(4096, seed=3)).cuda()), 2)
    enc = codec.encode(xt, n_ary=2, sync_syms=64)
    enc["table"].copy_(stale)
    codec.decode_into(enc, out)
    assert codec.decode_status() != 0   # stale decoder tables: reported
    enc = codec.encode(xt, n_ary=2, sync_syms=64)
    codec.decode_into(enc, out)
    assert codec.decode_status() == 0 and torch.equal(out, xt)
    codec.decode_into(enc, out)   # twice without a pack between
    assert codec.decode_status() == 0 and torch.equal(out, xt)


def _set_or_skip(c, name, value):
    """Select an A/B variant; the product library only has variant 0 (the alternatives are
    compiled in DC_AB_KERNELS diagnostic builds, tools/diag_build.sh)."""
    from data_compression_amd._lib import DcError
    try:
        c.set_option(name, value)
    except DcError:
        pytest.skip(f"{name}={value}: A/B kernels not in this build (DC_AB_KERNELS)")


@pytest.mark.parametrize("variant", [0, 1])
def test_decode_stale_tables_after_larger_decode(torch_cuda, variant):
    """a decode that finds its tables stale must leave the redo stage
    nothing to do. A large decode with many redo chunks first (its redo counter and masks
    stay behind), then a much smaller stream whose table was rebuilt by another context:
    reported, and nothing written past the smaller output (guard bytes intact); the next
    decodes on the context are exact again."""
    torch = torch_cuda
    from data_compression_amd import synth
    from data_compression_amd.device import Codec
    c = Codec(0)
    other = Codec(0)
    _set_or_skip(c, "decode_variant", variant)
    big = torch.from_numpy(_chain_stream(20, 5)).cuda()   # codes past the 15-bit table: many redo chunks
    enc = c.encode(big, n_ary=2, sync_syms=64)
    out = torch.empty_like(big)
    c.decode_into(enc, out)
    assert c.decode_status() == 0 and torch.equal(out, big)
    assert variant == 1 or c.decode_redo_count() > 0
    small = torch.from_numpy(synth.enwik_like(70_001, seed=33)).cuda()
    # another context's table (decoder tables never built: dec_ready 0), made BEFORE the encode
    # below and copied over the encode's table by plain bytes afterwards: the library sees no
    # table write after c's pack, so c keeps its tables for fresh and the decoder must catch it
    stale = other.table(other.hist(torch.from_numpy(synth.uniform_bytes(4096, seed=4)).cuda()), 2)
    enc_s = c.encode(small, n_ary=2, sync_syms=64)
    enc_s["table"].copy_(stale)
    guard = torch.full((small.numel() + 4096,), 0xA5, dtype=torch.uint8, device=small.device)
    c.decode_into(enc_s, guard[: small.numel()])
    assert c.decode_status() != 0
    assert bool((guard[small.numel():] == 0xA5).all()), "stale-table decode wrote past its output"
    for x in (small, big):
        e = c.encode(x, n_ary=2, sync_syms=64)
        o = torch.empty_like(x)
        c.decode_into(e, o)
        assert c.decode_status() == 0 and torch.equal(o, x)


def test_decode_table_rewritten_at_same_address(torch_cuda, codec):
    """the decoder tables a pack built are reused only while no table has
    been written since (process-wide generation, not the address alone). A new table written
    by another context into the buffer this context just packed with, and a stream under it
    (packed by the oracle, so no device pack builds its decoder tables), decodes exactly."""
    torch = torch_cuda
    from data_compression_amd import synth
    from data_compression_amd.device import Codec
    other = Codec(0)
    x1 = torch.from_numpy(synth.enwik_like(300_000, seed=91)).cuda()
    enc1 = codec.encode(x1, n_ary=2, sync_syms=64)   # codec's pack built this table's decoder tables
    T = enc1["table"]
    x2 = synth.english_like(200_003, seed=92)
    other.table(other.hist(torch.from_numpy(x2).cuda()), 2, out=T)   # same address, new table
    L, el, ev, code, nb, mx = _oracle_encode(x2, 2)
    payload, bits, idx = orc.huff_pack(x2, code, nb, sync_syms=64)
    words = torch.zeros(codec.words_needed(0, bits), dtype=torch.int32, device="cuda")
    words.view(torch.uint8)[: len(payload)] = torch.from_numpy(payload).cuda()
    lens = np.diff(np.append(idx, np.uint64(bits))).astype(np.int16)
    bases = idx[::64].astype(np.int64)
    sync = (torch.from_numpy(bases).cuda(), torch.from_numpy(lens).cuda())
    out = torch.empty(x2.size, dtype=torch.uint8, device="cuda")
    codec.decode(words, 0, sync, 64, x2.size, T, out)
    assert codec.decode_status() == 0 and np.array_equal(out.cpu().numpy(), x2)


def test_sharded_finalize_reads_its_own_plan(torch_cuda, codec):
    """finalize() of a stream reports that stream's pack outcome, not the
    latest encode's. Stream A into a words buffer far too small (the kernels write nothing and
    flag A's plan slot), then stream B encoded normally on the same context: finalize(A)
    raises, finalize(B) passes and B round-trips."""
    torch = torch_cuda
    from data_compression_amd import synth
    from data_compression_amd.dist import ShardedHuffman
    sh = ShardedHuffman(codec)
    xa = torch.from_numpy(synth.enwik_like(200_000, seed=5)).cuda()
    xb = torch.from_numpy(synth.enwik_like(150_000, seed=6)).cuda()
    tiny = torch.zeros(64, dtype=torch.int32, device="cuda")
    sa = sh.encode(xa, 2, 64, words=tiny, sync=codec.alloc_sync(xa.numel(), 64))
    sb = sh.encode(xb, 2, 64)
    with pytest.raises(RuntimeError):
        sh.finalize(sa)
    sh.finalize(sb)
    assert torch.equal(sh.decode(sb), xb)


@pytest.mark.parametrize("variant", [0, 1])
def test_decode_variants(torch_cuda, codec, variant):
    """The fast decoder's variants (0: one code per 15-bit lookup; 1: up to 3 per 13-bit
    lookup) on text, Zipf and flat bytes at n = 2, 3, 16, ragged sizes: exact round trips."""
    torch = torch_cuda
    from data_compression_amd import synth
    _set_or_skip(codec, "decode_variant", variant)
    try:
        for x, n_ary in ((synth.enwik_like(3 << 20, seed=61), 2), (synth.zipf_bytes((2 << 20) + 5, seed=62), 2),
                         (synth.english_like(1_000_003, seed=63), 3), (synth.enwik_like(777_777, seed=64), 16),
                         (synth.uniform_bytes(300_001, seed=65, lo=0, hi=255), 2)):
            xt = torch.from_numpy(x).cuda()
            enc = codec.encode(xt, n_ary=n_ary, sync_syms=64)
            out = torch.empty_like(xt)
            codec.decode_into(enc, out)
            assert codec.decode_status() == 0 and torch.equal(out, xt), (variant, n_ary, x.size)
    finally:
        codec.set_option("decode_variant", 0)


TEXT_CASES = [("base64url", 2), ("base16", 2), ("digits", 2), ("digits", 3), ("digits", 9), ("digits", 16),
              ("z85", 3), ("z85", 9), ("trits5", 3)]


@pytest.mark.parametrize("fmt,n_ary", TEXT_CASES)
def test_text_vs_oracle_and_roundtrip(torch_cuda, codec, fmt, n_ary):
    """Digit text of a real Huffman stream at bit offsets, byte-identical to
    the oracle's orc_text; text -> bits round trip; an invalid character is reported."""
    from data_compression_amd import synth
    from data_compression_amd._lib import DcError
    torch = torch_cuda
    fnum = codec.TEXT_FORMATS[fmt]
    x = synth.english_like(30011, seed=21)
    L, el, ev, code, nb, mx = _oracle_encode(x, n_ary)
    for bit_base in (0, 5, 32, 77):
        payload, bits, _ = orc.huff_pack(x, code, nb)
        enc = codec.encode(torch.from_numpy(x).cuda(), n_ary=n_ary, sync_syms=64, bit_base=bit_base)
        assert enc["bits"] == bits
        txt = codec.text(enc["words"], bit_base, bits, fmt, n_ary)
        want = orc.text(payload, bits, fnum, n_ary)
        assert txt.cpu().numpy().tobytes() == want, (fmt, n_ary, bit_base)
        back = codec.text_parse(txt, fmt, n_ary, bits)
        got = back.cpu().numpy().view(np.uint8)[: (bits + 7) // 8]
        assert np.array_equal(got, payload), (fmt, n_ary, bit_base)
    bad = txt.clone()
    bad[len(bad) // 2] = 0 if fmt == "trits5" else ord("~")
    with pytest.raises(DcError):
        codec.text_parse(bad, fmt, n_ary, bits)


def test_small_shard_bodies_concatenate_to_stream(torch_cuda, codec):
    """dc_small_compress_body on shards with 1-byte halos (dist.ShardedSmall's per-rank
    step): header + bodies == the reference front-end output of the whole stream; the
    body decoder inverts each body."""
    from data_compression_amd import synth
    torch = torch_cuda
    x = synth.log_like(300_001, seed=12)
    want = orc.small_compress(x.tobytes())
    cuts = [0, 1000, 1001, 77_777, 200_000, x.size]
    # a cut between ' ' and a letter (a pair straddling two shards)
    j = next(i for i in range(150_000, x.size) if x[i - 1] == ord(" ") and ord("a") <= x[i] <= ord("z"))
    cuts = sorted(set(cuts + [j]))
    xt = torch.from_numpy(x).cuda()
    parts = [bytes([8, x[0]])]
    for r in range(len(cuts) - 1):
        lo, hi = cuts[r], cuts[r + 1]
        y = xt[max(lo - 1, 0): min(hi + 1, x.size)]
        nelem = hi - lo - (1 if lo == 0 else 0)
        body = codec.small_body(y, lo > 0, nelem)
        parts.append(body.cpu().numpy().tobytes())
        back = codec.small_decompress_body(body).cpu().numpy()
        assert back.tobytes() == _small_body_decode_ref(body.cpu().numpy())
    assert b"".join(parts) == want


def _small_body_decode_ref(b):
    out = bytearray()
    for v in b.tolist():
        out += bytes([32, v - 0x80]) if v >= 0x80 else bytes([v])
    return bytes(out)


@pytest.mark.parametrize("fused", [True, False])
def test_sharded_small_single_rank_on_device(torch_cuda, codec, fused):
    """dist.ShardedSmall with the device engine (world size 1): C5 front-end + n=16
    Huffman equals the oracle's encoding of the reference front-end output; round trip. Both
    the one-pass encode + counted decode (dc_small_huff_*) and the two stages."""
    from data_compression_amd import synth
    from data_compression_amd.dist import ShardedSmall
    torch = torch_cuda
    x = synth.log_like(1 << 20, seed=13)
    sm = ShardedSmall(codec, fused=fused)
    s = sm.encode(torch.from_numpy(x).cuda(), n_ary=16, sync_syms=64)
    fe = np.frombuffer(orc.small_compress(x.tobytes()), np.uint8)
    L, el, ev, code, nb, mx = _oracle_encode(fe, 16)
    payload, bits, _ = orc.huff_pack(fe, code, nb, sync_syms=64)
    sm.h.finalize(s)
    assert s.bits == bits
    assert np.array_equal(s.words.cpu().numpy().view(np.uint8)[: len(payload)], payload)
    assert np.array_equal(sm.decode(s).cpu().numpy(), x)


def test_sharded_small_streams_own_their_buffers(torch_cuda, codec):
    """Two fused encodes of same-size inputs, then both decodes: the first stream's payload,
    sync index and table must survive the second encode (they were cached per size)."""
    from data_compression_amd import synth
    from data_compression_amd.dist import ShardedSmall
    torch = torch_cuda
    n = (3 << 16) + 11
    xs = [synth.log_like(n, seed=31), synth.log_like(n, seed=32)]
    sm = ShardedSmall(codec, fused=True)
    ss = [sm.encode(torch.from_numpy(x).cuda(), n_ary=16, sync_syms=64) for x in xs]
    for x, s in zip(xs, ss):
        assert np.array_equal(sm.decode(s).cpu().numpy(), x)


def test_static_body_after_adaptive_work(torch_cuda):
    """One context: an adaptive encode (it leaves first-touch records behind), then a static
    shard body on the same context must still encode (the static write passed the
    records on and tripped the unsettled-ranks guard)."""
    from data_compression_amd import synth
    from data_compression_amd.device import Codec
    from data_compression_amd.dist import ShardedNybble
    torch = torch_cuda
    c = Codec(0)
    x = synth.english_like(50_001, seed=3)
    xt = torch.from_numpy(x).cuda()
    assert c.nyb_compress(xt, True).cpu().numpy().tobytes() == orc.nybble_compress(x.tobytes(), True)
    c.nyb_body_plan(xt, True, dist_initial_lists())   # adaptive plan too
    seg, lit = ShardedNybble(c).compress(xt, False)
    assert not lit
    assert seg.cpu().numpy().tobytes() == orc.nybble_compress(x.tobytes(), False)


def dist_initial_lists():
    from data_compression_amd.dist import INITIAL_LISTS
    return INITIAL_LISTS.copy()


# ---------------------------------------------------------------- nybble: adaptive in parallel, shards
def _nyb_cases(torch):
    from data_compression_amd import synth
    rng = np.random.default_rng(77)
    cases = []
    for n in (1, 2, 3, 5, 17, 4096, 4097, 4098, 8193, 65_543, (1 << 20) + 3):
        cases.append(("text", synth.english_like(n, seed=n)))
    for n in (4099, 300_001):
        cases.append(("bytes", rng.integers(1, 256, size=n, dtype=np.uint8)))   # every context, non-ASCII
        cases.append(("skew", rng.choice(np.frombuffer(b"e tax\x80\x81", np.uint8), size=n)))
    # zero bytes (outside the reference's C-string domain; the restatement is length-based): the
    # walk pads short lists with zero bytes, so a touched zero must be told from a pad
    cases.append(("zeros", rng.integers(0, 256, size=300_001, dtype=np.uint8)))
    cases.append(("zskew", rng.choice(np.frombuffer(b"\x00\x00e t\x01", np.uint8), size=70_001)))
    z = synth.english_like(200_003, seed=5)
    z[rng.integers(0, z.size, size=300)] = 0   # rare zeros: pushed off, or still on a list
    cases.append(("zrare", z))
    cases.append(("log", synth.log_like(5 << 20, seed=9)))   # 1280 tiles: two reduce levels
    return cases


@pytest.mark.parametrize("modify", [True, False])
def test_nybble_encode_parallel_vs_oracle(torch_cuda, codec, modify):
    """Adaptive encode by per-tile move-to-front summaries (k_mtf_*), byte-exact against the
    reference restatement, at ragged sizes, every context, and misaligned device buffers (offset
    1: a tile's elements still start in its first granule dword, k_mtf_walk<2>; offset 5: they
    start in its second, the any-alignment walk k_mtf_walk<3>)."""
    torch = torch_cuda
    for kind, x in _nyb_cases(torch):
        ref = orc.nybble_compress(x.tobytes(), modify)
        xd = torch.from_numpy(x).cuda()
        b1 = torch.zeros(x.size + 1, dtype=torch.uint8, device="cuda")
        b1[1:] = xd
        b5 = torch.zeros(x.size + 5, dtype=torch.uint8, device="cuda")
        b5[5:] = xd
        for xt in (xd, b1[1:], b5[5:]):
            got = codec.nyb_compress(xt, modify).cpu().numpy().tobytes()
            assert got == ref, (kind, x.size)
        if modify and x.size < 400_000:
            # bytes >= 0x80 do not round-trip in the reference either: compare with
            # the reference decoder's output
            back = codec.nyb_decompress(torch.from_numpy(np.frombuffer(ref, np.uint8).copy()).cuda(), True)
            assert back.cpu().numpy().tobytes() == orc.nybble_decompress(ref, True), (kind, x.size)
            if kind in ("text", "log"):
                assert np.array_equal(back.cpu().numpy(), x), (kind, x.size)


@pytest.mark.parametrize("wtile_off", [0, 1])
def test_nybble_static_writers_vs_oracle(torch_cuda, wtile_off):
    """The nybble codec's two writers each way (and the adaptive encode's) (DC_OPT_NYB_WTILE_OFF: 0 = a wave per 4096-element
    tile, k_nyb_enc_wtile / k_nyb_dec_wtile; 1 = a workgroup per tile, k_fsm_write), byte-exact
    against the reference restatement (nybble_compression.c compress_bytestring and
    decompress_bytestring, modify = false) on the ragged, every-context and zero-byte cases, a
    LITERAL fallback, and odd element counts at tile edges."""
    from data_compression_amd.device import Codec
    torch = torch_cuda
    c = Codec(0)
    c.set_option("nyb_wtile_off", wtile_off)
    cases = _nyb_cases(torch)
    rng = np.random.default_rng(11)
    cases.append(("literal", rng.integers(128, 256, size=70_001, dtype=np.uint8)))   # no byte a hit
    for n in (4096 * 4 + 1, 4096 * 4 + 2, 4096 * 5 - 1, 64 * 3 + 2):
        cases.append(("edge", synth_text(n, seed=n)))
    for kind, x in cases:
        ref = orc.nybble_compress(x.tobytes(), False)
        got = c.nyb_compress(torch.from_numpy(x).cuda(), False).cpu().numpy().tobytes()
        assert got == ref, (kind, x.size, wtile_off)
        # the decode writers (k_nyb_dec_wtile / k_fsm_write<M_NYB_DEC>) on the reference's stream
        back = c.nyb_decompress(torch.from_numpy(np.frombuffer(ref, np.uint8).copy()).cuda(), False)
        assert back.cpu().numpy().tobytes() == orc.nybble_decompress(ref, False), (kind, x.size, wtile_off)
        if x.size < 2_000_000:   # the adaptive encode's writer (k_nyb_enc_wtile<true> / k_fsm_write)
            got = c.nyb_compress(torch.from_numpy(x).cuda(), True).cpu().numpy().tobytes()
            assert got == orc.nybble_compress(x.tobytes(), True), (kind, x.size, wtile_off, "adaptive")


def synth_text(n, seed):
    from data_compression_amd import synth
    return synth.english_like(n, seed=seed)


@pytest.mark.parametrize("v1", [0, 1, 3])
def test_nybble_adaptive_decode_edges(torch_cuda, codec, v1):
    """Adaptive decode (tokens by the static transducer, then the resolve in place: 0 = control
    words + k_nyb_resolve_c + the re-encode check, 3 = the exact k_nyb_resolve_s, 1 = the
    one-pass k_nyb_adec): every output size 1..200 and block-boundary sizes, output buffers at
    every offset mod 64 (the resolve kernels' first and last blocks), against the reference
    restatement."""
    torch = torch_cuda
    from data_compression_amd import synth
    _set_or_skip(codec, "nyb_adec_v1", int(v1))
    try:
        rng = np.random.default_rng(17)
        sizes = list(range(1, 201)) + [255, 256, 257, 4095, 4096, 4097, 65536 + 63, 200_001]
        for n in sizes:
            x = synth.english_like(n, seed=n) if n % 3 else rng.integers(1, 128, size=n, dtype=np.uint8)
            ref = orc.nybble_compress(x.tobytes(), True)
            comp = torch.from_numpy(np.frombuffer(ref, np.uint8).copy()).cuda()
            want = orc.nybble_decompress(ref, True)
            off = (n * 7) % 64
            big = torch.full((2 * len(ref) + off + 64,), 0xEE, dtype=torch.uint8, device="cuda")
            got = codec.nyb_decompress(comp, True, out=big[off: off + 2 * len(ref)])
            assert got.cpu().numpy().tobytes() == want, (n, off)
            tail = big[off + len(want):].cpu().numpy()
            assert (big[:off].cpu().numpy() == 0xEE).all() and (tail[: 2 * len(ref) - len(want)] == 0xEE).all(), n
    finally:
        codec.set_option("nyb_adec_v1", 0)


@pytest.mark.parametrize("v1", [0, 3])
def test_nybble_adaptive_decode_any_stream(torch_cuda, codec, v1):
    """Adaptive decode of arbitrary streams (random nybbles after the 0xAF header, and the
    encoder's streams with one byte changed to a literal that is in its list, which the
    reference decoder moves from where it is), for the control-word resolve and the plain-code
    one, against the reference restatement."""
    torch = torch_cuda
    from data_compression_amd import synth
    _set_or_skip(codec, "nyb_adec_v1", v1)
    try:
        rng = np.random.default_rng(23)
        for n in [3, 4, 17, 64, 65, 66, 130, 1000, 4097, 70_001]:
            for kind in ("random", "low", "patched"):
                if kind == "patched":
                    ref = bytearray(orc.nybble_compress(synth.english_like(n, seed=n).tobytes(), True))
                    if ref[0] != 0xAF or len(ref) < 4:
                        continue
                    k = 2 + int(rng.integers(0, len(ref) - 2))
                    ref[k] = 0x65   # a literal 'e' nybble pair where the stream had something else
                    comp = bytes(ref)
                else:
                    body = rng.integers(0, 256 if kind == "random" else 128, size=n, dtype=np.uint8)
                    comp = bytes([0xAF]) + body.tobytes()
                want = orc.nybble_decompress(comp, True)
                t = torch.from_numpy(np.frombuffer(comp, np.uint8).copy()).cuda()
                got = codec.nyb_decompress(t, True).cpu().numpy().tobytes()
                assert got == want, (n, kind)
    finally:
        codec.set_option("nyb_adec_v1", 0)


class _ThreadRanks:
    """world ranks as threads over one GPU (one Codec each), all_gather by a barrier: runs
    dist.ShardedNybble's orchestration unchanged on the device engine."""

    def __init__(self, world):
        import threading
        self.world, self.bar, self.slots = world, threading.Barrier(world), [None] * world

    def gather(self, rank, vals):
        self.slots[rank] = list(vals)
        self.bar.wait()
        out = [list(v) for v in self.slots]
        self.bar.wait()
        return out


@pytest.mark.parametrize("world,modify", [(2, False), (3, True), (4, False), (5, True)])
def test_sharded_nybble_on_device(torch_cuda, world, modify):
    import threading

    from data_compression_amd import synth
    from data_compression_amd.device import Codec
    from data_compression_amd.dist import ShardedNybble
    torch = torch_cuda
    x = synth.english_like(200_000 * world + 51, seed=world)
    rng = np.random.default_rng(world)
    cuts = [0] + sorted(int(v) for v in rng.choice(np.arange(2, x.size - 1), world - 1, replace=False)) + [x.size]
    ref = orc.nybble_compress(x.tobytes(), modify)
    whole = np.frombuffer(ref, np.uint8)
    dcut = [0] + sorted(int(v) for v in rng.choice(np.arange(3, whole.size - 1), world - 1, replace=False)) + \
        [whole.size]
    tr = _ThreadRanks(world)
    res, errs = [None] * world, []

    def run(r):
        try:
            torch.cuda.set_device(0)
            sn = ShardedNybble(Codec(0))
            sn.world, sn.rank = world, r
            sn._gather = lambda vals, dev: tr.gather(r, vals)
            seg, lit = sn.compress(torch.from_numpy(x[cuts[r]: cuts[r + 1]].copy()).cuda(), modify)
            out = None
            if not modify:
                out = sn.decompress(torch.from_numpy(whole[dcut[r]: dcut[r + 1]].copy()).cuda()).cpu().numpy()
            res[r] = (seg.cpu().numpy().tobytes(), lit, out)
        except Exception as e:   # noqa: BLE001
            errs.append(repr(e))
            tr.bar.abort()

    ths = [threading.Thread(target=run, args=(r,)) for r in range(world)]
    for t in ths:
        t.start()
    for t in ths:
        t.join(timeout=120)
    assert not errs, errs
    assert b"".join(r[0] for r in res) == ref
    if not modify:
        assert np.array_equal(np.concatenate([r[2] for r in res]), x)


@pytest.mark.parametrize("modify", [True, False])
def test_nybble_chunked_container(torch_cuda, codec, modify):
    """DCNK: every chunk is the reference's stream of that chunk (so it decodes alone), the
    container decodes chunk-parallel back to the input, and damage is reported."""
    import struct

    from data_compression_amd import synth
    from data_compression_amd._lib import DcError
    torch = torch_cuda
    for n, K in ((0, 64), (1, 16), (17, 16), (5000, 4096), (300_007, 4096), (3 << 20, 1 << 16)):
        x = synth.english_like(n, seed=n + 1) if n else np.zeros(0, np.uint8)
        xt = torch.from_numpy(x).cuda() if n else torch.zeros(0, dtype=torch.uint8, device="cuda")
        comp = codec.nyb_compress_chunked(xt, modify, K)
        c = comp.cpu().numpy().tobytes()
        magic, ver, mod, k, nn, nch = struct.unpack_from("<IIIIQQ", c)
        assert (magic, ver, mod, k, nn) == (0x4B4E4344, 1, int(modify), K, n)
        assert nch == (n + K - 1) // K
        off = np.frombuffer(c, np.uint64, nch + 1, 32)
        pay = c[32 + 8 * (nch + 1):]
        assert len(pay) == int(off[-1])
        for i in range(0, nch, max(1, nch // 7)):
            chunk = x[i * K: (i + 1) * K].tobytes()
            assert pay[int(off[i]): int(off[i + 1])] == orc.nybble_compress(chunk, modify), (n, K, i)
        if n:
            back = codec.nyb_decompress_chunked(comp)
            assert np.array_equal(back.cpu().numpy(), x), (n, K)
    bad = comp.clone()
    bad[32 + 8] = bad[32 + 8] + 1   # chunk 1 starts one byte late
    with pytest.raises(DcError):
        codec.nyb_decompress_chunked(bad)
    # shards that are multiples of K: the merged per-shard containers equal the whole one
    from data_compression_amd.dist import merge_chunked
    x = synth.log_like(5 * 65536 + 999, seed=3)
    parts = [x[:2 * 65536], x[2 * 65536: 4 * 65536], x[4 * 65536:]]
    per = [codec.nyb_compress_chunked(torch.from_numpy(p.copy()).cuda(), modify, 65536).cpu().numpy().tobytes()
           for p in parts]
    whole = codec.nyb_compress_chunked(torch.from_numpy(x).cuda(), modify, 65536).cpu().numpy().tobytes()
    assert merge_chunked(per) == whole


@pytest.mark.parametrize("modify", [True, False])
def test_nybble_batch_decode_vs_oracle(torch_cuda, codec, modify):
    """dc_nyb_decompress_batch (the many-stream throughput path beside DCNK):
    independent reference streams of mixed sizes, including empty ones, LITERAL-fallback
    streams (type ' '), streams of other type bytes (copied whole, :806), arbitrary nybble
    streams and one of every size 1..40, each decoded as the reference restatement does."""
    torch = torch_cuda
    from data_compression_amd import synth
    rng = np.random.default_rng(41)
    streams = [b""]
    for n in list(range(1, 41)) + [100, 4095, 4096, 4097, 65_537]:
        streams.append(orc.nybble_compress(synth.english_like(n, seed=n).tobytes(), modify))
    streams.append(orc.nybble_compress(bytes(rng.integers(1, 128, size=3000, dtype=np.uint8)), modify))  # often ' '
    streams.append(bytes([0x41]) + b"raw bytes under another type")
    streams.append(bytes([0xAF]) + rng.integers(0, 256, size=777, dtype=np.uint8).tobytes())
    streams.append(bytes([0xAF]))
    for _ in range(300):
        n = int(rng.integers(1, 2000))
        streams.append(orc.nybble_compress(synth.english_like(n, seed=int(rng.integers(1 << 30))).tobytes(), modify))
    off = np.zeros(len(streams) + 1, np.int64)
    off[1:] = np.cumsum([len(x) for x in streams])
    data = np.frombuffer(b"".join(streams), np.uint8).copy()
    out, out_off = codec.nyb_decompress_batch(torch.from_numpy(data).cuda(), torch.from_numpy(off).cuda(), modify)
    o, oo = out.cpu().numpy().tobytes(), out_off.cpu().numpy()
    for i, st in enumerate(streams):
        want = b"" if st == b"" else orc.nybble_decompress(st, modify) if st[0] != 0xAF or len(st) >= 2 else b""
        assert o[oo[i]: oo[i + 1]] == want, (i, len(st))


def _thread_collectives(sh, tr, r, world, torch):
    """ShardedHuffman collectives over thread ranks (all on one GPU)."""
    def all_reduce(t):
        tot = np.sum(np.array(tr.gather(r, t.cpu().tolist()), dtype=np.int64), axis=0)
        t.copy_(torch.from_numpy(tot).to(t.device))

    def all_gather_scalar(t):
        v = tr.gather(r, [int(t.item())])
        return torch.tensor([q[0] for q in v], dtype=t.dtype, device=t.device)

    def broadcast_table(t):
        v = tr.gather(r, t.cpu().numpy().tobytes())[world - 1]
        t.copy_(torch.from_numpy(np.array(v, dtype=np.uint8)).to(t.device))
    sh._all_reduce, sh._all_gather_scalar = all_reduce, all_gather_scalar
    sh._reduce_to_src, sh._broadcast_table = all_reduce, broadcast_table   # the sum: read by the table rank only


@pytest.mark.parametrize("world,n_ary,table_mode,prealloc", [(2, 2, "replicate", False), (3, 16, "replicate", False),
                                                             (3, 2, "broadcast", False), (3, 2, "replicate", True),
                                                             (4, 16, "broadcast", True)])
def test_sharded_huffman_on_device(torch_cuda, world, n_ary, table_mode, prealloc):
    """dist.ShardedHuffman on the device engine (thread ranks, collectives by a barrier):
    each rank packs at its global bit offset; the OR-merged shards equal the single-GPU
    stream of the whole input bit for bit, and every rank decodes its own shard. In
    broadcast mode the table bytes one rank's context built drive every other context.
    prealloc: words and sync index preallocated, so the rank's bit offset stays on the
    device (dc_huff_pack_async_dev / dc_huff_decode_dev: no host read in the encode)."""
    import threading

    from data_compression_amd import synth
    from data_compression_amd.device import Codec
    from data_compression_amd.dist import ShardedHuffman
    torch = torch_cuda
    S = 64
    shard = 64 * S * 37
    x = synth.enwik_like(shard * (world - 1) + 50_001, seed=world)
    tr = _ThreadRanks(world)
    res, errs = [None] * world, []

    def run(r):
        try:
            torch.cuda.set_device(0)
            c = Codec(0)
            sh = ShardedHuffman(c, table_mode=table_mode)
            sh.world, sh.rank = world, r
            sh.table_src = world - 1
            _thread_collectives(sh, tr, r, world, torch)
            lo = r * shard
            xs = torch.from_numpy(x[lo: x.size if r == world - 1 else lo + shard].copy()).cuda()
            if prealloc:
                words = torch.empty(c.words_needed(31, 32 * xs.numel()) + 8, dtype=torch.int32, device="cuda")
                s = sh.encode(xs, n_ary=n_ary, sync_syms=S, words=words, sync=c.alloc_sync(xs.numel(), S))
                assert s.bits == -1 and isinstance(s.bit_base, torch.Tensor)
                y = sh.decode(s)
                sh.finalize(s)
            else:
                s = sh.encode(xs, n_ary=n_ary, sync_syms=S)
                y = sh.decode(s)
            nw = (s.bit_base % 32 + s.bits + 31) // 32
            res[r] = (s.bit_base, s.bits, s.words[:nw].cpu().numpy().copy(), bool(torch.equal(y[: xs.numel()], xs)))
        except Exception as e:   # noqa: BLE001
            errs.append(repr(e))
            tr.bar.abort()

    ths = [threading.Thread(target=run, args=(r,)) for r in range(world)]
    for t in ths:
        t.start()
    for t in ths:
        t.join(timeout=120)
    assert not errs, errs
    assert all(r[3] for r in res)
    total = res[-1][0] + res[-1][1]
    merged = np.zeros((total + 31) // 32, np.uint32)
    for base, bits, w, _ in res:
        w0 = base // 32
        merged[w0: w0 + w.size] |= w.view(np.uint32)[: merged.size - w0]
    c = Codec(0)
    enc = c.encode(torch.from_numpy(x).cuda(), n_ary=n_ary, sync_syms=S)
    assert enc["bits"] == total
    ref = enc["words"].cpu().numpy().view(np.uint32)[: merged.size]
    assert np.array_equal(merged, ref)


@pytest.mark.parametrize("world,fused", [(2, False), (3, False), (2, True), (3, True), (4, True)])
def test_sharded_small_on_device(torch_cuda, world, fused):
    """dist.ShardedSmall on the device engine (thread ranks). Two stages: the halo elements
    settled on the host, bodies sized then written in place (dc_small_compress_body_plan/_write)
    at 16-B aligned re-cut segments. Fused: each shard's one-pass encode at its global offsets
    (dc_small_huff_shard_*), offsets on the device until finalize(). Either way the OR-merged
    Huffman shards equal the oracle's encoding of the reference front-end output, and the
    decoded segments concatenate to the input."""
    import threading

    from data_compression_amd import synth
    from data_compression_amd.device import Codec
    from data_compression_amd.dist import ShardedSmall
    torch = torch_cuda
    S, n_ary = 64, 16
    x = synth.log_like((1 << 20) * world + 777, seed=world)
    cuts = [0]
    for k in range(1, world):   # one cut inside a pair (' ' | letter), one just before a ' '
        c = k * x.size // world
        while not (x[c - 1] == ord(" ") and ord("a") <= x[c] <= ord("z")) if k % 2 else x[c] != ord(" "):
            c += 1
        cuts.append(c)
    cuts.append(x.size)
    tr = _ThreadRanks(world)
    slots = [None] * world
    res, errs = [None] * world, []

    def run(r):
        try:
            torch.cuda.set_device(0)
            sm = ShardedSmall(Codec(0), fused=fused)
            sm.world = sm.h.world = world
            sm.rank = sm.h.rank = r
            sm.h.table_src = world - 1
            _thread_collectives(sm.h, tr, r, world, torch)
            sm._gather_i64 = lambda vals: tr.gather(r, vals)

            def ag(t):   # (the fused path's device all_gather and all_reduce)
                v = tr.gather(r, t.reshape(-1).cpu().tolist())
                return torch.tensor(v, dtype=t.dtype, device=t.device).view((world,) + tuple(t.shape))

            def ar(t, op=None):
                v = np.array(tr.gather(r, t.reshape(-1).cpu().tolist()), dtype=np.int64)
                red = v.max(axis=0) if op is not None and op == torch.distributed.ReduceOp.MAX else v.sum(axis=0)
                t.copy_(torch.from_numpy(red).to(t.device).view(t.shape))
            sm._all_gather_dev, sm._all_reduce_dev = ag, ar

            def shift(send, recv):   # send to r + 1, receive from r - 1
                slots[r] = send.clone() if send is not None else None
                tr.bar.wait()
                if recv is not None and recv.numel():
                    recv.copy_(slots[r - 1])
                tr.bar.wait()
            sm._shift = shift
            s = sm.encode(torch.from_numpy(x[cuts[r]: cuts[r + 1]].copy()).cuda(), n_ary=n_ary, sync_syms=S)
            assert (getattr(s, "shard_fused", None) is not None) == fused
            sm.finalize(s) if fused else sm.h.finalize(s)
            y = sm.decode(s)
            nw = (s.bit_base % 32 + s.bits + 31) // 32
            res[r] = (s.bit_base, s.bits, s.words[:nw].cpu().numpy().copy(), y.cpu().numpy().copy())
        except Exception as e:   # noqa: BLE001
            errs.append(repr(e))
            tr.bar.abort()

    ths = [threading.Thread(target=run, args=(r,)) for r in range(world)]
    for t in ths:
        t.start()
    for t in ths:
        t.join(timeout=120)
    assert not errs, errs
    assert np.array_equal(np.concatenate([v[3] for v in res]), x)
    fe = np.frombuffer(orc.small_compress(x.tobytes()), np.uint8)
    L, el, ev, code, nb, mx = _oracle_encode(fe, n_ary)
    payload, bits, _ = orc.huff_pack(fe, code, nb, sync_syms=S)
    total = res[-1][0] + res[-1][1]
    assert total == bits
    merged = np.zeros((total + 31) // 32, np.uint32)
    for base, nbits, w, _ in res:
        w0 = base // 32
        merged[w0: w0 + w.size] |= w.view(np.uint32)[: merged.size - w0]
    assert np.array_equal(merged.view(np.uint8)[: len(payload)], payload)


def test_histogram_running_counters_skewed(torch_cuda, codec):
    """k_hist_blocks keeps running 8-bit wave counters across a workgroup's blocks (the
    block's counts are 32-bit differences): a single repeated byte makes every field wrap
    and carry many times; ragged tails and every bin value."""
    torch = torch_cuda
    for n, fill in ((64 << 20, 0x20), (64 << 20, 0xFF), ((48 << 20) + 12345, 0x00)):
        x = torch.full((n,), fill, dtype=torch.uint8, device="cuda")
        x[::4099] = torch.arange(256, device="cuda", dtype=torch.int64).repeat(n // 4099 // 256 + 1)[: x[::4099].numel()].to(torch.uint8)
        h = codec.hist(x)
        assert torch.equal(h, torch.bincount(x.to(torch.int64), minlength=256)), (n, fill)


@pytest.mark.gpu
def test_histogram_grids_and_repeats(torch_cuda):
    """The bins go through a per-context accumulator that the last workgroup out empties:
    any grid (1 workgroup, a few, more than the input's blocks), launches back to back on
    one context, a sub-block input in between, two contexts interleaved."""
    torch = torch_cuda
    from data_compression_amd.device import Codec
    from data_compression_amd import synth
    a, b = Codec(0), Codec(0)
    xs = [torch.from_numpy(synth.enwik_like((5 << 20) + 77, seed=s)).cuda() for s in (1, 2)]
    ref = [torch.bincount(x.to(torch.int64), minlength=256) for x in xs]
    tiny = xs[1][:100]   # under one block
    for grid in (1, 3, 64, 0):   # 0: the default grid
        a.set_option("hist_grid", grid)
        for k in range(3):
            assert torch.equal(a.hist(xs[k & 1]), ref[k & 1]), (grid, k)
            assert torch.equal(b.hist(xs[(k + 1) & 1]), ref[(k + 1) & 1]), (grid, k)
        assert torch.equal(a.hist(tiny), torch.bincount(tiny.to(torch.int64), minlength=256)), grid
        assert torch.equal(a.hist(xs[0]), ref[0]), grid
