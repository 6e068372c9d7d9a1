"""Codes of 4-bit digits (n = 9..16) whose lengths reach 4 digits (16 bits) and beyond: the fast
decoder's 15-bit first level escapes every such code, so those chunks go through the exact redo
(k_huff_decode8_fix, its second level and canonical search; n_ary_huffman.c:1540-1568: codes of
one length are consecutive base-n values, lengths ascending). Streams bit-exact against the
oracle's packer (the layout is build-defined, parity pinned at the table level); outputs against
the input; runs of 16-bit codes (three in one 4-symbol batch), codes of 5-6 digits, garbage.
(Round 6 also measured a redo-free form, a 16-bit one-byte table with the lengths from the
canonical limits: bit-exact on these tests but slower, profiles/r6e_n16_v2_ab.log.)"""
import numpy as np
import pytest

from oracle import oracle as orc

pytestmark = pytest.mark.gpu


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


def _oracle_stream(x, n, S=64):
    h = orc.histogram(x)
    L = orc.huffman_lengths(h, n)
    el, ev = orc.canonical(L, n)
    code, nb, mx = orc.bitcodes(el, ev, n)
    payload, bits, _ = orc.huff_pack(x, code, nb, sync_syms=S)
    return payload, bits, mx


def _skewed(n, seed, rare=240, frac=0.008):
    """Bytes whose n = 9/10 code has 4-digit (16-bit) codes, often several in a row (three in one
    4-symbol batch: the 48-bit case): 12 frequent symbols, 240 rare ones in bursts of 4."""
    rng = np.random.default_rng(seed)
    common = rng.choice(np.arange(32, 127), 12, replace=False).astype(np.uint8)
    rare_v = rng.choice(np.setdiff1d(np.arange(1, 256), common), rare, replace=False).astype(np.uint8)
    out = rng.choice(common, n)
    for p in rng.integers(0, n - 8, int(n * frac / 4)):
        out[p: p + 4] = rng.choice(rare_v, 4)
    return out.astype(np.uint8)


def _deep(base, reps, seed):
    """n = 16 needs a deep tree for 4-digit codes (256 symbols fit two digits): levels of 15
    symbols with counts base^5, base^4, ... (base 4: codes of 1-4 digits; base 6: up to 6)."""
    counts = np.array([base ** (5 - lvl) for lvl in range(6) for _ in range(15)], np.int64)
    v = np.repeat(np.arange(1, counts.size + 1, dtype=np.uint8), counts * reps)
    return np.random.default_rng(seed).permutation(v).astype(np.uint8)


@pytest.mark.parametrize("n_ary", [9, 10, 16])
@pytest.mark.parametrize("kind", ["text", "skewed"])
def test_digit4_decode_bit_exact(torch_cuda, codec, n_ary, kind):
    torch = torch_cuda
    from data_compression_amd import synth
    if kind == "text":
        x = synth.GENERATORS["C5"](1 << 20, seed=5)
    else:
        x = _deep(4, 40, seed=n_ary) if n_ary == 16 else _skewed(1 << 20, seed=n_ary)
    payload, bits, mx = _oracle_stream(x, n_ary)
    xt = torch.from_numpy(x).cuda()
    enc = codec.encode(xt, n_ary=n_ary, sync_syms=64)
    assert enc["bits"] == bits
    got = enc["words"].cpu().numpy().view(np.uint8)[: len(payload)]
    assert np.array_equal(got, payload)
    out = torch.empty_like(xt)
    codec.decode_into(enc, out)
    assert codec.decode_status() == 0
    assert torch.equal(out, xt)
    if mx <= 15:   # (every code within the 15-bit first level: nothing to redo, 1 MiB = whole tuples)
        assert codec.decode_redo_count() == 0


def test_digit4_c5_fused_decode(torch_cuda, codec):
    """The C5 path (small front-end + n = 16, fused encode, counted decode, the redo adding the
    redone chunks' pair counts): the output is the input."""
    torch = torch_cuda
    from data_compression_amd import synth
    x = synth.GENERATORS["C5"](4 << 20, seed=55)
    xt = torch.from_numpy(x).cuda()
    enc = codec.small_huff_encode(xt, 16, 64)
    y = codec.small_huff_decode(enc)
    assert torch.equal(y, xt)


def test_digit4_table_from_other_context_and_long_codes(torch_cuda, codec):
    """A table written by another context, and a 4-bit-digit code past 4 digits (up to 24 bits:
    the redo's canonical search): both decode exactly."""
    torch = torch_cuda
    from data_compression_amd.device import Codec
    other = Codec(0)
    x = _deep(4, 10, seed=77)
    xt = torch.from_numpy(x).cuda()
    enc = other.encode(xt, n_ary=16, sync_syms=64)
    out = torch.empty_like(xt)
    codec.decode_into(enc, out)   # (this context did not write that table)
    assert codec.decode_status() == 0 and torch.equal(out, xt)
    # n = 16 codes of up to 6 digits (24 bits)
    y = _deep(6, 2, seed=3)
    _, _, mx = _oracle_stream(y, 16)
    assert mx > 16
    yt = torch.from_numpy(y).cuda()
    enc = codec.encode(yt, n_ary=16, sync_syms=64)
    outy = torch.empty_like(yt)
    codec.decode_into(enc, outy)
    assert codec.decode_status() == 0 and torch.equal(outy, yt), mx


def test_digit4_corrupt_stream_returns(torch_cuda, codec):
    """Garbage payload under a valid index, 16-bit codes: the decoder and the redo stay in bounds
    and return (as test_decode_corrupt_stream_reports)."""
    torch = torch_cuda
    x = _deep(4, 10, seed=9)
    xt = torch.from_numpy(x).cuda()
    enc = codec.encode(xt, n_ary=16, sync_syms=64)
    g = torch.Generator(device="cpu").manual_seed(2)
    enc["words"].copy_(torch.randint(-2**31, 2**31 - 1, enc["words"].shape, generator=g, dtype=torch.int32).cuda())
    out = torch.empty_like(xt)
    codec.decode_into(enc, out)
    codec.decode_status()   # 0 or DC_E_STREAM; it must return
    torch.cuda.synchronize()
