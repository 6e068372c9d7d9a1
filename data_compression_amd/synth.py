"""Seeded synthetic workloads for the five BASELINE.json configs.

There is no network and no local enwik8, so every input is generated. The
generators are deterministic functions of (size, seed) and are used by the
parity tests (small sizes) and by bench.py (full sizes):

  C1 english_like  4 KiB English-like ASCII (nybble codec plumbing), seed 0xC1
  C2 enwik_like    wiki/XML markup text, ~1% multi-byte UTF-8, bytes 1..255, seed 0xC2
  C3 uniform_bytes i.i.d. uniform bytes (parity variant 1..255), seed 0xC3
  C4 zipf_bytes    Zipf(s=1) over 255 ranks through a fixed permutation, seed 0xC4+rank
  C5 log_like      syslog-like lines, 7-bit ASCII, seed 0xC5

Every generator except the extension variant of C3 avoids byte 0, because the
reference's C-string API (n_ary_huffman.c:482, nybble_compression.c:909) stops
at the first NUL.
"""
from __future__ import annotations

import numpy as np

_PIECE = 32 << 20  # generate in 32 MiB pieces to bound temporary memory

_WORDS = (
    "the of and to in a is that for it as was with be by on not he i this are or "
    "his from at which but have an they you were her she there one all we their "
    "has been if more when will would who so no can had its time only new some "
    "could these two may first then do any like my now over such our man me even "
    "most made after also did many before must through back years where much your "
    "way well down should because each just those people how too little state good "
    "very make world still own see men work long get here between both life being "
    "under never day same another know while last might us great old year off come "
    "since against go came right used take three banana test this is only data "
    "compression huffman table code length symbol block stream byte text string"
).split()

_MARKUP = [
    "[[", "]]", "{{", "}}", "<page>", "</page>", "<title>", "</title>", "<text>",
    "</text>", "<id>", "</id>", "|", "=", "==", "'''", "''", "&quot;", "&amp;",
    "&lt;", "&gt;", "*", "#", "http://", "www.", ".org", ".com", "/", ":", ";",
    "(", ")", "-", "_", "Category:", "File:", "ref", "cite", "\n", "\n\n",
]

# ~1% of bytes: multi-byte UTF-8 (Latin-1 letters, dashes, CJK)
_UTF8 = ["é", "ü", "ö", "ä", "ñ", "ç", "—", "–", "’", "“", "”", "日", "本", "中", "ß", "ø"]


def _vocab_arrays(tokens, weights):
    enc = [t.encode("utf-8") if isinstance(t, str) else t for t in tokens]
    lmax = max(len(t) for t in enc)
    arr = np.zeros((len(enc), lmax), dtype=np.uint8)
    lens = np.zeros(len(enc), dtype=np.int64)
    for i, t in enumerate(enc):
        arr[i, : len(t)] = np.frombuffer(t, dtype=np.uint8)
        lens[i] = len(t)
    w = np.asarray(weights, dtype=np.float64)
    return arr, lens, w / w.sum()


def _emit_tokens(n, rng, arr, lens, p):
    """Concatenate i.i.d. tokens drawn with probabilities p until n bytes exist."""
    out = np.empty(n, dtype=np.uint8)
    filled = 0
    avg = float((lens * p).sum())
    lmax = arr.shape[1]
    col = np.arange(lmax)[None, :]
    while filled < n:
        want = min(n - filled, _PIECE)
        ntok = int(want / avg * 1.05) + 64
        ids = rng.choice(len(lens), size=ntok, p=p)
        chunk = arr[ids][col < lens[ids][:, None]]
        take = min(chunk.size, n - filled)
        out[filled : filled + take] = chunk[:take]
        filled += take
    return out


def _zipf_weights(k, s=1.0):
    return 1.0 / np.arange(1, k + 1, dtype=np.float64) ** s


def _english_vocab():
    words = [w + " " for w in _WORDS] + [w + ", " for w in _WORDS[:20]] + [
        w + ". " for w in _WORDS[:20]] + [w.capitalize() + " " for w in _WORDS[:30]] + ["\n"]
    wts = list(_zipf_weights(len(_WORDS), 0.9)) + list(_zipf_weights(20) * 0.05) + list(
        _zipf_weights(20) * 0.05) + list(_zipf_weights(30) * 0.05) + [0.02]
    return _vocab_arrays(words, wts)


def english_like(n: int, seed: int = 0xC1) -> np.ndarray:
    return _emit_tokens(n, np.random.default_rng(seed), *_english_vocab())


def _enwik_vocab():
    toks = [w + " " for w in _WORDS] + [w.capitalize() + " " for w in _WORDS[:60]]
    wts = list(_zipf_weights(len(_WORDS), 1.0)) + list(_zipf_weights(60) * 0.15)
    toks += _MARKUP
    wts += list(_zipf_weights(len(_MARKUP), 0.8) * 0.12)
    toks += [str(d) for d in range(10)] + ["19", "20", "200", "1999", "2001"]
    wts += [0.01] * 15
    toks += [u + " " for u in _UTF8] + ["caf" + _UTF8[0] + " ", "na" + _UTF8[8] + "ve "]
    wts += list(_zipf_weights(len(_UTF8), 1.0) * 0.012) + [0.002, 0.001]
    # rare ASCII punctuation so that most printable bytes appear
    rare = [chr(c) for c in range(33, 127) if chr(c) not in "".join(toks)]
    toks += rare
    wts += [2e-4] * len(rare)
    toks += ["\t"]
    wts += [1e-3]
    return _vocab_arrays(toks, wts)


def enwik_like(n: int, seed: int = 0xC2) -> np.ndarray:
    return _emit_tokens(n, np.random.default_rng(seed), *_enwik_vocab())


def uniform_bytes(n: int, seed: int = 0xC3, lo: int = 1, hi: int = 255) -> np.ndarray:
    rng = np.random.default_rng(seed)
    out = np.empty(n, dtype=np.uint8)
    for s in range(0, n, _PIECE):
        e = min(n, s + _PIECE)
        out[s:e] = rng.integers(lo, hi + 1, size=e - s, dtype=np.uint16).astype(np.uint8)
    return out


def zipf_bytes(n: int, seed: int = 0xC4, s: float = 1.0) -> np.ndarray:
    rng = np.random.default_rng(seed)
    perm = np.random.default_rng(0xC4).permutation(255).astype(np.uint8) + 1  # fixed map
    p = _zipf_weights(255, s)
    cdf = np.cumsum(p / p.sum())
    # 2^16-entry inverse-CDF lookup table: byte = lut[u16]
    lut = perm[np.minimum(np.searchsorted(cdf, (np.arange(65536) + 0.5) / 65536.0), 254)]
    out = np.empty(n, dtype=np.uint8)
    for st in range(0, n, _PIECE):
        e = min(n, st + _PIECE)
        out[st:e] = lut[rng.integers(0, 65536, size=e - st, dtype=np.uint32)]
    return out


def _log_vocab():
    toks = [w + " " for w in _WORDS]
    wts = list(_zipf_weights(len(_WORDS), 1.0))
    stamps = ["2025-08-0%dT%02d:%02d:%02dZ " % (d, h, m, s)
              for d in range(1, 4) for h in (0, 7, 13, 23) for m in (5, 31) for s in (0, 17, 42)]
    hosts = ["host%02d app[%d]: " % (h, 1000 + 37 * h) for h in range(16)]
    toks += ["\n" + t for t in stamps] + hosts + ["error ", "warn ", "info ", "debug "]
    wts += [0.6 / len(stamps)] * len(stamps) + [0.6 / len(hosts)] * len(hosts) + [0.05] * 4
    return _vocab_arrays(toks, wts)


def log_like(n: int, seed: int = 0xC5) -> np.ndarray:
    return _emit_tokens(n, np.random.default_rng(seed), *_log_vocab())


GENERATORS = {
    "C1": english_like,
    "C2": enwik_like,
    "C3": uniform_bytes,
    "C4": zipf_bytes,
    "C5": log_like,
}


_VOCAB = {"C1": _english_vocab, "C2": _enwik_vocab, "C5": _log_vocab}


def device_text(cfg: str, n: int, seed: int, device):
    """Same token vocabulary and probabilities as the numpy generator of `cfg`, sampled
    on the GPU with torch (different random stream; used for the full-size bench inputs,
    where numpy would need tens of seconds per GiB)."""
    import torch

    if cfg == "C3":
        g = torch.Generator(device=device).manual_seed(seed)
        return torch.randint(1, 256, (n,), generator=g, device=device, dtype=torch.int32).to(torch.uint8)
    if cfg == "C4":
        p = _zipf_weights(255, 1.0)
        perm = np.random.default_rng(0xC4).permutation(255).astype(np.uint8) + 1
        cdf = torch.from_numpy(np.cumsum(p / p.sum())).to(device)
        g = torch.Generator(device=device).manual_seed(seed)
        u = torch.rand(n, generator=g, device=device, dtype=torch.float64)
        idx = torch.clamp(torch.searchsorted(cdf, u), max=254)
        return torch.from_numpy(perm).to(device)[idx]
    arr, lens, p = _VOCAB[cfg]()
    tok = torch.from_numpy(arr).to(device)
    tlen = torch.from_numpy(lens).to(device)
    cdf = torch.from_numpy(np.cumsum(p)).to(device)
    g = torch.Generator(device=device).manual_seed(seed)
    avg = float((lens * p).sum())
    out = torch.empty(n, dtype=torch.uint8, device=device)
    filled = 0
    while filled < n:
        want = min(n - filled, 64 << 20)
        ntok = int(want / avg * 1.05) + 64
        u = torch.rand(ntok, generator=g, device=device, dtype=torch.float64)
        ids = torch.clamp(torch.searchsorted(cdf, u), max=len(lens) - 1)
        # the sampled tokens' bytes, concatenated: a flat gather (token of each output byte by
        # repeat_interleave, its column = position - the token's exclusive offset). The same
        # bytes as the 2-D boolean-mask index tok[ids][col < tlen[ids][:, None]] it replaces,
        # which hung when 4 processes ran it at once on one GPU (tools/synth_stall.py)
        tl = tlen[ids].to(torch.int64)
        total = int(tl.sum())
        start = torch.cumsum(tl, 0) - tl
        which = torch.repeat_interleave(torch.arange(ntok, device=device), tl, output_size=total)
        pos = torch.arange(total, device=device) - start[which]
        chunk = tok[ids[which], pos]
        take = min(chunk.numel(), n - filled)
        out[filled : filled + take] = chunk[:take]
        filled += take
    return out
