"""Multi-GPU Huffman codec: one process per GPU, contiguous shards, one global code table.

SURVEY.md §8(e): the stream is split into contiguous shards, one per rank. The only
exchange steps are the ones the single global bitstream needs:

  1. local 256-bin histogram  -> all_reduce(SUM)           (2 KiB, RCCL over xGMI)
  2. every rank builds the same code table from the global histogram (deterministic)
  3. local payload bit count  -> all_gather                 (8 B per rank)
     rank r's stream starts at bit_base_r = sum of the bit counts of ranks < r
  4. each rank packs its shard at bit_base_r: the shard boundaries fall inside 32-bit
     words, whose halves are OR-merged when the payloads are gathered
  5. decode is local: every rank decodes its own shard from its own words
  6. (optional, timed separately) gather of the variable-size payloads to one rank

The result is bit-identical to the single-GPU stream of the concatenated input, at any
rank count, as long as every shard except the last holds a multiple of
64 * sync_syms symbols (so no sync group straddles two ranks).

The per-rank work is done by an *engine* with the interface of device.Codec
(hist/table/plan/pack_async/decode/...). The product engine is device.Codec (HIP kernels,
RCCL through torch.distributed "nccl"); the gloo tests plug in a CPU engine built on the
oracle, so the orchestration code tested on CPU is the code that runs on the GPUs.
"""
from __future__ import annotations

from dataclasses import dataclass

import torch
import torch.distributed as dist


@dataclass
class ShardStream:
    words: torch.Tensor      # int32 words; word 0 = global stream word bit_base // 32
    bit_base: int            # global bit offset of this shard's first code bit
    bits: int                # payload bits of this shard
    sync: tuple              # (int64 group bases, int16 chunk bit lengths), absolute bits
    sync_syms: int
    n: int                   # symbols in this shard
    table: torch.Tensor      # device code table (identical on every rank)


class ShardedHuffman:
    def __init__(self, engine, group=None):
        self.e = engine
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0

    # ---- collectives (no-ops at world size 1) -------------------------------------------
    def _all_reduce(self, t):
        if self.world > 1:
            dist.all_reduce(t, group=self.group)

    def _all_gather_scalar(self, t):
        if self.world == 1:
            return t.reshape(1)
        out = torch.empty(self.world, dtype=t.dtype, device=t.device)
        dist.all_gather_into_tensor(out, t.reshape(1), group=self.group)
        return out

    # ---- codec ----------------------------------------------------------------------------
    def plan(self, x, n_ary: int, hist=None, table=None, total=None):
        """Steps 1-3: global table and this rank's payload bit count (device tensors), and
        the gathered per-rank bit counts (device tensor; None at world size 1)."""
        hist = self.e.hist(x, out=hist) if hist is not None else self.e.hist(x)
        self._all_reduce(hist)
        tab = self.e.table(hist, n_ary, out=table) if table is not None else self.e.table(hist, n_ary)
        total = self.e.plan(tab, total=total) if total is not None else self.e.plan(tab)
        totals = self._all_gather_scalar(total) if self.world > 1 else None
        return tab, total, totals

    def encode(self, x, n_ary: int = 2, sync_syms: int = 64, words=None, sync=None, hist=None, table=None,
               total=None) -> ShardStream:
        """words/sync/hist/table/total: optional preallocated buffers. At world size 1 with
        preallocated words the encode issues no host synchronisation."""
        n = x.numel()
        if self.world > 1 and self.rank < self.world - 1 and n % (64 * sync_syms):
            raise ValueError("every shard but the last must hold a multiple of 64*sync_syms symbols")
        tab, tot, totals = self.plan(x, n_ary, hist, table, total)
        base, bits = 0, None
        if totals is not None:   # the rank's global bit offset: one small host read
            tv = totals.cpu().tolist()
            base, bits = int(sum(tv[: self.rank])), int(tv[self.rank])
        if words is None:
            bits = int(tot.item()) if bits is None else bits
            words = self.e.alloc_words(base, bits)
        if sync is None:
            sync = self.e.alloc_sync(n, sync_syms)
        self.e.pack_async(x, tab, base, words, sync, sync_syms)
        return ShardStream(words, base, bits if bits is not None else -1, sync, sync_syms, n, tab)

    def finalize(self, s: ShardStream):
        """Fill in the payload bit count (host read) if encode() skipped it."""
        if s.bits < 0:
            s.bits = int(self.e.plan_total())
        return s

    def decode(self, s: ShardStream, out=None):
        if out is None:
            out = self.e.alloc_bytes(s.n)
        self.e.decode(s.words, s.bit_base, s.sync, s.sync_syms, s.n, s.table, out)
        return out

    # ---- step 6: gather the whole stream to one rank (timed separately by bench.py) -------
    def gather(self, s: ShardStream, dst: int = 0):
        """Returns (words, bits, bases, lens) of the whole stream on rank dst, None elsewhere.
        Boundary words shared by two ranks are OR-merged."""
        nw = (s.bit_base % 32 + s.bits + 31) // 32
        meta = torch.tensor([s.bit_base, s.bits, nw, s.sync[0].numel(), s.sync[1].numel()],
                            dtype=torch.int64, device=s.words.device)
        if self.world == 1:
            return s.words[:nw], s.bits, s.sync[0], s.sync[1]
        allm = [torch.empty_like(meta) for _ in range(self.world)]
        dist.all_gather(allm, meta, group=self.group)
        allm = [m.cpu().tolist() for m in allm]
        mw = max(m[2] for m in allm)
        mg = max(m[3] for m in allm)
        mc = max(m[4] for m in allm)
        dev = s.words.device
        wpad = torch.zeros(mw, dtype=torch.int32, device=dev)
        wpad[:nw] = s.words[:nw]
        gpad = torch.zeros(mg, dtype=torch.int64, device=dev)
        gpad[: s.sync[0].numel()] = s.sync[0]
        cpad = torch.zeros(mc, dtype=torch.int32, device=dev)   # int16 is not a gloo dtype
        cpad[: s.sync[1].numel()] = s.sync[1].to(torch.int32) & 0xFFFF
        W = [torch.empty_like(wpad) for _ in range(self.world)]
        Gs = [torch.empty_like(gpad) for _ in range(self.world)]
        Cs = [torch.empty_like(cpad) for _ in range(self.world)]
        dist.all_gather(W, wpad, group=self.group)
        dist.all_gather(Gs, gpad, group=self.group)
        dist.all_gather(Cs, cpad, group=self.group)
        if self.rank != dst:
            return None
        total_bits = allm[-1][0] + allm[-1][1]
        out = torch.zeros((total_bits + 31) // 32, dtype=torch.int32, device=dev)
        for r, m in enumerate(allm):
            w0 = m[0] // 32
            k = min(m[2], out.numel() - w0)
            out[w0: w0 + k] |= W[r][:k]
        bases = torch.cat([Gs[r][: allm[r][3]] for r in range(self.world)])
        lens = torch.cat([Cs[r][: allm[r][4]] for r in range(self.world)]).to(torch.int16)
        return out, total_bits, bases, lens


class ShardedSmall:
    """C5 (BASELINE configs[4]): small_compression.c front-end + n-ary Huffman, sharded.

    SURVEY.md §8(e) "Small front-end: pairs never overlap (' ' is never the second byte of
    a pair), so the only halo is one byte at the shard start" (and one at its end, for a
    pair that starts on a shard's last byte). Steps:
      1. all_gather of every rank's (first byte, last byte): the 1-byte halos
      2. each rank's front-end body (dc_small_compress_body); rank 0 prefixes the header
         (type byte 8, raw first byte, small_compression.c:582-665)
      3. all_gather of the body lengths: the LITERAL fallback (output >= input, :655-662)
         is decided over the whole stream, as the single-stream encoder decides it
      4. the front-end stream is re-cut at multiples of 64 * sync_syms (each rank sends its
         < 64 * sync_syms tail bytes to the next rank: one point-to-point exchange), so the
         Huffman stage (ShardedHuffman) sees the layout it needs
      5. ShardedHuffman encodes the front-end stream: bit-identical to the single-GPU
         encoding of the whole front-end output
    Decode: Huffman decode of the rank's segment, then the front-end inverse (per byte,
    stateless); the ranks' decoded segments concatenate to the input.
    """

    def __init__(self, engine, group=None):
        self.e = engine
        self.h = ShardedHuffman(engine, group)
        self.group = group
        self.world, self.rank = self.h.world, self.h.rank

    def _gather_i64(self, vals):
        t = torch.tensor(vals, dtype=torch.int64, device=self._dev)
        if self.world == 1:
            return [vals]
        out = [torch.empty_like(t) for _ in range(self.world)]
        dist.all_gather(out, t, group=self.group)
        return [o.cpu().tolist() for o in out]

    def frontend(self, x, sync_syms: int = 64):
        """Steps 1-4: this rank's segment of the global front-end stream (device bytes),
        its global start, and whether the stream fell back to LITERAL."""
        self._dev = x.device
        n = x.numel()
        if n < 2:
            raise ValueError("each shard needs >= 2 bytes")
        ends = self._gather_i64([int(x[0]), int(x[-1]), n])
        left = ends[self.rank - 1][1] if self.rank > 0 else None
        right = ends[self.rank + 1][0] if self.rank < self.world - 1 else None
        n_total = sum(e[2] for e in ends)
        parts = ([torch.tensor([left], dtype=torch.uint8, device=x.device)] if left is not None else []) + [x] + \
                ([torch.tensor([right], dtype=torch.uint8, device=x.device)] if right is not None else [])
        y = torch.cat(parts) if len(parts) > 1 else x
        # body of stream bytes: rank 0 -> x[1..n-1] (x[0] is the raw first byte); rank r ->
        # all of x (y[0] is the left halo)
        nelem = n - 1 if self.rank == 0 else n
        body = self.e.small_body(y, self.rank > 0, nelem)
        lens = self._gather_i64([body.numel()])
        total = 2 + sum(v[0] for v in lens)
        literal = total >= n_total
        if literal:   # ' ' + raw input, as the single-stream encoder falls back
            seg = torch.cat([torch.tensor([ord(" ")], dtype=torch.uint8, device=x.device), x]) if self.rank == 0 else x
        else:
            seg = torch.cat([torch.tensor([8, int(x[0])], dtype=torch.uint8, device=x.device), body]) \
                if self.rank == 0 else body
        sizes = [v[0] for v in self._gather_i64([seg.numel()])]
        return self._recut(seg, sizes, 64 * sync_syms), literal

    def _recut(self, seg, sizes, q):
        """Move each rank's bytes past the next multiple of q (global position) to the next
        rank, so every segment but the last starts and ends on a multiple of q."""
        off = [sum(sizes[:r]) for r in range(self.world + 1)]
        cut = [0] + [(off[r] // q) * q for r in range(1, self.world)] + [off[self.world]]
        if any(cut[r] < off[r - 1] for r in range(1, self.world)):
            raise ValueError("front-end segments too short to re-cut at 64 * sync_syms")
        r = self.rank
        send = seg[cut[r + 1] - off[r]:] if r < self.world - 1 else seg[:0]
        keep = seg[: cut[r + 1] - off[r]] if r < self.world - 1 else seg
        recv = torch.empty(off[r] - cut[r], dtype=torch.uint8, device=seg.device)
        if self.world > 1:   # < q bytes to the next rank (gloo: even ranks send first)
            ops = []
            if r < self.world - 1 and send.numel():
                ops.append(dist.P2POp(dist.isend, send.contiguous(), r + 1, group=self.group))
            if r > 0 and recv.numel():
                ops.append(dist.P2POp(dist.irecv, recv, r - 1, group=self.group))
            if ops:
                for w in dist.batch_isend_irecv(ops):
                    w.wait()
        return torch.cat([recv, keep]) if recv.numel() else keep

    def encode(self, x, n_ary: int = 16, sync_syms: int = 64):
        seg, literal = self.frontend(x, sync_syms)
        s = self.h.encode(seg, n_ary=n_ary, sync_syms=sync_syms)
        s.literal = literal
        return s

    def decode(self, s):
        seg = self.h.decode(s)[: s.n]
        if self.rank == 0:
            return self.e.small_decompress(seg)
        return seg if s.literal else self.e.small_decompress_body(seg)
