"""Multi-GPU Huffman codec: one process per GPU, contiguous shards, one global code table.

SURVEY.md §8(e): the stream is split into contiguous shards, one per rank. The only
exchange steps are the ones the single global bitstream needs:

  1. local 256-bin histogram  -> all_reduce(SUM)           (2 KiB, RCCL over xGMI)
  2. every rank builds the same code table from the global histogram (deterministic;
     table_mode="replicate", the default), or rank table_src builds it from a reduce(SUM)
     of the histograms and broadcasts the table bytes to the others (table_mode="broadcast",
     the north star's "RCCL broadcast of the shared code table": one 2 KiB reduce and one
     table-sized broadcast instead of an all_reduce and a table build on every rank)
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

import numpy as np
import torch
import torch.distributed as dist


@dataclass
class ShardStream:
    words: torch.Tensor      # int32 words; word 0 = global stream word bit_base // 32
    bit_base: object         # global bit offset of this shard's first code bit: an int, or (an
                             # encode into preallocated buffers at world size > 1) a one-element
                             # int64 device tensor the kernels read; finalize() makes it an int
    bits: int                # payload bits of this shard (-1 until finalize())
    sync: tuple              # (int64 group bases, int16 chunk bit lengths), absolute bits
    sync_syms: int
    n: int                   # symbols in this shard
    table: torch.Tensor      # device code table (identical on every rank)
    totals: torch.Tensor = None   # the ranks' payload bits (device), when bit_base is a tensor
    total: torch.Tensor = None    # this shard's payload bits (device), as planned
    plan_gen: int = None          # the engine's plan identity (pack_status of THIS encode)
    status_ok: bool = False       # finalize() has checked this stream's pack status


class ShardedHuffman:
    def __init__(self, engine, group=None, table_mode: str = "replicate", table_src: int = 0):
        if table_mode not in ("replicate", "broadcast"):
            raise ValueError(f"table_mode must be 'replicate' or 'broadcast', not {table_mode!r}")
        self.e = engine
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        if not 0 <= table_src < self.world:
            raise ValueError(f"table_src {table_src} outside the group of {self.world} ranks")
        self.table_mode = table_mode
        self.table_src = table_src

    # ---- collectives (no-ops at world size 1) -------------------------------------------
    def _all_reduce(self, t):
        if self.world > 1:
            dist.all_reduce(t, group=self.group)

    def _src_global(self):
        return self.table_src if self.group is None else dist.get_global_rank(self.group, self.table_src)

    def _reduce_to_src(self, t):
        dist.reduce(t, dst=self._src_global(), group=self.group)

    def _broadcast_table(self, t):
        dist.broadcast(t, src=self._src_global(), group=self.group)

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
        if self.world == 1 and getattr(self.e, "fused_plan", False):   # no exchange: one fused launch
            hist, tab, total = self.e.encode_plan(x, n_ary, hist=hist, table=table, total=total)
            return tab, total, None
        hist = self.e.hist(x, out=hist) if hist is not None else self.e.hist(x)
        fused = hasattr(self.e, "table_plan")   # table + this shard's plan in one launch
        if self.table_mode == "broadcast" and self.world > 1:
            self._reduce_to_src(hist)
            if self.rank == self.table_src and fused:   # table + its own plan, one launch
                tab, total = self.e.table_plan(hist, n_ary, out=table, total=total)
                self._broadcast_table(tab)
            else:
                if self.rank == self.table_src:
                    tab = self.e.table(hist, n_ary, out=table) if table is not None else self.e.table(hist, n_ary)
                else:
                    tab = table if table is not None else self.e.alloc_table()
                self._broadcast_table(tab)
                total = self.e.plan(tab, total=total) if total is not None else self.e.plan(tab)
        else:
            self._all_reduce(hist)
            if fused:
                tab, total = self.e.table_plan(hist, n_ary, out=table, total=total)
            else:
                tab = self.e.table(hist, n_ary, out=table) if table is not None else self.e.table(hist, n_ary)
                total = self.e.plan(tab, total=total) if total is not None else self.e.plan(tab)
        totals = self._all_gather_scalar(total) if self.world > 1 else None
        return tab, total, totals

    def encode(self, x, n_ary: int = 2, sync_syms: int = 64, words=None, sync=None, hist=None, table=None,
               total=None) -> ShardStream:
        """words/sync/hist/table/total: optional preallocated buffers. With preallocated words
        and sync the encode issues no host synchronisation at any world size: the rank's bit
        offset (the exclusive prefix of the gathered bit counts) stays on the device and the
        pack kernels read it there (dc_huff_pack_async_dev)."""
        n = x.numel()
        if self.world > 1 and self.rank < self.world - 1 and n % (64 * sync_syms):
            raise ValueError("every shard but the last must hold a multiple of 64*sync_syms symbols")
        tab, tot, totals = self.plan(x, n_ary, hist, table, total)
        base, bits = 0, None
        if totals is not None:
            if words is not None and sync is not None:
                base = totals[: self.rank].sum().reshape(1)   # device int64, no host read
                bits = -1
            else:   # buffers sized here: one small host read
                tv = totals.cpu().tolist()
                base, bits = int(sum(tv[: self.rank])), int(tv[self.rank])
        if words is None:
            bits = int(tot.item()) if bits is None else bits
            words = self.e.alloc_words(base, bits)
        if sync is None:
            sync = self.e.alloc_sync(n, sync_syms)
        gen = self.e.plan_gen()   # this encode's plan: finalize() reads its own pack status
        self.e.pack_async(x, tab, base, words, sync, sync_syms)
        return ShardStream(words, base, bits if bits is not None else -1, sync, sync_syms, n, tab,
                           totals if not isinstance(base, int) else None, tot, gen)

    def finalize(self, s: ShardStream):
        """Host values of the bit offset and payload bit count (one host read) if encode()
        left them on the device, and the pack's outcome: with the offset on the device, a
        preallocated `words` too small for bit_base % 32 + bits (size it with
        words_needed(31, bits)) makes the kernels write nothing, which is raised here
        rather than gathered as an empty stream. The status and bit count are this stream's
        own (its plan's slot and total), whatever the engine encoded after it."""
        if s.totals is not None:
            tv = s.totals.cpu().tolist()
            s.bit_base, s.bits, s.totals = int(sum(tv[: self.rank])), int(tv[self.rank]), None
        elif s.bits < 0:
            s.bits = int(s.total.item()) if s.total is not None else int(self.e.plan_total())
        if not s.status_ok:
            st = self.e.pack_status(s.table, s.plan_gen)
            if st != 0:
                raise RuntimeError(f"rank {self.rank}: pack failed with status {st} (dc_huff_pack_status)")
            s.status_ok = True
        return s

    def decode(self, s: ShardStream, out=None):
        if out is None:
            out = self.e.alloc_bytes(s.n)
        self.e.decode(s.words, s.bit_base, s.sync, s.sync_syms, s.n, s.table, out)
        return out

    # ---- step 6: gather the whole stream to one rank (timed separately by bench.py) -------
    def gather(self, s: ShardStream, dst: int = 0):
        """Returns (words, bits, bases, lens) of the whole stream on rank dst, None elsewhere.
        One small all_gather of the shapes, then point-to-point sends to dst only (grouped
        send/recv): the interior words of each rank land in place in the merged
        stream; the two words a rank may share with its neighbours travel separately and are
        OR-merged."""
        self.finalize(s)
        nw = (s.bit_base % 32 + s.bits + 31) // 32 if s.bits > 0 else 0
        if self.world == 1:
            return s.words[:nw], s.bits, s.sync[0], s.sync[1]
        ng, nc = s.sync[0].numel(), s.sync[1].numel()
        meta = torch.tensor([s.bit_base, s.bits, nw, ng, nc], dtype=torch.int64, device=s.words.device)
        allm = [torch.empty_like(meta) for _ in range(self.world)]
        dist.all_gather(allm, meta, group=self.group)
        allm = [m.cpu().tolist() for m in allm]
        dst_g = dst if self.group is None else dist.get_global_rank(self.group, dst)

        def pieces(words, m):   # (head word, interior, tail word) views of a rank's words
            k = m[2]
            return (words[0:min(k, 1)], words[1:max(k - 1, 1)], words[max(k - 1, 1):k])

        if self.rank != dst:
            h, body, tl = pieces(s.words, allm[self.rank])
            lens = s.sync[1].view(torch.uint8)   # int16 travels as bytes (not every backend has it)
            ops = [dist.P2POp(dist.isend, t.contiguous(), dst_g, group=self.group)
                   for t in (h, body, tl, s.sync[0], lens) if t.numel()]
            for w in dist.batch_isend_irecv(ops) if ops else []:
                w.wait()
            return None
        dev = s.words.device
        total_bits = allm[-1][0] + allm[-1][1]
        out = torch.zeros((total_bits + 31) // 32, dtype=torch.int32, device=dev)
        bases = torch.empty(sum(m[3] for m in allm), dtype=torch.int64, device=dev)
        lens = torch.empty(sum(m[4] for m in allm), dtype=torch.int16, device=dev)
        lens8 = lens.view(torch.uint8)
        ops, edges = [], []
        g0 = c0 = 0
        for r, m in enumerate(allm):
            w0, k = m[0] // 32, m[2]
            if r == self.rank:
                h, body, tl = pieces(s.words, m)
                if body.numel():
                    out[w0 + 1: w0 + k - 1] = body
                edges.append((w0, h, w0 + k - 1, tl))
                bases[g0: g0 + m[3]] = s.sync[0]
                lens[c0: c0 + m[4]] = s.sync[1]
            else:
                e = torch.zeros(2, dtype=torch.int32, device=dev)
                h, tl = e[0:min(k, 1)], e[1:1 + max(min(k - 1, 1), 0)]
                body = out[w0 + 1: w0 + max(k - 1, 1)]
                for t in (h, body, tl, bases[g0: g0 + m[3]], lens8[2 * c0: 2 * (c0 + m[4])]):
                    if t.numel():
                        ops.append(dist.P2POp(dist.irecv, t, r if self.group is None else
                                              dist.get_global_rank(self.group, r), group=self.group))
                edges.append((w0, h, w0 + k - 1, tl))
            g0 += m[3]
            c0 += m[4]
        for w in dist.batch_isend_irecv(ops) if ops else []:
            w.wait()
        for w0, h, wl, tl in edges:   # words shared with a neighbouring rank: OR-merged
            if h.numel():
                out[w0: w0 + 1] |= h
            if tl.numel():
                out[wl: wl + 1] |= tl
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

    Fused (the default where the engine has dc_small_huff_*): at world size 1 the front-end and
    the Huffman code in one pass over x (_encode_fused). At world size > 1 the same one pass per
    shard, with no re-cut and no host read in the encode (_encode_fused_shards):
      1. all_gather of every rank's (first byte, last byte, n): the 1-byte halos, on the device
      2. the shard's histogram of M (dc_small_huff_shard_hist: the halo bytes are read by the
         kernel) -> all_reduce -> the stream's table and this shard's bits (dc_huff_table_plan)
      3. all_gather of every rank's (bits, symbols) -> this shard's global bit offset and first
         symbol index, on the device
      4. dc_small_huff_shard_pack_async: the shard's codes at that global bit, its local sync
         index (its own decode) and its part of the stream's sync index (chunks at multiples of
         S of the global symbol index; the gather adds the parts of the chunks two shards share)
    finalize() (before the decode or the gather) reads the offsets back once per step and
    agrees the fallbacks over the ranks (LITERAL output of the whole stream, a shard whose pack
    cannot run fused): then every rank re-encodes with the two stages.
    """

    def __init__(self, engine, group=None, table_mode: str = "replicate", table_src: int = 0, fused: bool = True):
        """fused: at world size 1, the one-pass encode and the counted decode (dc_small_huff_*)
        when the engine has them; False keeps the two stages (front-end, then Huffman)."""
        self.e = engine
        self.h = ShardedHuffman(engine, group, table_mode=table_mode, table_src=table_src)
        self.group = group
        self.world, self.rank = self.h.world, self.h.rank
        self.fused = fused

    def _gather_i64(self, vals):
        t = torch.tensor(vals, dtype=torch.int64, device=self._dev)
        if self.world == 1:
            return [vals]
        out = [torch.empty_like(t) for _ in range(self.world)]
        dist.all_gather(out, t, group=self.group)
        return [o.cpu().tolist() for o in out]

    @staticmethod
    def _lower(v):
        return ord("a") <= v <= ord("z")

    def frontend(self, x, sync_syms: int = 64):
        """Steps 1-4: this rank's segment of the global front-end stream (device bytes, 16-B
        aligned) and whether the stream fell back to LITERAL.
        No copy of the shard: the body kernel reads x itself (elements x[1..], x[0] its left
        context), and the two elements whose output depends on a neighbour's byte are settled
        on the host from the gathered halo bytes: x[0] (the second byte of a pair that starts
        on the previous shard's last byte, or the start of a pair with x[1]) is written as
        the body's head, and x[-1] (' ' starting a pair with the next shard's first byte)
        patches the body's last byte. The body is sized first (dc_small_compress_body_plan),
        so every rank knows the re-cut before writing: it writes its body once, at the offset
        where the bytes received from the previous rank complete an aligned segment."""
        self._dev = x.device
        n = x.numel()
        if n < 2:
            raise ValueError("each shard needs >= 2 bytes")
        x0, x1, xl = x[[0, 1, n - 1]].tolist()
        ends = self._gather_i64([x0, xl, n])
        left = ends[self.rank - 1][1] if self.rank > 0 else None
        right = ends[self.rank + 1][0] if self.rank < self.world - 1 else None
        n_total = sum(e[2] for e in ends)
        if self.rank == 0:
            head = bytes([8, x0])                       # type byte, raw first byte
        elif left == ord(" ") and self._lower(x0):
            head = b""                                  # x[0] closes the previous shard's pair
        elif x0 == ord(" ") and self._lower(x1):
            head = bytes([0x80 + x1])                   # x[0] x[1] is a pair
        else:
            head = bytes([x0])
        hb = 2 if self.rank == 0 else 0                 # header bytes (not body)
        nb = len(head) - hb + self.e.small_body_plan(x, self.rank > 0, n - 1)
        lens = self._gather_i64([nb])
        total = 2 + sum(v[0] for v in lens)
        literal = total >= n_total
        sizes = [v[0] + 2 for v in lens[:1]] + [v[0] for v in lens[1:]]
        if literal:   # ' ' + raw input, as the single-stream encoder falls back
            sizes = [e[2] + (1 if r == 0 else 0) for r, e in enumerate(ends)]
        q = 64 * sync_syms
        cut, nrecv, keep = self._cuts(sizes, q)
        m = sizes[self.rank]
        buf = self.e.alloc_bytes(nrecv + m + 16)        # [received | own segment]
        if literal:
            k = 0
            if self.rank == 0:
                buf[nrecv: nrecv + 1].fill_(ord(" "))
                k = 1
            buf[nrecv + k: nrecv + k + n] = x
        else:
            body = self.e.small_body_write(x, self.rank > 0, n - 1, buf[nrecv:], head=head)
            if right is not None and xl == ord(" ") and self._lower(right):
                body[-1:].fill_(0x80 + right)           # x[-1] starts a pair with the next shard
        return self._exchange(buf, nrecv, m, keep), literal

    def _cuts(self, sizes, q):
        """Re-cut of the segments (sizes, in rank order) at multiples of q (global position):
        each rank's bytes past the next multiple of q move to the next rank, so every segment
        but the last starts and ends on a multiple of q. Returns (cuts, bytes this rank
        receives, bytes it keeps of its own)."""
        off = [sum(sizes[:r]) for r in range(self.world + 1)]
        cut = [0] + [(off[r] // q) * q for r in range(1, self.world)] + [off[self.world]]
        if any(cut[r] < off[r - 1] for r in range(1, self.world)):
            raise ValueError("front-end segments too short to re-cut at 64 * sync_syms")
        r = self.rank
        keep = cut[r + 1] - off[r] if r < self.world - 1 else sizes[r]
        return cut, off[r] - cut[r], keep

    def _exchange(self, buf, nrecv, m, keep):
        """buf = [nrecv bytes to receive | own segment of m bytes]: send own bytes past `keep`
        to the next rank, receive the previous rank's into the front (in place, no copy).
        Returns the re-cut segment buf[: nrecv + keep]."""
        r = self.rank
        if self.world > 1:   # < q bytes to the next rank
            self._shift(buf[nrecv + keep: nrecv + m] if r < self.world - 1 else None,
                        buf[:nrecv] if r > 0 else None)
        return buf[: nrecv + keep]

    def _shift(self, send, recv):
        """send (or None) to rank + 1 and recv (or None) from rank - 1, grouped."""
        ops = []
        if send is not None and send.numel():
            ops.append(dist.P2POp(dist.isend, send, self.rank + 1, group=self.group))
        if recv is not None and recv.numel():
            ops.append(dist.P2POp(dist.irecv, recv, self.rank - 1, group=self.group))
        for w in dist.batch_isend_irecv(ops) if ops else []:
            w.wait()

    def encode(self, x, n_ary: int = 16, sync_syms: int = 64, words=None, sync=None, table=None, total=None,
               gsync=None):
        """words/sync/table/total (gsync: world > 1): optional caller-owned buffers for the fused
        path (the stream points into them, so a caller that keeps several streams passes
        distinct ones; without them every encode allocates its own)."""
        if self.fused and self.world == 1 and hasattr(self.e, "small_huff_plan") and x.numel() >= 2:
            s = self._encode_fused(x, n_ary, sync_syms, words, sync, table, total)
            if s is not None:
                return s
        if self.fused and self.world > 1 and hasattr(self.e, "small_shard_hist"):
            return self._encode_fused_shards(x, n_ary, sync_syms, words, sync, gsync, table, total)
        return self._encode_two_stage(x, n_ary, sync_syms)

    def _encode_two_stage(self, x, n_ary, sync_syms):
        seg, literal = self.frontend(x, sync_syms)
        s = self.h.encode(seg, n_ary=n_ary, sync_syms=sync_syms)
        s.literal = literal
        return s

    def _encode_fused(self, x, n_ary, S, words=None, sync=None, table=None, total=None):
        """World size 1: the front-end and the Huffman code in one pass over x, the front-end
        output never written (dc_small_huff_plan + dc_small_huff_pack_async): the stream equals
        frontend() + ShardedHuffman.encode() bit for bit. None when the fused path does not
        apply (LITERAL output, every byte value present, DC_E_FALLBACK): the caller runs the
        two stages. Only the histogram (scratch the stream does not keep) is reused across
        calls; the words, sync index, table and total belong to the returned stream."""
        from ._lib import DcError
        n = x.numel()
        hist = getattr(self, "_fhist", None)
        if hist is None:
            hist = self._fhist = self.e._t(256, torch.int64)
        tab = table if table is not None else self.e.alloc_table()
        tot = total if total is not None else self.e._t(1, torch.int64)
        if sync is None:
            sync = self.e.alloc_sync(n + 1, S)
        try:
            _, tab, tot = self.e.small_huff_plan(x, n_ary, hist=hist, table=tab, total=tot)
        except DcError as err:
            if err.rc != -8:
                raise
            return None
        bits = int(tot.item())
        need = self.e.words_needed(0, bits)
        if words is None or words.numel() < need:
            words = self.e._t(need + need // 16, torch.int32)
        buf = {"words": words, "sync": sync}
        gen = self.e.plan_gen()
        self.e.small_huff_pack_async(x, tab, 0, buf["words"], buf["sync"], S)
        st = self.e.pack_status(tab, gen)
        if st == -8:
            return None
        if st != 0:
            raise RuntimeError(f"dc_small_huff_pack_async failed with status {st}")
        m = self.e.small_huff_symbols()
        ng, nch = self.e.sync_sizes(m, S)   # the index of m symbols (the buffers hold n + 1)
        sync = (buf["sync"][0][: max(ng, 1)], buf["sync"][1][: max(nch, 1)])
        s = ShardStream(buf["words"], 0, bits, sync, S, m, tab, None, tot, gen)
        s.literal = False
        s.fused = True
        return s

    # ---- fused encode of a shard (world > 1) -----------------------------------------------
    def _all_gather_dev(self, t):   # every rank's t, stacked (device, no host read)
        out = torch.empty(self.world * t.numel(), dtype=t.dtype, device=t.device)
        dist.all_gather_into_tensor(out, t.reshape(-1).contiguous(), group=self.group)
        return out.view((self.world,) + tuple(t.shape))

    def _all_reduce_dev(self, t, op=dist.ReduceOp.SUM):
        dist.all_reduce(t, op=op, group=self.group)

    def _encode_fused_shards(self, x, n_ary, S, words=None, sync=None, gsync=None, table=None, total=None):
        n = x.numel()
        if n < 2:
            raise ValueError("each shard needs >= 2 bytes")
        if x.data_ptr() % 16:
            # the fused kernels read the shard as 16-B granules (dc_small_huff_shard_hist returns
            # DC_E_ARG otherwise); an aligned copy keeps this rank in step with the others'
            # collectives below, where a raise here would leave them waiting in the all_reduce
            x = x.clone()
        dev, r, e = x.device, self.rank, self.e
        # 1. halos: every rank's first and last byte and size, gathered on the device
        ends = self._all_gather_dev(torch.stack([x[0].to(torch.int64), x[n - 1].to(torch.int64),
                                                 torch.tensor(n, dtype=torch.int64, device=dev)]))
        neg = torch.full((), -1, dtype=torch.int64, device=dev)
        shard = torch.stack([neg, neg, ends[r - 1, 1] if r > 0 else neg,
                             ends[r + 1, 0] if r < self.world - 1 else neg]).contiguous()
        # 2. the shard's histogram of M, the stream's table, this shard's bits under it
        hist = e.small_shard_hist(x, shard)
        hg = hist.clone()
        self._all_reduce_dev(hg)
        if self.h.table_mode == "broadcast":
            tab = table if table is not None else e.alloc_table()
            if r == self.h.table_src:
                tab = e.table(hg, n_ary, out=tab) if table is not None else e.table(hg, n_ary)
            self.h._broadcast_table(tab)
            tot = e.plan(tab, total=total) if total is not None else e.plan(tab)
        else:
            tab, tot = e.table_plan(hg, n_ary, out=table, total=total)
        # 3. every shard's (bits, symbols): this shard's global bit and first symbol
        m = hist.sum()
        bm = self._all_gather_dev(torch.stack([tot.reshape(()).to(torch.int64), m]))
        shard[0] = bm[:r, 0].sum()
        shard[1] = bm[:r, 1].sum()
        literal = bm[:, 1].sum() >= ends[:, 2].sum()   # the whole stream's LITERAL test
        # 4. the pack; buffers: the words sized here need the bits (one host read)
        if words is None:
            words = e.alloc_words(0, int(tot.item()) + 32)
        if sync is None:
            sync = e.alloc_sync(n + 1, S)
        if gsync is None:
            gsync = e.alloc_sync(n + 1 + 2 * S, S)
        gen = e.plan_gen()
        e.small_shard_pack_async(x, tab, shard, words, sync, gsync, S)
        s = ShardStream(words, shard[0:1], -1, sync, S, -1, tab, None, tot, gen)
        s.literal = False
        s.fused = True
        s.shard_fused = {"x": x, "n_ary": n_ary, "shard": shard, "m": m, "gsync": gsync, "literal": literal}
        return s

    def finalize(self, s):
        """The host values of a fused shard stream (one read of 4 device scalars) and the
        fallbacks agreed over the ranks: a LITERAL stream or a shard whose fused pack did not
        run (DC_E_FALLBACK) makes every rank re-encode with the two stages."""
        fs = getattr(s, "shard_fused", None)
        if fs is None or fs.get("done"):
            return s
        st = self.e.pack_status(s.table, s.plan_gen)
        v = torch.stack([fs["shard"][0], fs["shard"][1], s.total.reshape(()).to(torch.int64), fs["m"],
                         fs["literal"].to(torch.int64)]).cpu().tolist()
        flags = torch.tensor([1 if (st == -8 or v[4]) else 0, 1 if st not in (0, -8) else 0], dtype=torch.int64,
                             device=fs["shard"].device)
        self._all_reduce_dev(flags, dist.ReduceOp.MAX)
        fb, bad = flags.tolist()
        if bad:
            raise RuntimeError(f"rank {self.rank}: fused shard pack failed with status {st} (a rank's plan/pack)")
        if fb:   # every rank: the two stages
            t = self._encode_two_stage(fs["x"], fs["n_ary"], s.sync_syms)
            self.h.finalize(t)
            s.__dict__.update(t.__dict__)
            s.shard_fused = None
            s.fused = False
            return s
        s.bit_base, s.bits, s.n, s.totals = int(v[0]), int(v[2]), int(v[3]), None
        ng, nch = self.e.sync_sizes(s.n, s.sync_syms)
        s.sync = (s.sync[0][: max(ng, 1)], s.sync[1][: max(nch, 1)])
        fs["M"] = int(v[1])
        fs["done"] = True
        return s

    def gather(self, s, dst: int = 0):
        """The whole stream on rank dst (ShardedHuffman.gather's words), with, for a fused shard
        stream, the stream's sync index assembled from the shards' parts: the chunks two shards
        share are the sums of their parts, each group base comes from the shard it starts in."""
        self.finalize(s)
        fs = getattr(s, "shard_fused", None)
        if fs is None:
            return self.h.gather(s, dst)
        dev = s.words.device
        # (this stream's own plan generation and total: finalize() above already checked its
        # pack status, and the words gather must not read a later plan's on this context)
        empty = ShardStream(s.words, s.bit_base, s.bits, (torch.empty(0, dtype=torch.int64, device=dev),
                                                          torch.empty(0, dtype=torch.int16, device=dev)),
                            s.sync_syms, s.n, s.table, None, s.total, s.plan_gen, True)
        g = self.h.gather(empty, dst)
        S = s.sync_syms
        M, mm = fs["M"], s.n
        c0 = M // S
        c0e = c0 & ~1
        nl = (M + mm - 1) // S - c0 + 1 if mm else 0
        g0, g1 = -(-M // (64 * S)), -(-(M + mm) // (64 * S))
        gl = fs["gsync"][1][c0 - c0e: c0 - c0e + nl]
        gb = fs["gsync"][0][: g1 - g0]
        meta = self._all_gather_dev(torch.tensor([c0, nl, g0, g1 - g0], dtype=torch.int64, device=dev))
        metas = meta.cpu().tolist()
        dst_g = dst if self.group is None else dist.get_global_rank(self.group, dst)
        if self.rank != dst:
            ops = [dist.P2POp(dist.isend, t.contiguous(), dst_g, group=self.group)
                   for t in (gl.view(torch.uint8), gb) if t.numel()]
            for w in dist.batch_isend_irecv(ops) if ops else []:
                w.wait()
            return None
        nchunk = max(mt[0] + mt[1] for mt in metas)
        ngroup = (nchunk + 63) // 64
        lens32 = torch.zeros(nchunk, dtype=torch.int32, device=dev)
        bases = torch.empty(ngroup, dtype=torch.int64, device=dev)
        parts, ops = [], []
        for q, (qc0, qnl, qg0, qng) in enumerate(metas):
            if q == self.rank:
                parts.append((qc0, gl.clone()))
                bases[qg0: qg0 + qng] = gb
                continue
            src = q if self.group is None else dist.get_global_rank(self.group, q)
            t = torch.empty(qnl, dtype=torch.int16, device=dev)
            if qnl:
                ops.append(dist.P2POp(dist.irecv, t.view(torch.uint8), src, group=self.group))
            if qng:
                ops.append(dist.P2POp(dist.irecv, bases[qg0: qg0 + qng], src, group=self.group))
            parts.append((qc0, t))
        for w in dist.batch_isend_irecv(ops) if ops else []:
            w.wait()
        for qc0, t in parts:
            lens32[qc0: qc0 + t.numel()] += t.to(torch.int32) & 0xFFFF
        return g[0], g[1], bases, (lens32 - ((lens32 >= 32768).to(torch.int32) << 16)).to(torch.int16)   # u16 bits

    def decode(self, s, out=None):
        """out: optional buffer of >= 2 * s.n bytes for the front-end inverse (the result is a
        view of it, or of the Huffman output when a later rank's segment is LITERAL)."""
        self.finalize(s)
        kw = {} if out is None else {"out": out}
        if (self.fused and self.world == 1 and not s.literal and hasattr(self.e, "small_huff_decode")
                and isinstance(s.bit_base, int)):
            # world 1: the decoder counts the pair symbols per group, and the front-end inverse
            # takes those counts (dc_small_huff_decode: no counting pass over the decoded stream)
            enc = {"words": s.words, "bit_base": s.bit_base, "sync": s.sync, "S": s.sync_syms, "n": s.n,
                   "table": s.table}
            mb = getattr(self, "_mbuf", None)
            if mb is None or mb.numel() < s.n + 16:
                mb = self._mbuf = self.e.alloc_bytes(s.n + 16)
            return self.e.small_huff_decode(enc, mbuf=mb, **kw)
        seg = self.h.decode(s)[: s.n]
        if self.rank == 0:
            return self.e.small_decompress(seg, **kw)
        return seg if s.literal else self.e.small_decompress_body(seg, **kw)


INITIAL_LISTS = np.frombuffer(b" etaoins" * 16, np.uint8).reshape(16, 8)   # initialize_dictionary


def compose_summaries(la, ca, lb, cb):
    """Summary of (stretch A then stretch B) from theirs (each started empty): per context,
    first 8 distinct of (B's list, A's list)."""
    out = np.zeros((16, 8), np.uint8)
    cnt = np.zeros(16, np.uint8)
    for c in range(16):
        seen = []
        for v in list(lb[c][: int(cb[c])]) + list(la[c][: int(ca[c])]):
            if v not in seen:
                seen.append(v)
            if len(seen) == 8:
                break
        out[c, : len(seen)] = seen
        cnt[c] = len(seen)
    return out, cnt


def compose_lists(lists, summ, cnt):
    """Move-to-front lists after a shard whose summary (started empty) is (summ, cnt):
    first 8 distinct of (summary list, lists) per context (update_context,
    nybble_compression.c:665-687). Host side of the adaptive shard exchange."""
    out = np.empty_like(lists)
    for c in range(16):
        seen = []
        for v in list(summ[c][: int(cnt[c])]) + list(lists[c]):
            if v not in seen:
                seen.append(v)
            if len(seen) == 8:
                break
        out[c] = seen
    return out


class ShardedNybble:
    """nybble_compression.c's compress_bytestring / decompress_bytestring, sharded.

    SURVEY.md §8(e): "Nybble static: shards need a 1-byte halo (x[start-1] for the seed and
    context) and the carried run parity of the previous shard's trailing hit-run"; "Nybble
    adaptive: encode can be sharded with a halo of context history; decode: replicas only".
    Encode (both modes), per rank:
      1. all_gather of (first byte, last byte, n): the 1-byte left halo and the stream size
      2. adaptive only: the rank's move-to-front summary (dc_nyb_mtf_summary, 144 B) is
         all-gathered and each rank composes its entry lists from the initial " etaoins"
         lists and the summaries of the ranks before it
      3. the rank's transducer plan (dc_nyb_body_plan: bytes out and exit state from either
         entry state, the rank of its last element) is all-gathered; each rank derives its
         entry state (is a hit nybble pending, and that byte's rank) and the stream total
      4. LITERAL fallback (output >= input, :1018-1037) decided over the whole stream
      5. each rank writes its body (dc_nyb_body_write); rank 0 prefixes 0xAF, x[0]
    The ranks' segments concatenate to the single-stream compress_bytestring output.
    Decode (static): the compressed stream is cut anywhere; each rank's segment needs one
    byte of right halo and the entry state "start at the low nybble", found the same way
    (dc_nyb_dbody_plan, all_gather, dc_nyb_dbody_write). The decoded segments concatenate
    to the input. Adaptive decode is sequential by definition (each byte's list depends on
    every byte before it): decode_replica gathers the stream and decodes it whole.
    """

    def __init__(self, engine, group=None, table_mode: str = "replicate", table_src: int = 0):
        if table_mode not in ("replicate", "broadcast"):
            raise ValueError(f"table_mode must be 'replicate' or 'broadcast', not {table_mode!r}")
        self.e = engine
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        if not 0 <= table_src < self.world:
            raise ValueError(f"table_src {table_src} outside the group of {self.world} ranks")
        self.table_mode = table_mode
        self.table_src = table_src

    def _gather(self, vals, dev):
        if self.world == 1:
            return [list(vals)]
        t = torch.tensor(vals, dtype=torch.int64, device=dev)
        out = [torch.empty_like(t) for _ in range(self.world)]
        dist.all_gather(out, t, group=self.group)
        return [o.cpu().tolist() for o in out]

    def _u8(self, vals, dev):
        return torch.tensor(vals, dtype=torch.uint8, device=dev)

    _STATIC = b" etaoins"

    @staticmethod
    def _fsm_elem(hit):
        """(c0, c1, s0, s1) of one element (dc_core.hip elem_fsm, M_NYB_ENC): a hit flips
        the pending state and emits 1 byte when it closes a pair; a miss emits itself (and a
        pending byte raw before it)."""
        return (0, 1, 1, 0) if hit else (1, 2, 0, 0)

    @staticmethod
    def _then(a, b):
        """Composition of transducer plans (a then b), as fsm_then."""
        c0 = a[0] + (b[1] if a[2] else b[0])
        s0 = b[3] if a[2] else b[2]
        c1 = a[1] + (b[1] if a[3] else b[0])
        s1 = b[3] if a[3] else b[2]
        return (c0, c1, s0, s1)

    def compress(self, x, modify: bool):
        """This rank's segment of the compressed stream, and whether it is LITERAL.
        No copy of the shard: the kernels walk x itself (elements x[1..], context x[0]); the
        element x[0], whose context is the previous shard's last byte (the 1-byte halo), is
        coded on the host (its rank from the entry lists, its transducer step) and its
        output written as the body's head."""
        dev, n = x.device, x.numel()
        if n < 1 or (self.rank == 0 and n < 2):
            raise ValueError("shards need >= 1 byte (rank 0: >= 2)")
        x0, xl = x[[0, n - 1]].tolist()
        ends = self._gather([x0, xl, n], dev)
        n_total = sum(e[2] for e in ends)
        r = self.rank
        left = ends[r - 1][1] if r > 0 else None
        lists = None
        if modify:
            summ, cnt = self.e.nyb_mtf_summary(x)   # elements x[1..] from empty lists
            if r > 0:   # x[0] touched into its context's list first: summary = (x0) then (x[1..])
                first = np.zeros((16, 8), np.uint8)
                fcnt = np.zeros(16, np.uint8)
                first[(left >> 3) & 15, 0] = x0
                fcnt[(left >> 3) & 15] = 1
                summ, cnt = compose_summaries(first, fcnt, summ, cnt)
            allsum = self._gather(list(summ.reshape(-1)) + list(cnt), dev)
            lists = INITIAL_LISTS.copy()
            for q in range(r):
                a = np.asarray(allsum[q], np.uint8)
                lists = compose_lists(lists, a[:128].reshape(16, 8), a[128:])
        r0 = 0xFF
        if r > 0:   # x[0]: its rank under the entry lists, then touched
            if modify:
                c = (left >> 3) & 15
                row = list(lists[c])
                r0 = row.index(x0) if x0 in row else 0xFF
                lists[c] = [x0] + [v for v in row if v != x0][:7]
            else:
                r0 = self._STATIC.index(bytes([x0])) if bytes([x0]) in self._STATIC else 0xFF
        plan = self.e.nyb_body_plan(x, modify, lists)   # (c0, c1, s0, s1, last rank) of x[1..]
        if r > 0:
            comp = self._then(self._fsm_elem(r0 != 0xFF), tuple(plan[:4]))
            plan = list(comp) + [plan[4] if n > 1 else r0]
        plans = self._gather(plan, dev)
        s, pend, total = 0, -1, 2
        for q in range(self.world):
            c0, c1, s0, s1, last = plans[q]
            if q == r:
                my_s, my_pend = s, pend
            total += c1 if s else c0
            s = s1 if s else s0
            pend = last if s else -1
        total += s                      # odd tail: the last pending byte is written raw
        literal = total >= n_total
        if literal:
            seg = torch.cat([self._u8([ord(" ")], dev), x]) if r == 0 else x
            return seg, True
        is_last = r == self.world - 1
        if r == 0:
            head, s_in, p_in = bytes([0xAF, x0]), 0, -1
        else:   # x[0]'s output from the entry state (compress_byte_index, :819-884)
            s_in, p_in = my_s, my_pend if my_s else -1
            if r0 != 0xFF:
                if s_in:
                    head, s_in, p_in = bytes([((8 | p_in) << 4) | (8 | r0)]), 0, -1
                else:
                    head, s_in, p_in = b"", 1, r0
            else:
                head = bytes([left, x0]) if s_in else bytes([x0])
                s_in, p_in = 0, -1
        if n == 1:   # x[0] alone: its head, and on the last shard a pending byte written raw
            tail = bytes([x0]) if is_last and s_in else b""
            return self._u8(list(head + tail), dev), False
        body = self.e.nyb_body_write(x, modify, p_in if s_in else -1, is_last, head=head)
        return body, False

    def decompress(self, seg):
        """Static-mode decode of this rank's segment of a compressed stream (as compress
        cut it, or cut anywhere) -> this rank's decoded bytes. No copy of the segment: the
        one byte of right halo (the next segment's first byte) only completes this segment's
        last output byte when the walk ends "at the low nybble" (it supplies that byte's low
        half), which is patched after the body is written."""
        dev, m = seg.device, seg.numel()
        b0, b1 = (seg[[0, 1]].tolist() if m > 1 else ([int(seg[0]), -1] if m else [-1, -1]))
        info = self._gather([m, b0, b1], dev)
        typ = info[0][1]
        if typ == ord(" "):
            return seg[1:] if self.rank == 0 else seg
        if typ != 0xAF:
            raise ValueError("not a nybble stream (type byte %r)" % typ)
        if self.rank == 0 and m < 2:
            raise ValueError("rank 0's segment must hold the 2-byte header")
        body = seg[2:] if self.rank == 0 else seg
        right = next((info[q][1] for q in range(self.rank + 1, self.world) if info[q][0] > 0), None)
        mb = body.numel()
        plans = self._gather(self.e.nyb_dbody_plan(body, mb), dev)
        s = 0
        for q in range(self.rank):
            c0, c1, s0, s1 = plans[q]
            s = s1 if s else s0
        head = bytes([info[0][2]]) if self.rank == 0 else b""   # the raw first byte
        out = self.e.nyb_dbody_write(body, mb, s, head=head)
        s_out = plans[self.rank][3] if s else plans[self.rank][2]
        if right is not None and s_out == 1 and mb:
            out[-1:].add_(right >> 4)   # (l & 7) << 4 + the next byte's high nybble (:753-795)
        return out

    def decode_replica(self, seg, sizes, modify: bool):
        """Adaptive (or any) decode by replicas: every rank gathers the whole stream, decodes
        it, and keeps its own byte range (sizes = the ranks' input sizes)."""
        dev, m = seg.device, seg.numel()
        ms = [v[0] for v in self._gather([m], dev)]
        if self.world > 1:
            buf = torch.zeros(max(ms), dtype=torch.uint8, device=dev)
            buf[:m] = seg
            parts = [torch.empty_like(buf) for _ in range(self.world)]
            dist.all_gather(parts, buf, group=self.group)
            whole = torch.cat([p[:k] for p, k in zip(parts, ms)])
        else:
            whole = seg
        out = self.e.nyb_decompress(whole, modify)
        a = sum(sizes[: self.rank])
        return out[a: a + sizes[self.rank]]

    # ---- independent-chunk framing (DCNK): the adaptive decode that shards -------------------
    def compress_chunked(self, x, modify: bool, chunk: int = 1 << 16):
        """This rank's DCNK container (no exchange: chunks are independent). With every shard
        but the last a multiple of `chunk` bytes, merge_chunked of the ranks' containers is
        byte-identical to the single-GPU container of the whole input."""
        return self.e.nyb_compress_chunked(x, modify, chunk)

    def decompress_chunked(self, comp):
        return self.e.nyb_decompress_chunked(comp)


def merge_chunked(containers):
    """Concatenate per-rank DCNK containers (host bytes, in rank order) into one."""
    import struct
    heads = [struct.unpack_from("<IIIIQQ", c) for c in containers]
    magic, ver, mod, K = heads[0][:4]
    offs, pays, base = [], [], 0
    for c, h in zip(containers, heads):
        assert h[:4] == (magic, ver, mod, K), "containers differ in format"
        nch = h[5]
        o = np.frombuffer(c, np.uint64, nch + 1, 32)
        offs.append(o[:-1] + np.uint64(base))
        pays.append(c[32 + 8 * (nch + 1): 32 + 8 * (nch + 1) + int(o[-1])])
        base += int(o[-1])
    n = sum(h[4] for h in heads)
    nch = sum(h[5] for h in heads)
    head = struct.pack("<IIIIQQ", magic, ver, mod, K, n, nch)
    return head + np.concatenate(offs + [np.array([base], np.uint64)]).astype(np.uint64).tobytes() + b"".join(pays)
