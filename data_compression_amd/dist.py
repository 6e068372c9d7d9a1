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
    bit_base: int            # global bit offset of this shard's first code bit
    bits: int                # payload bits of this shard
    sync: tuple              # (int64 group bases, int16 chunk bit lengths), absolute bits
    sync_syms: int
    n: int                   # symbols in this shard
    table: torch.Tensor      # device code table (identical on every rank)


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
        hist = self.e.hist(x, out=hist) if hist is not None else self.e.hist(x)
        if self.table_mode == "broadcast" and self.world > 1:
            self._reduce_to_src(hist)
            if self.rank == self.table_src:
                tab = self.e.table(hist, n_ary, out=table) if table is not None else self.e.table(hist, n_ary)
            else:
                tab = table if table is not None else self.e.alloc_table()
            self._broadcast_table(tab)
        else:
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
        head = bytes([8, ends[0][0]]) if self.rank == 0 else b""   # type byte, raw first byte
        body = self.e.small_body(y, self.rank > 0, nelem, head=head)
        lens = self._gather_i64([body.numel() - len(head)])
        total = 2 + sum(v[0] for v in lens)
        literal = total >= n_total
        if literal:   # ' ' + raw input, as the single-stream encoder falls back
            seg = torch.cat([torch.tensor([ord(" ")], dtype=torch.uint8, device=x.device), x]) if self.rank == 0 else x
        else:
            seg = body   # rank 0's already starts with the header
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

    def decode(self, s, out=None):
        """out: optional buffer of >= 2 * s.n bytes for the front-end inverse (the result is a
        view of it, or of the Huffman output when a later rank's segment is LITERAL)."""
        seg = self.h.decode(s)[: s.n]
        kw = {} if out is None else {"out": out}
        if self.rank == 0:
            return self.e.small_decompress(seg, **kw)
        return seg if s.literal else self.e.small_decompress_body(seg, **kw)


INITIAL_LISTS = np.frombuffer(b" etaoins" * 16, np.uint8).reshape(16, 8)   # initialize_dictionary


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

    def compress(self, x, modify: bool):
        """This rank's segment of the compressed stream, and whether it is LITERAL."""
        dev, n = x.device, x.numel()
        if n < 1 or (self.rank == 0 and n < 2):
            raise ValueError("shards need >= 1 byte (rank 0: >= 2)")
        ends = self._gather([int(x[0]), int(x[-1]), n], dev)
        n_total = sum(e[2] for e in ends)
        y = torch.cat([self._u8([ends[self.rank - 1][1]], dev), x]) if self.rank > 0 else x
        lists = None
        if modify:
            summ, cnt = self.e.nyb_mtf_summary(y)
            allsum = self._gather(list(summ.reshape(-1)) + list(cnt), dev)
            lists = INITIAL_LISTS.copy()
            for q in range(self.rank):
                a = np.asarray(allsum[q], np.uint8)
                lists = compose_lists(lists, a[:128].reshape(16, 8), a[128:])
        plan = self.e.nyb_body_plan(y, modify, lists)
        plans = self._gather(plan, dev)
        s, pend, total = 0, -1, 2
        for q in range(self.world):
            c0, c1, s0, s1, last = plans[q]
            if q == self.rank:
                my_s, my_pend = s, pend
            total += c1 if s else c0
            s = s1 if s else s0
            pend = last if s else -1
        total += s                      # odd tail: the last pending byte is written raw
        literal = total >= n_total
        if literal:
            seg = torch.cat([self._u8([ord(" ")], dev), x]) if self.rank == 0 else x
            return seg, True
        body = self.e.nyb_body_write(y, modify, my_pend if my_s else -1, self.rank == self.world - 1)
        if self.rank == 0:
            body = torch.cat([self._u8([0xAF, int(x[0])], dev), body])
        return body, False

    def decompress(self, seg):
        """Static-mode decode of this rank's segment of a compressed stream (as compress
        cut it, or cut anywhere) -> this rank's decoded bytes."""
        dev, m = seg.device, seg.numel()
        info = self._gather([m, int(seg[0]) if m else -1], dev)
        typ = info[0][1]
        if typ == ord(" "):
            return seg[1:] if self.rank == 0 else seg
        if typ != 0xAF:
            raise ValueError("not a nybble stream (type byte %r)" % typ)
        body = seg[2:] if self.rank == 0 else seg
        if self.rank == 0 and m < 2:
            raise ValueError("rank 0's segment must hold the 2-byte header")
        right = next((info[q][1] for q in range(self.rank + 1, self.world) if info[q][0] > 0), None)
        y = torch.cat([body, self._u8([right], dev)]) if right is not None else body
        mb = body.numel()
        plans = self._gather(self.e.nyb_dbody_plan(y, mb), dev)
        s = 0
        for q in range(self.rank):
            c0, c1, s0, s1 = plans[q]
            s = s1 if s else s0
        out = self.e.nyb_dbody_write(y, mb, s)
        return torch.cat([seg[1:2], out]) if self.rank == 0 else out

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
