"""Cell-range sharding of the entity index across the GPUs of one node.

SURVEY.md s8(e): the reference's postings table `scd_cells_operations` is
range-partitioned by `cell_id` inside CockroachDB
(pkg/scd/store/cockroach/store.go:140-147).  Here the same partition is an
explicit one-process-per-GPU layout:

  * `cell_splitters` cuts the uint64 cell-id space into `parts` contiguous
    ranges at posting-count quantiles (hot cells never straddle two ranks, so
    a skewed airspace still balances by postings, not by id span);
  * rank r builds `dssg_index_build_range` over its range: postings only for
    its cells, every entity's cell list whole;
  * `ShardedSearch` (the device path, one process per GPU): each rank covers
    its own query batch; `dssg_route_plan/fill_device` packs, per query, one
    row + its whole cell list for every shard owning one of its cells; an
    all-to-all (RCCL over xGMI) delivers them; the shard unpacks them
    (`dssg_unpack_queries_device`) and joins them against its cell-range
    index with the single-GPU join kernel; `dssg_route_pairs_*` sends every
    pair back to its query's home rank (second all-to-all).  Because the
    smallest-shared-cell rule sees whole cell lists on both sides, every
    (query, entity) pair is emitted by exactly one shard -- no cross-shard
    dedupe.  xGMI is point-to-point, so the exchange is a direct all-to-all
    (one peer per link), never a ring of the whole batch.
  * `allgather_csr` / `gather_pairs`: the simpler broadcast-style exchange
    (every rank sees the whole batch), kept for the CPU protocol test.

Only the exchange steps are collectives; every byte they move is packed and
unpacked by HIP kernels behind the C ABI.  torch.distributed is plumbing: the
process group and the collectives over caller-owned device tensors.
"""
from __future__ import annotations

import ctypes as C
from typing import List, Sequence, Tuple

import numpy as np

U64_MAX = 2**64 - 1


QUAD_SPAN = 1 << 37  # ids under one level-12 cell (a quad of the index): [k * 2^37, (k + 1) * 2^37)


def quad_end(c: int) -> int:
    """The last id of the quad (level-12 cell) span holding id c."""
    return int(c) | (QUAD_SPAN - 1)


def cell_splitters(cells: np.ndarray, parts: int) -> List[Tuple[int, int]]:
    """Inclusive uint64 ranges [lo, hi], in order, partitioning the whole id
    space into `parts`; each cut falls at the end of the quad (level-12 cell:
    the index keeps one posting per (entity, quad), so a shard holds whole
    quads, dssg_index_build_range) holding the distinct cell where the running
    posting count reaches r/parts of the total (a hot cell is never split).
    Parts beyond the number of distinct quads hold no cell."""
    if parts < 1:
        raise ValueError("parts must be >= 1")
    cells = np.asarray(cells, dtype=np.uint64)
    his: List[int] = []
    if len(cells):
        u, cnt = np.unique(cells, return_counts=True)
        cum = np.cumsum(cnt)
        total = int(cum[-1])
        for r in range(1, parts):
            k = int(np.searchsorted(cum, total * r / parts, side="left"))
            his.append(int(u[min(k, len(u) - 1)]))
    else:
        his = [0] * (parts - 1)
    ranges, lo, prev = [], 0, -1
    for hi in his:
        room = (parts - len(ranges) - 1) * QUAD_SPAN  # a quad span for each part still to come
        hi = min(quad_end(max(hi, prev + 1)), U64_MAX - room)  # strictly increasing, quad-aligned
        ranges.append((lo, hi))
        lo, prev = hi + 1, hi
    ranges.append((lo, U64_MAX))
    return ranges


def owner_of(ranges: Sequence[Tuple[int, int]], cell: int) -> int:
    """Rank whose range holds `cell` (the first one, for degenerate tails)."""
    for r, (lo, hi) in enumerate(ranges):
        if lo <= cell <= hi:
            return r
    raise ValueError("cell outside every range")


# ------------------------------------------------------------- collectives
def _dist():
    import torch.distributed as dist  # plumbing only
    return dist


def allgather_csr(offs, cells, *attrs, group=None):
    """All-gather a CSR batch (offs[n+1] int64, cells[C] int64 bit patterns of
    the uint64 ids, per-row attribute tensors).  Returns the concatenated
    batch in rank order plus the row offset of every rank."""
    import torch
    dist = _dist()
    world = dist.get_world_size(group)
    dev = cells.device
    n = offs.numel() - 1
    sizes = torch.tensor([n, cells.numel()], dtype=torch.int64, device=dev)
    all_sizes = [torch.empty_like(sizes) for _ in range(world)]
    dist.all_gather(all_sizes, sizes, group=group)
    all_sizes = [tuple(int(v) for v in s.tolist()) for s in all_sizes]
    max_n = max(s[0] for s in all_sizes)
    max_c = max(s[1] for s in all_sizes)

    def gather_padded(t, length, maxlen):
        buf = torch.zeros((maxlen,) + tuple(t.shape[1:]), dtype=t.dtype, device=dev)
        buf[:length] = t[:length]
        outs = [torch.empty_like(buf) for _ in range(world)]
        dist.all_gather(outs, buf, group=group)
        return outs

    counts = offs[1:] - offs[:-1]
    g_counts = gather_padded(counts, n, max(max_n, 1))
    g_cells = gather_padded(cells, cells.numel(), max(max_c, 1))
    g_attrs = [gather_padded(a, n, max(max_n, 1)) for a in attrs]
    cnt = torch.cat([g_counts[r][: all_sizes[r][0]] for r in range(world)])
    out_offs = torch.zeros(cnt.numel() + 1, dtype=torch.int64, device=dev)
    out_offs[1:] = torch.cumsum(cnt, 0)
    out_cells = torch.cat([g_cells[r][: all_sizes[r][1]] for r in range(world)])
    out_attrs = [torch.cat([ga[r][: all_sizes[r][0]] for r in range(world)]) for ga in g_attrs]
    row_base = np.concatenate([[0], np.cumsum([s[0] for s in all_sizes])])[:-1].tolist()
    return out_offs, out_cells, out_attrs, row_base


def gather_pairs(q, e, group=None):
    """All-gather every rank's (query, entity) pair set (uint32 ids carried
    in int64 tensors).  Returns the concatenation in rank order."""
    import torch
    dist = _dist()
    world = dist.get_world_size(group)
    dev = q.device
    n = torch.tensor([q.numel()], dtype=torch.int64, device=dev)
    ns = [torch.empty_like(n) for _ in range(world)]
    dist.all_gather(ns, n, group=group)
    ns = [int(x.item()) for x in ns]
    m = max(max(ns), 1)
    pk = torch.zeros(m, dtype=torch.int64, device=dev)
    pk[: q.numel()] = (q.to(torch.int64) << 32) | e.to(torch.int64)
    outs = [torch.empty_like(pk) for _ in range(world)]
    dist.all_gather(outs, pk, group=group)
    allp = torch.cat([outs[r][: ns[r]] for r in range(world)])
    return allp >> 32, allp & 0xFFFFFFFF


# ------------------------------------------------------- device sharded path
def part_his(ranges: Sequence[Tuple[int, int]]) -> np.ndarray:
    """Inclusive upper bounds of the parts (dssg_route_plan_device's
    part_hi), uint64, the last one UINT64_MAX."""
    his = np.array([hi for _, hi in ranges], dtype=np.uint64)
    if len(his) == 0 or int(his[-1]) != U64_MAX:
        raise ValueError("ranges must end at UINT64_MAX")
    return his


def all_to_all(send, send_counts: Sequence[int], group=None, stage_host: bool = False):
    """All-to-all of a part-major 1-D tensor (send_counts[d] elements for rank
    d).  Returns (received tensor, source-major; per-source counts).  Counts
    travel first (one all-to-all of world int64s).  stage_host: bounce
    through host memory (gloo)."""
    import torch
    dist = _dist()
    dev = send.device
    cdev = "cpu" if stage_host else dev
    sc = torch.tensor(list(send_counts), dtype=torch.int64, device=cdev)
    rc = torch.empty_like(sc)
    dist.all_to_all_single(rc, sc, group=group)
    recv_counts = [int(x) for x in rc.tolist()]
    src = send.cpu() if stage_host else send
    out = torch.empty(sum(recv_counts), dtype=send.dtype, device=cdev)
    dist.all_to_all_single(out, src, recv_counts, [int(x) for x in send_counts], group=group)
    return (out.to(dev) if stage_host else out), recv_counts


class ShardedSearch:
    """One rank of the cell-range sharded 4D search.

    `index` is this rank's dssg_index_build_range[_device] shard over
    `ranges[rank]`; `step` takes this rank's covered query batch (device CSR
    + attributes, tlo already max(start, now)) and returns, on the same rank,
    the (query, entity) pairs of its own queries as one int64 tensor packed
    (query << 32 | entity) -- exactly the pair set a single-GPU search of the
    batch against the whole index returns."""

    def __init__(self, ctx, index, ranges, group=None, stage_host: bool = False):
        import torch
        from . import device as D
        dist = _dist()
        self.ctx, self.index, self.group = ctx, index, group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        if len(ranges) != self.world:
            raise ValueError("one cell range per rank")
        self.stage_host = stage_host
        self.dev = torch.device("cuda", torch.cuda.current_device())
        self.part_hi = torch.as_tensor(part_his(ranges).view(np.int64), device=self.dev)
        self._D = D
        self.times = {}

    def _mark(self, name, t0, sync):
        import time
        import torch
        if sync:
            torch.cuda.synchronize()
            t = time.perf_counter()
            self.times[name] = self.times.get(name, 0.0) + (t - t0)
            return t
        return t0

    def step(self, offs_ptr, cells_ptr, nq, alo, ahi, tlo, thi, timed: bool = False):
        """The routing protocol of dssgpu.h (the one dssg_sharded_search_device
        runs), with torch.distributed doing the two all-to-alls: fused
        [rows | cells] query segments out, pairs home.  Returns this rank's
        pairs packed (query << 32 | entity) as one int64 tensor."""
        import time
        import torch
        from . import _lib
        D, ctx, L = self._D, self.ctx, self.ctx.L
        W, me = self.world, self.rank
        st = D._stream_ptr()
        t = time.perf_counter()
        if timed:
            torch.cuda.synchronize()
            t = time.perf_counter()
        # (1) route this rank's queries to the shards owning their cells: one
        # fused segment per shard
        rc = (C.c_int64 * _lib.MAX_PARTS)()
        cc = (C.c_int64 * _lib.MAX_PARTS)()
        sb = (C.c_int64 * _lib.MAX_PARTS)()
        ctx.check(L.dssg_route_plan_device(ctx.h, nq, C.c_void_p(offs_ptr), C.c_void_p(cells_ptr), W,
                                           D._ptr(self.part_hi), st, rc, cc, sb))
        seg_words = [sb[d] // 8 for d in range(W)]
        send = torch.empty(sum(seg_words) + 4, dtype=torch.int64, device=self.dev)
        ctx.check(L.dssg_route_fill_device(ctx.h, nq, C.c_void_p(offs_ptr), C.c_void_p(cells_ptr), D._ptr(alo),
                                           D._ptr(ahi), D._ptr(tlo), D._ptr(thi), st, D._ptr(send)))
        # counts travel with a small all-gather (rows, cells per destination)
        mine = torch.tensor([rc[d] for d in range(W)] + [cc[d] for d in range(W)], dtype=torch.int64,
                            device="cpu" if self.stage_host else self.dev)
        allc = [torch.zeros_like(mine) for _ in range(W)]
        _dist().all_gather(allc, mine, group=self.group)
        allc = [x.cpu() for x in allc]
        src_rows = [int(allc[p][me]) for p in range(W)]
        src_cells = [int(allc[p][W + me]) for p in range(W)]
        t = self._mark("route", t, timed)
        # (2) one exchange of the fused segments (all-to-all over xGMI)
        recv, _ = all_to_all(send[:sum(seg_words)], seg_words, self.group, self.stage_host)
        t = self._mark("exchange_queries", t, timed)
        # (3) unpack + join against this rank's shard
        batch = _lib.Batch()
        recv = recv if recv.numel() else torch.empty(4, dtype=torch.int64, device=self.dev)
        ctx.check(L.dssg_unpack_queries_device(ctx.h, D._ptr(recv), W, (C.c_int64 * _lib.MAX_PARTS)(*src_rows),
                                               (C.c_int64 * _lib.MAX_PARTS)(*src_cells), st, C.byref(batch)))
        pairs = _lib.Pairs()
        ctx.check(L.dssg_search_device(ctx.h, self.index, batch.n, C.c_void_p(batch.offs), C.c_void_p(batch.cells),
                                       C.c_void_p(batch.alt_lo), C.c_void_p(batch.alt_hi), C.c_void_p(batch.tlo),
                                       C.c_void_p(batch.thi), C.c_void_p(0), st, C.byref(pairs)))
        t = self._mark("join", t, timed)
        if timed:  # roofline accounting: postings of the distinct cells this shard was asked for
            tch = C.c_int64()
            ctx.check(L.dssg_search_touched_device(ctx.h, self.index, batch.n, C.c_void_p(batch.offs),
                                                   C.c_void_p(batch.cells), st, C.byref(tch)))
            self.last_touched = int(tch.value)
            t = time.perf_counter()
        # (4) pairs home: this rank's own straight to its output, the others'
        # packed and all-to-all'd back
        pc = (C.c_int64 * _lib.MAX_PARTS)()
        ctx.check(L.dssg_route_pairs_plan_device(ctx.h, C.byref(batch), C.byref(pairs), W, me, st, pc))
        pn = [pc[d] for d in range(W)]
        send_pairs = torch.empty(sum(pn) - pn[me] + 1, dtype=torch.int64, device=self.dev)
        self_q = torch.empty(pn[me] + 1, dtype=torch.int32, device=self.dev)
        self_e = torch.empty(pn[me] + 1, dtype=torch.int32, device=self.dev)
        ctx.check(L.dssg_route_pairs_fill_device(ctx.h, C.byref(batch), C.byref(pairs), st, D._ptr(send_pairs),
                                                 D._ptr(self_q), D._ptr(self_e)))
        t = self._mark("route_pairs", t, timed)
        got, _ = all_to_all(send_pairs[:-1], [0 if d == me else pn[d] for d in range(W)], self.group,
                            self.stage_host)
        own = (self_q[:pn[me]].to(torch.int64) << 32) | (self_e[:pn[me]].to(torch.int64) & 0xFFFFFFFF)
        out = torch.cat([own, got])
        self._mark("exchange_pairs", t, timed)
        self.last_bytes = {"query_bytes_sent": 8 * (sum(seg_words) - seg_words[me]),
                           "query_bytes_recv": 8 * (int(recv.numel()) - seg_words[me]) if sum(src_rows) else 0,
                           "pair_bytes_sent": 8 * (sum(pn) - pn[me]), "pair_bytes_recv": 8 * int(got.numel())}
        self.last_rows = int(batch.n)
        self.last_recv_cells = recv[:0]
        self.last_recv_ncells = sum(src_cells)
        self.last_shard_pairs = int(pairs.n)
        return out


class NativeComm:
    """A dssg_comm: the library's own RCCL communicator (no torch in the
    exchange).  `unique_id()` on one rank, shared out of band, then
    `NativeComm(ctx, nranks, rank, uid)` on every rank."""

    def __init__(self, ctx, nranks: int, rank: int, uid: bytes):
        from . import _lib
        if len(uid) != _lib.COMM_ID_BYTES:
            raise ValueError("a dssg_comm id is %d bytes" % _lib.COMM_ID_BYTES)
        self.ctx = ctx
        self.nranks, self.rank = nranks, rank
        buf = (C.c_uint8 * len(uid)).from_buffer_copy(uid)
        h = C.c_void_p()
        ctx.check(ctx.L.dssg_comm_init(ctx.h, nranks, rank, buf, C.byref(h)))
        self.h = h

    @staticmethod
    def unique_id(ctx) -> bytes:
        from . import _lib
        buf = (C.c_uint8 * _lib.COMM_ID_BYTES)()
        ctx.check(ctx.L.dssg_comm_unique_id(buf))
        return bytes(buf)

    def close(self):
        if getattr(self, "h", None):
            self.ctx.L.dssg_comm_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class NativeShardedSearch:
    """`ShardedSearch` with the whole step in the library
    (dssg_sharded_search_device: route, RCCL all-to-alls, shard join, pairs
    home).  step() returns this rank's (query, entity) pairs as device
    pointers (a _lib.Pairs, valid until the next step).

    With `xcomm` (a second NativeComm) and `xstream` (a torch stream) the
    step is dssg_sharded_search_async_device: the pairs' trip home runs on
    xstream over xcomm, overlapping the next step's routing and join; the
    returned pairs are complete once xstream's queued work has run and stay
    valid until the second next step.  Every collective of a rank must be
    issued by one host thread (dssgpu.h)."""

    def __init__(self, ctx, comm: NativeComm, index, ranges: Sequence[Tuple[int, int]], xcomm: NativeComm = None,
                 xstream=None):
        import torch
        if len(ranges) != comm.nranks:
            raise ValueError("one cell range per rank")
        if (xcomm is None) != (xstream is None):
            raise ValueError("xcomm and xstream go together")
        self.ctx, self.comm, self.index = ctx, comm, index
        self.xcomm, self.xstream = xcomm, xstream
        self.part_hi = torch.as_tensor(part_his(ranges).view(np.int64),
                                       device=torch.device("cuda", torch.cuda.current_device()))

    def step(self, offs_ptr, cells_ptr, nq, alo, ahi, tlo, thi):
        from . import _lib, device as D
        ctx = self.ctx
        out = _lib.Pairs()
        args = (D._ptr(self.part_hi), nq, C.c_void_p(offs_ptr), C.c_void_p(cells_ptr), D._ptr(alo), D._ptr(ahi),
                D._ptr(tlo), D._ptr(thi), D._stream_ptr())
        if self.xcomm is None:
            ctx.check(ctx.L.dssg_sharded_search_device(ctx.h, self.comm.h, self.index, *args, C.byref(out)))
        else:
            ctx.check(ctx.L.dssg_sharded_search_async_device(ctx.h, self.comm.h, self.xcomm.h, self.index, *args,
                                                             C.c_void_p(self.xstream.cuda_stream), C.byref(out)))
        return out

    def stats(self):
        """dssg_sharded_stats of the most recent step on this context: phase
        ms (route, exchange_queries, join, route_pairs, exchange_pairs; timing
        on) and the bytes / rows / pairs it moved."""
        ms = (C.c_double * 5)()
        cnt = (C.c_int64 * 8)()
        self.ctx.check(self.ctx.L.dssg_sharded_stats(self.ctx.h, ms, cnt))
        names = ["route", "exchange_queries", "join", "route_pairs", "exchange_pairs"]
        keys = ["query_bytes_sent", "query_bytes_recv", "pair_bytes_sent", "pair_bytes_recv", "rows", "shard_pairs",
                "cells", "touched"]
        return dict(zip(names, list(ms))), dict(zip(keys, [int(v) for v in cnt]))

    def close(self):
        self.comm.close()
        if self.xcomm is not None:
            self.xcomm.close()
