"""Cell-range sharding protocol on CPU with gloo, world 2.

What runs here is the protocol the product ships (include/dssgpu.h, routing
section; dssg_sharded_search_device): each rank routes its covered queries
into fused [rows | cells] segments, one all-to-all delivers them, the shard
unpacks and joins them, its own queries' pairs stay home and the others' go
back in a second all-to-all.  The device kernels are restated in numpy by
oracle/route_oracle.py and the shard join is the oracle's search filtered to
the pairs whose smallest shared cell lies in the rank's range -- the checker
standing in for route.hip and k_join (tests/test_gpu_shard.py runs the real
kernels against it).  Plus the invariant the design rests on: with whole cell
lists, the smallest-shared-cell rule puts every (query, entity) pair on
exactly one shard.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from dss_amd import shard, workload as W


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_splitters_partition_and_balance():
    rng = np.random.default_rng(0)
    cells = (rng.integers(0, 1000, 20000).astype(np.uint64) << np.uint64(40)) | np.uint64(1 << 34)
    for parts in (1, 2, 3, 8):
        r = shard.cell_splitters(cells, parts)
        assert len(r) == parts and r[0][0] == 0 and r[-1][1] == 2**64 - 1
        assert all(r[k][1] + 1 == r[k + 1][0] for k in range(parts - 1))
        own = np.array([shard.owner_of(r, int(c)) for c in np.unique(cells)])
        _, cnt = np.unique(cells, return_counts=True)
        load = np.bincount(own, weights=cnt, minlength=parts)
        assert load.max() <= len(cells) / parts + cnt.max()  # quantile cuts: off by at most one cell


def test_splitters_hot_cell_and_few_cells():
    cells = np.array([7] * 100 + [9, 11], dtype=np.uint64)
    r = shard.cell_splitters(cells, 4)
    assert len(r) == 4 and r[-1][1] == 2**64 - 1
    assert sum(1 for lo, hi in r if lo <= 7 <= hi) == 1
    assert shard.cell_splitters(np.zeros(0, np.uint64), 3)[-1][1] == 2**64 - 1


def _smallest_shared(qc, ec):
    s = np.intersect1d(qc, ec)
    return int(s[0]) if len(s) else None


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oracle import oracle as O, route_oracle as R
        O.build()
        _, qs, qa, it, ia, now = W.config(0, scale=0.03)
        ioffs, icells, _, _ = O.cover_batch(it.kind, it.voff, it.lat, it.lng, it.radius_m, nthreads=2)
        ranges = shard.cell_splitters(icells, world)
        part_hi = shard.part_his(ranges)
        tlo_all, thi_all = W.query_bounds(qa, now)
        # this rank covers its contiguous slice of the query batch
        n = qs.n
        lo, hi = rank * n // world, (rank + 1) * n // world
        sub = qs.subset(np.arange(lo, hi))
        qo, qcells, _, _ = O.cover_batch(sub.kind, sub.voff, sub.lat, sub.lng, sub.radius_m, nthreads=2)
        alo, ahi, tlo, thi = qa.alt_lo[lo:hi], qa.alt_hi[lo:hi], tlo_all[lo:hi], thi_all[lo:hi]
        # (1) route: fused segments + counts
        send, rows_n, cells_n, seg = R.route(qo, qcells, alo, ahi, tlo, thi, part_hi)
        assert seg == [32 * r + 32 * ((c + 3) // 4) for r, c in zip(rows_n, cells_n)]
        mine = torch.tensor(rows_n + cells_n, dtype=torch.int64)
        allc = [torch.zeros_like(mine) for _ in range(world)]
        dist.all_gather(allc, mine)
        src_rows = [int(allc[p][rank]) for p in range(world)]
        src_cells = [int(allc[p][world + rank]) for p in range(world)]
        # (2) one all-to-all of the segments
        rseg = [R.segment_bytes(r, c) for r, c in zip(src_rows, src_cells)]
        recv = torch.empty(sum(rseg), dtype=torch.uint8)
        dist.all_to_all_single(recv, torch.from_numpy(send), rseg, seg)
        # (3) unpack + shard join (oracle as the stand-in for k_join): the
        # pairs whose smallest shared cell lies in this rank's range
        b = R.unpack(recv.numpy(), src_rows, src_cells)
        assert len(b["qid"]) == sum(src_rows) and b["offs"][-1] == sum(src_cells)
        rq, re = O.search(ioffs, icells, ia.alt_lo, ia.alt_hi, ia.t0, ia.t1, None, b["offs"], b["cells"], b["alo"],
                          b["ahi"], b["tlo"], b["thi"])
        keep = np.array([shard.owner_of(ranges, _smallest_shared(b["cells"][b["offs"][rq[k]]:b["offs"][rq[k] + 1]],
                                                                icells[ioffs[re[k]]:ioffs[re[k] + 1]])) == rank
                         for k in range(len(rq))], dtype=bool)
        rq, re = rq[keep], re[keep]
        # (4) pairs home: own ones kept, the others all-to-all'd back
        oq, oe, packed, pcounts = R.route_pairs(b, rq, re, world, rank)
        sc = [0 if d == rank else int(pcounts[d]) for d in range(world)]
        pcs = torch.tensor([int(x) for x in pcounts], dtype=torch.int64)
        allp = [torch.zeros_like(pcs) for _ in range(world)]
        dist.all_gather(allp, pcs)
        rc = [0 if p == rank else int(allp[p][rank]) for p in range(world)]
        got_p = torch.empty(sum(rc), dtype=torch.int64)
        dist.all_to_all_single(got_p, torch.from_numpy(packed.view(np.int64)), rc, sc)
        gq, ge = R.unpack_pairs(got_p.numpy().view(np.uint64))
        got = np.sort((np.concatenate([oq, gq]).astype(np.uint64) << np.uint64(32)) |
                      np.concatenate([oe, ge]).astype(np.uint64))
        fq, fe = O.search(ioffs, icells, ia.alt_lo, ia.alt_hi, ia.t0, ia.t1, None, qo, qcells, alo, ahi, tlo, thi)
        want = np.sort((fq.astype(np.uint64) << np.uint64(32)) | fe.astype(np.uint64))
        q.put((rank, bool(np.array_equal(got, want)), int(len(want)), int(len(rq)), int(len(oq)), sum(rows_n)))
    finally:
        dist.destroy_process_group()


def test_sharded_protocol_gloo_world2():
    world = 2
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=300)
    res = sorted(q.get(timeout=5) for _ in range(world))
    assert all(p.exitcode == 0 for p in procs)
    assert all(ok for _, ok, _, _, _, _ in res), res
    # every pair computed on exactly one shard: the shards' pairs add up to
    # the pairs delivered home
    assert sum(r[3] for r in res) == sum(r[2] for r in res) > 0
    # both paths carried pairs: some stayed home, some crossed
    assert 0 < sum(r[4] for r in res) < sum(r[2] for r in res)
    assert all(r[5] > 0 for r in res)
