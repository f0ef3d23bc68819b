"""Cell-range sharding protocol (dss_amd/shard.py) on CPU with gloo, world 2.

What runs here is the host side of SURVEY.md s8(e): splitters, the
all-gather of a covered query batch, the pair gather, and the invariant the
whole design rests on -- with whole cell lists, the smallest-shared-cell rule
puts every (query, entity) pair on exactly one shard.  The shard-local join
is the device kernel in production (tests/test_gpu_shard.py checks it on a
GPU); here the oracle plays it, as the checker.
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
        from oracle import oracle as O
        O.build()
        _, qs, qa, it, ia, now = W.config(0, scale=0.004)
        ioffs, icells, _, _ = O.cover_batch(it.kind, it.voff, it.lat, it.lng, it.radius_m, nthreads=2)
        ranges = shard.cell_splitters(icells, world)
        # this rank covers its contiguous slice of the query batch
        n = qs.n
        lo, hi = rank * n // world, (rank + 1) * n // world
        sub = qs.subset(np.arange(lo, hi))
        qo, qcells, _, _ = O.cover_batch(sub.kind, sub.voff, sub.lat, sub.lng, sub.radius_m, nthreads=2)
        tlo, thi = W.query_bounds(qa, now)
        t = lambda a: torch.as_tensor(np.ascontiguousarray(a))  # noqa: E731
        offs, cells, attrs, base = shard.allgather_csr(t(qo), t(qcells.view(np.int64)), t(qa.alt_lo[lo:hi]),
                                                       t(qa.alt_hi[lo:hi]), t(tlo[lo:hi]), t(thi[lo:hi]))
        assert base == [r * n // world for r in range(world)]
        fo, fc, _, _ = O.cover_batch(qs.kind, qs.voff, qs.lat, qs.lng, qs.radius_m, nthreads=2)
        assert np.array_equal(offs.numpy(), fo) and np.array_equal(cells.numpy().view(np.uint64), fc)
        assert np.array_equal(attrs[2].numpy(), tlo) and np.array_equal(attrs[1].numpy(), qa.alt_hi)
        # shard-local join (oracle as the stand-in for the device kernel):
        # the pairs whose smallest shared cell lies in this rank's range
        rq, re = O.search(ioffs, icells, ia.alt_lo, ia.alt_hi, ia.t0, ia.t1, None, fo, fc, qa.alt_lo, qa.alt_hi,
                          tlo, thi)
        keep = []
        for k in range(len(rq)):
            c = _smallest_shared(fc[fo[rq[k]]:fo[rq[k] + 1]], icells[ioffs[re[k]]:ioffs[re[k] + 1]])
            keep.append(shard.owner_of(ranges, c) == rank)
        keep = np.array(keep, dtype=bool)
        gq, ge = shard.gather_pairs(t(rq[keep].astype(np.int64)), t(re[keep].astype(np.int64)))
        got = np.sort((gq.numpy() << 32) | ge.numpy())
        want = np.sort((rq.astype(np.int64) << 32) | re.astype(np.int64))
        q.put((rank, bool(np.array_equal(got, want)), int(len(got)), int(keep.sum())))
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
    assert all(ok for _, ok, _, _ in res)
    assert sum(k for _, _, _, k in res) == res[0][2]  # disjoint: every pair on exactly one rank
    assert res[0][2] > 0
