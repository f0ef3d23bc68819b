"""GPU: cell-range sharded search == the single-index search.

Two levels:
  * one process, N simulated shards: route (HIP) -> per-shard unpack + join
    against a dssg_index_build_range shard -> pairs routed home; the union is
    the full pair set and the shards' pair sets are disjoint;
  * two processes on the one GPU, gloo collectives (the exchange is staged
    through host memory; RCCL replaces gloo on a multi-GPU node): the full
    `ShardedSearch.step` protocol, checked against the CPU oracle.
"""
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _keys(q, e):
    return np.sort((np.asarray(q, np.uint64) << np.uint64(32)) | np.asarray(e, np.uint64))


def _covered(scale, cfg=0):
    from dss_amd import geo, workload as W
    _, q, qa, it, ia, now = W.config(cfg, scale=scale)
    ci = geo.cover_batch(it.kind, it.voff, it.lat, it.lng, it.radius_m)
    cq = geo.cover_batch(q.kind, q.voff, q.lat, q.lng, q.radius_m)
    tlo, thi = W.query_bounds(qa, now)
    return ci, cq, qa, ia, tlo, thi


# configs[0] (compact footprints) and configs[4] (corridors: long x long pairs
# meet on several shards and must still come back exactly once)
@pytest.mark.parametrize("cfg,scale,nparts", [(0, 0.05, 1), (0, 0.05, 3), (0, 0.05, 8), (4, 0.0004, 3), (4, 0.0004, 8)])
def test_routed_shards_equal_full_search(cfg, scale, nparts):
    import ctypes as C
    import torch
    from dss_amd import _lib, device as D, shard
    from dss_amd.store import EntityIndex
    ci, cq, qa, ia, tlo, thi = _covered(scale, cfg)
    full = EntityIndex(ci.offs, ci.cells, ia.alt_lo, ia.alt_hi, ia.t0, ia.t1)
    fq, fe = full.search_batch(cq.offs, cq.cells, qa.alt_lo, qa.alt_hi, tlo, thi)
    assert len(fq) > 0
    ranges = shard.cell_splitters(ci.cells, nparts)
    ctx = _lib.context()
    L = ctx.L
    dev = "cuda"
    t = lambda a: torch.as_tensor(np.ascontiguousarray(a), device=dev)  # noqa: E731
    offs, cells = t(cq.offs), t(cq.cells.view(np.int64))
    alo, ahi, dtlo, dthi = t(qa.alt_lo), t(qa.alt_hi), t(tlo), t(thi)
    part_hi = t(shard.part_his(ranges).view(np.int64))
    st = D._stream_ptr()
    nq = len(cq.offs) - 1
    rc = (C.c_int64 * _lib.MAX_PARTS)()
    cc = (C.c_int64 * _lib.MAX_PARTS)()
    sb = (C.c_int64 * _lib.MAX_PARTS)()
    ctx.check(L.dssg_route_plan_device(ctx.h, nq, D._ptr(offs), D._ptr(cells), nparts, D._ptr(part_hi), st, rc, cc,
                                       sb))
    rows_n, cells_n, seg = [rc[d] for d in range(nparts)], [cc[d] for d in range(nparts)], [sb[d] for d in range(nparts)]
    # every query goes to exactly the parts owning one of its cells
    want_rows = [0] * nparts
    for q in range(nq):
        for d in {shard.owner_of(ranges, int(c)) for c in cq.cells[cq.offs[q]:cq.offs[q + 1]]}:
            want_rows[d] += 1
    assert rows_n == want_rows
    assert seg == [32 * r + 32 * ((c + 3) // 4) for r, c in zip(rows_n, cells_n)]  # the fused layout of dssgpu.h
    send = torch.empty(sum(seg) // 8 + 4, dtype=torch.int64, device=dev)
    ctx.check(L.dssg_route_fill_device(ctx.h, nq, D._ptr(offs), D._ptr(cells), D._ptr(alo), D._ptr(ahi), D._ptr(dtlo),
                                       D._ptr(dthi), st, D._ptr(send)))
    got, per_part = [], []
    w0 = 0
    for d in range(nparts):
        idx = EntityIndex(ci.offs, ci.cells, ia.alt_lo, ia.alt_hi, ia.t0, ia.t1, cell_range=ranges[d])
        seg_d = send[w0: w0 + seg[d] // 8].clone()  # part d's segment, as the exchange delivers it
        w0 += seg[d] // 8
        if rows_n[d] == 0:
            per_part.append(0)
            continue
        batch = _lib.Batch()
        ctx.check(L.dssg_unpack_queries_device(ctx.h, D._ptr(seg_d), 1, (C.c_int64 * _lib.MAX_PARTS)(rows_n[d]),
                                               (C.c_int64 * _lib.MAX_PARTS)(cells_n[d]), st, C.byref(batch)))
        # the received rows carry the home batch's cell lists and attributes
        ro = D.copy_back(ctx, batch.offs, rows_n[d] + 1, np.int64)
        rq = D.copy_back(ctx, batch.qid, rows_n[d], np.uint32)
        rcl = D.copy_back(ctx, batch.cells, int(ro[-1]), np.uint64)
        assert int(ro[-1]) == cells_n[d]
        for k in range(0, rows_n[d], max(1, rows_n[d] // 50)):
            q = int(rq[k])
            assert np.array_equal(rcl[ro[k]:ro[k + 1]], cq.cells[cq.offs[q]:cq.offs[q + 1]])
        pairs = _lib.Pairs()
        ctx.check(L.dssg_search_device(ctx.h, idx.h, batch.n, C.c_void_p(batch.offs), C.c_void_p(batch.cells),
                                       C.c_void_p(batch.alt_lo), C.c_void_p(batch.alt_hi), C.c_void_p(batch.tlo),
                                       C.c_void_p(batch.thi), C.c_void_p(0), st, C.byref(pairs)))
        # pairs home, both ways: home part 0 as this rank's own (straight to
        # the output arrays) and as another rank's (packed for the exchange)
        pc = (C.c_int64 * _lib.MAX_PARTS)()
        ctx.check(L.dssg_route_pairs_plan_device(ctx.h, C.byref(batch), C.byref(pairs), 2, 0, st, pc))
        assert pc[0] == pairs.n and pc[1] == 0
        sq = torch.empty(pairs.n + 1, dtype=torch.int32, device=dev)
        se = torch.empty(pairs.n + 1, dtype=torch.int32, device=dev)
        ctx.check(L.dssg_route_pairs_fill_device(ctx.h, C.byref(batch), C.byref(pairs), st, C.c_void_p(0), D._ptr(sq),
                                                 D._ptr(se)))
        own = _keys(sq[: pairs.n].cpu().numpy().view(np.uint32), se[: pairs.n].cpu().numpy().view(np.uint32))
        ctx.check(L.dssg_route_pairs_plan_device(ctx.h, C.byref(batch), C.byref(pairs), 2, 1, st, pc))
        outp = torch.empty(pairs.n + 1, dtype=torch.int64, device=dev)
        ctx.check(L.dssg_route_pairs_fill_device(ctx.h, C.byref(batch), C.byref(pairs), st, D._ptr(outp),
                                                 C.c_void_p(0), C.c_void_p(0)))
        uq = torch.empty(pairs.n + 1, dtype=torch.int32, device=dev)
        ue = torch.empty(pairs.n + 1, dtype=torch.int32, device=dev)
        ctx.check(L.dssg_unpack_pairs_device(ctx.h, pairs.n, D._ptr(outp), D._ptr(uq), D._ptr(ue), st))
        torch.cuda.synchronize()
        pk = np.sort(outp[: pairs.n].cpu().numpy().view(np.uint64))
        assert np.array_equal(pk, own)
        assert np.array_equal(_keys(uq[: pairs.n].cpu().numpy().view(np.uint32),
                                    ue[: pairs.n].cpu().numpy().view(np.uint32)), own)
        got.append(pk)
        per_part.append(len(pk))
        idx.free()
    allp = np.sort(np.concatenate(got)) if got else np.zeros(0, np.uint64)
    assert len(np.unique(allp)) == len(allp), "a pair was emitted by two shards"
    assert np.array_equal(allp, _keys(fq, fe))
    if nparts > 1:
        assert sum(1 for x in per_part if x > 0) > 1  # the work really is spread


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank(rank, world, port, q):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), HSA_ENABLE_IPC_MODE_LEGACY="0")
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.cuda.set_device(0)
        from dss_amd import _lib, device as D, shard, workload as W
        from oracle import oracle as O
        O.build()
        _, qs, qa, it, ia, now = W.config(0, scale=0.02)
        ctx = _lib.context(0)
        dev = "cuda:0"
        t = lambda a: torch.as_tensor(np.ascontiguousarray(a), device=dev)  # noqa: E731
        icells = D.cover(ctx, D.DeviceFootprints.upload(it, dev))
        i_offs = D.copy_back(ctx, icells.offs, it.n + 1, np.int64)
        i_cells = D.copy_back(ctx, icells.cells, int(i_offs[-1]), np.uint64)
        ranges = shard.cell_splitters(i_cells, world)
        lo, hi = ranges[rank]
        attrs = [t(ia.alt_lo), t(ia.alt_hi), t(ia.t0), t(ia.t1)]  # alive for the whole build
        h = D.build_index(ctx, icells, *attrs, cell_range=(lo, hi))
        # this rank's query slice
        n = qs.n
        a, b = rank * n // world, (rank + 1) * n // world
        sub = qs.subset(np.arange(a, b))
        tlo, thi = W.query_bounds(qa, now)
        qc = D.cover(ctx, D.DeviceFootprints.upload(sub, dev))
        ss = shard.ShardedSearch(ctx, h, ranges, stage_host=True)
        qattrs = [t(qa.alt_lo[a:b]), t(qa.alt_hi[a:b]), t(tlo[a:b]), t(thi[a:b])]
        out = ss.step(qc.offs, qc.cells, sub.n, *qattrs)
        torch.cuda.synchronize()
        got = np.sort(out.cpu().numpy().view(np.uint64))
        so, sc, _, _ = O.cover_batch(sub.kind, sub.voff, sub.lat, sub.lng, sub.radius_m, nthreads=2)
        io, ic, _, _ = O.cover_batch(it.kind, it.voff, it.lat, it.lng, it.radius_m, nthreads=2)
        oq, oe = O.search(io, ic, ia.alt_lo, ia.alt_hi, ia.t0, ia.t1, None, so, sc, qa.alt_lo[a:b], qa.alt_hi[a:b],
                          tlo[a:b], thi[a:b])
        want = _keys(oq, oe)
        q.put((rank, bool(np.array_equal(got, want)), len(want), ss.last_rows, ss.last_shard_pairs))
        ctx.L.dssg_index_free(h)
    finally:
        dist.destroy_process_group()


def test_sharded_search_two_ranks_gloo():
    import torch.multiprocessing as mp
    world = 2
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_rank, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=100)
    for p in procs:
        if p.is_alive():
            p.kill()
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    res = sorted(q.get(timeout=5) for _ in range(world))
    assert all(ok for _, ok, _, _, _ in res), res
    assert all(n > 0 for _, _, n, _, _ in res)
    # pairs computed on the shards == pairs delivered home
    assert sum(r[4] for r in res) == sum(r[2] for r in res)


def test_native_rccl_one_rank_equals_full_search():
    """The library's own RCCL exchange (dssg_comm_*, dssg_sharded_search_device)
    on a one-rank communicator: route -> grouped send/recv to itself -> join
    -> pairs home, equal to the whole-index search.  (More ranks need more
    GPUs: the multi-GPU node at round end.)"""
    import torch
    from dss_amd import _lib, device as D, shard
    from dss_amd.store import EntityIndex
    ci, cq, qa, ia, tlo, thi = _covered(0.05)
    full = EntityIndex(ci.offs, ci.cells, ia.alt_lo, ia.alt_hi, ia.t0, ia.t1)
    fq, fe = full.search_batch(cq.offs, cq.cells, qa.alt_lo, qa.alt_hi, tlo, thi)
    ctx = _lib.context()
    uid = shard.NativeComm.unique_id(ctx)
    comm = shard.NativeComm(ctx, 1, 0, uid)
    ranges = shard.cell_splitters(ci.cells, 1)
    idx = EntityIndex(ci.offs, ci.cells, ia.alt_lo, ia.alt_hi, ia.t0, ia.t1, cell_range=ranges[0])
    t = lambda a: torch.as_tensor(np.ascontiguousarray(a), device="cuda")  # noqa: E731
    offs, cells = t(cq.offs), t(cq.cells.view(np.int64))
    ns = shard.NativeShardedSearch(ctx, comm, idx.h, ranges)
    try:
        # identity routing (one part), then the general path forced: route,
        # own segment copied, unpack, join, own pairs straight to the output
        for identity in (1, 0):
            ctx.set_tuning("route_identity", identity)
            for _ in range(2):  # a second step reuses the communicator's buffers
                p = ns.step(offs.data_ptr(), cells.data_ptr(), len(cq.offs) - 1, t(qa.alt_lo), t(qa.alt_hi), t(tlo),
                            t(thi))
                gq = D.copy_back(ctx, p.q, int(p.n), np.uint32)
                ge = D.copy_back(ctx, p.e, int(p.n), np.uint32)
                assert np.array_equal(_keys(gq, ge), _keys(fq, fe))
    finally:
        ctx.set_tuning("route_identity", 1)
    comm.close()
    idx.free()


def test_native_async_exchange_stream_one_rank():
    """dssg_sharded_search_async_device: the pairs' trip home on a second
    communicator and stream.  On one rank, identity and general routing:
    every step equals the whole-index search once the exchange stream has
    run, and a step's output stays valid through the next step (two buffer
    sets) -- the steps alternate between the batch and its first half, so a
    reread of an overwritten buffer would show the other batch's pairs
    (the identity path returned the engine's own buffers); the
    stats report the routed rows and no bytes to other ranks."""
    import torch
    from dss_amd import _lib, device as D, shard
    from dss_amd.store import EntityIndex
    ci, cq, qa, ia, tlo, thi = _covered(0.05)
    full = EntityIndex(ci.offs, ci.cells, ia.alt_lo, ia.alt_hi, ia.t0, ia.t1)
    nq = len(cq.offs) - 1
    half = nq // 2
    wants = [_keys(*full.search_batch(cq.offs, cq.cells, qa.alt_lo, qa.alt_hi, tlo, thi)),
             _keys(*full.search_batch(cq.offs[:half + 1], cq.cells[:int(cq.offs[half])], qa.alt_lo[:half],
                                      qa.alt_hi[:half], tlo[:half], thi[:half]))]
    assert len(wants[1]) < len(wants[0])
    ctx = _lib.context()
    comms = [shard.NativeComm(ctx, 1, 0, shard.NativeComm.unique_id(ctx)) for _ in range(2)]
    ranges = shard.cell_splitters(ci.cells, 1)
    idx = EntityIndex(ci.offs, ci.cells, ia.alt_lo, ia.alt_hi, ia.t0, ia.t1, cell_range=ranges[0])
    t = lambda a: torch.as_tensor(np.ascontiguousarray(a), device="cuda")  # noqa: E731
    offs, cells = t(cq.offs), t(cq.cells.view(np.int64))
    qargs = (t(qa.alt_lo), t(qa.alt_hi), t(tlo), t(thi))
    xs = torch.cuda.Stream()
    ns = shard.NativeShardedSearch(ctx, comms[0], idx.h, ranges, xcomm=comms[1], xstream=xs)
    with pytest.raises(ValueError):
        shard.NativeShardedSearch(ctx, comms[0], idx.h, ranges, xcomm=comms[1])
    try:
        for identity in (1, 0):
            ctx.set_tuning("route_identity", identity)
            prev = None
            for k in range(4):
                which = k % 2
                p = ns.step(offs.data_ptr(), cells.data_ptr(), half if which else nq, *qargs)
                torch.cuda.synchronize()
                got = _keys(D.copy_back(ctx, p.q, int(p.n), np.uint32), D.copy_back(ctx, p.e, int(p.n), np.uint32))
                assert np.array_equal(got, wants[which]), (identity, k)
                if prev is not None:  # the previous step's output (the other batch), read after this step
                    pq_, pn_, pw = prev
                    again = _keys(D.copy_back(ctx, pq_.q, pn_, np.uint32), D.copy_back(ctx, pq_.e, pn_, np.uint32))
                    assert np.array_equal(again, wants[pw]), (identity, k)
                prev = (p, int(p.n), which)
            ms, cnt = ns.stats()
            if identity == 0:
                assert cnt["rows"] > 0
                assert cnt["query_bytes_sent"] == 0 and cnt["pair_bytes_sent"] == 0
                assert cnt["shard_pairs"] == len(wants[1])  # (the last step: the half batch)
        # timing on: phases measured, touched postings counted
        ctx.set_tuning("route_identity", 0)
        ctx.L.dssg_set_timing(ctx.h, 1)
        p = ns.step(offs.data_ptr(), cells.data_ptr(), len(cq.offs) - 1, *qargs)
        ctx.L.dssg_set_timing(ctx.h, 0)
        ms, cnt = ns.stats()
        assert ms["join"] > 0 and ms["exchange_pairs"] >= 0 and cnt["touched"] > 0
        torch.cuda.synchronize()
    finally:
        ctx.set_tuning("route_identity", 1)
    ns.close()
    idx.free()
