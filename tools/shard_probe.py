#!/usr/bin/env python3
"""One rank's shard join at world size N, in one process (profiling only, not
product code): the k_join a rank of an N-GPU sharded run launches, without N
processes sharing the one GPU of a profiling box (a rocprofv3 PMC pass counts
whatever runs on the chip, so a same-device multi-rank rehearsal would mix the
ranks' joins in its FETCH_SIZE / WRITE_SIZE).

The shard: rank R's cell range of N (shard.cell_splitters over the config's
intent postings, quad-aligned), built as in bench.py.  Its batch: the union of
the N ranks' query batches (bench.py's seeds), covered -- a shard receives
every query that touches its range with its whole cell list, and the cells
outside the range find no postings, so the join's units and records are the
shard's own.  Each step searches that batch against the shard (HIP events on
the search); the per-launch k_join counters come from rocprofv3 around this
script (tools/profile.sh with PROBE=N).

usage: python tools/shard_probe.py N [--config 2] [--rank 0] [--steps 4] [--warmup 1]"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def concat(fps):
    from dss_amd.workload import Footprints
    voff, base = [np.zeros(1, np.int64)], 0
    for f in fps:
        voff.append(f.voff[1:] + base)
        base += int(f.voff[-1])
    return Footprints(np.concatenate([f.kind for f in fps]), np.concatenate(voff),
                      np.concatenate([f.lat for f in fps]), np.concatenate([f.lng for f in fps]),
                      np.concatenate([f.radius_m for f in fps]))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("world", type=int)
    ap.add_argument("--config", type=int, default=2)
    ap.add_argument("--rank", type=int, default=0)
    ap.add_argument("--steps", type=int, default=4)
    ap.add_argument("--warmup", type=int, default=1)
    a = ap.parse_args()
    import torch
    import bench
    from dss_amd import _lib, device as D, shard, workload as W
    dev = "cuda:0"
    ctx = _lib.context(0)
    t = lambda x: torch.as_tensor(x, device=dev)  # noqa: E731
    qs, qas = [], []
    for r in range(a.world):
        q, qa, intents, ia, now, rid = W.config_split(a.config, r)
        qs.append(q)
        qas.append(qa)
    queries = concat(qs)
    nq, ni = queries.n, intents.n
    alo = np.concatenate([x.alt_lo for x in qas])
    ahi = np.concatenate([x.alt_hi for x in qas])
    tlo = np.maximum(np.concatenate([x.t0 for x in qas]), now)
    thi = np.concatenate([x.t1 for x in qas])
    i_offs_t, i_cells_t = bench.cover_chunked(ctx, D, torch, intents, dev)
    icells = _lib.Cells(ni, int(i_offs_t.data_ptr()), int(i_cells_t.data_ptr()), 0, 0, int(i_cells_t.numel()))
    ranges = shard.cell_splitters(i_cells_t.cpu().numpy().view(np.uint64), a.world)
    index = D.build_index(ctx, icells, t(ia.alt_lo), t(ia.alt_hi), t(ia.t0), t(ia.t1), cell_range=ranges[a.rank])
    q_offs_t, q_cells_t = bench.cover_chunked(ctx, D, torch, queries, dev)
    qcells = _lib.Cells(nq, int(q_offs_t.data_ptr()), int(q_cells_t.data_ptr()), 0, 0, int(q_cells_t.numel()))
    qargs = (t(alo), t(ahi), t(tlo), t(thi))
    torch.cuda.synchronize()
    import ctypes as C
    ms = []
    for k in range(a.warmup + a.steps):
        ctx.L.dssg_set_timing(ctx.h, 1)
        p = D.search(ctx, index, qcells, *qargs)
        torch.cuda.synchronize()
        ca, cb, cc = C.c_double(), C.c_double(), C.c_double()
        ctx.L.dssg_phase_times(ctx.h, C.byref(ca), C.byref(cb), C.byref(cc))
        if k >= a.warmup:
            ms.append((cb.value, cc.value, int(p.n)))
    ctx.L.dssg_set_timing(ctx.h, 0)
    touched = bench.touched_postings(ctx, D, index, qcells)
    print(json.dumps({"world": a.world, "rank": a.rank, "config": a.config, "queries_all_ranks": nq, "intents": ni,
                      "shard_postings": int(ctx.L.dssg_index_num_postings(index)), "P_touched": touched,
                      "join_ms": float(np.mean([m[0] for m in ms])),
                      "join_kernel_ms": float(np.mean([m[1] for m in ms])), "pairs": ms[-1][2],
                      "range": [str(x) for x in ranges[a.rank]]}), flush=True)


if __name__ == "__main__":
    main()
