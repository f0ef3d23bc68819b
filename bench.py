#!/usr/bin/env python3
"""Benchmark: 4D conflict queries/s against a resident N-intent airspace.

BASELINE.json metric "4D conflict queries/sec vs N-intent airspace
(1/2/4/8 GPU); coverings/sec".  Default workload configs[2], the north-star
airspace: 1M polygon/circle query footprints per GPU step against a
10M-intent index over California (70 % around 4 hotspots), seeded synthetic
data (SURVEY.md s8(d) generator).  --config 1 is the 1M x 1M metro config.

One step = cover the rank's 1M query footprints on the GPU (level-13 S2
coverings) -> overlap join against the HBM-resident index -> fused
altitude/time/now filter -> deduplicated (query, intent) pairs resident in
HBM.  The index (intent coverings + posting lists) is built before timing.

Ranks: one process per GPU.  Under torchrun (WORLD_SIZE set) each process is
one rank; `--gpus N` without a launcher starts the N rank processes itself
(self_launch) before anything touches a GPU.  --mode:
  replica (the default at every N): each rank holds the whole index (a few
    GB of its 288 GB of HBM) and covers + joins its own 1M-query batch; the
    query batches are the units sharded across ranks, with no collective on
    the data path.  "scaling": "weak" (1M queries per GPU).
  sharded (--mode sharded; BASELINE's cell-range layout): the
    intent index is split into N uint64 cell ranges at posting quantiles, one
    shard per GPU.  Each rank covers its own 1M queries, routes every query
    (row + whole cell list) to the shards owning its cells (all-to-all over
    RCCL/xGMI, the library's own communicator), joins what it receives
    against its shard, and routes the pairs back to their queries' home ranks
    (second all-to-all).  The replica rate is reported beside it.  Not the
    default: at N = 8 about 7/8 of a step's ~256M pairs cross ranks, ~1.8 GB
    per rank per step against a ~4 ms step, while the whole index fits every
    GPU many times over.
Timing: barrier + synchronize on both sides of exactly --steps steps, max
over ranks.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0      # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
FP64_PEAK_TFLOPS = 78.6    # MI355X FP64 vector (spec)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


_STAGE = ["start", time.time()]
_JSON_FD = [None]
# Stages with collectives in them: one that runs past its limit is taken to be
# hung (a peer that never issued its side of a collective); the process exits
# non-zero instead of holding its GPU until an outside timeout (the launcher
# then stops the other ranks).
STAGE_LIMIT_S = {"native exchange init": 300, "warmup": 900, "timed steps": 900,
                 "replica rate beside the sharded one": 900, "sharded phases": 900}
# The sharded leg of an N > 1 replica run (sharded_leg): a stage of it that
# runs past its limit ends the rank with status 0 -- the replica line is
# complete -- and rank 0 prints that line with sharded.error set.
LEG_LIMIT_S = 120  # (each legit stage of the leg takes seconds at full size; a hang costs at most this)
_PENDING = [None, 0]  # rank 0's finished replica line while the sharded leg runs; this rank


def keep_stdout_for_json():
    """Only the result line goes to stdout: native libraries (RCCL's init
    banner) write to fd 1 directly, so fd 1 is pointed at stderr and the
    original stdout is kept for emit()."""
    sys.stdout.flush()
    _JSON_FD[0] = os.dup(1)
    os.dup2(2, 1)


def emit(result):
    line = (json.dumps(result) + "\n").encode()
    if _JSON_FD[0] is None:
        sys.stdout.write(line.decode())
        sys.stdout.flush()
    else:
        os.write(_JSON_FD[0], line)


def stage(name):
    """Name the current stage (the heartbeat reports it)."""
    _STAGE[0] = name
    _STAGE[1] = time.time()
    log(f"[bench] {name}")


def heartbeat(every=30.0):
    """A stderr line every `every` s while the process runs (long configs)."""
    import threading
    t0 = time.time()

    def run():
        while True:
            time.sleep(every)
            log(f"[bench] alive {time.time() - t0:.0f}s, stage: {_STAGE[0]}")
            if _STAGE[0].startswith("sharded leg") and time.time() - _STAGE[1] > LEG_LIMIT_S:
                log(f"[bench] stage '{_STAGE[0]}' exceeded {LEG_LIMIT_S}s: the sharded leg is abandoned")
                if _PENDING[0] is not None and _PENDING[1] == 0:
                    _PENDING[0]["sharded"] = {"error": f"stage '{_STAGE[0]}' exceeded {LEG_LIMIT_S}s (a collective "
                                                       f"presumed hung); the replica line stands"}
                    emit(_PENDING[0])
                os._exit(0)
            limit = STAGE_LIMIT_S.get(_STAGE[0])
            if limit and time.time() - _STAGE[1] > limit:
                log(f"[bench] stage '{_STAGE[0]}' exceeded {limit}s: exiting (a collective is presumed hung)")
                os._exit(3)
    threading.Thread(target=run, daemon=True).start()


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1,
                    help="GPUs (ranks) of one node.  Under a launcher (torchrun: WORLD_SIZE set) each process is one "
                         "rank; without one, N > 1 starts N rank processes itself (before any GPU call here) and "
                         "relays rank 0's result line")
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", type=int, default=2,
                    help="BASELINE.json configs[i]; default 2: the north-star airspace (10M intents, 1M-query batches "
                         "per GPU), the layout BASELINE's 1/2/4/8-GPU metric is quoted on")
    ap.add_argument("--scale", type=float, default=1.0, help="shrink the workload (debug only; invalid for the metric)")
    ap.add_argument("--query-scale", type=float, default=1.0,
                    help="queries per step relative to the config's 1M (configs[4] at full size: 0.1, since its output "
                         "grows with batch x airspace density: ~5.7k pairs per query against 50M corridors)")
    ap.add_argument("--cpu-sample", type=int, default=-1,
                    help="queries in the CPU-baseline sample (-1: auto -- the whole step's batch for configs[0]..[3], a "
                         "bounded sample of ~10-30 s of CPU work for configs[4]; 0: skip).  The sample's "
                         "cells and pairs are compared with the GPU step's (parity on the sampled queries)")
    ap.add_argument("--parity-sample", type=int, default=20000,
                    help="ranks other than 0 (N > 1): queries of their own batch whose cells and pairs are compared "
                         "with the oracle after the timed steps (0: skip)")
    ap.add_argument("--no-verify", action="store_true", help="skip the full-size GPU-vs-oracle parity check")
    ap.add_argument("--survey-model", type=int, default=1, help="also count SURVEY s8(d)'s per-query byte model")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="CPU-baseline threads (0: the process's CPU share -- the affinity mask, capped by "
                         "OMP_NUM_THREADS, which the GPU box sets to its per-GPU share of 16)")
    ap.add_argument("--mode", choices=["sharded", "replica"], default=None,
                    help="multi-GPU layout: replica (index on every GPU, query batches split across ranks, no "
                         "data-path collective; the default) or sharded (index split by S2 cell range, queries and "
                         "pairs exchanged by all-to-all, BASELINE's layout, with the replica rate reported beside it)")
    ap.add_argument("--sharded-leg", type=int, default=1,
                    help="N > 1, replica mode: after the replica line's steps, the same ranks time the cell-range "
                         "shards (BASELINE's layout) over the library's RCCL exchange and attach them as the line's "
                         "`sharded` record (value stays the replica rate); 0: skip")
    ap.add_argument("--exchange", choices=["native", "torch"], default=None,
                    help="sharded mode's all-to-alls: native (the library's own RCCL communicator, "
                         "dssg_sharded_search_device) or torch (torch.distributed; the instrumented path).  Default: "
                         "native with --dist-backend nccl, torch otherwise")
    ap.add_argument("--dist-backend", default="nccl", help="nccl (RCCL) on a multi-GPU node; gloo for rehearsals")
    ap.add_argument("--tune", action="append", default=[], metavar="KEY=VALUE",
                    help="dssg_set_tuning knob for every pipeline's context (e.g. lazy_sig_recs=0)")
    ap.add_argument("--pipelines", type=int, default=3,
                    help="batch pipelines per GPU, each its own engine context + stream + host thread.  replica: P "
                         "independent cover+join pipelines (one batch's FP64 covering overlaps another's join, as "
                         "concurrent RPCs would); sharded: P-1 contexts cover the next batches ahead while the "
                         "exchange + shard join runs the batches in step order on one communicator")
    ap.add_argument("--latency", type=int, default=1,
                    help="also time single requests (cover + search of one footprint): alone, and 64 concurrent "
                         "callers through the micro-batcher (dssg_batcher)")
    ap.add_argument("--same-device", action="store_true",
                    help="rehearsal: every rank on cuda:0 (one-GPU box, gloo backend)")
    ap.add_argument("--launch-probe", default=None, metavar="DIR",
                    help="test hook: each rank writes its launch environment to DIR/rank<r>.json and exits before "
                         "importing torch (checks the self-launch on a machine without GPUs)")
    return ap.parse_args(argv)


def self_launch(args, argv):
    """`--gpus N` (N > 1) with no launcher around this process: start N rank
    processes of this same command line, one per GPU (RANK / LOCAL_RANK /
    WORLD_SIZE / MASTER_* in their environment, rendezvous on 127.0.0.1), the
    way torchrun would.  Nothing here touches the GPU: the children own the
    devices.  Rank 0's stdout (the result line) is relayed; if a rank fails,
    the others are stopped (their exact PIDs) and its exit status returned."""
    import socket
    import subprocess
    import threading
    n = args.gpus
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    log(f"[bench] self-launch: {n} ranks, rendezvous 127.0.0.1:{port}")
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, "-u", os.path.join(ROOT, "bench.py")] + list(argv), env=env,
                                      stdout=subprocess.PIPE if r == 0 else None))

    def relay():
        for line in procs[0].stdout:
            sys.stdout.write(line.decode(errors="replace"))
            sys.stdout.flush()
    th = threading.Thread(target=relay, daemon=True)
    th.start()
    rc, alive, deadline = 0, set(range(n)), None
    while alive:
        for r in sorted(alive):
            c = procs[r].poll()
            if c is None:
                continue
            alive.discard(r)
            if c != 0 and rc == 0:
                rc = c if c > 0 else 128 - c
                log(f"[bench] rank {r} exited with status {c}; stopping the other ranks")
                for q in alive:
                    procs[q].terminate()
                deadline = time.time() + 30
        if deadline is not None and time.time() > deadline:
            for q in alive:
                procs[q].kill()
            deadline = None
        time.sleep(0.1)
    th.join(timeout=10)
    return rc


def launch_probe(path):
    """--launch-probe: record this rank's launch environment (no torch, no GPU)."""
    os.makedirs(path, exist_ok=True)
    rank = int(os.environ.get("RANK", 0))
    rec = {k.lower(): os.environ.get(k) for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")}
    rec["pid"] = os.getpid()
    rec["torch_imported"] = "torch" in sys.modules
    with open(os.path.join(path, f"rank{rank}.json"), "w") as f:
        json.dump(rec, f)
    if rank == 0:
        print(json.dumps({"launch_probe": rec}), flush=True)


def allreduce_vals(dist, torch, vals, op):
    """All-reduce a few float64 control values over the process group (on the
    GPU when the group is RCCL, else on the host); returns a list."""
    dev = f"cuda:{torch.cuda.current_device()}" if dist.get_backend() == "nccl" else "cpu"
    t = torch.tensor([float(v) for v in vals], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=op)
    return t.cpu().tolist()


def timed(torch, dist, dev, world, fn):
    """Barrier + synchronize on both sides of fn(); the max over ranks (s)."""
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    fn()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        tt = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
    return elapsed


class StepFailure(RuntimeError):
    """A pipeline failed inside the timed region: no result line may be
    printed for the run (a rate over steps that did not finish is not a
    measurement), and the process exits non-zero."""


def replica_steps(torch, D, ctx, workers, d_q, index, qargs, steps):
    """`steps` replica steps (cover + join against the whole index) over the
    main context and the worker pipelines; the steps are handed out one at a
    time, so no pipeline idles while another still has a queue (the tail is
    at most one step).  A pipeline that raises stops every other one from
    taking further steps; the first error is re-raised as StepFailure after
    all threads have joined, and so is a count of finished steps short of
    `steps` -- the caller never divides `steps` by a time in which fewer
    finished."""
    import threading
    tickets = [0]
    finished = [0]
    errors = []
    lock = threading.Lock()

    def take():
        with lock:
            if errors:
                return False
            t = tickets[0]
            tickets[0] += 1
        return t < steps

    def run(wctx, wstream):
        try:
            with torch.cuda.stream(wstream):
                while take():
                    D.search(wctx, index, D.cover(wctx, d_q), *qargs)
                    with lock:
                        finished[0] += 1
                wstream.synchronize()
        except BaseException as e:  # noqa: BLE001 -- re-raised below, on the calling thread
            with lock:
                errors.append(e)

    threads = [threading.Thread(target=run, args=w) for w in workers]
    for th in threads:
        th.start()
    run(ctx, torch.cuda.current_stream())
    for th in threads:
        th.join()
    if errors:
        raise StepFailure(f"{len(errors)} pipeline(s) failed in the timed steps ({finished[0]} of {steps} steps "
                          f"finished): {type(errors[0]).__name__}: {errors[0]}") from errors[0]
    if finished[0] != steps:
        raise StepFailure(f"{finished[0]} of {steps} steps finished")


HBM_RESERVE = 4 << 30  # kept free beside the pipelines' steady-state buffers


def add_pipelines(args, torch, D, _lib, local, dev, tunes, d_q, join):
    """Up to --pipelines - 1 worker pipelines beside the main context.  Each
    new context is warmed with two full steps (cover + join when `join` =
    (index, qargs) is given; the second step settles buffers the first one
    sized, such as the pair buffer after a long x long overflow) and kept only
    if the HBM left after it still holds another context of the same size
    plus HBM_RESERVE -- so the timed steps never allocate.  A context whose
    warm-up runs out of memory is dropped.  Returns (workers, note)."""
    workers = []
    foot = 0
    want = max(0, args.pipelines - 1)
    note = None
    for _ in range(want):
        free0, _t = torch.cuda.mem_get_info(local)
        if workers and free0 < foot + HBM_RESERVE:
            note = f"{len(workers) + 1} of {args.pipelines} pipelines: {free0 / 2**30:.1f} GiB free, one more " \
                   f"pipeline holds {foot / 2**30:.1f} GiB"
            break
        wctx = _lib.Context(local)
        ws = torch.cuda.Stream(device=dev)
        try:
            for k, v in tunes:
                wctx.set_tuning(k, v)
            with torch.cuda.stream(ws):
                for _rep in range(2):
                    c = D.cover(wctx, d_q)
                    if join is not None:
                        D.search(wctx, join[0], c, *join[1])
                ws.synchronize()
        except _lib.DssgError as e:
            wctx.close()
            torch.cuda.synchronize()
            note = f"{len(workers) + 1} of {args.pipelines} pipelines: warming pipeline {len(workers) + 2} failed " \
                   f"({e})"
            break
        free1, _t = torch.cuda.mem_get_info(local)
        foot = max(foot, free0 - free1)
        workers.append((wctx, ws))
        if free1 < HBM_RESERVE:  # this one fits only without the reserve: drop it
            wctx.close()
            workers.pop()
            torch.cuda.synchronize()
            note = f"{len(workers) + 1} of {args.pipelines} pipelines: the last one left " \
                   f"{free1 / 2**30:.1f} GiB free"
            break
    if note:
        log(f"[bench] {note}")
    return workers, note


def cover_ahead_steps(torch, D, ctx, covers, d_q, steps, search_fn):
    """`steps` sharded steps: step k's batch is covered by covers[k % P] (own
    context, stream and host thread) ahead of time, and the exchange + shard
    join (`search_fn(cells)`) runs on the calling thread in step order -- one
    communicator, so every rank issues its collectives in the same order.  A
    cover context re-covers only after the search that read its last batch
    (host semaphore + a stream wait on that search's event)."""
    import queue
    import threading
    P = len(covers)
    if P == 0:  # one pipeline: cover inline on the main context
        for _ in range(steps):
            search_fn(D.cover(ctx, d_q))
        return
    ready = [queue.Queue() for _ in range(P)]
    free = [threading.Semaphore(1) for _ in range(P)]
    done = [None] * P
    err = []
    stop = threading.Event()

    def cover_loop(p):
        wctx, ws = covers[p]
        try:
            with torch.cuda.stream(ws):
                for _ in range(p, steps, P):
                    free[p].acquire()
                    if stop.is_set():
                        return
                    if done[p] is not None:
                        ws.wait_event(done[p])
                    c = D.cover(wctx, d_q)
                    ev = torch.cuda.Event()
                    ev.record(ws)
                    ready[p].put((c, ev))
                ws.synchronize()
        except BaseException as e:  # noqa: BLE001 -- handed to the search thread
            err.append(e)
            ready[p].put(None)

    threads = [threading.Thread(target=cover_loop, args=(p,), daemon=True) for p in range(P)]
    for th in threads:
        th.start()
    # an explicit stream (never the default one, whose handle 0 sends the
    # library to the context's own non-blocking stream, which the waits
    # below would not order): the step's kernels run after its covering
    main = torch.cuda.Stream()
    finished = 0
    try:
        with torch.cuda.stream(main):
            for k in range(steps):
                item = ready[k % P].get()
                if item is None:
                    raise StepFailure(f"a cover pipeline failed in the timed steps ({finished} of {steps} steps "
                                      f"finished): {type(err[0]).__name__}: {err[0]}") from err[0]
                c, ev = item
                main.wait_event(ev)
                search_fn(c)
                finished += 1
                ev_done = torch.cuda.Event()
                ev_done.record(main)
                done[k % P] = ev_done
                free[k % P].release()
    finally:
        if finished != steps:  # release the cover threads so they end
            stop.set()
            for f in free:
                f.release()
    for th in threads:
        th.join()


def main():
    argv = sys.argv[1:]
    args = parse_args(argv)
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(self_launch(args, argv))
    if args.launch_probe:
        launch_probe(args.launch_probe)
        return

    heartbeat()
    keep_stdout_for_json()
    import torch
    import torch.distributed as dist

    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    if world != args.gpus:
        log(f"[bench] note: --gpus {args.gpus} but WORLD_SIZE {world}; the line reports n_gpus = WORLD_SIZE")
    local = 0 if args.same_device else int(os.environ.get("LOCAL_RANK", 0))
    mode = args.mode or "replica"
    exchange = args.exchange or ("native" if args.dist_backend == "nccl" else "torch")
    torch.cuda.set_device(local)
    # The process group is the control plane (rendezvous, barriers, the
    # timing max, parity flags).  With the library's own RCCL exchange it is
    # gloo, so each process holds one RCCL (the library's); the torch
    # exchange (fallback / rehearsals) runs over the PG or an RCCL subgroup.
    leg = mode == "replica" and world > 1 and args.sharded_leg != 0
    native_wanted = (mode == "sharded" or leg) and exchange == "native"
    pg_backend = "gloo" if native_wanted else args.dist_backend
    _PENDING[1] = rank
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")   # single-process sharded runs (no launcher)
    os.environ.setdefault("MASTER_PORT", "29533")
    if world > 1 or mode == "sharded":
        if pg_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local), rank=rank, world_size=world)
        else:
            dist.init_process_group(pg_backend, rank=rank, world_size=world)

    from dss_amd import _lib, device as D, workload as W

    ctx = _lib.context(local)
    dev = f"cuda:{local}"
    tunes = [(kv.split("=", 1)[0], int(kv.split("=", 1)[1])) for kv in args.tune]
    for k, v in tunes:
        ctx.set_tuning(k, v)

    # ---------------------------------------------------------------- setup
    t_setup = time.time()
    # same airspace on every rank (config seed), a rank-private query batch
    queries, qa, intents, ia, now, rid = W.config_split(args.config, rank, args.scale, args.query_scale)
    nq, ni = queries.n, intents.n
    tlo = np.maximum(qa.t0, now)  # operations.go:398-402 COALESCE(ends_at >= start) AND ends_at >= now
    t = lambda a: torch.as_tensor(a, device=dev)  # noqa: E731
    d_int = D.DeviceFootprints.upload(intents, dev)
    d_q = D.DeviceFootprints.upload(queries, dev)
    q_alo, q_ahi, q_tlo, q_thi = t(qa.alt_lo), t(qa.alt_hi), t(tlo), t(qa.t1)
    qargs = (q_alo, q_ahi, q_tlo, q_thi)
    i_alo, i_ahi, i_t0, i_t1 = t(ia.alt_lo), t(ia.alt_hi), t(ia.t0), t(ia.t1)
    torch.cuda.synchronize()
    tb = time.time()
    # the intents' coverings, covered in chunks and kept in torch-owned HBM
    # (the next cover() call reuses the library's own output buffers)
    i_offs_t, i_cells_t = cover_chunked(ctx, D, torch, intents, dev)
    icells = _lib.Cells(ni, int(i_offs_t.data_ptr()), int(i_cells_t.data_ptr()), 0, 0, int(i_cells_t.numel()))
    del d_int
    cover_i_s = time.time() - tb
    tb = time.time()
    ranges = full_index = None
    large = i_cells_t.numel() > LARGE_POSTINGS
    if mode == "sharded":
        from dss_amd import shard
        # splitters from the intent postings (host), then this rank's shard
        i_cells_h = i_cells_t.cpu().numpy().view(np.uint64)
        ranges = shard.cell_splitters(i_cells_h, world)
        # the whole index beside the shard: the replica rate and the parity reference
        full_index = D.build_index(ctx, icells, i_alo, i_ahi, i_t0, i_t1)
        tb = time.time()
        index = D.build_index(ctx, icells, i_alo, i_ahi, i_t0, i_t1, cell_range=ranges[rank])
    else:
        index = D.build_index(ctx, icells, i_alo, i_ahi, i_t0, i_t1)
    torch.cuda.synchronize()
    build_s = time.time() - tb
    n_post = int(ctx.L.dssg_index_num_postings(index))
    free_b, total_b = torch.cuda.mem_get_info(local)
    log(f"[rank {rank}] mode {mode}, setup {time.time() - t_setup:.1f}s, intent cover {cover_i_s:.2f}s, index build "
        f"{build_s:.2f}s, postings {n_post}, HBM free {free_b / 2**30:.1f} of {total_b / 2**30:.1f} GiB")
    sort_ph = None
    if rank == 0 and mode != "sharded":
        sort_ph = (sort_phase(ctx, torch, dev, i_offs_t, i_cells_t) if not large else
                   {"skipped": f"{i_cells_t.numel()} postings: the sort's scratch on top of the index would not fit "
                               f"beside it; the build's sorts are inside index_build_s"})
    sharded = native = None
    if mode == "sharded":
        native, sharded, exchange = make_exchange(args, ctx, dist, torch, dev, rank, index, ranges, exchange,
                                                  native_wanted, pg_backend)

    def shard_search(cells, timed_phases=False):
        if native is not None:
            return native.step(cells.offs, cells.cells, nq, *qargs)
        return sharded.step(cells.offs, cells.cells, nq, *qargs, timed=timed_phases)

    def step(timed=False):
        cells = D.cover(ctx, d_q)
        if mode == "sharded":
            return cells, shard_search(cells, timed)
        return cells, D.search(ctx, index, cells, *qargs)

    stage("warmup")
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()

    # extra pipelines: each its own context (engine scratch), stream and host
    # thread, warmed to its steady-state buffers and kept only if HBM holds it
    # (sharded: they cover ahead; every collective is issued by this thread)
    workers, pipe_note = add_pipelines(args, torch, D, _lib, local, dev, tunes, d_q,
                                       None if mode == "sharded" else (index, qargs))

    # ------------------------------------------------------------ timed steps
    stage("timed steps")
    general = None
    if mode == "sharded":
        elapsed = timed(torch, dist, dev, world,
                        lambda: cover_ahead_steps(torch, D, ctx, workers, d_q, args.steps, shard_search))
        if world == 1 and native is not None:
            # one rank: the library routes by the identity; the general path
            # (route, own segment copied, unpack, join, own pairs to the
            # output, pairs on the exchange stream) timed beside it
            ctx.set_tuning("route_identity", 0)
            cover_ahead_steps(torch, D, ctx, workers, d_q, 2, shard_search)
            gt = timed(torch, dist, dev, world,
                       lambda: cover_ahead_steps(torch, D, ctx, workers, d_q, args.steps, shard_search))
            ctx.set_tuning("route_identity", 1)
            general = {"value": world * nq * args.steps / gt, "ms_per_step": 1000.0 * gt / max(1, args.steps),
                       "note": "one rank with the routing forced through the general path (route_identity=0)"}
    else:
        elapsed = timed(torch, dist, dev, world,
                        lambda: replica_steps(torch, D, ctx, workers, d_q, index, qargs, args.steps))
    ms_per_step = 1000.0 * elapsed / max(1, args.steps)
    value = world * nq * args.steps / elapsed

    if mode == "sharded":
        # the replica layout beside it: every rank joins its own batch against
        # the whole index, same pipelines, no exchange
        stage("replica rate beside the sharded one")
        replica_steps(torch, D, ctx, workers, d_q, full_index, qargs, max(1, args.warmup))
        rt = timed(torch, dist, dev, world,
                   lambda: replica_steps(torch, D, ctx, workers, d_q, full_index, qargs, args.steps))
        replica = {"value": world * nq * args.steps / rt, "ms_per_step": 1000.0 * rt / max(1, args.steps),
                   "pipelines_per_gpu": 1 + len(workers),
                   "note": "whole index on every GPU, each rank's batch joined locally (no exchange)"}
        if general is not None:
            replica["sharded_general_path"] = general
        for wctx, _ in workers:
            wctx.close()
        sharded_report(args, ctx, D, dist, torch, sharded, native, step, full_index, i_offs_t, i_cells_t, ranges, rank,
                       world, nq, ni, n_post, build_s, value, ms_per_step, qargs, queries, qa, intents, ia, now,
                       exchange=exchange, replica=replica, pipelines=1 + len(workers), pipe_note=pipe_note)
        if native is not None:
            native.close()
        ctx.L.dssg_index_free(index)
        dist.destroy_process_group()
        return
    for wctx, _ in workers:
        wctx.close()

    # ------------------------------------------- phase timing + roofline
    stage(f"phase timing ({value:.4g} queries/s over the timed steps)")
    import ctypes as C
    ctx.L.dssg_set_timing(ctx.h, 1)
    cover_ms, join_ms, kern_ms = [], [], []
    ctx.join_profile()  # (a counting build: clear what the timed steps summed)
    for _ in range(5):
        cells, pairs = step()
        ca, cb, cc = C.c_double(), C.c_double(), C.c_double()
        ctx.L.dssg_phase_times(ctx.h, C.byref(ca), C.byref(cb), C.byref(cc))
        cover_ms.append(ca.value)
        join_ms.append(cb.value)
        kern_ms.append(cc.value)
    ctx.L.dssg_set_timing(ctx.h, 0)
    jprof = ctx.join_profile()
    if jprof:  # per search (the 5 phase-timing steps, one pipeline)
        jprof = {k: v / 5 for k, v in jprof.items()}
        jprof["yield"] = jprof["kept"] / max(1.0, jprof["lane_tests"])
    n_keys, n_units, n_runs, n_iters, n_tests = (C.c_int64() for _ in range(5))
    ctx.check(ctx.L.dssg_search_counters(ctx.h, C.byref(n_keys), C.byref(n_units), C.byref(n_runs), C.byref(n_iters),
                                         C.byref(n_tests)))
    n_fl, n_mg, n_ml, n_tg = (C.c_int64() for _ in range(4))
    ctx.check(ctx.L.dssg_join_events(ctx.h, C.byref(n_fl), C.byref(n_mg), C.byref(n_ml), C.byref(n_tg)))
    n_lq, n_lp = C.c_int64(), C.c_int64()
    ctx.check(ctx.L.dssg_join_longs(ctx.h, C.byref(n_lq), C.byref(n_lp)))
    c_tot = int(cells.total_cells)
    r_tot = int(pairs.n)
    kern_avg_ms = float(np.mean(kern_ms))
    cover_avg = float(np.mean(cover_ms))
    join_avg = float(np.mean(join_ms))
    # Algorithmic bytes of one k_join launch: the batch's query
    # inputs (24 B attributes + 8 B per covering cell), every posting of a
    # cell the batch touches read once (28 B: entity id, alt pair, time
    # pair), and the output pairs (8 B).
    stage("cover roofline counts")
    c_offs_h = D.copy_back(ctx, cells.offs, nq + 1, np.int64)
    cover_rl = cover_roofline(queries, c_offs_h, D.copy_back(ctx, cells.cells, int(c_offs_h[-1]), np.uint64),
                              cover_avg)
    stage("touched postings")
    p_touched = touched_postings(ctx, D, index, cells)
    join_bytes = 24 * nq + 8 * c_tot + 28 * p_touched + 8 * r_tot
    achieved = join_bytes / (kern_avg_ms * 1e-3) / 1e9
    # SURVEY s8(d) per-query model (B_q summed over queries, each query
    # charged for its own matched postings): what a query-at-a-time join
    # would move; reported for reference, not as the roofline.
    m_tot, d_tot = C.c_int64(), C.c_int64()
    if args.survey_model:
        stage("survey model counts")
        ctx.check(ctx.L.dssg_search_stats_device(ctx.h, index, cells.n, C.c_void_p(cells.offs),
                                                 C.c_void_p(cells.cells), D._stream_ptr(), C.byref(m_tot),
                                                 C.byref(d_tot)))
    survey_bytes = 8 * c_tot + 12 * m_tot.value + 24 * d_tot.value + 8 * r_tot
    stage("device copy bandwidth")
    copy_bw = copy_bandwidth(ctx, torch, dev)

    # every rank: its step's covering and pairs against the oracle (rank 0:
    # the timed CPU baseline on its --cpu-sample; the others: --parity-sample
    # queries), the flags reduced over ranks
    stage("oracle parity" + (" + cpu baseline" if rank == 0 else ""))
    cpu, parity = oracle_leg(args, ctx, D, dist, torch, dev, rank, world, queries, qa, intents, ia, now, i_offs_t,
                             i_cells_t, cells, pairs)
    result = None
    if rank == 0:
        latency = None  # (measured last, below)
        traffic = pmc_traffic("k_join", nq, ni)
        result = {
            "metric": "4D conflict queries/sec vs N-intent airspace",
            "value": value,
            "unit": "queries/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_per_step,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (seeded SURVEY s8(d) generator; no datasets)",
            "config": {"workload": f"configs[{args.config}]: {nq} query footprints/GPU/step vs {ni}-entity resident "
                                   f"index, {W.CONFIG_NAMES[args.config]}, S2 level 13"
                                   + (" (SearchISAs semantics)" if rid else ""),
                       "queries_per_gpu_step": nq, "intents": ni, "postings": n_post, "index": index_info(ctx, index),
                       "parallelism": f"query-sharded x{world}, index replicated"
                                      + ("; the cell-range shards timed after by the same ranks: `sharded`" if leg else ""),
                       "scale": args.scale,
                       "pipelines_per_gpu": 1 + len(workers), "pipelines_note": pipe_note},
            "coverings_per_s": world * nq / (cover_avg * 1e-3),
            "phase_ms": {"cover": cover_avg, "join": join_avg, "join_kernel": kern_avg_ms},
            "pairs_per_step": r_tot,
            "join_work": {"keys": n_keys.value, "units": n_units.value, "runs": n_runs.value,
                          "wave_iters": n_iters.value, "lane_tests": n_tests.value, "flushes": n_fl.value,
                          "exact_merges": n_mg.value, "exact_merge_lanes": n_ml.value,
                          "long_pair_occurrences": n_tg.value, "long_queries": n_lq.value,
                          "long_postings": n_lp.value,
                          "yield": r_tot / max(1, n_tests.value),
                          "predicates": jprof},
            "index_build_s": build_s,
            "sort_phase": sort_ph,
            "cover_fp64": cover_fp64(nq, ni),
            "cover_roofline": cover_rl,
            "request_latency": latency,
            "roofline": {"kernel": "k_join (overlap join + fused altitude/time filter)", "bound": "hbm",
                         "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS,
                         "hbm_copy_measured_GBs": copy_bw,
                         "frac_of_measured_copy": achieved / copy_bw if copy_bw else None,
                         "traffic": traffic["bytes_per_launch"] if traffic else None,
                         "traffic_source": traffic["source"] if traffic else None,
                         "algorithmic_bytes": join_bytes, "launch_ms": kern_avg_ms,
                         "counts": {"queries": nq, "C": c_tot, "P_touched": p_touched, "R": r_tot},
                         "survey_per_query_model": {"bytes": survey_bytes, "M": m_tot.value, "D": d_tot.value,
                                                    "equiv_GBs": survey_bytes / (kern_avg_ms * 1e-3) / 1e9}
                         if args.survey_model else None},
            "cpu_baseline": cpu,
            "parity": parity,
        }
        _PENDING[0] = result
    if leg:
        # BASELINE configs[2]'s layout timed by the same ranks after the
        # replica line's steps (the line's value stays the replica rate)
        rec = sharded_leg(args, ctx, D, dist, torch, dev, _lib, local, tunes, rank, world, nq, d_q, qargs, index,
                          icells, (i_alo, i_ahi, i_t0, i_t1), i_cells_t, exchange, native_wanted, pg_backend)
        if rank == 0:
            result["sharded"] = rec
    if rank == 0:
        # last: the per-request calls reuse the context's cover / search
        # buffers that `cells` and `pairs` point into
        if args.latency:
            stage("single-request latency")
            result["request_latency"] = request_latency(ctx, D, index, queries, qa, now)
        _PENDING[0] = None
        emit(result)
    ctx.L.dssg_index_free(index)
    if world > 1:
        dist.destroy_process_group()


def make_exchange(args, ctx, dist, torch, dev, rank, index, ranges, exchange, native_wanted, pg_backend, tag=""):
    """The sharded step's exchange: the library's own communicators (queries;
    pairs home on a second stream) when wanted, else -- or if any rank cannot
    open them (no RCCL to dlopen, init error; every rank falls back together,
    agreed by one all-reduce, and the line says so) -- the torch-collective
    exchange over RCCL (a subgroup beside the gloo control group) or staged
    through host memory (gloo rehearsals).  Returns (native, sharded, exchange)."""
    from dss_amd import _lib, shard
    native = sharded = None
    world = dist.get_world_size()
    if native_wanted:
        stage(tag + "native exchange init")
        ok = torch.ones(1)
        err = None
        # the ids travel once over the control group, with rank 0's success
        # flag: every rank takes part in every broadcast, and no rank starts a
        # communicator init another rank will not join
        uids = torch.zeros(2, _lib.COMM_ID_BYTES + 1, dtype=torch.uint8)
        if rank == 0:
            try:
                for k in range(2):
                    uids[k, :-1].copy_(torch.frombuffer(bytearray(shard.NativeComm.unique_id(ctx)), dtype=torch.uint8))
                    uids[k, -1] = 1
            except Exception as e:  # noqa: BLE001 -- reported in the result line
                err = f"{type(e).__name__}: {e}"
        dist.broadcast(uids, 0)
        if int(uids[:, -1].min()) == 1:
            try:
                comms = [shard.NativeComm(ctx, world, rank, bytes(uids[k, :-1].numpy())) for k in range(2)]
                native = shard.NativeShardedSearch(ctx, comms[0], index, ranges, xcomm=comms[1],
                                                   xstream=torch.cuda.Stream(device=dev))
            except Exception as e:  # noqa: BLE001 -- reported in the result line
                err = f"{type(e).__name__}: {e}"
                ok.zero_()
        else:
            err = err or "rank 0 could not make an RCCL id"
            ok.zero_()
        dist.all_reduce(ok, op=dist.ReduceOp.MIN)
        if ok.item() < 1:
            log(f"[rank {rank}] native exchange unavailable ({err}); using the torch exchange")
            native = None
            exchange = f"torch (native exchange init failed on some rank: {err})"
    if native is None:
        group = None
        if pg_backend != "nccl" and args.dist_backend == "nccl":
            group = dist.new_group(backend="nccl")
        sharded = shard.ShardedSearch(ctx, index, ranges, group=group, stage_host=group is None and pg_backend != "nccl")
    return native, sharded, exchange


_ORACLE_SAMPLE = {}  # this rank's oracle pair keys of its parity sample (cpu_baseline), for the sharded leg


def sharded_leg(args, ctx, D, dist, torch, dev, _lib, local, tunes, rank, world, nq, d_q, qargs, index, icells, iattrs,
                i_cells_t, exchange, native_wanted, pg_backend):
    """N > 1, replica mode: the cell-range shards BASELINE configs[2] names
    (partitioned like the reference's scd_cells_operations PK
    (cell_id, operation_id), pkg/scd/store/cockroach/store.go:140-147), timed
    by the same rank processes after the replica steps -- under torchrun
    there is no parent of ours to start a second set.  Each rank builds its
    shard, opens the library's RCCL communicators (the control group is gloo,
    so the library's RCCL is the process's only one), runs --warmup steps and
    then exactly --steps sharded steps (cover ahead on the other pipelines,
    route -> query all-to-all -> shard join -> pairs home on the exchange
    stream), barrier + synchronize around them, max over ranks.  Parity on
    every rank: its delivered pairs of its oracle sample == the oracle's pair
    keys kept from the replica leg (exact), and its whole delivered set ==
    the replica index's search of the same covering (count + checksum).
    Returns the `sharded` record; {"error": ...} if the leg raised (a hung
    collective ends the rank through the stage watchdog, LEG_LIMIT_S)."""
    import traceback

    from dss_amd import shard
    rec = {"layout": f"cell-range shards x{world}: the intent index split at posting quantiles into {world} S2 "
                     f"cell-id ranges (whole quads), one per GPU; queries routed to the shards owning their cells "
                     f"and pairs routed home by all-to-all"}
    shard_index = native = sharded = None
    workers = []
    try:
        stage("sharded leg: shard build")
        ranges = shard.cell_splitters(i_cells_t.cpu().numpy().view(np.uint64), world)
        tb = time.time()
        shard_index = D.build_index(ctx, icells, *iattrs, cell_range=ranges[rank])
        torch.cuda.synchronize()
        rec["index_build_s_rank0"] = time.time() - tb
        rec["postings_rank0"] = int(ctx.L.dssg_index_num_postings(shard_index))
        native, sharded, exchange = make_exchange(args, ctx, dist, torch, dev, rank, shard_index, ranges, exchange,
                                                  native_wanted, pg_backend, tag="sharded leg: ")
        rec["exchange"] = "the library's RCCL communicators (dssg_sharded_search_async_device)" \
            if native is not None else exchange

        def shard_search(cells, timed_phases=False):
            if native is not None:
                return native.step(cells.offs, cells.cells, nq, *qargs)
            return sharded.step(cells.offs, cells.cells, nq, *qargs, timed=timed_phases)

        stage("sharded leg: warmup")
        for _ in range(max(1, args.warmup)):
            shard_search(D.cover(ctx, d_q))
        torch.cuda.synchronize()
        workers, note = add_pipelines(args, torch, D, _lib, local, dev, tunes, d_q, None)
        stage("sharded leg: timed steps")
        el = timed(torch, dist, dev, world,
                   lambda: cover_ahead_steps(torch, D, ctx, workers, d_q, args.steps, shard_search))
        rec.update({"value": world * nq * args.steps / el, "unit": "queries/s", "ms_per_step": 1000.0 * el / args.steps,
                    "steps": args.steps, "warmup": max(1, args.warmup), "pipelines_per_gpu": 1 + len(workers),
                    "pipelines_note": note})
        for wctx, _ in workers:
            wctx.close()
        workers = []
        # one instrumented step: phases (max over ranks) and bytes moved
        stage("sharded leg: phases")
        names = ["route", "exchange_queries", "join", "route_pairs", "exchange_pairs"]
        ctx.L.dssg_set_timing(ctx.h, 1)
        if sharded is not None:
            sharded.times = {}
        cells = D.cover(ctx, d_q)
        out = shard_search(cells, True)
        torch.cuda.synchronize()
        ctx.L.dssg_set_timing(ctx.h, 0)
        if native is not None:
            ms, cnt = native.stats()
            moved = {k: cnt[k] for k in ("query_bytes_sent", "query_bytes_recv", "pair_bytes_sent", "pair_bytes_recv")}
            ph = [ms[k] for k in names]
        else:
            ph = [1000.0 * sharded.times.get(k, 0.0) for k in names]
            moved = dict(sharded.last_bytes)
        rec["phase_ms_max_over_ranks"] = dict(zip(names, allreduce_vals(dist, torch, ph, dist.ReduceOp.MAX)))
        rec["bytes_per_step_rank0"] = moved
        # parity
        stage("sharded leg: parity")
        gq, ge = sample_pairs_host(ctx, D, torch, dev, out, nq)
        got = (gq.astype(np.uint64) << np.uint64(32)) | ge.astype(np.uint64)
        n_s, okeys = _ORACLE_SAMPLE.get("n", 0), _ORACLE_SAMPLE.get("keys")
        o_ok = okeys is not None and np.array_equal(np.sort(got[gq < n_s]), okeys)
        rp = D.search(ctx, index, cells, *qargs)
        fq, fe = sample_pairs_host(ctx, D, torch, dev, rp, nq)
        want = (fq.astype(np.uint64) << np.uint64(32)) | fe.astype(np.uint64)
        w_ok = len(want) == len(got) and pair_checksum(want) == pair_checksum(got)
        local_v = [1.0 if o_ok else 0.0, 1.0 if w_ok else 0.0, float(n_s), float(len(got)),
                   float(sum(moved.values()))]
        mins = allreduce_vals(dist, torch, local_v, dist.ReduceOp.MIN)
        sums = allreduce_vals(dist, torch, local_v, dist.ReduceOp.SUM)
        rec["bytes_per_step_all_ranks"] = sums[4]
        rec["pairs_per_step_all_ranks"] = sums[3]
        rec["parity"] = {"oracle_all_ranks_equal": bool(mins[0] == 1.0), "oracle_queries_all_ranks": int(sums[2]),
                         "oracle_check": "per rank: its delivered pairs of the queries in its oracle sample (rank 0: "
                                         "the CPU baseline's, the others: --parity-sample) == the oracle's pairs of "
                                         "those queries, exactly",
                         "all_ranks_equal": bool(mins[1] == 1.0),
                         "whole_index_check": "per rank: count + sum(splitmix64(q << 32 | e)) of the delivered pairs "
                                              "== the replica index's search of the same covering"}
    except Exception as e:  # noqa: BLE001 -- reported in the line; the replica line stands
        log(traceback.format_exc())
        rec["error"] = f"{type(e).__name__}: {e}"
    finally:
        for wctx, _ in workers:
            wctx.close()
        if native is not None:
            native.close()
        if shard_index is not None:
            ctx.L.dssg_index_free(shard_index)
        torch.cuda.synchronize()
    return rec


def mix64(x: np.ndarray) -> np.ndarray:
    """splitmix64 finalizer (uint64, wrapping): an order-independent pair-set
    checksum is sum(mix64(q << 32 | e)) mod 2^64."""
    with np.errstate(over="ignore"):
        z = x.astype(np.uint64) + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def pair_checksum(keys: np.ndarray) -> int:
    tot = np.uint64(0)
    with np.errstate(over="ignore"):
        for k in range(0, len(keys), 1 << 24):
            tot = tot + mix64(keys[k:k + (1 << 24)]).sum(dtype=np.uint64)
    return int(tot)


def sharded_report(args, ctx, D, dist, torch, sh, native, step, full, i_offs_t, i_cells_t, ranges, rank, world, nq,
                   ni, n_post, build_s, value, ms_per_step, qargs, queries, qa, intents, ia, now, exchange="torch",
                   replica=None, pipelines=1, pipe_note=None):
    """Phase breakdown (synchronised passes, max over ranks), the exchanged
    bytes, the shard join's roofline, and parity: every rank's delivered pair
    set (a) == a whole-index search of its own queries (count +
    order-independent checksum) and (b) against the oracle, cells and pairs
    compared exactly (rank 0: the timed CPU baseline on its --cpu-sample; the
    others: --parity-sample queries)."""
    import ctypes as C

    from dss_amd import workload as W
    dev = f"cuda:{torch.cuda.current_device()}"
    names = ["route", "exchange_queries", "join", "route_pairs", "exchange_pairs"]
    stage("sharded phases")
    ctx.L.dssg_set_timing(ctx.h, 1)
    if sh is not None:
        sh.times = {}
    reps = 5
    cover_ms, kern_ms, ph_sum, moved = [], [], dict.fromkeys(names, 0.0), {}
    shard_rows = shard_cells = shard_pairs = touched = 0
    for _ in range(reps):
        cells, out = step(timed=True)
        ca, cb, cc = C.c_double(), C.c_double(), C.c_double()
        ctx.L.dssg_phase_times(ctx.h, C.byref(ca), C.byref(cb), C.byref(cc))
        cover_ms.append(ca.value)
        kern_ms.append(cc.value)
        if native is not None:
            ms, cnt = native.stats()
            for k in names:
                ph_sum[k] += ms[k]
            moved = {k: cnt[k] for k in ("query_bytes_sent", "query_bytes_recv", "pair_bytes_sent", "pair_bytes_recv")}
            shard_rows, shard_cells, shard_pairs, touched = cnt["rows"], cnt["cells"], cnt["shard_pairs"], cnt["touched"]
    ctx.L.dssg_set_timing(ctx.h, 0)
    if native is None:
        ph_sum = {k: 1000.0 * sh.times.get(k, 0.0) for k in names}
        moved = dict(sh.last_bytes)
        shard_rows, shard_cells, shard_pairs, touched = sh.last_rows, sh.last_recv_ncells, sh.last_shard_pairs, \
            sh.last_touched
    torch.cuda.synchronize()
    ph = [float(np.mean(cover_ms))] + [ph_sum[k] / reps for k in names] + [float(np.mean(kern_ms))]
    phase = dict(zip(["cover"] + names + ["join_kernel"], allreduce_vals(dist, torch, ph, dist.ReduceOp.MAX)))
    # shard join roofline (DESIGN.md s5 byte model over what this shard joined)
    jb = 24 * shard_rows + 8 * shard_cells + 28 * touched + 8 * shard_pairs
    kern = float(np.mean(kern_ms))
    n_out = int(out.numel()) if torch.is_tensor(out) else int(out.n)
    local = [jb / (kern * 1e-3) / 1e9, shard_rows, shard_cells, shard_pairs, n_out, sum(moved.values()),
             moved.get("pair_bytes_recv", 0)]
    mins = allreduce_vals(dist, torch, local, dist.ReduceOp.MIN)
    sums = allreduce_vals(dist, torch, local, dist.ReduceOp.SUM)
    # parity (a): whole-index search of this rank's own queries (the same
    # covering `cells` the last sharded step routed)
    parity = {}
    gq, ge = sample_pairs_host(ctx, D, torch, dev, out, nq)
    if full is not None:
        pairs = D.search(ctx, full, cells, *qargs)
        fq, fe = sample_pairs_host(ctx, D, torch, dev, pairs, nq)
        want = (fq.astype(np.uint64) << np.uint64(32)) | fe.astype(np.uint64)
        got = (gq.astype(np.uint64) << np.uint64(32)) | ge.astype(np.uint64)
        ok = len(want) == len(got) and pair_checksum(want) == pair_checksum(got)
        t = allreduce_vals(dist, torch, [1.0 if ok else 0.0], dist.ReduceOp.MIN)
        parity["whole_index_check"] = "per rank: count + sum(splitmix64(q << 32 | e)) of the delivered pairs == a " \
                                      "whole-index GPU search of the rank's own queries"
        parity["all_ranks_equal"] = bool(t[0] == 1.0)
        del want, got, fq, fe
        ctx.L.dssg_index_free(full)
    # parity (b) + the CPU baseline: the oracle on every rank
    stage("oracle parity" + (" + cpu baseline" if rank == 0 else ""))
    cpu, opar = oracle_leg(args, ctx, D, dist, torch, dev, rank, world, queries, qa, intents, ia, now, i_offs_t,
                           i_cells_t, cells, None, host_pairs=(gq, ge))
    if opar:
        parity.update(opar)
    traffic = pmc_traffic("k_join", nq, ni, world=world, mode="sharded")
    if rank != 0:
        return
    result = {
        "metric": "4D conflict queries/sec vs N-intent airspace",
        "value": value,
        "unit": "queries/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (seeded SURVEY s8(d) generator; no datasets)",
        "config": {"workload": f"configs[{args.config}]: {nq} query footprints/GPU/step vs a {ni}-entity index "
                               f"sharded by S2 cell range over {world} GPU(s), {W.CONFIG_NAMES[args.config]}, S2 level 13",
                   "queries_per_gpu_step": nq, "intents": ni, "postings_rank0": n_post,
                   "parallelism": f"cell-range shards x{world}; queries routed to shards and pairs routed home by "
                                  f"all-to-all ({'the library RCCL communicators' if exchange == 'native' else exchange})",
                   "exchange": exchange, "scale": args.scale, "pipelines_per_gpu": pipelines,
                   "pipelines_note": pipe_note or ("the other pipelines cover ahead; one host thread issues every "
                                                   "collective (route, query all-to-all, join on the step stream; "
                                                   "pairs home on the exchange stream, overlapping the next step)")},
        "replica": replica,
        "coverings_per_s": world * nq / (phase["cover"] * 1e-3),
        "phase_ms_max_over_ranks": phase,
        "exchanged": {"bytes_per_step_rank0": moved, "bytes_per_step_all_ranks": sums[5],
                      "pair_bytes_per_returned_pair": sums[6] / max(1.0, sums[4]),
                      "pair_format": "8 B (home-local query << 32 | entity) per pair that crosses ranks; a rank's "
                                     "own queries' pairs move no bytes"},
        "routed": {"rows_total": sums[1], "rows_min_rank": mins[1], "cells_total": sums[2],
                   "pairs_total": sums[4]},
        "index_build_s": build_s,
        "roofline": {"kernel": "k_join on the shard (overlap join + fused altitude/time filter)", "bound": "hbm",
                     "achieved": local[0], "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": local[0] / HBM_PEAK_GBS,
                     "traffic": traffic["bytes_per_launch"] if traffic else None,
                     "traffic_source": traffic["source"] if traffic else None, "rank": 0,
                     "algorithmic_bytes": jb, "launch_ms": kern,
                     "counts": {"rows": shard_rows, "C": shard_cells, "P_touched": touched, "R": shard_pairs}},
        "cpu_baseline": cpu,
        "parity": parity,
    }
    emit(result)


def sample_pairs_host(ctx, D, torch, dev, pairs, n):
    """(q, e) host arrays of the pairs whose query index is < n, filtered on
    the GPU; `pairs` is a _lib.Pairs (device q / e arrays) or an int64
    tensor packed (q << 32 | e)."""
    import ctypes as C
    if torch.is_tensor(pairs):
        sel = pairs[(pairs >> 32) < n]
        h = sel.cpu().numpy()
        return (h >> 32).astype(np.uint32), (h & 0xFFFFFFFF).astype(np.uint32)
    m = int(pairs.n)
    if m == 0:
        return np.zeros(0, np.uint32), np.zeros(0, np.uint32)
    q = torch.empty(m, dtype=torch.int32, device=dev)
    e = torch.empty(m, dtype=torch.int32, device=dev)
    torch.cuda.synchronize()
    ctx.check(ctx.L.dssg_copy_device(ctx.h, C.c_void_p(q.data_ptr()), C.c_void_p(pairs.q), 4 * m, D._stream_ptr()))
    ctx.check(ctx.L.dssg_copy_device(ctx.h, C.c_void_p(e.data_ptr()), C.c_void_p(pairs.e), 4 * m, D._stream_ptr()))
    # (the copies run on the library stream when torch's is the default one:
    # a device-wide sync orders them before torch reads the tensors)
    torch.cuda.synchronize()
    keep = q < n  # query ids < 2^24: no sign issue in int32
    return q[keep].cpu().numpy().view(np.uint32), e[keep].cpu().numpy().view(np.uint32)


def oracle_leg(args, ctx, D, dist, torch, dev, rank, world, queries, qa, intents, ia, now, i_offs_t, i_cells_t, cells,
               pairs, host_pairs=None):
    """The oracle on every rank, after the timed steps: rank 0 runs the CPU
    baseline (timed; --cpu-sample queries, -1 = the config's auto sample),
    every other rank --parity-sample queries of its own batch; each compares
    the oracle's cells and pairs of its sample with its GPU step exactly
    (`cells` = the step's covering, `pairs` or `host_pairs` its pairs).  The
    flags are reduced over ranks.  Returns (rank 0's cpu_baseline or None,
    parity dict or None)."""
    n = args.cpu_sample if rank == 0 else args.parity_sample
    if n < 0:
        auto = AUTO_CPU_SAMPLE.get(args.config)
        n = queries.n if auto is None else auto
    n = min(n, queries.n)
    if world > 1:  # one build of the checker (a no-op when prebuilt), then every rank loads it
        from oracle import oracle as O
        if rank == 0:
            O.build()
        dist.barrier()
    cpu = parity = None
    if n > 0 and not (args.no_verify and rank != 0):
        g_offs = D.copy_back(ctx, cells.offs, n + 1, np.int64)
        g_c = D.copy_back(ctx, cells.cells, int(g_offs[-1]), np.uint64)
        gq, ge = host_pairs if host_pairs is not None else sample_pairs_host(ctx, D, torch, dev, pairs, n)
        keep = gq < n
        gq, ge = gq[keep], ge[keep]
        cpu, parity = cpu_baseline(args, rank, n, intents, ia, queries, qa, now,
                                   lambda sc, sub: intent_csr(torch, i_offs_t, i_cells_t, sc, subset=sub),
                                   g_offs, g_c, gq, ge)
    if world > 1:
        ok = parity is not None and parity["cells_equal"] and parity["pairs_equal"]
        f = [1.0 if ok else 0.0, n, parity["gpu_pairs"] if parity else 0]
        fmin = allreduce_vals(dist, torch, f, dist.ReduceOp.MIN)
        fsum = allreduce_vals(dist, torch, f, dist.ReduceOp.SUM)
        parity = dict(parity or {}, rank0_check="oracle cells + pairs of rank 0's sample (exact)",
                      oracle_all_ranks_equal=bool(fmin[0] == 1.0), oracle_ranks=world,
                      oracle_queries_all_ranks=int(fsum[1]), oracle_pairs_all_ranks=int(fsum[2]),
                      oracle_note=f"every rank compared the oracle's cells and pairs of its first queries "
                                  f"(rank 0: {n}, the others: --parity-sample {args.parity_sample}) with what its "
                                  f"GPU step delivered, exactly")
    return cpu, parity


def copy_bandwidth(ctx, torch, dev, nbytes=4 << 30):
    """Measured device copy (the library's 16-B-vector copy kernel,
    dssg_copy_device) in GB/s of read + write, beside the 8 TB/s spec
    (SURVEY.md s8(d)); HIP events on the copy's own stream."""
    import ctypes as C
    try:
        a = torch.empty(nbytes // 8, dtype=torch.int64, device=dev)
        b = torch.empty_like(a)
    except RuntimeError:
        return None
    a.fill_(1)
    torch.cuda.synchronize()
    st = torch.cuda.Stream(device=dev)  # events and the copy on one explicit stream
    times = []
    for _ in range(6):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        ctx.check(ctx.L.dssg_copy_device(ctx.h, C.c_void_p(b.data_ptr()), C.c_void_p(a.data_ptr()), nbytes,
                                         C.c_void_p(st.cuda_stream)))
        e1.record(st)
        e1.synchronize()
        times.append(e0.elapsed_time(e1))
    del a, b
    torch.cuda.empty_cache()
    return 2 * nbytes / (float(np.median(times[1:])) * 1e-3) / 1e9


LARGE_POSTINGS = 600_000_000  # above: no host copy of the intents' cells, no standalone sort-phase run


def cover_chunked(ctx, D, torch, fp, dev, chunk=4_000_000):
    """Cover footprints chunk by chunk on the GPU; the CSR lands in torch
    tensors (offs int64 [n+1], cells int64 bit patterns [P])."""
    import ctypes as C
    n = fp.n
    offs = torch.zeros(n + 1, dtype=torch.int64, device=dev)
    parts = []
    for a in range(0, n, chunk):
        b = min(n, a + chunk)
        sub = fp.slice(a, b) if (a, b) != (0, n) else fp
        d = D.DeviceFootprints.upload(sub, dev)
        c = D.cover(ctx, d)
        o = torch.empty(b - a + 1, dtype=torch.int64, device=dev)
        x = torch.empty(max(1, int(c.total_cells)), dtype=torch.int64, device=dev)
        ctx.check(ctx.L.dssg_copy_device(ctx.h, C.c_void_p(o.data_ptr()), C.c_void_p(c.offs), 8 * (b - a + 1),
                                         D._stream_ptr()))
        if c.total_cells:
            ctx.check(ctx.L.dssg_copy_device(ctx.h, C.c_void_p(x.data_ptr()), C.c_void_p(c.cells),
                                             8 * int(c.total_cells), D._stream_ptr()))
        parts.append((a, b, o, x[: int(c.total_cells)]))
        del d
    torch.cuda.synchronize()
    total = sum(int(x.numel()) for _, _, _, x in parts)
    cells = torch.empty(max(1, total), dtype=torch.int64, device=dev)
    base = 0
    for a, b, o, x in parts:
        offs[a + 1: b + 1] = o[1:] + base
        cells[base: base + x.numel()] = x
        base += int(x.numel())
    parts = x = o = None
    torch.cuda.synchronize()
    torch.cuda.empty_cache()  # the chunk copies' memory back to the device for the index build
    return offs, cells[:total]


def intent_csr(torch, offs_t, cells_t, sample_cells, subset=False):
    """Host CSR of the intents the CPU baseline's index needs: all of them,
    or -- for airspaces past LARGE_POSTINGS -- only those sharing a cell with
    the sample's queries (the only ones that can pair with them), found on the
    GPU.  Returns (offs, cells, entity ids)."""
    if cells_t.numel() <= LARGE_POSTINGS and not subset:
        offs = offs_t.cpu().numpy()
        return offs, cells_t.cpu().numpy().view(np.uint64), np.arange(len(offs) - 1, dtype=np.int64)
    dev = cells_t.device
    # int64 order (cell ids of faces 4, 5 are negative as int64): searchsorted needs it
    sc = torch.as_tensor(np.unique(np.asarray(sample_cells, np.uint64).view(np.int64)), device=dev)
    hit = torch.zeros(offs_t.numel() - 1, dtype=torch.bool, device=dev)
    step = 1 << 26  # chunked: a few GB of scratch beside the resident index
    for a in range(0, cells_t.numel(), step):
        x = cells_t[a: a + step]
        i = torch.searchsorted(sc, x).clamp_(max=sc.numel() - 1)
        pos = torch.nonzero(sc[i] == x).squeeze(1) + a
        del i
        hit[torch.searchsorted(offs_t, pos, right=True) - 1] = True
        del pos
    ents = torch.nonzero(hit).squeeze(1)
    del hit
    offs_parts, cell_parts, base = [np.zeros(1, np.int64)], [], 0
    for a in range(0, ents.numel(), 1 << 20):  # the selected entities' cells, block by block to the host
        en = ents[a: a + (1 << 20)]
        starts, lens = offs_t[en], offs_t[en + 1] - offs_t[en]
        o = torch.cumsum(lens, 0)
        idx = torch.repeat_interleave(starts - (o - lens), lens) + torch.arange(int(o[-1]), device=dev)
        cell_parts.append(cells_t[idx].cpu().numpy().view(np.uint64))
        offs_parts.append(o.cpu().numpy() + base)
        base += int(o[-1])
    return np.concatenate(offs_parts), np.concatenate(cell_parts), ents.cpu().numpy()


def sort_phase(ctx, torch, dev, i_offs_t, i_cells_t):
    """Sort-phase roofline: the index build's (cell, entity)
    radix sort (radix.hip) on this airspace's own postings, timed with HIP
    events on the library's stream.  Algorithmic bytes: 24 B per posting
    (8 B key + 4 B payload, read and written once)."""
    import ctypes as C
    P = int(i_cells_t.numel())
    if P == 0:
        return None
    keys = i_cells_t
    n = i_offs_t.numel() - 1
    vals = torch.repeat_interleave(torch.arange(n, dtype=torch.int32, device=dev), i_offs_t[1:] - i_offs_t[:-1])
    ko, vo = torch.empty_like(keys), torch.empty_like(vals)
    torch.cuda.synchronize()
    ms = C.c_double(0)
    times = []
    for _ in range(6):
        ctx.check(ctx.L.dssg_radix_sort_device(ctx.h, 8, P, 64, C.c_void_p(keys.data_ptr()), C.c_void_p(ko.data_ptr()),
                                               C.c_void_p(vals.data_ptr()), C.c_void_p(vo.data_ptr()), None,
                                               C.byref(ms)))
        times.append(ms.value)
    t = float(np.median(times[1:]))
    alg = 24 * P
    passes = 4
    phys = 32 * P  # per pass: k_rs_hist reads the 8-B keys, k_rs_scatter reads and writes key + value (12 + 12 B)
    return {"kernel": "radix sort of (cell, entity) postings (k_rs_hist/k_rs_scan/k_rs_scatter)", "bound": "hbm",
            "postings": P, "ms": t, "achieved": alg / t / 1e6, "peak": 8000.0, "unit": "GB/s",
            "frac": alg / t / 1e6 / 8000.0, "algorithmic_bytes": alg,
            "passes": passes, "physical_bytes_per_pass": phys,
            "per_pass_physical_GBs": phys / (t / passes) / 1e6,
            "per_pass_physical_frac": phys / (t / passes) / 1e6 / 8000.0,
            "note": "level-13 ids vary in bits 35..63 only: 4 digit passes of <= 8 bits; the 24-B model counts one "
                    "read + one write of each posting, each pass moves 32 B of it"}


def touched_postings(ctx, D, index, cells):
    """Postings of the distinct cells the batch's queries cover, each counted
    once (dssg_search_touched_device)."""
    import ctypes as C
    out = C.c_int64()
    ctx.check(ctx.L.dssg_search_touched_device(ctx.h, index, cells.n, C.c_void_p(cells.offs), C.c_void_p(cells.cells),
                                               D._stream_ptr(), C.byref(out)))
    return int(out.value)


def index_info(ctx, index):
    import ctypes as C
    v = [C.c_int64() for _ in range(6)]
    ctx.check(ctx.L.dssg_index_info(index, *[C.byref(x) for x in v]))
    d = dict(zip(["postings", "groups", "long_duration_postings", "long_footprint_postings", "max_group_postings",
                  "dcap_us"], [x.value for x in v]))
    d["grain_level"] = int(ctx.L.dssg_index_grain(index))  # 12: (entity, quad) postings; 13: (entity, cell)
    return d


def pmc_traffic(kernel, nq, ni, world=1, mode="replica"):
    """HBM bytes per launch of `kernel` from the committed rocprofv3 PMC
    summary (tools/pmc_summary.py --json; FETCH_SIZE x2 + WRITE_SIZE, the
    gfx950 correction of MI355X_MICROARCH.md s HBM), if one exists for this
    workload size."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return None
    if d.get("queries") != nq or d.get("intents") != ni:
        return None
    if mode == "sharded" and world > 1:
        # a shard's k_join (rank 0's cell range, the queries routed to it),
        # profiled per world size in a same-device rehearsal
        d = d.get("sharded", {}).get(str(world))
        if not d:
            return None
    k = d.get("kernels", {}).get(kernel)
    if not k:
        return None
    return {"bytes_per_launch": k["hbm_bytes_per_launch"], "source": d.get("source", path)}


_POS_IJ = np.array([[(0x874B78B4 >> (8 * o + 2 * p)) & 3 for p in range(4)] for o in range(4)], np.uint64)
_POS_OR = np.array([(0xC1 >> (2 * p)) & 3 for p in range(4)], np.uint64)


def decode13(cells):
    """Level-13 S2 cell ids -> (face, i, j) (cellid.go faceIJOrientation,
    one level at a time; the same walk as search.hip decode13)."""
    c = np.asarray(cells, np.uint64)
    face = (c >> np.uint64(61)).astype(np.int64)
    o = (face & 1).astype(np.uint64)
    i = np.zeros(len(c), np.int64)
    j = np.zeros(len(c), np.int64)
    for lvl in range(13):
        pos = (c >> np.uint64(59 - 2 * lvl)) & np.uint64(3)
        ij = _POS_IJ[o, pos]
        i = (i << 1) | (ij >> np.uint64(1)).astype(np.int64)
        j = (j << 1) | (ij & np.uint64(1)).astype(np.int64)
        o = o ^ _POS_OR[pos]
    return face, i, j


def cover_roofline(fp, offs, cells, cover_ms):
    """SURVEY.md s8(d)'s covering model: F_p = 48 E_p (|C_p| + |R_p|) + 40 V_p
    summed over the step's footprints, against the FP64 vector peak.  E_p =
    V_p = the loop's vertices (a circle's RegularLoop has 20; the closing
    edge included), C_p = its output cells, R_p = the level-13 edge
    neighbours of C_p outside C_p (a neighbour across a cube face is counted
    as rejected: exact within a face, an over-count of at most the cells
    that touch a face edge)."""
    n = len(offs) - 1
    if n == 0 or len(cells) == 0:
        return None
    nv = np.where(fp.kind == 1, 20, np.diff(fp.voff)).astype(np.int64)
    cp = np.diff(offs).astype(np.int64)
    owner = np.repeat(np.arange(n, dtype=np.int64), cp)
    face, i, j = decode13(cells)
    key = (owner << 30) | (face << 26) | (i << 13) | j
    own = np.sort(key)
    nb = []
    for di, dj in ((1, 0), (-1, 0), (0, 1), (0, -1)):
        ii, jj = i + di, j + dj
        inside = (ii >= 0) & (ii < 8192) & (jj >= 0) & (jj < 8192)
        k = (owner << 30) | (face << 26) | (np.clip(ii, 0, 8191) << 13) | np.clip(jj, 0, 8191)
        nb.append(np.where(inside, k, -1 - np.arange(len(k), dtype=np.int64) * 4 - len(nb)))  # cross-face: unique
    nb = np.unique(np.concatenate(nb))
    pos = np.searchsorted(own, nb)
    hit = (pos < len(own)) & (own[np.minimum(pos, len(own) - 1)] == nb)
    rej = nb[~hit]
    rp = np.zeros(n, np.int64)
    inface = rej >= 0
    np.add.at(rp, rej[inface] >> 30, 1)
    # cross-face neighbours: attribute to their cells' footprints
    xf = (-1 - rej[~inface]) // 4
    np.add.at(rp, owner[xf], 1)
    flops = float(np.sum(48 * nv * (cp + rp) + 40 * nv))
    achieved = flops / (cover_ms * 1e-3) / 1e12
    return {"model": "SURVEY s8(d): F_p = 48 E_p (|C_p| + |R_p|) + 40 V_p", "bound": "fp64-valu",
            "flops": flops, "achieved": achieved, "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
            "frac": achieved / FP64_PEAK_TFLOPS, "cover_ms": cover_ms,
            "counts": {"footprints": n, "E": int(nv.sum()), "C": int(cp.sum()), "R": int(rp.sum())}}


def request_latency(ctx, D, index, queries, qa, now, n_alone=3000, callers=64, seconds=2.0):
    """The per-RPC path the reference runs (one covering + one SQL search per
    request, pkg/scd/operations_handler.go:118-168), driven by native caller
    threads (tools/loadgen.c; Python threads could not issue the calls at
    this rate):
      alone:  one request at a time through the unbatched ABI
              (dssg_cover_batch, then dssg_search_operations: host buffers in
              and out, the capacity protocol), as the Go binding calls it;
      single: one caller through the micro-batcher (dssg_batcher);
      batched: `callers` threads issuing requests back to back through the
              batcher (2 workers, each its own context and stream).
    p50 / p99 request latency in ms and requests/s."""
    import ctypes as C
    from dss_amd.store import Batcher
    lg = C.CDLL(os.path.join(ROOT, "tools", "libloadgen.so"))
    vp = C.c_void_p
    n = queries.n
    a = lambda x, t: np.ascontiguousarray(x, dtype=t)  # noqa: E731
    kind, voff = a(queries.kind, np.int32), a(queries.voff, np.int64)
    la, ln, rad = a(queries.lat, np.float64), a(queries.lng, np.float64), a(queries.radius_m, np.float32)
    alo, ahi, t0, t1 = a(qa.alt_lo, np.float32), a(qa.alt_hi, np.float32), a(qa.t0, np.int64), a(qa.t1, np.int64)
    work = [n] + [x.ctypes.data_as(vp) for x in (kind, voff, la, ln, rad, alo, ahi, t0, t1)] + [int(now)]
    lg.dssl_alone.argtypes = [vp, vp, C.c_int64, C.c_int64] + [vp] * 9 + [C.c_int64, vp, vp]
    lg.dssl_batched.argtypes = [vp, C.c_int, C.c_double, C.c_int64] + [vp] * 9 + [C.c_int64, C.c_int64, vp, vp, vp,
                                                                                    vp, vp]
    lat_a = np.zeros(n_alone)
    nerr = C.c_int64()
    ctx.check(lg.dssl_alone(ctx.h, index, n_alone, *work, lat_a.ctypes.data_as(vp), C.byref(nerr)))
    alone = lat_a[min(200, n_alone // 4):]
    import types
    b = Batcher(types.SimpleNamespace(h=index), max_batch=4096, max_wait_us=0)  # (an index handle holder)

    def run(threads, secs):
        cap = 1 << 22
        lat = np.zeros(cap)
        ns, nr, ne, wall = C.c_int64(), C.c_int64(), C.c_int64(), C.c_double()
        nreq0, nb0 = b.stats()
        ctx.check(lg.dssl_batched(b.h, threads, secs, *work, cap, lat.ctypes.data_as(vp), C.byref(ns), C.byref(nr),
                                  C.byref(ne), C.byref(wall)))
        nreq1, nb1 = b.stats()
        lat = lat[: ns.value]
        return {"callers": threads, "requests": int(nr.value), "errors": int(ne.value),
                "batches": int(nb1 - nb0), "mean_batch": float((nreq1 - nreq0) / max(1, nb1 - nb0)),
                "p50_ms": float(np.percentile(lat, 50)), "p99_ms": float(np.percentile(lat, 99)),
                "requests_per_s": float(nr.value / wall.value)}
    run(1, 0.3)  # warm the workers' contexts
    single = run(1, 1.0)
    batched = run(callers, seconds)
    b.close()
    return {"alone": {"requests": len(alone), "errors": int(nerr.value), "p50_ms": float(np.percentile(alone, 50)),
                      "p99_ms": float(np.percentile(alone, 99)), "requests_per_s": float(1000.0 / alone.mean())},
            "single": single, "batched": batched,
            "note": "one request = cover 1 footprint + searchOperations, host buffers in and out (the RPC path); "
                    "native caller threads (tools/loadgen.c); batched: dssg_batcher, 2 workers, no fixed wait"}


def cover_fp64(nq, ni):
    """FP64 VALU throughput of the covering kernels (the
    covering is FP64-VALU-bound) from the committed rocprofv3 pass
    (tools/fp64_summary.py: 64 x (2 FMA + ADD + MUL) F64 wave instructions
    per launch over the launch's duration), if one exists for this size."""
    try:
        with open(os.path.join(ROOT, "profiles", "fp64_cover.json")) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return None
    if d.get("queries") != nq or d.get("intents") != ni:
        return None
    top = max(d["kernels"].items(), key=lambda kv: kv[1]["avg_ms"])
    return {"kernel": top[0], "bound": "fp64-valu", "achieved": top[1]["tflops"], "peak": d["peak_tflops"],
            "unit": "TFLOP/s", "frac": top[1]["frac_of_fp64_peak"], "source": d["source"],
            "all": {k: round(v["tflops"], 2) for k, v in d["kernels"].items() if v["tflops"] > 0.5}}


def cpu_info():
    """Host CPU facts for the baseline line: model (lscpu / /proc/cpuinfo),
    logical CPUs of the machine (nproc) and of this process (affinity)."""
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        aff = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        aff = os.cpu_count() or 1
    return {"model": model, "nproc": os.cpu_count(), "affinity": aff}


def cpu_threads(args):
    if args.cpu_threads > 0:
        return args.cpu_threads
    info = cpu_info()
    share = info["affinity"]
    omp = os.environ.get("OMP_NUM_THREADS")
    if omp and omp.isdigit() and int(omp) > 0:
        share = min(share, int(omp))
    return max(1, share)


# CPU-baseline sample per config when --cpu-sample is -1 (auto): the oracle's
# cost per query grows with the airspace density, so the bounded samples keep
# the baseline near 10-30 s of CPU work on 16 cores.
AUTO_CPU_SAMPLE = {0: None, 1: None, 2: None, 3: None, 4: 20000}


def cpu_baseline(args, rank, n, intents, ia, queries, qa, now, intent_csr_fn, g_offs, g_c, gq, ge):
    """The CPU restatement (oracle/, kind "port": pthreads over the process's
    CPU share) on the first n queries of the rank's batch: cover them, search
    them against the intents' posting list (built untimed; for the largest
    airspaces, and on ranks other than 0, only the intents sharing a cell
    with the sample, which are the only ones that can pair with it), and
    compare every cell and every pair with the GPU step's (g_offs / g_c: the
    GPU covering of those queries, gq / ge: the GPU pairs with q < n).  Rank
    0 also reports the timing as the baseline: queries/s on `cores` threads,
    the one-thread rate and a per-request sample."""
    from oracle import oracle as O
    O.build()
    sub = queries if n == queries.n else queries.subset(np.arange(n))
    th = cpu_threads(args)
    t0 = time.perf_counter()
    qo, qc, _, _ = O.cover_batch(sub.kind, sub.voff, sub.lat, sub.lng, sub.radius_m, nthreads=th)
    t1 = time.perf_counter()
    stage(f"oracle: {n} queries covered in {t1 - t0:.1f}s; intents for the oracle index")
    i_offs, i_cells, ents = intent_csr_fn(qc, rank != 0)
    stage(f"oracle: index over {len(ents)} intents, {len(i_cells)} postings")
    sel = lambda a: a[ents] if len(ents) != len(a) else a  # noqa: E731
    idx = O.Index(i_offs, i_cells, sel(ia.alt_lo), sel(ia.alt_hi), sel(ia.t0), sel(ia.t1))
    tlo = np.maximum(qa.t0[:n], now)
    t2 = time.perf_counter()
    stage("oracle: search")
    rq, re = idx.search(qo, qc, qa.alt_lo[:n], qa.alt_hi[:n], tlo, qa.t1[:n], nthreads=th)
    t3 = time.perf_counter()
    stage(f"oracle: search {t3 - t2:.1f}s; parity")
    re = ents[re]
    gk = np.sort((gq.astype(np.uint64) << np.uint64(32)) | ge.astype(np.uint64))
    ok = (rq.astype(np.uint64) << np.uint64(32)) | re.astype(np.uint64)
    ok.sort()
    _ORACLE_SAMPLE.update(n=n, keys=ok)  # (the sharded leg checks its delivered pairs against these)
    parity = None
    if not args.no_verify:
        parity = {"queries": n, "of_batch": queries.n, "cells_equal": bool(np.array_equal(g_offs, qo) and
                                                                            np.array_equal(g_c, qc)),
                  "pairs_equal": bool(np.array_equal(gk, ok)), "gpu_pairs": int(len(gk)), "oracle_pairs": int(len(ok)),
                  "cells": int(len(qc)), "unique": bool(len(gk) == 0 or np.all(gk[1:] != gk[:-1]))}
    if rank != 0 or args.cpu_sample == 0:
        return None, parity
    # the reference's per-request shape on the CPU: one covering + one search
    # per request, one thread (ctypes call overhead included, ~10 us); the
    # same loop gives the one-thread rate
    req_ms = []
    for k in range(min(400, n)):
        v0, v1 = int(sub.voff[k]), int(sub.voff[k + 1])
        tr = time.perf_counter()
        o1, c1, _, _ = O.cover_batch(sub.kind[k:k + 1], np.array([0, v1 - v0]), sub.lat[v0:v1], sub.lng[v0:v1],
                                     sub.radius_m[k:k + 1], nthreads=1)
        idx.search(o1, c1, qa.alt_lo[k:k + 1], qa.alt_hi[k:k + 1], tlo[k:k + 1], qa.t1[k:k + 1], nthreads=1)
        req_ms.append(1000.0 * (time.perf_counter() - tr))
    info = cpu_info()
    secs = (t1 - t0) + (t3 - t2)
    one_thread = 1000.0 / float(np.mean(req_ms)) if req_ms else None
    cpu = {"value": n / secs, "unit": "queries/s", "cores": th, "kind": "port",
           "sample": f"{n} of the step's {queries.n} queries (cover + search) vs the {intents.n}-intent index"
                     + ("" if len(ents) == intents.n else f" (the {len(ents)} intents sharing a cell with the sample)"),
           "coverings_per_s": n / (t1 - t0), "seconds": secs, "cpu_model": info["model"],
           "single_request": {"requests": len(req_ms), "p50_ms": float(np.percentile(req_ms, 50)),
                              "p99_ms": float(np.percentile(req_ms, 99)), "threads": 1},
           "one_thread_queries_per_s": one_thread,
           "all_affinity_estimate": {"cpus": info["affinity"],
                                     "queries_per_s_upper_bound": (n / secs) / th * info["affinity"],
                                     "how": "the measured rate per thread x every CPU in the process's affinity mask "
                                            "(linear scaling: an upper bound); not run, since the GPU box's pool "
                                            "gives a process a CPU share of OMP_NUM_THREADS"},
           "nproc": info["nproc"], "affinity_cpus": info["affinity"],
           "threads_note": "threads = the process's CPU share on the GPU box (OMP_NUM_THREADS / affinity)"}
    return cpu, parity


if __name__ == "__main__":
    main()
