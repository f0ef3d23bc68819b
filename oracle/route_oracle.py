"""Test infrastructure (the checker, never the product): a numpy restatement
of the cell-range routing protocol of include/dssgpu.h / route.hip -- the
fused [rows | cells] query segments, the source-major unpack, and the pairs
home with the rank's own pairs kept out of the exchange.  The CPU world-2
test (tests/test_shard.py) drives the product's protocol through it over
gloo, with the oracle's search standing in for the shard join.

Reference partitioning: scd_cells_operations keyed (cell_id, operation_id),
range-split by CockroachDB (/root/reference/pkg/scd/store/cockroach/
store.go:140-147); the SQL layer fans `cell_id = ANY($cells)` out to the
ranges (operations.go:384-390).
"""
from __future__ import annotations

import numpy as np

ROW = np.dtype([("tlo", "<i8"), ("thi", "<i8"), ("alo", "<f4"), ("ahi", "<f4"), ("qid", "<u4"), ("ncells", "<u4")])
assert ROW.itemsize == 32  # DSSG_ROUTE_ROW_BYTES


def part_of(cells: np.ndarray, part_hi: np.ndarray) -> np.ndarray:
    """First part d with c <= part_hi[d] (route.hip part_of)."""
    return np.searchsorted(part_hi, np.asarray(cells, np.uint64), side="left")


def segment_bytes(rows: int, cells: int) -> int:
    """dssgpu.h: 32 * rows + 32 * ceil(cells / 4)."""
    return 32 * rows + 32 * ((cells + 3) // 4)


def route(offs, cells, alo, ahi, tlo, thi, part_hi):
    """The send buffer (uint8) of part-major fused segments and the per-part
    (rows, cells, segment bytes).  Rows of a segment in query order (the
    device's order is unspecified; only the layout is fixed)."""
    offs = np.asarray(offs, np.int64)
    cells = np.asarray(cells, np.uint64)
    np_ = len(part_hi)
    nq = len(offs) - 1
    owner = part_of(cells, part_hi)
    qof = np.repeat(np.arange(nq), np.diff(offs))
    dest = [np.unique(owner[offs[q]:offs[q + 1]]) for q in range(nq)]
    segs, rows_n, cells_n = [], [], []
    for d in range(np_):
        qs = np.array([q for q in range(nq) if d in dest[q]], dtype=np.int64)
        r = np.zeros(len(qs), ROW)
        if len(qs):
            r["tlo"], r["thi"], r["alo"], r["ahi"] = tlo[qs], thi[qs], alo[qs], ahi[qs]
            r["qid"] = qs
            r["ncells"] = offs[qs + 1] - offs[qs]
        cl = np.concatenate([cells[offs[q]:offs[q + 1]] for q in qs]) if len(qs) else np.zeros(0, np.uint64)
        body = r.tobytes() + cl.astype("<u8").tobytes()
        nb = segment_bytes(len(qs), len(cl))
        segs.append(body + b"\0" * (nb - len(body)))
        rows_n.append(len(qs))
        cells_n.append(len(cl))
    del qof
    seg = [len(x) for x in segs]
    return np.frombuffer(b"".join(segs), np.uint8).copy(), rows_n, cells_n, seg


def unpack(recv: np.ndarray, src_rows, src_cells):
    """Received segments (source-major) -> batch dict: offs, cells, alo, ahi,
    tlo, thi, home (source part), qid (home-local query)."""
    buf = np.asarray(recv, np.uint8).tobytes()
    off = 0
    rows, cl, home = [], [], []
    for s, (nr, nc) in enumerate(zip(src_rows, src_cells)):
        r = np.frombuffer(buf, ROW, count=nr, offset=off)
        c = np.frombuffer(buf, "<u8", count=nc, offset=off + 32 * nr)
        rows.append(r)
        cl.append(c)
        home.append(np.full(nr, s, np.uint32))
        off += segment_bytes(nr, nc)
    r = np.concatenate(rows) if rows else np.zeros(0, ROW)
    offs = np.zeros(len(r) + 1, np.int64)
    np.cumsum(r["ncells"].astype(np.int64), out=offs[1:])
    return {"offs": offs, "cells": np.concatenate(cl).astype(np.uint64) if cl else np.zeros(0, np.uint64),
            "alo": r["alo"].copy(), "ahi": r["ahi"].copy(), "tlo": r["tlo"].copy(), "thi": r["thi"].copy(),
            "home": np.concatenate(home) if home else np.zeros(0, np.uint32), "qid": r["qid"].copy()}


def route_pairs(batch, pq, pe, nparts: int, self_part: int):
    """The shard's pairs home: (own q, own e) for self_part's queries, and the
    part-major packed send buffer (home-local qid << 32 | entity) with the
    per-part counts (self_part's counted, sent as 0)."""
    pq = np.asarray(pq, np.int64)
    pe = np.asarray(pe, np.uint64)
    home = batch["home"][pq].astype(np.int64)
    qid = batch["qid"][pq].astype(np.uint64)
    counts = np.bincount(home, minlength=nparts)[:nparts]
    mine = home == self_part
    send = []
    for d in range(nparts):
        if d == self_part:
            continue
        m = home == d
        send.append((qid[m] << np.uint64(32)) | pe[m])
    packed = np.concatenate(send) if send else np.zeros(0, np.uint64)
    return qid[mine].astype(np.uint32), pe[mine].astype(np.uint32), packed, counts


def unpack_pairs(packed: np.ndarray):
    p = np.asarray(packed, np.uint64)
    return (p >> np.uint64(32)).astype(np.uint32), (p & np.uint64(0xFFFFFFFF)).astype(np.uint32)
