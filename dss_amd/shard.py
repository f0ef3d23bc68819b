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
  * each rank covers its slice of the query batch and `allgather_csr` gives
    every rank the whole covered batch (RCCL all-gather over xGMI; gloo on
    CPU in the tests);
  * each rank joins the whole batch against its shard.  Because the
    smallest-shared-cell rule sees whole cell lists, every (query, entity)
    pair is emitted by exactly one rank -- no cross-shard dedupe;
  * `gather_pairs` collects the pair sets (all-gather of counts, then of the
    padded buffers).

Only the exchange steps are collectives; the join itself is the same HIP
kernel as the single-GPU path.  torch.distributed is plumbing: the process
group and the collectives; the tensors it moves are the C ABI's buffers.
"""
from __future__ import annotations

from typing import List, Sequence, Tuple

import numpy as np

U64_MAX = 2**64 - 1


def cell_splitters(cells: np.ndarray, parts: int) -> List[Tuple[int, int]]:
    """Inclusive uint64 ranges [lo, hi], in order, partitioning the whole id
    space into `parts`; each cut falls right after the distinct cell where
    the running posting count reaches r/parts of the total (a hot cell is
    never split).  Parts beyond the number of distinct cells hold no cell."""
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
        hi = min(max(hi, prev + 1), U64_MAX - (parts - len(ranges)))  # strictly increasing, room left
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
