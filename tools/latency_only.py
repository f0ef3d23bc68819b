"""The per-request leg alone (analysis tool): build configs[2]'s index the way
bench.py does, then run request_latency's batched leg (64 native callers
through dssg_batcher) for a few seconds -- so a rocprofv3 kernel trace sees
only the per-request path.  usage: python tools/latency_only.py [TREE] [SECONDS]
(TREE: the repository root whose bench.py / dss_amd to use, e.g. ab/r04)"""
import json
import os
import sys

tree = os.path.abspath(sys.argv[1] if len(sys.argv) > 1 else os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
secs = float(sys.argv[2]) if len(sys.argv) > 2 else 2.0
sys.path.insert(0, tree)
os.chdir(tree)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from dss_amd import _lib, device as D, workload as W  # noqa: E402

ctx = _lib.context(0)
dev = "cuda:0"
queries, qa, intents, ia, now, rid = W.config_split(2, 0, 1.0, 1.0)
t = lambda a: torch.as_tensor(a, device=dev)  # noqa: E731
i_offs_t, i_cells_t = bench.cover_chunked(ctx, D, torch, intents, dev)
icells = _lib.Cells(intents.n, int(i_offs_t.data_ptr()), int(i_cells_t.data_ptr()), 0, 0, int(i_cells_t.numel()))
index = D.build_index(ctx, icells, t(ia.alt_lo), t(ia.alt_hi), t(ia.t0), t(ia.t1))
torch.cuda.synchronize()
res = bench.request_latency(ctx, D, index, queries, qa, now, n_alone=400, seconds=secs)
print(json.dumps({"tree": tree, "request_latency": res}), flush=True)
