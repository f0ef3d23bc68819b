"""Assemble profiles/pmc_traffic.json (the traffic bench.py's lines cite) from
one round's rocprofv3 summaries: the replica join's (tools/gpu.sh prof:2 ->
TAG/prof_c2/pmc_traffic.json) and the shard-join probes' at world sizes 2, 4
and 8 (tools/gpu.sh probe:N -> TAG/probeN/{pmc_traffic,probe}.json).

usage: python tools/merge_traffic.py profiles/TAG > profiles/pmc_traffic.json"""
import json
import os
import sys


def main():
    base = sys.argv[1].rstrip("/")
    with open(os.path.join(base, "prof_c2", "pmc_traffic.json")) as f:
        out = json.load(f)
    out["source"] = f"{base}/prof_c2"
    out["sharded"] = {}
    for n in (2, 4, 8):
        d = os.path.join(base, f"probe{n}")
        try:
            with open(os.path.join(d, "pmc_traffic.json")) as f:
                t = json.load(f)
            with open(os.path.join(d, "probe.json")) as f:
                probe = json.loads(f.read().strip().splitlines()[-1])
        except (OSError, ValueError, IndexError):
            continue
        out["sharded"][str(n)] = {
            "source": d, "probe": probe,
            "note": "rank 0's shard join at world size N in one process (tools/shard_probe.py): the union of the N "
                    "ranks' 1M-query batches against rank 0's cell-range shard",
            "kernels": t["kernels"]}
    json.dump(out, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main()
