#!/bin/bash
# Per-request A/B on one box: the round-4 tree (ab/r04,
# built from commit c0c28fd by the caller; git-ignored) and the head, each a
# short configs[2] bench line whose request_latency leg (tools/loadgen.c's
# native callers: alone, single through the batcher, 64 callers batched) is
# what is compared; interleaved A B A B so box drift shows as run-to-run noise.
# Results under gpurun_out/TAG/.   usage: bash tools/latency_ab.sh TAG
set -o pipefail
TAG=${1:-ab}
cd "$GRAFT_REPO_ROOT" || exit 1
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p "$O"
ARGS="--steps 3 --warmup 1 --cpu-sample 0 --no-verify --survey-model 0 --pipelines 1"
for rep in 1 2; do
    (cd ab/r04 && timeout -k 10 300 python -u bench.py $ARGS > "$O/r04_$rep.json" 2> "$O/r04_$rep.err") \
        || { echo R04_FAILED; tail -20 "$O/r04_$rep.err"; exit 1; }
    timeout -k 10 300 python -u bench.py $ARGS > "$O/head_$rep.json" 2> "$O/head_$rep.err" \
        || { echo HEAD_FAILED; tail -20 "$O/head_$rep.err"; exit 1; }
    for v in r04 head; do
        python3 - "$O/${v}_$rep.json" "$v.$rep" <<'EOF'
import json, sys
d = json.load(open(sys.argv[1]))["request_latency"]
print(sys.argv[2], "alone p50 %.3f" % d["alone"]["p50_ms"], "single p50 %.3f" % d["single"]["p50_ms"],
      "batched %.1fk req/s p99 %.2f mean batch %.1f" % (d["batched"]["requests_per_s"] / 1e3, d["batched"]["p99_ms"],
                                                       d["batched"]["mean_batch"]))
EOF
    done
done
echo all_done
