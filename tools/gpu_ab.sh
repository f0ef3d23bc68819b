#!/bin/bash
# A/B run through gpurun: a few GPU test files, then short bench lines per
# config (no CPU baseline / latency legs).
#   usage: TESTS="tests/test_gpu_search.py" CFGS="2 1" XARGS="..." bash tools/gpu_ab.sh TAG
set -o pipefail
TAG=${1:-ab}
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/$TAG
mkdir -p "$O"
if [ -n "$TESTS" ]; then
  timeout -k 10 400 python -u -m pytest $TESTS -x -q --timeout 120 --timeout-method thread > "$O/tests.log" 2>&1 \
      || { echo TESTS_FAILED; tail -30 "$O/tests.log"; exit 1; }
  tail -1 "$O/tests.log"
fi
for c in ${CFGS:-2 1}; do
  case $c in 4) CA="--config 4 --scale 0.2" ;; *) CA="--config $c" ;; esac
  timeout -k 10 300 python -u bench.py $CA --steps ${STEPS:-10} --warmup 2 --cpu-sample 0 --latency 0 --survey-model 0 $XARGS > "$O/c$c.json" 2> "$O/c$c.err" \
      || { echo BENCH_FAILED c$c; tail -20 "$O/c$c.err"; exit 1; }
  python3 -c "import json;d=json.load(open('$O/c$c.json'));print('c$c', round(d['value']/1e6,2), 'Mq/s', {k:round(x,3) for k,x in d['phase_ms'].items()}, 'rl', round(d['roofline']['frac'],3), 'cover', round(d['cover_roofline']['frac'],3), 'parity', d.get('parity',{}).get('pairs_equal') if d.get('parity') else None)"
done
echo all_done
