#!/bin/bash
# One gpurun call: (optionally) the GPU tests, then bench.py on the configs
# named on the command line, each under its own time limit; results under
# gpurun_out/<tag>/.  Usage (through gpurun):
#   bash tools/gpu_bench_configs.sh TAG [tests] "CONFIG[:extra bench args]" ...
# e.g. bash tools/gpu_bench_configs.sh r02a tests "1" "2:--steps 10"
set -o pipefail
TAG=$1
shift
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
if [ "$1" = "tests" ]; then
    shift
    timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
        > "$OUT/gpu_tests.log" 2>&1 || { echo TESTS_FAILED; tail -40 "$OUT/gpu_tests.log"; exit 1; }
    tail -2 "$OUT/gpu_tests.log"
fi
for spec in "$@"; do
    cfg=${spec%%:*}
    extra=""
    [ "$spec" != "$cfg" ] && extra=${spec#*:}
    name=$(echo "config_${cfg}_${extra}" | tr -c 'A-Za-z0-9_.=\n-' '_')
    echo "== bench config $cfg $extra"
    timeout -k 10 ${BENCH_TIMEOUT:-600} python -u bench.py --config "$cfg" $extra > "$OUT/$name.json" 2> "$OUT/$name.err" \
        || { echo "BENCH_FAILED $cfg"; tail -20 "$OUT/$name.err"; exit 1; }
    cut -c1-600 "$OUT/$name.json"
done
echo done
