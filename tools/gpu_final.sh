# Round-end evidence in one gpurun call: the GPU tests, the default bench
# line (configs[2]), then the rocprofv3 kernel trace + FETCH/WRITE + FP64
# passes of the same workload (tools/profile.sh, one pipeline), summaries
# copied to gpurun_out/<tag>/ (the raw traces exceed gpurun's copy-back limit).
#   usage (through gpurun): bash tools/gpu_final.sh TAG
set -o pipefail
TAG=${1:-final}
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1 \
    || { echo TESTS_FAILED; tail -30 "$OUT/gpu_tests.log"; exit 1; }
tail -1 "$OUT/gpu_tests.log"
timeout -k 10 500 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { echo BENCH_FAILED; tail "$OUT/bench.err"; exit 1; }
cut -c1-300 "$OUT/bench.json"
FP64=1 STEPS=4 BENCH_ARGS="--config 2" NI=10000000 bash tools/profile.sh "$TAG" > "$OUT/profile.log" 2>&1 || { echo PROF_FAILED; tail "$OUT/profile.log"; exit 1; }
P=gpurun_out/prof/$TAG
cp "$P/summary.csv" "$OUT/pmc_summary.csv"
cp "$P/pmc_traffic.json" "$OUT/pmc_traffic.json"
cp "$P/fp64_cover.json" "$P/fp64.txt" "$OUT/" 2>/dev/null
KS=$(find "$P" -name 'kt_kernel_stats.csv' | head -1)
[ -n "$KS" ] && cp "$KS" "$OUT/kernel_stats.csv"
rm -rf gpurun_out/prof
head -6 "$OUT/pmc_summary.csv" | cut -c1-200
echo done
