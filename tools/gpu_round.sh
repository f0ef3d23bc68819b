# One gpurun call: GPU tests, the bench line, then rocprofv3 (trace + PMC).
#   usage (through gpurun): bash tools/gpu_round.sh TAG [skip-tests]
set -o pipefail
TAG=${1:-r01}
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/$TAG
if [ "$2" != "skip-tests" ]; then
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/$TAG/gpu_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/$TAG/gpu_tests.log; exit 1; }
tail -2 gpurun_out/$TAG/gpu_tests.log
fi
timeout -k 10 400 python -u bench.py > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err || { echo BENCH_FAILED; tail gpurun_out/$TAG/bench.err; exit 1; }
cat gpurun_out/$TAG/bench.json
if [ "$3" != "noprof" ]; then
bash tools/profile.sh $TAG || { echo PROF_FAILED; exit 1; }
fi
echo done
