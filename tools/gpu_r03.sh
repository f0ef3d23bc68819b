# One gpurun call for round 3: GPU tests, the default bench line (configs[2],
# N=1), the 2-rank same-device gloo rehearsal of the self-launched sharded
# path, and the 1-rank native RCCL sharded path.
#   usage (through gpurun): bash tools/gpu_r03.sh TAG [skip-tests]
set -o pipefail
TAG=${1:-r03}
cd $GRAFT_REPO_ROOT
O=gpurun_out/$TAG
mkdir -p $O
if [ "$2" != "skip-tests" ]; then
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
fi
timeout -k 10 500 python -u bench.py --steps 20 --warmup 3 > $O/bench.json 2> $O/bench.err || { echo BENCH_FAILED; tail $O/bench.err; exit 1; }
cut -c1-600 $O/bench.json
timeout -k 10 400 python -u bench.py --gpus 2 --same-device --dist-backend gloo --scale 0.05 --steps 3 --warmup 1 > $O/gloo2.json 2> $O/gloo2.err || { echo GLOO2_FAILED; tail -30 $O/gloo2.err; exit 1; }
cut -c1-400 $O/gloo2.json
timeout -k 10 300 python -u bench.py --mode sharded --exchange native --scale 0.1 --steps 5 --warmup 1 > $O/native1.json 2> $O/native1.err || { echo NATIVE1_FAILED; tail -30 $O/native1.err; exit 1; }
cut -c1-400 $O/native1.json
echo done
