set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/s55
timeout -k 10 200 python -u -m pytest tests/test_gpu_radix.py -x -v --timeout 120 --timeout-method thread > gpurun_out/s55/radix.log 2>&1 || { echo RADIX_FAILED; tail -40 gpurun_out/s55/radix.log; exit 1; }
tail -3 gpurun_out/s55/radix.log
timeout -k 10 200 python -u tools/sort_bench.py > gpurun_out/s55/sort.json 2>&1 || { echo SORTB_FAILED; tail -20 gpurun_out/s55/sort.json; exit 1; }
cat gpurun_out/s55/sort.json
bash tools/gpu_round.sh s55 skip-tests noprof
