set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu_final.sh r03final || exit 1
bash tools/gpu_bench_configs.sh r03final_cfg "1:--latency 0" "3:--latency 0" "4:--scale 0.2 --latency 0"
