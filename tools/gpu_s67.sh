set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/s67
timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 12 --same-device --dist-backend gloo --cpu-sample 0 > gpurun_out/s67/rep2.json 2> gpurun_out/s67/rep2.err || { echo REP_FAILED; grep -E "Error|error" gpurun_out/s67/rep2.err | head; exit 1; }
cat gpurun_out/s67/rep2.json
