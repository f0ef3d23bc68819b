# Other BASELINE configs and the sharded path (2 ranks on one GPU over gloo),
# each with its built-in GPU-vs-oracle parity check.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/s59
timeout -k 10 240 python -u bench.py --config 0 --steps 10 --pipelines 1 > gpurun_out/s59/c0.json 2> gpurun_out/s59/c0.err || { echo C0_FAILED; tail gpurun_out/s59/c0.err; exit 1; }
timeout -k 10 300 python -u bench.py --config 3 --scale 0.2 --steps 10 --cpu-sample 20000 > gpurun_out/s59/c3.json 2> gpurun_out/s59/c3.err || { echo C3_FAILED; tail gpurun_out/s59/c3.err; exit 1; }
timeout -k 10 300 python -u bench.py --config 4 --scale 0.05 --steps 5 --cpu-sample 5000 > gpurun_out/s59/c4.json 2> gpurun_out/s59/c4.err || { echo C4_FAILED; tail gpurun_out/s59/c4.err; exit 1; }
timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 3 --same-device --dist-backend gloo --scale 0.25 --cpu-sample 0 > gpurun_out/s59/sh2.json 2> gpurun_out/s59/sh2.err || { echo SH_FAILED; tail gpurun_out/s59/sh2.err; exit 1; }
echo ok
