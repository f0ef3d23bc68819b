set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r02zg
timeout -k 10 300 python -u bench.py --config 2 --scale 0.1 --mode sharded --exchange native --steps 5 --warmup 1 > gpurun_out/r02zg/native1.json 2> gpurun_out/r02zg/native1.err || { echo NATIVE_FAILED; tail -20 gpurun_out/r02zg/native1.err; exit 1; }
cut -c1-400 gpurun_out/r02zg/native1.json
timeout -k 10 400 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 bench.py --config 2 --scale 0.05 --dist-backend gloo --same-device --steps 3 --warmup 1 > gpurun_out/r02zg/gloo2.json 2> gpurun_out/r02zg/gloo2.err || { echo GLOO_FAILED; tail -30 gpurun_out/r02zg/gloo2.err; exit 1; }
cut -c1-400 gpurun_out/r02zg/gloo2.json
