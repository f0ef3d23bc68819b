set -e
mkdir -p gpurun_out/v3
timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/v3/pytest.log 2>&1
tail -1 gpurun_out/v3/pytest.log
timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 --cpu-sample 0 --survey-model 0 --pipelines 1 > gpurun_out/v3/c1.json 2>gpurun_out/v3/c1.err
python3 -c "import json; d=json.loads(open('gpurun_out/v3/c1.json').read().strip().splitlines()[-1]); print(round(d['value']/1e6,2), d['phase_ms'], d['parity'])"
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/v3/prof -o kt --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 --cpu-sample 0 --survey-model 0 --pipelines 1 --no-verify > $GRAFT_REPO_ROOT/gpurun_out/v3/prof.log 2>&1
