set -e
mkdir -p gpurun_out/v8
timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/v8/pytest.log 2>&1
tail -1 gpurun_out/v8/pytest.log
for p in 1 3; do
  timeout -k 10 200 python3 bench.py --steps 21 --warmup 2 --cpu-sample 0 --survey-model 0 --no-verify --pipelines $p > gpurun_out/v8/p$p.json 2>gpurun_out/v8/p$p.err
  python3 -c "import json; d=json.loads(open('gpurun_out/v8/p$p.json').read().strip().splitlines()[-1]); print($p, round(d['value']/1e6,2), d['ms_per_step'], d['phase_ms'])"
done
