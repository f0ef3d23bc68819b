set -e
mkdir -p gpurun_out/v2
timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/v2/pytest.log 2>&1
tail -1 gpurun_out/v2/pytest.log
for c in 1 4; do
  S=1.0; [ $c = 4 ] && S=0.2
  timeout -k 10 200 python3 bench.py --steps 5 --warmup 2 --cpu-sample 0 --survey-model 0 --pipelines 1 --config $c --scale $S > gpurun_out/v2/c$c.json 2>gpurun_out/v2/c$c.err
  python3 -c "import json; d=json.loads(open('gpurun_out/v2/c$c.json').read().strip().splitlines()[-1]); print($c, round(d['value']/1e6,2), d['phase_ms'], d['parity'], d['join_work'])"
done
