#!/bin/bash
# Knob sweep through gpurun: one short bench line per variant (name:args;...)
#   usage: CFG=2 VARS="p3:--pipelines 3;p4:--pipelines 4" bash tools/gpu_knobs.sh TAG
set -o pipefail
TAG=${1:-knobs}
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/$TAG
mkdir -p "$O"
IFS=';' read -ra VS <<< "$VARS"
for v in "${VS[@]}"; do
  name=${v%%:*}; vargs=${v#*:}
  timeout -k 10 300 python -u bench.py --config ${CFG:-2} --steps ${STEPS:-12} --warmup 2 --cpu-sample 0 --latency 0 --survey-model 0 $vargs > "$O/$name.json" 2> "$O/$name.err" \
      || { echo BENCH_FAILED $name; tail -20 "$O/$name.err"; exit 1; }
  python3 -c "import json;d=json.load(open('$O/$name.json'));print('$name', round(d['value']/1e6,2), 'Mq/s', round(d['ms_per_step'],3), 'ms', {k:round(x,3) for k,x in d['phase_ms'].items()})"
done
echo all_done
