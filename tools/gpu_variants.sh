#!/bin/bash
# k_join timing of library variants (tools/variants.sh) on one config, one
# pipeline, HIP-event kernel times from the bench line.
#   usage: CFG=2 VARIANTS="base noemit" bash tools/gpu_variants.sh TAG
set -o pipefail
TAG=${1:-var}
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/$TAG
mkdir -p "$O"
for v in ${VARIANTS:-base}; do
  if [ "$v" = base ]; then unset DSS_AMD_LIB; else export DSS_AMD_LIB=$GRAFT_REPO_ROOT/dss_amd/variants/$v.so; fi
  timeout -k 10 300 python -u bench.py --config ${CFG:-2} --steps ${STEPS:-8} --warmup 2 --pipelines 1 --cpu-sample 0 --latency 0 --survey-model 0 --no-verify $XARGS > "$O/$v.json" 2> "$O/$v.err" \
      || { echo BENCH_FAILED $v; tail -20 "$O/$v.err"; exit 1; }
  python3 -c "import json;d=json.load(open('$O/$v.json'));print('$v', round(d['value']/1e6,2), 'Mq/s', {k:round(x,3) for k,x in d['phase_ms'].items()})"
done
unset DSS_AMD_LIB
echo all_done
