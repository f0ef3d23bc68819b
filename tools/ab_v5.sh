set -e
mkdir -p gpurun_out/v5
B="python3 bench.py --steps 10 --warmup 2 --cpu-sample 0 --survey-model 0 --no-verify --pipelines 1"
for v in base noorigin; do
  if [ $v = base ]; then L=""; else L="DSS_AMD_LIB=dss_amd/variants/$v.so"; fi
  env $L timeout -k 10 120 $B > gpurun_out/v5/$v.json 2>gpurun_out/v5/$v.err
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/v5/$v.json').read().strip().splitlines()[-1]); print('$v', round(d['value']/1e6,1), d['phase_ms'])"
done
cd /tmp && export TMPDIR=/tmp && DSS_AMD_LIB=$GRAFT_REPO_ROOT/dss_amd/variants/noorigin.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/v5/prof -o kt --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 --cpu-sample 0 --survey-model 0 --pipelines 1 --no-verify > $GRAFT_REPO_ROOT/gpurun_out/v5/prof.log 2>&1
