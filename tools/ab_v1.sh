set -e
mkdir -p gpurun_out/v1
B="python3 bench.py --steps 10 --warmup 2 --cpu-sample 0 --survey-model 0 --no-verify --pipelines 1"
for v in base nolong base nolong; do
  if [ $v = base ]; then L=""; else L="DSS_AMD_LIB=dss_amd/variants/$v.so"; fi
  env $L timeout -k 10 120 $B > gpurun_out/v1/$v.json 2>gpurun_out/v1/$v.err
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/v1/$v.json').read().strip().splitlines()[-1]); print('$v', round(d['value']/1e6,1), d['phase_ms'])"
done
