# A/B timing of join variants (tools/variants.sh builds them) on configs[1]
# and configs[4] at scale 0.2; one JSON line per run under gpurun_out/$TAG.
set -e
TAG=${TAG:-xp}
mkdir -p gpurun_out/$TAG
for v in ${VARIANTS:-base noemit nosig nohull notest}; do
  L=""; [ $v != base ] && L="DSS_AMD_LIB=dss_amd/variants/$v.so"
  for c in ${CONFIGS:-1 4}; do
    S=""; [ $c = 4 ] && S="--scale 0.2"
    env $L timeout -k 10 150 python bench.py --config $c $S --steps 5 --latency 0 --cpu-sample 0 > gpurun_out/$TAG/c${c}_$v.json 2> gpurun_out/$TAG/c${c}_$v.err
    python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[1],round(d['value']/1e6,2),d['phase_ms'],(d.get('parity') or {}).get('pairs_equal'))" gpurun_out/$TAG/c${c}_$v.json
  done
done
