#!/bin/bash
# Whole-step A/B with 3 pipelines (the bench line's own setting, where the
# kernels of different pipelines overlap): bench.py on configs[CFG, default 2] under each
# library, alternating, twice; then one PMC pass per library (VALU, SALU, LDS
# instructions and waves per kernel).  base = the in-tree library; others from
# dss_amd/variants/ (tools/variants.sh).  Results under gpurun_out/TAG/.
#   usage: [CFG=N] [NO_PMC=1] bash tools/ab_step.sh TAG V1,V2,...   (V = base, a variant name,
#          or tune=KEY=VALUE: the in-tree library with dssg_set_tuning KEY=VALUE)
set -o pipefail
TAG=${1:-ab_step}
VS=${2:-base}
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/$TAG; mkdir -p $O
A="--config ${CFG:-2} --steps 40 --warmup 5 --no-verify --cpu-sample 0 --latency 0 --survey-model 0"
for r in 1 2; do
  for v in ${VS//,/ }; do
    X=""
    if [ $v = base ]; then unset DSS_AMD_LIB
    elif [ "${v#tune=}" != "$v" ]; then unset DSS_AMD_LIB; X="--tune ${v#tune=}"  # tune=KEY=VALUE: the in-tree library with a knob
    else export DSS_AMD_LIB=$GRAFT_REPO_ROOT/dss_amd/variants/$v.so; fi
    timeout -k 10 240 python -u bench.py $A $X > $O/ab_${v}_$r.json 2> $O/ab_${v}_$r.err || { echo BENCH_FAILED $v; tail -5 $O/ab_${v}_$r.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/ab_${v}_$r.json')); print('$v', $r, round(d['value']/1e6,2), round(d['ms_per_step'],4), {k: round(x,3) for k,x in d['phase_ms'].items()})"
  done
done
unset DSS_AMD_LIB
cd /tmp && export TMPDIR=/tmp
[ -n "$NO_PMC" ] && { echo all_done; exit 0; }
for v in ${VS//,/ }; do
  [ "${v#tune=}" != "$v" ] && continue
  if [ $v = base ]; then unset DSS_AMD_LIB; else export DSS_AMD_LIB=$GRAFT_REPO_ROOT/dss_amd/variants/$v.so; fi
  timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_INSTS_SALU SQ_INSTS_LDS -d $GRAFT_REPO_ROOT/$O/pmc_$v -o pmc --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --config 2 --steps 3 --warmup 1 --no-verify --cpu-sample 0 --latency 0 --survey-model 0 --pipelines 1 > $GRAFT_REPO_ROOT/$O/pmc_$v.log 2>&1 || { echo PMC_FAILED $v; exit 1; }
done
echo all_done
