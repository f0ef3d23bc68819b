#!/bin/bash
# A/B of library variants (tools/variants.sh) on the configs[1] kernel trace:
# per variant a KT_ONLY profile; compare k_setup / k_cand_test averages.
set -e
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/xpc
for v in ${VARIANTS:-setup64}; do
  cd /tmp && export TMPDIR=/tmp
  DSS_AMD_LIB=$R/dss_amd/variants/$v.so timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/xpc/$v -o kt --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --cpu-sample 0 --survey-model 0 --pipelines 1 --latency 0 ${BENCH_ARGS} > $R/gpurun_out/xpc/$v.log 2>&1
done
