#!/bin/bash
# Kernel-trace A/B of library variants (tools/variants.sh) on one config:
#   VARIANTS="base wpe5" CFG=1 bash tools/gpu_kt.sh TAG     (through gpurun)
# "base" is the in-tree dss_amd/libdss_amd.so.  One rocprofv3 kernel-trace
# run per variant (tools/profile.sh, KT_ONLY), summaries under
# gpurun_out/prof/TAG_<variant>/.
set -o pipefail
TAG=${1:-kt}
cd $GRAFT_REPO_ROOT
CFG=${CFG:-1}
NI=${NI:-1000000}
[ "$CFG" = 2 ] && NI=10000000
for v in ${VARIANTS:-base}; do
  if [ "$v" = base ]; then unset DSS_AMD_LIB; else export DSS_AMD_LIB=$GRAFT_REPO_ROOT/dss_amd/variants/$v.so; fi
  KT_ONLY=1 STEPS=${STEPS:-4} BENCH_ARGS="--config $CFG $XARGS" NI=$NI bash tools/profile.sh ${TAG}_$v > gpurun_out/kt_${TAG}_$v.log 2>&1 || { echo KT_FAILED $v; tail -20 gpurun_out/kt_${TAG}_$v.log; exit 1; }
  echo "== $v"
  head -${TOP:-22} gpurun_out/prof/${TAG}_$v/summary.csv | cut -c1-100
done
unset DSS_AMD_LIB
echo all_done
