#!/bin/bash
# rocprofv3 evidence of the bench command in one gpurun call: per config,
# the kernel trace + FETCH/WRITE passes (+ the FP64 VALU pass with FP64=1),
# summaries kept under gpurun_out/<tag>_c<cfg>/, raw traces dropped (they
# exceed gpurun's copy-back limit).
#   usage (through gpurun): CFGS="2 1" FP64=1 bash tools/gpu_prof.sh TAG
set -o pipefail
TAG=${1:-prof}
cd "$GRAFT_REPO_ROOT" || exit 1
for c in ${CFGS:-2 1}; do
  case $c in 1) NI=1000000 ;; 2) NI=10000000 ;; 3) NI=5000000 ;; *) NI=0 ;; esac
  T=${TAG}_c$c
  STEPS=${STEPS:-4} BENCH_ARGS="--config $c $XARGS" NI=$NI bash tools/profile.sh "$T" > "gpurun_out/prof_$T.log" 2>&1 \
      || { echo PROF_FAILED $T; tail -20 "gpurun_out/prof_$T.log"; exit 1; }
  P=gpurun_out/prof/$T
  O=gpurun_out/$T
  mkdir -p "$O"
  cp "$P/summary.csv" "$O/pmc_summary.csv"
  cp "$P/pmc_traffic.json" "$O/pmc_traffic.json" 2>/dev/null
  cp "$P/fp64_cover.json" "$P/fp64.txt" "$O/" 2>/dev/null
  KS=$(find "$P" -name 'kt_kernel_stats.csv' | head -1)
  [ -n "$KS" ] && cp "$KS" "$O/kernel_stats.csv"
  rm -rf "$P"
  echo "== $T"
  head -18 "$O/pmc_summary.csv" | cut -c1-150
  [ -f "$O/fp64.txt" ] && head -8 "$O/fp64.txt"
done
echo all_done
