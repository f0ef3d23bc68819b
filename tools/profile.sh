#!/bin/bash
# rocprofv3 evidence for bench.py on one MI355X (run through gpurun):
#   kernel trace + stats, then separate PMC passes (never mixed with trace
#   domains, never more counters per block than one pass holds).  Output
#   under gpurun_out/prof/<tag>; summarize with tools/pmc_summary.py.
set -eo pipefail
TAG=${1:-prof}
STEPS=${STEPS:-3}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/prof/$TAG
mkdir -p "$OUT"
B="$R/bench.py --steps $STEPS --warmup 1 --cpu-sample 0 --survey-model 0 --pipelines 1 --latency 0 --no-verify $BENCH_ARGS"
# PROBE=N: one rank's shard join at world size N (tools/shard_probe.py, one process)
[ -n "$PROBE" ] && B="$R/tools/shard_probe.py $PROBE --steps $STEPS --warmup 1 $PROBE_ARGS"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT" -o kt --output-format csv -- python3 $B > "$OUT/kt.log" 2>&1
[ -n "$KT_ONLY" ] || timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d "$OUT" -o pmc_fetch --output-format csv -- python3 $B > "$OUT/pmc_fetch.log" 2>&1
[ -n "$KT_ONLY" ] || timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d "$OUT" -o pmc_write --output-format csv -- python3 $B > "$OUT/pmc_write.log" 2>&1
if [ -n "$FULL_PMC" ] || [ -n "$FP64" ]; then
# FP64 VALU work of the covering kernels (TOTAL_64_OPS's terms, without MFMA)
timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT64 -d "$OUT" -o pmc_f64 --output-format csv -- python3 $B > "$OUT/pmc_f64.log" 2>&1
fi
if [ -n "$FULL_PMC" ]; then
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_WAIT_INST_ANY -d "$OUT" -o pmc_sq --output-format csv -- python3 $B > "$OUT/pmc_sq.log" 2>&1
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_SALU GRBM_GUI_ACTIVE -d "$OUT" -o pmc_cyc --output-format csv -- python3 $B > "$OUT/pmc_cyc.log" 2>&1
fi
cd "$R"
python3 tools/pmc_summary.py "$OUT" --skip-first ${SKIP:-2} --json "$OUT/pmc_traffic.json" --queries ${NQ:-1000000} --intents ${NI:-10000000} --source "profiles/$TAG" > "$OUT/summary.csv"
if [ -n "$FULL_PMC" ] || [ -n "$FP64" ]; then
python3 tools/fp64_summary.py "$OUT" "$OUT/fp64_cover.json" ${NQ:-1000000} ${NI:-10000000} ${SKIP:-2} "profiles/$TAG" > "$OUT/fp64.txt"
fi
cat "$OUT/summary.csv" | head -30
