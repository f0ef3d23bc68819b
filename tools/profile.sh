#!/bin/bash
# rocprofv3 evidence for bench.py on one MI355X (run through gpurun):
#   kernel trace + stats, then separate PMC passes (never mixed with trace
#   domains).  Output under gpurun_out/prof/<tag>; summarize with
#   tools/pmc_summary.py.
set -eo pipefail
TAG=${1:-prof}
STEPS=${STEPS:-3}
OUT=$GRAFT_REPO_ROOT/gpurun_out/prof/$TAG
mkdir -p "$OUT"
B="$GRAFT_REPO_ROOT/bench.py --steps $STEPS --warmup 1 --cpu-sample 0"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT" -o kt --output-format csv -- python3 $B > "$OUT/kt.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d "$OUT" -o pmc_fetch --output-format csv -- python3 $B > "$OUT/pmc_fetch.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d "$OUT" -o pmc_write --output-format csv -- python3 $B > "$OUT/pmc_write.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_WAIT_INST_ANY -d "$OUT" -o pmc_sq --output-format csv -- python3 $B > "$OUT/pmc_sq.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_SALU GRBM_GUI_ACTIVE -d "$OUT" -o pmc_cyc --output-format csv -- python3 $B > "$OUT/pmc_cyc.log" 2>&1
find "$OUT" -name '*.csv' | head -50
