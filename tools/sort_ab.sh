#!/bin/bash
# Radix-sort variants A/B on one box: tools/sort_bench.py under each library
# (base = the in-tree one; others built by tools/variants.sh into
# dss_amd/variants/), then a kernel-trace summary of the base.  Results under
# gpurun_out/TAG/.   usage: bash tools/sort_ab.sh TAG V1,V2,...
set -o pipefail
TAG=${1:-sortab}
cd "$GRAFT_REPO_ROOT" || exit 1
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p "$O"
for v in ${2//,/ }; do
    if [ "$v" = base ]; then unset DSS_AMD_LIB; else export DSS_AMD_LIB=$GRAFT_REPO_ROOT/dss_amd/variants/$v.so; fi
    timeout -k 10 240 python -u tools/sort_bench.py > "$O/sort_$v.jsonl" 2> "$O/sort_$v.err" \
        || { echo SORT_FAILED $v; tail -20 "$O/sort_$v.err"; exit 1; }
    echo "-- $v"; python3 -c "
import json,sys
for l in open('$O/sort_$v.jsonl'):
    if l.startswith('{'):
        d=json.loads(l); print('%-62s %8.3f ms %7.1f GB/s ok=%s' % (d['shape'][:62], d['ms'], d['GBs'], d['sorted_equal_torch']))"
done
unset DSS_AMD_LIB
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/kt" -o kt --output-format csv -- python3 "$GRAFT_REPO_ROOT/tools/sort_bench.py" > "$O/kt.log" 2>&1 \
    || { echo KT_FAILED; tail -20 "$O/kt.log"; exit 1; }
f=$(find "$O/kt" -name 'kt_kernel_stats.csv' | head -1); cp "$f" "$O/kernel_stats.csv"; rm -rf "$O/kt"
head -12 "$O/kernel_stats.csv" | cut -d, -f1-4 | cut -c1-150
echo all_done
