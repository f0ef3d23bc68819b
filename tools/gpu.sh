#!/bin/bash
# The one GPU runner (through gpurun): a list of steps, each under its own
# time limit, stopping at the first failure.  Results under gpurun_out/TAG/.
#   usage: bash tools/gpu.sh TAG STEP [STEP ...]
# steps:
#   tests[:FILES]         pytest -m gpu (all GPU tests, or the named files)
#   bench:CFG[:ARGS]      a full bench.py line (CPU baseline, parity, latency unless ARGS say otherwise)
#   quick:CFG[:ARGS]      a short bench.py line (no CPU baseline / latency / survey counts), one summary line
#   var:CFG:V1,V2[:ARGS]  quick lines of library variants (tools/variants.sh builds dss_amd/variants/V.so;
#                         "base" is the in-tree library), one pipeline
#   prof:CFG[:ARGS]       rocprofv3 kernel trace + FETCH/WRITE (+ FP64 with FP64=1) of the bench command
#                         (tools/profile.sh, one pipeline); summaries kept, raw traces dropped
#   gloo2[:ARGS]          2 ranks on cuda:0 over gloo, sharded (the self-launched path), scale 0.05 unless ARGS
#   native1[:ARGS]        1 rank, sharded over the library's own RCCL communicator
# env: BENCH_TIMEOUT (s, default 600 for bench, 300 for quick/var), STEPS for quick/var (default 10)
set -o pipefail
TAG=$1
shift
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/$TAG
mkdir -p "$O"

summary() {  # one line per bench json
    python3 - "$1" "$2" <<'EOF'
import json, sys
d = json.load(open(sys.argv[1]))
ph = d.get("phase_ms") or d.get("phase_ms_max_over_ranks") or {}
rl, cr, par = d.get("roofline") or {}, d.get("cover_roofline") or {}, d.get("parity") or {}
print(sys.argv[2], f"{d['value'] / 1e6:.2f} Mq/s", f"{d['ms_per_step']:.3f} ms/step",
      {k: round(v, 3) for k, v in ph.items()}, "rl", round(rl.get("frac", 0), 3), "cover", round(cr.get("frac", 0), 3),
      "pipes", d.get("config", {}).get("pipelines_per_gpu"),
      "parity", {k: v for k, v in par.items() if isinstance(v, bool)})
EOF
}

for step in "$@"; do
    kind=${step%%:*}
    rest=""
    [ "$step" != "$kind" ] && rest=${step#*:}
    name=$(echo "$step" | tr -c 'A-Za-z0-9_.=\n-' '_' | cut -c1-80)
    echo "== $step"
    case $kind in
    tests)
        rest=${rest:-tests}
        timeout -k 10 ${TESTS_TIMEOUT:-600} python -u -m pytest ${rest//,/ } -m gpu -x -v --timeout 120 \
            --timeout-method thread > "$O/$name.log" 2>&1 || { echo TESTS_FAILED; tail -40 "$O/$name.log"; exit 1; }
        tail -1 "$O/$name.log" ;;
    bench|quick)
        cfg=${rest%%:*}
        args=""
        [ "$rest" != "$cfg" ] && args=${rest#*:}
        args=${args//:/ }  # (several bench args: ARG1:ARG2)
        extra=""
        lim=${BENCH_TIMEOUT:-600}
        if [ $kind = quick ]; then
            extra="--steps ${STEPS:-10} --warmup 2 --cpu-sample 0 --latency 0 --survey-model 0"
            lim=${BENCH_TIMEOUT:-300}
        fi
        timeout -k 10 $lim python -u bench.py --config "$cfg" $extra $args > "$O/$name.json" 2> "$O/$name.err" \
            || { echo BENCH_FAILED; tail -30 "$O/$name.err"; exit 1; }
        summary "$O/$name.json" "$name" ;;
    var)
        cfg=${rest%%:*}
        r2=${rest#*:}
        vs=${r2%%:*}
        args=""
        [ "$r2" != "$vs" ] && args=${r2#*:}
        args=${args//:/ }
        for v in ${vs//,/ }; do
            if [ "$v" = base ]; then unset DSS_AMD_LIB; else export DSS_AMD_LIB=$GRAFT_REPO_ROOT/dss_amd/variants/$v.so; fi
            timeout -k 10 ${BENCH_TIMEOUT:-300} python -u bench.py --config "$cfg" --steps ${STEPS:-10} --warmup 2 \
                --pipelines 1 --cpu-sample 0 --latency 0 --survey-model 0 --no-verify $args > "$O/${name}_$v.json" \
                2> "$O/${name}_$v.err" || { echo BENCH_FAILED $v; tail -30 "$O/${name}_$v.err"; exit 1; }
            summary "$O/${name}_$v.json" "$v"
        done
        unset DSS_AMD_LIB ;;
    prof)
        cfg=${rest%%:*}
        args=""
        [ "$rest" != "$cfg" ] && args=${rest#*:}
        case $cfg in 1) NI=1000000 ;; 2) NI=10000000 ;; 3) NI=5000000 ;; *) NI=0 ;; esac
        T=${TAG}_c$cfg
        STEPS=${PSTEPS:-4} BENCH_ARGS="--config $cfg $args" NI=$NI bash tools/profile.sh "$T" > "$O/prof_c$cfg.log" 2>&1 \
            || { echo PROF_FAILED; tail -30 "$O/prof_c$cfg.log"; exit 1; }
        P=gpurun_out/prof/$T
        D=$O/prof_c$cfg
        mkdir -p "$D"
        cp "$P/summary.csv" "$D/pmc_summary.csv"
        cp "$P/pmc_traffic.json" "$D/" 2>/dev/null
        cp "$P/fp64_cover.json" "$P/fp64.txt" "$D/" 2>/dev/null
        KS=$(find "$P" -name 'kt_kernel_stats.csv' | head -1)
        [ -n "$KS" ] && cp "$KS" "$D/kernel_stats.csv"
        rm -rf "$P"
        head -${TOP:-20} "$D/pmc_summary.csv" | cut -c1-160 ;;
    probe)  # probe:N -- rocprofv3 passes over one rank's shard join at world size N (tools/shard_probe.py)
        T=${TAG}_probe$rest
        PROBE=$rest STEPS=${PSTEPS:-4} NQ=1000000 NI=10000000 bash tools/profile.sh "$T" > "$O/probe$rest.log" 2>&1 \
            || { echo PROBE_FAILED; tail -30 "$O/probe$rest.log"; exit 1; }
        P=gpurun_out/prof/$T
        D=$O/probe$rest
        mkdir -p "$D"
        cp "$P/summary.csv" "$D/pmc_summary.csv"
        cp "$P/pmc_traffic.json" "$D/" 2>/dev/null
        grep '^{' "$P/kt.log" > "$D/probe.json" || true
        KS=$(find "$P" -name 'kt_kernel_stats.csv' | head -1)
        [ -n "$KS" ] && cp "$KS" "$D/kernel_stats.csv"
        rm -rf "$P"
        cat "$D/probe.json"; head -${TOP:-8} "$D/pmc_summary.csv" | cut -c1-160 ;;
    kt)  # kt:CFG:V1,V2[:ARGS] -- kernel-trace summaries of library variants (one pipeline)
        cfg=${rest%%:*}
        r2=${rest#*:}
        vs=${r2%%:*}
        args=""
        [ "$r2" != "$vs" ] && args=${r2#*:}
        for v in ${vs//,/ }; do
            if [ "$v" = base ]; then unset DSS_AMD_LIB; else export DSS_AMD_LIB=$GRAFT_REPO_ROOT/dss_amd/variants/$v.so; fi
            T=${TAG}_kt_$v
            KT_ONLY=1 STEPS=${PSTEPS:-4} BENCH_ARGS="--config $cfg $args" bash tools/profile.sh "$T" > "$O/kt_$v.log" 2>&1 \
                || { echo KT_FAILED $v; tail -30 "$O/kt_$v.log"; exit 1; }
            mkdir -p "$O/kt_$v"
            cp gpurun_out/prof/$T/summary.csv "$O/kt_$v/pmc_summary.csv"
            KS=$(find gpurun_out/prof/$T -name 'kt_kernel_stats.csv' | head -1)
            [ -n "$KS" ] && cp "$KS" "$O/kt_$v/kernel_stats.csv"
            rm -rf gpurun_out/prof/$T
            echo "-- $v"
            head -${TOP:-16} "$O/kt_$v/pmc_summary.csv" | cut -c1-110
        done
        unset DSS_AMD_LIB ;;
    gloo2)
        timeout -k 10 ${BENCH_TIMEOUT:-400} python -u bench.py --gpus 2 --same-device --dist-backend gloo \
            ${rest:---scale 0.05 --steps 3 --warmup 1} > "$O/$name.json" 2> "$O/$name.err" \
            || { echo GLOO2_FAILED; tail -30 "$O/$name.err"; exit 1; }
        summary "$O/$name.json" "$name" ;;
    native1)
        timeout -k 10 ${BENCH_TIMEOUT:-400} python -u bench.py --mode sharded --exchange native \
            ${rest:---scale 0.1 --steps 5 --warmup 1} > "$O/$name.json" 2> "$O/$name.err" \
            || { echo NATIVE1_FAILED; tail -30 "$O/$name.err"; exit 1; }
        summary "$O/$name.json" "$name" ;;
    *)
        echo "unknown step $step"
        exit 2 ;;
    esac
done
echo all_done
