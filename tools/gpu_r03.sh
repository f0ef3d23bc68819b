# One gpurun call for round 3: GPU tests, the default bench line (configs[2],
# N=1), the 2-rank same-device gloo rehearsal of the self-launched sharded
# path, and the 1-rank native RCCL sharded path.
#   usage (through gpurun): bash tools/gpu_r03.sh TAG [skip-tests]
set -o pipefail
TAG=${1:-r03}
cd $GRAFT_REPO_ROOT
O=gpurun_out/$TAG
mkdir -p $O
if [ "$2" != "skip-tests" ]; then
# test failures do not stop the call (the bench checks its own parity); a crash, hang or kill does
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?
tail -2 $O/gpu_tests.log
grep -E "FAILED|ERROR" $O/gpu_tests.log | head -20
[ $rc -le 1 ] || { echo TESTS_CRASHED rc=$rc; exit 1; }
fi
timeout -k 10 500 python -u bench.py --steps 20 --warmup 3 > $O/bench.json 2> $O/bench.err || { echo BENCH_FAILED; tail $O/bench.err; exit 1; }
cut -c1-600 $O/bench.json
timeout -k 10 400 python -u bench.py --gpus 2 --same-device --dist-backend gloo --scale 0.05 --steps 3 --warmup 1 > $O/gloo2.json 2> $O/gloo2.err || { echo GLOO2_FAILED; tail -30 $O/gloo2.err; exit 1; }
cut -c1-400 $O/gloo2.json
timeout -k 10 300 python -u bench.py --mode sharded --exchange native --scale 0.1 --steps 5 --warmup 1 > $O/native1.json 2> $O/native1.err || { echo NATIVE1_FAILED; tail -30 $O/native1.err; exit 1; }
cut -c1-400 $O/native1.json
echo done
if [ -n "$AB" ]; then
# variants: name=bench args (ABV="name1:args1;name2:args2")
IFS=';' read -ra VS <<< "${ABV:-base:}"
for v in "${VS[@]}"; do
name=${v%%:*}; vargs=${v#*:}
for c in 1 2; do
DSS_COVER_STATS=1 timeout -k 10 300 python -u bench.py --config $c --steps 20 --warmup 3 --cpu-sample 0 --latency 0 --survey-model 0 $vargs > $O/ab_${name}_c${c}.json 2> $O/ab_${name}_c${c}.err || { echo AB_FAILED $name c$c; tail -20 $O/ab_${name}_c${c}.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/ab_${name}_c${c}.json'));print('AB $name c$c', round(d['value']/1e6,1), 'Mq/s', {k:round(x,3) for k,x in d['phase_ms'].items()}, round(d['roofline']['frac'],3), round(d['cover_roofline']['frac'],3))"
done; done
grep -h "\[cover\]" $O/ab_*_c*.err | sort | uniq -c | sort -rn | head -6
fi
if [ -n "$LAT" ]; then
for w in 2 4; do
DSSG_BATCHER_WORKERS=$w DSSG_BATCHER_PROFILE=1 timeout -k 10 300 python -u bench.py --config 1 --steps 3 --warmup 1 --cpu-sample 0 --survey-model 0 > $O/lat_w$w.json 2> $O/lat_w$w.err || { echo LAT_FAILED w$w; tail -20 $O/lat_w$w.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/lat_w$w.json'));r=d['request_latency'];print('LAT w$w', json.dumps({k:{kk:round(vv,3) for kk,vv in v.items() if isinstance(vv,float)} for k,v in r.items() if isinstance(v,dict)}))"
grep "dssg_batcher" $O/lat_w$w.err | tail -2
done
fi
if [ -n "$PROF" ]; then
STEPS=4 BENCH_ARGS="--config 2" NI=10000000 bash tools/profile.sh ${TAG}_c2 > $O/prof_c2.log 2>&1 || { echo PROF_C2_FAILED; tail -20 $O/prof_c2.log; exit 1; }
head -25 gpurun_out/prof/${TAG}_c2/summary.csv | cut -c1-160
KT_ONLY=1 STEPS=4 BENCH_ARGS="--config 1" NI=1000000 bash tools/profile.sh ${TAG}_c1 > $O/prof_c1.log 2>&1 || { echo PROF_C1_FAILED; tail -20 $O/prof_c1.log; exit 1; }
head -25 gpurun_out/prof/${TAG}_c1/summary.csv | cut -c1-120
fi
echo all_done
