set -e
mkdir -p gpurun_out/r02zq
for v in ${VARIANTS:-base noemit nosig nohull both}; do
  L=""; [ $v != base ] && L="DSS_AMD_LIB=dss_amd/variants/$v.so"
  for c in 4 1; do
    S=""; [ $c = 4 ] && S="--scale 0.2"
    env $L timeout -k 10 150 python bench.py --config $c $S --steps 5 --latency 0 --cpu-sample 0 > gpurun_out/r02zq/c${c}_$v.json 2> gpurun_out/r02zq/c${c}_$v.err
  done
done
