set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/s56
for v in base it8 it4; do
  if [ $v = base ]; then L=""; else L=dss_amd/variants/$v.so; fi
  DSS_AMD_LIB=$L timeout -k 10 200 python -u tools/sort_bench.py > gpurun_out/s56/sort_$v.json 2>&1 || { echo SORTB_FAILED $v; tail -20 gpurun_out/s56/sort_$v.json; exit 1; }
  echo "== $v"; grep shape gpurun_out/s56/sort_$v.json | cut -c1-160
done
