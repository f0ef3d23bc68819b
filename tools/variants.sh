#!/bin/bash
# Build differently-tuned copies of libdss_amd.so into dss_amd/variants/
# (git-ignored, but shipped to the GPU box) for A/B timing with
#   DSS_AMD_LIB=dss_amd/variants/<name>.so python bench.py ...
#   usage: tools/variants.sh name "-DFLAG=1 ..." [name "flags"]...
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
C=$R/dss_amd/csrc
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math -Wno-unused-function"
mkdir -p $R/dss_amd/variants $R/build/variants
while [ $# -ge 2 ]; do
  name=$1; defs=$2; shift 2
  O=$R/build/variants/$name; mkdir -p $O
  for f in cover.hip ingress.hip radix.hip search.hip subs.hip store.hip route.hip scan.hip selftest.hip capi.cpp; do
    /opt/rocm/bin/hipcc $FLAGS $defs -c $C/$f -o $O/$f.o &
  done
  wait
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $R/dss_amd/variants/$name.so $O/*.o
  echo built $name
done
