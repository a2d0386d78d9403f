#!/bin/bash
# Alternating rocprofv3 kernel traces of two librbx builds on the C2 bench (add pipeline kernels):
#   bash tools/kt_ab.sh <old.so>   -> gpurun_out/kt_{old,new}_{1,2}/
set -u
OLD=${1:?old librbx.so}
R=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
cd /tmp || exit 1
for i in 1 2; do
  for tag in old new; do
    if [ $tag = old ]; then L=$OLD; else L=$R/redisson_amd/librbx.so; fi
    RBX_LIB_PATH=$L timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/kt_${tag}_$i -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline > $R/gpurun_out/kt_${tag}_$i.log 2>&1 || exit 1
  done
done
