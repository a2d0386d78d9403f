#!/bin/bash
# Kernel-trace stats of one bench.py workload per (library, tune):
#   bash tools/kstats_bench.sh <workload> <tag> <lib|-> <tune|-> [<lib|-> <tune|-> ...]
#   -> gpurun_out/kstb_<tag>.txt
set -u
W=$1; TAG=$2; shift 2
R=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
cd /tmp || exit 1
i=0
while [ $# -ge 2 ]; do
  lib=$1; tune=$2; shift 2
  i=$((i+1))
  [ "$tune" = "-" ] && tune=""
  D=$R/gpurun_out/kstb_${TAG}_$i
  if [ "$lib" = "-" ]; then unset RBX_LIB_PATH; else export RBX_LIB_PATH=$R/$lib; fi
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$D" -o run -- python3 "$R/bench.py" --workload "$W" --steps 3 --warmup 1 --no-cpu-baseline --no-hostpath --legs none --tune "$tune" > "$D.log" 2>&1 || exit 1
  f=$(find "$D" -name "*kernel_stats.csv" | head -1)
  python3 -c "
import csv,sys
print('== lib', sys.argv[2], 'tune', sys.argv[3])
for r in csv.DictReader(open(sys.argv[1])):
    if 'rbx' in r['Name']: print('%-44s %5s %9.4f ms' % (r['Name'][:44], r['Calls'], float(r['AverageNs'])/1e6))
" "$f" "$lib" "$tune" >> "$R/gpurun_out/kstb_$TAG.txt" || exit 1
  rm -rf "$D"
done
