#!/bin/bash
# Kernel-trace stats of one microbench run per rbx_tune setting:
#   bash tools/kstats.sh <bench> <tag> <tune> [<tune> ...]  -> gpurun_out/kstats_<tag>.txt
# (a tune is "key=value[,key=value]"; "-" = defaults)
set -u
BENCH=$1; TAG=$2; shift 2
R=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
cd /tmp || exit 1
i=0
for t in "$@"; do
  i=$((i+1))
  tune=$t; [ "$t" = "-" ] && tune=""
  D=$R/gpurun_out/kst_${TAG}_$i
  RBX_TUNE=$tune timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$D" -o run -- python3 "$R/tools/microbench.py" "$BENCH" > "$D.log" 2>&1 || exit 1
  f=$(find "$D" -name "*kernel_stats.csv" | head -1)
  python3 -c "
import csv,sys
print('== tune', sys.argv[2])
for r in csv.DictReader(open(sys.argv[1])):
    if 'rbx' in r['Name']: print('%-44s %4s %9.4f ms' % (r['Name'][:44], r['Calls'], float(r['AverageNs'])/1e6))
" "$f" "$t" >> "$R/gpurun_out/kstats_$TAG.txt" || exit 1
done
