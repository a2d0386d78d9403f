#!/bin/bash
# C5 stream timing per rbx_tune setting: bash tools/c5_sweep.sh <tag> <tune> [<tune> ...]
#   -> gpurun_out/c5sweep_<tag>.jsonl (one line per setting: tune, ms_per_step, ops/s)
# (a tune is "key=value[,key=value]"; "-" = defaults)
set -u
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/c5sweep_$TAG.jsonl
: > "$O"
for t in "$@"; do
  tune=$t; [ "$t" = "-" ] && tune=""
  timeout -k 10 240 python3 "$R/bench.py" --workload c5 --steps 5 --warmup 1 --no-cpu-baseline --tune "$tune" \
      > "$R/gpurun_out/c5sweep_${TAG}_run.json" 2> "$R/gpurun_out/c5sweep_${TAG}_run.err" || exit 1
  python3 -c "
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(json.dumps({'tune': sys.argv[2], 'ms_per_step': d['ms_per_step'], 'value': d['value']}))" \
      "$R/gpurun_out/c5sweep_${TAG}_run.json" "$t" >> "$O" || exit 1
done
