#!/bin/bash
# Interleaved same-box A/B of rbx_tune settings on one bench workload:
#   bash tools/ab_tune.sh <workload> <rounds> <tuneA> <tuneB> [...]  -> gpurun_out/abt_<workload>.jsonl
# (a tune is "key=value[,key=value]"; "-" = defaults)
set -u
W=$1; N=$2; shift 2
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out"
for i in $(seq "$N"); do
  for t in "$@"; do
    tune=$t; [ "$t" = "-" ] && tune=""
    timeout -k 10 240 python3 "$R/bench.py" --workload "$W" --steps 10 --warmup 2 --no-cpu-baseline --no-hostpath --legs none \
      --tune "$tune" > "$R/gpurun_out/abt_run.log" 2>&1 || exit 1
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(json.dumps({'tune': sys.argv[2], 'ms_per_step': d['ms_per_step'], 'value': d['value'], 'add_ms': d.get('extra', {}).get('add_ms')}))" \
      "$R/gpurun_out/abt_run.log" "$t" >> "$R/gpurun_out/abt_$W.jsonl" || exit 1
  done
done
