#!/bin/bash
# Interleaved same-box A/B of two librbx builds on one bench workload:
#   bash tools/ab.sh <old.so> <workload> [rounds]   -> gpurun_out/ab_<workload>.jsonl
set -u
OLD=$1; W=$2; N=${3:-2}
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out"
for i in $(seq "$N"); do
  for lib in "$OLD" "$R/redisson_amd/librbx.so"; do
    RBX_LIB_PATH=$lib timeout -k 10 240 python3 "$R/bench.py" --workload "$W" --steps 10 --warmup 2 --no-cpu-baseline --no-hostpath --legs none \
      > "$R/gpurun_out/ab_run.log" 2>&1 || exit 1
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(json.dumps({'lib': sys.argv[2], 'ms_per_step': d['ms_per_step'], 'value': d['value'], 'add_ms': (d.get('add') or {}).get('ms_per_step')}))" \
      "$R/gpurun_out/ab_run.log" "$lib" >> "$R/gpurun_out/ab_$W.jsonl" || exit 1
  done
done
