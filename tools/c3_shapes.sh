#!/bin/bash
# A/B of the contains kernels on C3 (multi-tenant): staged doubling (stage1 4) vs the per-lane
# slot kernel (stage1 5) over shapes (P*10+Q) and grids.  Usage: c3_shapes.sh "shapes" "grids" [reps]
# -> gpurun_out/c3_shapes/runs.jsonl (one line per run: stage1, shape, grid, ms)
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/c3_shapes
SHAPES=${1:-"22 32 42"}
GRIDS=${2:-"2048 4096 8192"}
REPS=${3:-1}
mkdir -p "$O"
row() {  # stage1 shape grid json-file
  python3 -c "import json,sys; d=json.load(open('$4')); print(json.dumps({'stage1': $1, 'shape': $2, 'grid': $3, 'ms': d['ms_per_step'], 'keys_per_s': d['value']}))" >> "$O/runs.jsonl"
}
for r in $(seq $REPS); do
  timeout -k 10 120 python "$R/bench.py" --workload c3 --stage1 4 --no-cpu-baseline --steps 10 > "$O/last.json" 2>> "$O/err.log" || exit 1
  row 4 0 0 "$O/last.json"
  for sh in $SHAPES; do
    for g in $GRIDS; do
      timeout -k 10 120 python "$R/bench.py" --workload c3 --stage1 5 --tune contains_qshape=$sh,contains_qgrid=$g \
        --no-cpu-baseline --steps 10 > "$O/last.json" 2>> "$O/err.log" || exit 1
      row 5 $sh $g "$O/last.json"
    done
  done
done
echo done
