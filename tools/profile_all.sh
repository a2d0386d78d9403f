#!/bin/bash
# Bench lines + rocprof kernel stats + PMC traffic for every workload -> gpurun_out/
# Run through gpurun:  bash tools/profile_all.sh <tag>
set -u
TAG=${1:-r01c}
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out"
for w in c2 c3 c4 c5; do
  timeout -k 10 400 python3 "$R/bench.py" --workload $w > "$R/gpurun_out/bench_${TAG}_$w.json" 2> "$R/gpurun_out/bench_${TAG}_$w.err" || exit 1
  echo "bench $w ok"
  timeout -k 10 1200 bash "$R/tools/profile_round.sh" "${TAG}_$w" --workload $w || exit 1
done
echo "profile_all $TAG ok"
