#!/bin/bash
# r04: per-kernel C5 times with a fresh stream per step (rocprofv3 kernel trace; L2 is perturbed by
# the per-dispatch completion signals, so totals are above the unprofiled ones)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
export TMPDIR=/tmp
for v in "c5_fresh=1" "c5_fresh=1,stream_table8=0"; do
  d=$(echo "$v" | tr ',=' '__')
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/r04fr/$d" -o run -- \
    python3 "$R/bench.py" --workload c5 --steps 3 --warmup 1 --no-cpu-baseline --tune "$v" \
    > "$R/gpurun_out/r04fr_$d.json" 2> "$R/gpurun_out/r04fr_$d.err" || { echo "$v failed"; tail -5 "$R/gpurun_out/r04fr_$d.err"; exit 1; }
  find "$R/gpurun_out/r04fr/$d" -type f ! -name "*kernel_stats.csv" -delete
  echo "$v done"
done
