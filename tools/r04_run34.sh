#!/bin/bash
# r04: C1 leg kernel trace (what a 1M-key add spends its 0.19 ms on)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/r04c1" -o run -- \
  python3 bench.py --legs c1 --steps 1 --warmup 1 --no-cpu-baseline --no-hostpath --leg-steps 10 \
  > gpurun_out/c1prof.json 2> gpurun_out/c1prof.err || { echo "run failed"; tail -5 gpurun_out/c1prof.err; exit 1; }
find "$R/gpurun_out/r04c1" -type f ! -name "*kernel_stats.csv" -delete
echo ok
