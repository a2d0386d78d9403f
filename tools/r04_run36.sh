#!/bin/bash
# r04: C1 calls alone under a kernel trace
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/r04c1b" -o run -- \
  python3 tools/c1_only.py 12 > gpurun_out/c1only.log 2>&1 || { echo "run failed"; tail -5 gpurun_out/c1only.log; exit 1; }
find "$R/gpurun_out/r04c1b" -type f ! -name "*kernel_stats.csv" -delete
echo ok
