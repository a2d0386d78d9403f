#!/bin/bash
# r04: per-kernel C5 times at three prefilter sizes (rocprofv3 kernel trace)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
export TMPDIR=/tmp
for pf in 16 23 0; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/r04pf/pf$pf" -o run -- \
    python3 "$R/bench.py" --workload c5 --steps 3 --warmup 1 --no-cpu-baseline --tune "stream_prefilter=$pf" \
    > "$R/gpurun_out/r04pf_$pf.json" 2> "$R/gpurun_out/r04pf_$pf.err" || { echo "pf $pf failed"; tail -5 "$R/gpurun_out/r04pf_$pf.err"; exit 1; }
  find "$R/gpurun_out/r04pf/pf$pf" -type f ! -name "*kernel_stats.csv" -delete
  echo "pf $pf done"
done
find "$R/gpurun_out/r04pf" -name "*kernel_stats.csv" | sort
