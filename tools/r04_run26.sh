#!/bin/bash
# r04: C5 probe claims batched vs serial -- C5 tests, then the fresh-stream A/B
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04
mkdir -p "$O"
cd "$R"
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_c5_stream_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > "$O/gpu_tests26.log" 2>&1
rc=$?
echo "tests rc=$rc"; tail -3 "$O/gpu_tests26.log"
[ $rc -eq 0 ] || exit 1
bash tools/c5_sweep.sh r04b - stream_probe_batch=0 - stream_probe_batch=0 - || { echo sweep failed; exit 1; }
cat gpurun_out/c5sweep_r04b.jsonl
