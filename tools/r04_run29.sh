#!/bin/bash
# r04: C5 8-byte table scale -- C5 tests, then the fresh-stream A/B
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04
mkdir -p "$O"
cd "$R"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_c5_stream_gpu.py -m gpu -x -q --timeout 400 --timeout-method thread > "$O/gpu_tests29.log" 2>&1
rc=$?
echo "tests rc=$rc"; tail -3 "$O/gpu_tests29.log"
[ $rc -eq 0 ] || exit 1
bash tools/c5_sweep.sh r04s - stream_table_scale=2 stream_table_scale=4 - stream_table_scale=2 stream_table_scale=4 || { echo sweep failed; exit 1; }
cat gpurun_out/c5sweep_r04s.jsonl
