#!/bin/bash
# r04: C5 chunks sized by the 8-byte table's position field -- C5 tests, then the fresh-stream A/B
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04
mkdir -p "$O"
cd "$R"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_c5_stream_gpu.py -m gpu -x -v --timeout 400 --timeout-method thread > "$O/gpu_tests28.log" 2>&1
rc=$?
echo "tests rc=$rc"; grep -E "PASS|FAIL|passed|failed" "$O/gpu_tests28.log" | tail -4
[ $rc -eq 0 ] || exit 1
bash tools/c5_sweep.sh r04d - stream_chunk=6710784 - stream_chunk=6710784 || { echo sweep failed; exit 1; }
cat gpurun_out/c5sweep_r04d.jsonl
