#!/bin/bash
# r04: C5 defaults (fresh stream, no prefilter): C5 parity tests, then the default bench line
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04
mkdir -p "$O"
cd "$R"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_c5_stream_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > "$O/gpu_tests22.log" 2>&1
rc=$?
echo "tests rc=$rc"; tail -3 "$O/gpu_tests22.log"
[ $rc -eq 0 ] || exit 1
timeout -k 10 400 python -u bench.py > "$O/bench22.json" 2> "$O/bench22.err" || { echo "bench failed"; tail -20 "$O/bench22.err"; exit 1; }
tail -c 300 "$O/bench22.json"
echo done
