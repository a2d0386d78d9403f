#!/bin/bash
# r04: full GPU suite (node worker pool, every parity test) + the default bench line
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04
mkdir -p "$O"
cd "$R"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$O/gpu_tests11.log" 2>&1
rc=$?
echo "tests rc=$rc" | tee -a "$O/gpu_tests11.log"
tail -5 "$O/gpu_tests11.log"
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
timeout -k 10 400 python -u bench.py > "$O/bench11.json" 2> "$O/bench11.err" || { echo "bench failed"; tail -20 "$O/bench11.err"; exit 1; }
tail -c 400 "$O/bench11.json"
echo done
