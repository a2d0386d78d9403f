#!/bin/bash
# r04 first GPU call: GPU tests, the default bench line, the gather-rate sweep, the counter list.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04
mkdir -p "$O"
cd "$R"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$O/gpu_tests.log" 2>&1
rc=$?
echo "tests rc=$rc" | tee -a "$O/gpu_tests.log"
tail -15 "$O/gpu_tests.log"
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1   # a crash or a time limit: no further GPU step
timeout -k 10 400 python -u bench.py > "$O/bench.json" 2> "$O/bench.err" || { echo "bench failed"; tail -20 "$O/bench.err"; exit 1; }
timeout -k 10 300 python -u tools/microbench.py gather > "$O/gather_sweep.jsonl" 2>&1 || { echo "gather failed"; exit 1; }
(cd /tmp && timeout -k 10 120 rocprofv3 -L > "$O/rocprofv3_list.txt" 2>&1) || echo "list rc=$?"
echo done
