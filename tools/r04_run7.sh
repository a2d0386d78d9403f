#!/bin/bash
# r04: full GPU suite, sparse-HLL first batch timing, default bench line
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04
mkdir -p "$O"
cd "$R"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$O/gpu_tests7.log" 2>&1
rc=$?
echo "tests rc=$rc" | tee -a "$O/gpu_tests7.log"
tail -5 "$O/gpu_tests7.log"
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
timeout -k 10 300 python -u tools/microbench.py hllfirst --keys 1000 > "$O/hllfirst7.jsonl" 2>&1 || { echo hllfirst failed; tail "$O/hllfirst7.jsonl"; exit 1; }
cat "$O/hllfirst7.jsonl"
timeout -k 10 400 python -u bench.py > "$O/bench7.json" 2> "$O/bench7.err" || { echo "bench failed"; tail -20 "$O/bench7.err"; exit 1; }
tail -c 600 "$O/bench7.json"
echo done
