#!/bin/bash
# r04: full GPU suite (node worker pool, every parity test) + the default bench line
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04
mkdir -p "$O"
cd "$R"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$O/gpu_tests38.log" 2>&1
rc=$?
echo "tests rc=$rc" | tee -a "$O/gpu_tests38.log"
tail -5 "$O/gpu_tests38.log"
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")" || { echo "smoke failed"; exit 1; }
timeout -k 10 400 python -u bench.py > "$O/bench38.json" 2> "$O/bench38.err" || { echo "bench failed"; tail -20 "$O/bench38.err"; exit 1; }
tail -c 400 "$O/bench38.json"
echo done
