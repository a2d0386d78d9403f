#!/bin/bash
# r04: sparse-HLL shortcut parity + timing; XCD-routed C5 counters
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04
mkdir -p "$O"
cd "$R"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_hll_gpu.py tests/test_spring_data_gpu.py tests/test_node_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > "$O/gpu_tests6.log" 2>&1
rc=$?
echo "tests rc=$rc" | tee -a "$O/gpu_tests6.log"
tail -5 "$O/gpu_tests6.log"
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
timeout -k 10 300 python -u tools/microbench.py hllfirst --keys 1000 > "$O/hllfirst.jsonl" 2>&1 || { echo hllfirst failed; tail "$O/hllfirst.jsonl"; exit 1; }
cat "$O/hllfirst.jsonl"
bash tools/profile_round.sh r04_c5xr --workload c5 || { echo profile failed; exit 1; }
echo done
