#!/bin/bash
# r04 second call: the new C5 / node tests, then a C5 A/B (8-byte table vs r03 table, replies on/off)
# and a C5 profile with atomic counters.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04
mkdir -p "$O"
cd "$R"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_c5_stream_gpu.py tests/test_node_gpu.py tests/test_hll_gpu.py tests/test_lifecycle_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > "$O/gpu_tests2.log" 2>&1
rc=$?
echo "tests rc=$rc" | tee -a "$O/gpu_tests2.log"
tail -15 "$O/gpu_tests2.log"
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
bash tools/c5_sweep.sh r04a - stream_table8=0 c5_replies=0 stream_table8=0,c5_replies=0 - stream_table8=0 || { echo sweep failed; exit 1; }
cat gpurun_out/c5sweep_r04a.jsonl
bash tools/profile_round.sh r04_c5 --workload c5 || { echo profile failed; exit 1; }
echo done
