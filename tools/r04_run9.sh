#!/bin/bash
# r04: HLL tests + warm first-batch timing; C5 PMC for both first-setter tables (atomics)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04
mkdir -p "$O"
cd "$R"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_hll_gpu.py tests/test_lifecycle_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > "$O/gpu_tests9.log" 2>&1
rc=$?
echo "tests rc=$rc" | tee -a "$O/gpu_tests9.log"
tail -3 "$O/gpu_tests9.log"
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
timeout -k 10 300 python -u tools/microbench.py hllfirst --keys 1000 > "$O/hllfirst9.jsonl" 2>&1 || { echo hllfirst failed; tail "$O/hllfirst9.jsonl"; exit 1; }
cat "$O/hllfirst9.jsonl"
bash tools/profile_round.sh r04_c5t16 --workload c5 --tune stream_table8=0 || { echo profile c5t16 failed; exit 1; }
bash tools/profile_round.sh r04_c5 --workload c5 || { echo profile c5 failed; exit 1; }
echo done
