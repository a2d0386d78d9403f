#!/bin/bash
# r04: k = 20 / variable-key stream parity; C5 A/B of sc1 (L2-dropping) reply stores vs plain
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04
mkdir -p "$O"
cd "$R"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_c5_stream_gpu.py -m gpu -x -q -k "k20" --timeout 200 --timeout-method thread > "$O/gpu_tests12.log" 2>&1
rc=$?
echo "tests rc=$rc" | tee -a "$O/gpu_tests12.log"
tail -3 "$O/gpu_tests12.log"
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
: > "$O/c5_sc1_ab.jsonl"
for lib in librbx.so librbx_sc1.so librbx.so librbx_sc1.so; do
  RBX_LIB_PATH="$R/redisson_amd/$lib" timeout -k 10 240 python3 bench.py --workload c5 --steps 5 --warmup 1 --no-cpu-baseline > "$O/c5ab_run.json" 2> "$O/c5ab_run.err" || { echo "bench $lib failed"; tail "$O/c5ab_run.err"; exit 1; }
  python3 -c "
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(json.dumps({'lib': sys.argv[2], 'ms_per_step': d['ms_per_step'], 'value': d['value']}))" "$O/c5ab_run.json" "$lib" | tee -a "$O/c5_sc1_ab.jsonl"
done
echo done
