#!/bin/bash
# r04: rebucket's empty-item search vectorized -- Bloom parity suite, then the C1 leg and the C2 add
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04
mkdir -p "$O"
cd "$R"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_bloom_gpu.py -m gpu -x -q --timeout 400 --timeout-method thread > "$O/gpu_tests35.log" 2>&1
rc=$?
echo "tests rc=$rc"; tail -2 "$O/gpu_tests35.log"
[ $rc -eq 0 ] || exit 1
: > gpurun_out/c1ab35.jsonl
for i in 1 2; do
  timeout -k 10 300 python3 bench.py --legs c1 --steps 2 --warmup 1 --no-cpu-baseline --no-hostpath --leg-steps 20 \
    > gpurun_out/c1ab.json 2> gpurun_out/c1ab.err || { echo "run failed"; tail -5 gpurun_out/c1ab.err; exit 1; }
  python3 -c "
import json
d=json.loads(open('gpurun_out/c1ab.json').read().strip().splitlines()[-1])
c=d['legs']['c1']; print(json.dumps({'c2_add_ms': d['extra']['add_ms'], 'c1': c['value'], 'add_ms': c['add_ms'], 'contains_ms': c['contains_ms']}))" | tee -a gpurun_out/c1ab35.jsonl
done
