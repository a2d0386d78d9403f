#!/bin/bash
# r04: C1 leg -- partitioned add vs first-setter table add at launch scale (1M keys, 12 MB bitmap)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
export TMPDIR=/tmp
for t in "" "add_partition=0" "" "add_partition=0"; do
  timeout -k 10 300 python3 bench.py --legs c1 --steps 2 --warmup 1 --no-cpu-baseline --no-hostpath --leg-steps 20 --tune "$t" \
    > gpurun_out/c1ab.json 2> gpurun_out/c1ab.err || { echo "run failed"; tail -5 gpurun_out/c1ab.err; exit 1; }
  python3 -c "
import json,sys
d=json.loads(open('gpurun_out/c1ab.json').read().strip().splitlines()[-1])
c=d['legs']['c1']; print(json.dumps({'tune': sys.argv[1], 'value': c['value'], 'add_ms': c['add_ms'], 'contains_ms': c['contains_ms']}))" "$t" | tee -a gpurun_out/c1ab.jsonl
done
