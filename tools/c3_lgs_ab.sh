set -u
mkdir -p gpurun_out/c3lgs
for t in add_multi_seg_lgs=12 add_multi_seg_lgs=11 add_multi_seg_lgs=12 add_multi_seg_lgs=11; do
  timeout -k 10 300 python bench.py --workload c3 --steps 6 --warmup 2 --no-cpu-baseline --no-hostpath --legs none --tune $t > gpurun_out/c3lgs/run.json 2> gpurun_out/c3lgs/run.err || exit 1
  python3 -c "
import json,sys
d=json.loads(open('gpurun_out/c3lgs/run.json').read().strip().splitlines()[-1])
a=d.get('add') or d.get('extra',{}).get('add') or {}
print(json.dumps({'tune': sys.argv[1], 'contains_ms': d['ms_per_step'], 'add_ms': a.get('ms_per_step'), 'add_new': a.get('new_keys_per_step')}))" $t >> gpurun_out/c3lgs/ab.jsonl || exit 1
done
