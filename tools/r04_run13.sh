#!/bin/bash
# r04 experiment: C5 with the stream contains' key loads through buffer loads with cache-policy
# bits (a19: sc0 nt sc1, a17: sc0 sc1) vs the shipped global nt loads; interleaved, one process each
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04
mkdir -p "$O"
cd "$R"
export TMPDIR=/tmp
: > "$O/c5_keyaux_ab.jsonl"
for lib in librbx.so librbx_a19.so librbx_a17.so librbx.so librbx_a19.so librbx_a17.so; do
  RBX_LIB_PATH="$R/redisson_amd/$lib" timeout -k 10 240 python3 bench.py --workload c5 --steps 5 --warmup 1 --no-cpu-baseline > "$O/c5ab_run.json" 2> "$O/c5ab_run.err" || { echo "bench $lib failed"; tail "$O/c5ab_run.err"; exit 1; }
  python3 -c "
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(json.dumps({'lib': sys.argv[2], 'ms_per_step': d['ms_per_step'], 'value': d['value']}))" "$O/c5ab_run.json" "$lib" | tee -a "$O/c5_keyaux_ab.jsonl"
done
for lib in librbx.so librbx_a19.so; do
  (cd /tmp && RBX_LIB_PATH="$R/redisson_amd/$lib" timeout -s KILL 240 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum --kernel-trace --output-format csv -d "$O/pmc_$lib" -o p -- python3 "$R/bench.py" --workload c5 --steps 3 --warmup 1 --no-cpu-baseline > "$O/pmc_$lib.log" 2>&1) || { echo "pmc $lib failed"; exit 1; }
  f=$(find "$O/pmc_$lib" -name "*counter_collection.csv" | head -1); { head -1 "$f"; grep "k_stream_contains_q" "$f" | cat; } > "$O/pmc_keyaux_$lib.csv"; rm -rf "$O/pmc_$lib"
done
echo done
