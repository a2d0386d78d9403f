#!/bin/bash
# Round-2 exploration on one GPU: slice-probe / region-gather rooflines, emit2 workgroup A/B,
# then C3 and C4 profiles.  Run through gpurun:  bash tools/r02_explore.sh
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
cd "$R" || exit 1
timeout -k 10 300 python3 tools/microbench.py slices regions --keys 1000000 > "$O/r02c_micro.jsonl" 2> "$O/r02c_micro.err" || exit 1
echo micro-ok
for i in 1 2; do
  for nt in 1024 512; do
    timeout -k 10 200 python3 bench.py --legs none --no-cpu-baseline --no-hostpath --tune contains_emit2_nt=$nt \
      > "$O/r02c_ab_emit2_${nt}_$i.json" 2>> "$O/r02c_ab.err" || exit 1
  done
done
echo ab-ok
RBX_STREAM_BYTES="k_bloom_contains_q=1.6e9 k_bloom_contains_multi=1.6e9" \
  timeout -k 10 700 bash tools/profile_round.sh r02c_c3 --workload c3 > "$O/r02c_prof_c3.log" 2>&1 || exit 1
echo prof-c3-ok
