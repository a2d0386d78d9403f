#!/bin/bash
# rocprof kernel stats + PMC traffic for the C2 headline and the C3 / C4 / C5 legs -> gpurun_out/,
# merged into gpurun_out/traffic_<tag>.json (copy to profiles/traffic.json to feed bench.py).
# Run through gpurun:  bash tools/profile_all.sh <tag>
set -u
TAG=${1:-r02}
ONLY=${2:-c2,c3,c4,c5}  # subset of workloads (a gpurun call has 20 minutes)
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out"
if [[ ",$ONLY," == *",c2,"* ]]; then
RBX_STREAM_BYTES="k_bk_stage1=3.2e9 k_bloom_contains=3.2e9" \
  timeout -k 10 1200 bash "$R/tools/profile_round.sh" "${TAG}_c2" --workload c2 || exit 1
fi
if [[ ",$ONLY," == *",c3,"* ]]; then
RBX_STREAM_BYTES="k_bloom_contains_q=1.6e9 k_bloom_contains_multi=1.6e9 k_maddx_gather=1.333e8 k_madd_seg=1.6e9" \
  timeout -k 10 1200 bash "$R/tools/profile_round.sh" "${TAG}_c3" --workload c3 || exit 1
fi
[[ ",$ONLY," == *",c4,"* ]] && { timeout -k 10 1200 bash "$R/tools/profile_round.sh" "${TAG}_c4" --workload c4 || exit 1 ; }
if [[ ",$ONLY," == *",c5,"* ]]; then
RBX_STREAM_BYTES="k_stream_contains_q=4.84e8 k_stream_probe=5.37e7 k_stream_probe8=5.37e7 k_stream_commit=5.37e7" \
  timeout -k 10 1200 bash "$R/tools/profile_round.sh" "${TAG}_c5" --workload c5 || exit 1
fi
python3 - "$R/gpurun_out" "$TAG" <<'PY'
import json, sys
d, tag = sys.argv[1], sys.argv[2]
out = {}
for w in ("c2", "c3", "c4", "c5"):
    try:
        out.update(json.load(open(f"{d}/profile_{tag}_{w}/traffic.json")))
    except OSError:
        pass
json.dump(out, open(f"{d}/traffic_{tag}.json", "w"), indent=1, sort_keys=True)
PY
echo "profile_all $TAG ok"
