#!/bin/bash
# r04: C5 fresh stream at the 2^24 table -- occupancy filter and staged contains re-checked
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
export TMPDIR=/tmp
bash tools/c5_sweep.sh r04k - stream_occupancy=1 stream_contains_slots=0 - stream_occupancy=1 stream_contains_slots=0 || { echo sweep failed; exit 1; }
cat gpurun_out/c5sweep_r04k.jsonl
