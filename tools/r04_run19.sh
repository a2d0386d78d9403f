#!/bin/bash
# r04: C5 with a fresh stream per step (new (tenant, key) pairs) vs the replayed stream; prefilter sizes
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
export TMPDIR=/tmp
bash tools/c5_sweep.sh r04f - c5_fresh=1 c5_fresh=1,stream_prefilter=16 c5_fresh=1,stream_prefilter=20 c5_fresh=1,stream_prefilter=0 c5_fresh=1,stream_prefilter=24 - c5_fresh=1 || { echo sweep failed; exit 1; }
cat gpurun_out/c5sweep_r04f.jsonl
