#!/bin/bash
# r04: C5 fresh stream -- prefilter size A/B, interleaved twice
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
export TMPDIR=/tmp
bash tools/c5_sweep.sh r04g c5_fresh=1 c5_fresh=1,stream_prefilter=0 c5_fresh=1,stream_prefilter=24 c5_fresh=1,stream_prefilter=25 c5_fresh=1,stream_prefilter=22 c5_fresh=1 c5_fresh=1,stream_prefilter=0 c5_fresh=1,stream_prefilter=24 c5_fresh=1,stream_prefilter=25 || { echo sweep failed; exit 1; }
cat gpurun_out/c5sweep_r04g.jsonl
