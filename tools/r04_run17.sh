#!/bin/bash
# r04: C5 prefilter below 2^20 bits (interleaved repeats)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
export TMPDIR=/tmp
bash tools/c5_sweep.sh r04q stream_prefilter=20 stream_prefilter=19 stream_prefilter=18 stream_prefilter=17 stream_prefilter=16 - stream_prefilter=18 stream_prefilter=20 stream_prefilter=19 || { echo sweep failed; exit 1; }
cat gpurun_out/c5sweep_r04q.jsonl
