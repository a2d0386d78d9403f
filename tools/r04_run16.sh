#!/bin/bash
# r04: C5 prefilter size re-swept with the 8-byte first-setter table (interleaved repeats)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
export TMPDIR=/tmp
bash tools/c5_sweep.sh r04p - stream_prefilter=22 stream_prefilter=21 stream_prefilter=20 stream_prefilter=0 - stream_prefilter=22 stream_prefilter=20 stream_prefilter=24 || { echo sweep failed; exit 1; }
cat gpurun_out/c5sweep_r04p.jsonl
