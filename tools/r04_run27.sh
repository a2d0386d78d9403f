#!/bin/bash
# r04: C5 fresh stream -- chunk size
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
export TMPDIR=/tmp
bash tools/c5_sweep.sh r04c - stream_chunk=3355392 stream_chunk=1677696 - stream_chunk=3355392 || { echo sweep failed; exit 1; }
cat gpurun_out/c5sweep_r04c.jsonl
