#!/bin/bash
# r04: C5 fresh stream -- slot contains grid
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
export TMPDIR=/tmp
bash tools/c5_sweep.sh r04gq - stream_qgrid=1536 stream_qgrid=2048 stream_qgrid=768 - stream_qgrid=1536 stream_qgrid=2048 || { echo sweep failed; exit 1; }
cat gpurun_out/c5sweep_r04gq.jsonl
