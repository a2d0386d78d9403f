#!/bin/bash
# r04: C5 -- does the 8.4M-command chunk win by fewer chunks or by the table's lower load?
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
export TMPDIR=/tmp
bash tools/c5_sweep.sh r04l stream_chunk=6710784,stream_table_scale=2 stream_chunk=6710784 - stream_chunk=6710784,stream_table_scale=2 stream_chunk=6710784 - || { echo sweep failed; exit 1; }
cat gpurun_out/c5sweep_r04l.jsonl
