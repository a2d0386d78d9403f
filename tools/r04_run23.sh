#!/bin/bash
# r04: C5 PMC profile on the fresh stream (the new default)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
export TMPDIR=/tmp
bash tools/profile_all.sh r04f c5 || { echo profile failed; exit 1; }
ls gpurun_out/profile_r04f_c5/
