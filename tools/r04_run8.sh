#!/bin/bash
# r04: PMC of the C5 stream with the r03 first-setter table (atomic counts for the A/B), then the
# shipped tree's C2 profile (kernel stats + PMC incl. atomics)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
export TMPDIR=/tmp
bash tools/profile_round.sh r04_c5t16 --workload c5 --tune stream_table8=0 || { echo profile c5t16 failed; exit 1; }
bash tools/profile_round.sh r04_c5 --workload c5 || { echo profile c5 failed; exit 1; }
bash tools/profile_round.sh r04_c2 || { echo profile c2 failed; exit 1; }
echo done
