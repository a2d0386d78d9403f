#!/bin/bash
# One SQ counter pass over a microbench run:  bash tools/sqpmc.sh <bench> <tag> [lib]
#   -> gpurun_out/sq_<tag>.txt (per-kernel sums of the counters for rbx kernels)
# SQ_COUNTERS overrides the counter list (at most 8 SQ_ counters per pass).
set -u
BENCH=$1; TAG=$2; LIBP=${3:-}
R=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
cd /tmp || exit 1
D=$R/gpurun_out/sq_$TAG
[ -n "$LIBP" ] && export RBX_LIB_PATH=$LIBP
CTRS=${SQ_COUNTERS:-SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY}
timeout -s KILL 120 rocprofv3 --pmc $CTRS \
  --kernel-trace --output-format csv -d "$D" -o p -- python3 "$R/tools/microbench.py" "$BENCH" > "$D.log" 2>&1 || exit 1
f=$(find "$D" -name "*counter_collection.csv" | head -1)
python3 - "$f" "$R/gpurun_out/sq_$TAG.txt" <<'PY'
import csv, sys, collections
acc = collections.defaultdict(lambda: collections.defaultdict(float))
for r in csv.DictReader(open(sys.argv[1])):
    n = r.get("Kernel_Name", "")
    if "rbx::" not in n:
        continue
    acc[n[:40]][r["Counter_Name"]] += float(r["Counter_Value"])
with open(sys.argv[2], "w") as o:
    for k, v in acc.items():
        o.write(k + "  " + "  ".join(f"{c}={int(x)}" for c, x in sorted(v.items())) + "\n")
PY
