#!/bin/bash
# One PMC pass (non-SQ counters) over a microbench run: bash tools/pmc_one.sh <bench> <tag> <counters...>
#   -> gpurun_out/pmc_<tag>.txt (per-kernel averages per launch for rbx kernels)
set -u
BENCH=$1; TAG=$2; shift 2
R=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
cd /tmp || exit 1
D=$R/gpurun_out/pmc_$TAG
timeout -s KILL 120 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d "$D" -o p -- python3 "$R/tools/microbench.py" "$BENCH" > "$D.log" 2>&1 || exit 1
f=$(find "$D" -name "*counter_collection.csv" | head -1)
python3 - "$f" "$R/gpurun_out/pmc_$TAG.txt" <<'PY'
import csv, sys, collections
acc = collections.defaultdict(lambda: collections.defaultdict(float))
n = collections.defaultdict(set)
for r in csv.DictReader(open(sys.argv[1])):
    k = r.get("Kernel_Name", "")
    if "rbx::" not in k:
        continue
    acc[k[:40]][r["Counter_Name"]] += float(r["Counter_Value"])
    n[k[:40]].add(r.get("Dispatch_Id", r.get("Correlation_Id", "")))
with open(sys.argv[2], "w") as o:
    for k, v in acc.items():
        c = max(1, len(n[k]))
        o.write(k + "  launches=%d  " % c + "  ".join(f"{x}={y / c:.4g}" for x, y in sorted(v.items())) + "\n")
PY
rm -rf "$D"
