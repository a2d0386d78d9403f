#!/bin/bash
# Profiles one bench workload on one GPU: kernel-trace stats + separate PMC passes (FETCH_SIZE /
# WRITE_SIZE / TCC hit+miss / EA read+write requests / TCC + EA atomic requests) -> gpurun_out/profile_<tag>/, then the
# per-access-class traffic (tools/pmc_traffic.py) -> gpurun_out/profile_<tag>/traffic.json.
# Run through gpurun:  bash tools/profile_round.sh <tag> [--workload c2|c3|c4|c5 ...]
# RBX_STREAM_BYTES: "kernel=bytes ..." streamed (key) bytes per launch of the mixed-class kernels
# (default: C2's 100M x 32-byte keys through k_bk_stage1 and the direct kernel).
set -u
TAG=${1:-r02}; shift || true
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/profile_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp || exit 1
B="$R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-hostpath --legs none $*"
SB=${RBX_STREAM_BYTES:-"k_bk_stage1=3.2e9 k_bloom_contains=3.2e9"}
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- python3 $B > "$OUT/trace.log" 2>&1 || exit 1
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$OUT/pmc_fetch" -o p -- python3 $B > "$OUT/pmc_fetch.log" 2>&1 || exit 1
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d "$OUT/pmc_write" -o p -- python3 $B > "$OUT/pmc_write.log" 2>&1 || exit 1
timeout -s KILL 240 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace --output-format csv -d "$OUT/pmc_tcc" -o p -- python3 $B > "$OUT/pmc_tcc.log" 2>&1 || exit 1
timeout -s KILL 240 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum --kernel-trace --output-format csv -d "$OUT/pmc_req" -o p -- python3 $B > "$OUT/pmc_req.log" 2>&1 || exit 1
# atomic requests at the L2 and those executed at memory (EA): the atomic-throughput evidence
timeout -s KILL 240 rocprofv3 --pmc TCC_ATOMIC_sum TCC_EA0_ATOMIC_sum --kernel-trace --output-format csv -d "$OUT/pmc_atomic" -o p -- python3 $B > "$OUT/pmc_atomic.log" 2>&1 || exit 1
# API calls per bench run: warmup 2 + steps 5 of the measured op; C2 also adds twice (scratch warm-up + setup),
# and its tryInit(448_089_842, 0.01) filter adds once and contains 4 times (extra.c2_tryinit_nonpow2)
python3 "$R/tools/pmc_traffic.py" "$OUT/pmc_fetch" "$OUT/pmc_write" "$OUT/pmc_tcc" "$OUT/pmc_req" "$OUT/pmc_atomic" -o "$OUT/traffic.json" \
  --calls contains_pipeline=11 add_pipeline=3 stream_pipeline=7 madd_pipeline=7 maddx_pipeline=7 --stream-bytes $SB > /dev/null || exit 1
# keep summaries only (gpurun copies back <= 64 MiB): stats CSVs, our kernels' counter rows
for d in pmc_fetch pmc_write pmc_tcc pmc_req pmc_atomic; do
  f=$(find "$OUT/$d" -name "*counter_collection.csv" | head -1)
  [ -n "$f" ] && { head -1 "$f"; grep -E "rbx::" "$f" | cat; } > "$OUT/${d}_rbx_rows.csv"
done
find "$OUT" -name "*kernel_stats.csv" -exec cp {} "$OUT/kernel_stats.csv" \;
rm -rf "$OUT/pmc_fetch" "$OUT/pmc_write" "$OUT/pmc_tcc" "$OUT/pmc_req" "$OUT/pmc_atomic" "$OUT/trace"
echo "profile $TAG ok"
