#!/bin/bash
# r04: C5 reply bit-ring -- parity, A/B sweep, per-kernel stats
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04
mkdir -p "$O"
cd "$R"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_c5_stream_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > "$O/gpu_tests10.log" 2>&1
rc=$?
echo "tests rc=$rc" | tee -a "$O/gpu_tests10.log"
tail -5 "$O/gpu_tests10.log"
[ $rc -eq 0 ] || exit 1
bash tools/c5_sweep.sh r04g - stream_reply_ring=0 - stream_reply_ring=0 || { echo sweep failed; exit 1; }
cat gpurun_out/c5sweep_r04g.jsonl
for t in stream_reply_ring=1 stream_reply_ring=0; do
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/ks_$t" -o run -- python3 "$R/bench.py" --workload c5 --steps 5 --warmup 1 --no-cpu-baseline --tune "$t" > "$O/ks_$t.log" 2>&1) || { echo "kstats $t failed"; exit 1; }
  f=$(find "$O/ks_$t" -name "*kernel_stats.csv" | head -1); cp "$f" "$O/kstats_c5_$t.csv"; rm -rf "$O/ks_$t"
done
echo done
