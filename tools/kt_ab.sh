set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
cd /tmp || exit 1
for i in 1 2; do
  for tag in old new; do
    if [ $tag = old ]; then L=$R/tools/_ab/librbx_r01k.so; else L=$R/redisson_amd/librbx.so; fi
    RBX_LIB_PATH=$L timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/kt_${tag}_$i -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline > $R/gpurun_out/kt_${tag}_$i.log 2>&1 || exit 1
    f=$(find $R/gpurun_out/kt_${tag}_$i -name "*kernel_stats.csv" | head -1)
    grep -E "k_ba_" "$f" | awk -F'","' -v t=$tag '{print t, substr($1,1,40), $4}' >> $R/gpurun_out/kt_summary.txt
  done
done
