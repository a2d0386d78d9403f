set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05o
mkdir -p $O
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/trace -o run -- python3 $R/tools/c1_only.py 20 > $O/trace.log 2>&1 || { tail -20 $O/trace.log; exit 1; }
find $O/trace -name "*.csv" -exec ls -la {} \;
for f in $(find $O/trace -name "*kernel_trace.csv" -o -name "*memory_copy_trace.csv"); do cp $f $O/; done
rm -rf $O/trace
echo done
