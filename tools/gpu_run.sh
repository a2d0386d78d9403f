#!/bin/bash
# One parameterized GPU call (replaces the per-call rNN_run*.sh lease scripts):
#   bash tools/gpu_run.sh <tag> <step> [<step> ...]      -> gpurun_out/<tag>/
# ('+' inside an argument stands for a space)
# steps (run in order; the first failure, time limit or crash ends the call -- no GPU step after it):
#   tests            the whole -m gpu suite              tests=<pytest -k expr>   a subset
#   smoke            __graft_entry__.smoke()
#   bench            python bench.py (default line)      bench=<args, '+' for ' '>
#   kstats=<args>    rocprofv3 --kernel-trace --stats of bench.py <args> (summary CSV kept)
#   profile=<args>   tools/profile_round.sh <tag> <args> (kernel stats + PMC passes + traffic.json)
#   micro=<args>     python tools/microbench.py <args>
set -u
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R" || exit 1
export TMPDIR=/tmp
i=0
for step in "$@"; do
  i=$((i+1))
  name=${step%%=*}
  arg=""
  [ "$name" != "$step" ] && arg=${step#*=}
  arg=${arg//+/ }
  echo "[$TAG] step $i: $name $arg"
  case $name in
    tests)
      if [ -n "$arg" ]; then k=(-k "$arg"); else k=(); fi
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "${k[@]}" \
        > "$O/tests_$i.log" 2>&1
      rc=$?
      tail -4 "$O/tests_$i.log"
      [ $rc -eq 0 ] || { echo "tests rc=$rc"; grep -E "FAILED|Error|assert" "$O/tests_$i.log" | head -20; exit 1; } ;;
    smoke)
      timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke_$i.log" 2>&1 \
        || { echo "smoke failed"; tail -20 "$O/smoke_$i.log"; exit 1; }
      tail -1 "$O/smoke_$i.log" ;;
    bench)
      timeout -k 10 600 python -u bench.py $arg > "$O/bench_$i.json" 2> "$O/bench_$i.err" \
        || { echo "bench failed"; tail -20 "$O/bench_$i.err"; exit 1; }
      tail -c 600 "$O/bench_$i.json"; echo ;;
    kstats)
      D=$O/kstats_$i
      (cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$D" -o run -- \
        python3 "$R/bench.py" --no-cpu-baseline --no-hostpath $arg > "$D.log" 2>&1) \
        || { echo "kstats failed"; tail -20 "$D.log"; exit 1; }
      f=$(find "$D" -name "*kernel_stats.csv" | head -1)
      cp "$f" "$O/kernel_stats_$i.csv" && rm -rf "$D"
      python3 -c "
import csv,sys
for r in csv.DictReader(open(sys.argv[1])):
    if 'rbx' in r['Name']: print('%-60s %6s %9.4f ms' % (r['Name'][:60], r['Calls'], float(r['AverageNs'])/1e6))
" "$O/kernel_stats_$i.csv" ;;
    profile)
      bash tools/profile_round.sh "${TAG}_$i" $arg || { echo "profile failed"; exit 1; } ;;
    micro)
      timeout -k 10 600 python -u tools/microbench.py $arg > "$O/micro_$i.jsonl" 2> "$O/micro_$i.err" \
        || { echo "microbench failed"; tail -20 "$O/micro_$i.err"; exit 1; }
      tail -c 800 "$O/micro_$i.jsonl"; echo ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo "[$TAG] done"
