#!/bin/bash
# Interleaved A/B of two builds of the library on one bench workload (each run a fresh process):
#   bash tools/lib_ab.sh <tag> <libA> <libB> <reps> <bench args...>      -> gpurun_out/<tag>/
set -e
TAG=$1; A=$2; B=$3; REPS=$4; shift 4
R=$(pwd); O=$R/gpurun_out/$TAG; mkdir -p $O
for rep in $(seq 1 $REPS); do
  for lib in $A $B; do
    RBX_LIB_PATH=$R/redisson_amd/$lib timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-hostpath "$@" \
      > $O/${lib}_$rep.json 2> $O/${lib}_$rep.err
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(json.dumps({'lib': sys.argv[2], 'rep': int(sys.argv[3]), 'ms_per_step': d['ms_per_step'], 'value': d['value']}))" \
      $O/${lib}_$rep.json $lib $rep | tee -a $O/ab.jsonl
  done
done
