#!/bin/bash
# Bench variants (no CPU baseline) on one GPU: one line per configuration.
# Usage: tools/perf_sweep.sh TAG "args1" "args2" ...   (each step time-limited)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
TAG=$1; shift
mkdir -p $OUT
cd $R
for a in "$@"; do
  echo "== bench $a"
  timeout -k 10 300 python3 bench.py --no-cpu-baseline $a >> $OUT/sweep_$TAG.jsonl 2>> $OUT/sweep_$TAG.err
  rc=$?; tail -1 $OUT/sweep_$TAG.jsonl | cut -c1-400; [ $rc -ne 0 ] && { tail -5 $OUT/sweep_$TAG.err; exit $rc; }
done
exit 0
