#!/bin/bash
# One line per SURVEY §8 configuration besides the headline bench (each step
# time-limited; stops at the first failure).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
TAG=${1:-r1}
shift
W=${@:-"nrc restir prims pssmlt"}
mkdir -p $OUT
cd $R
for w in $W; do
  echo "== workload $w"
  timeout -k 10 900 python3 bench.py --workload $w --steps 1 --cpu-seconds 8 >> $OUT/workloads_$TAG.jsonl 2>> $OUT/workloads_$TAG.err
  rc=$?; tail -1 $OUT/workloads_$TAG.jsonl | cut -c1-300; [ $rc -ne 0 ] && { tail -8 $OUT/workloads_$TAG.err; exit $rc; }
done
exit 0
