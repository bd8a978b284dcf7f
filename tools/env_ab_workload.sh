#!/bin/bash
# Interleaved A/B of MTX_* environment settings on one bench workload.
# Usage: tools/env_ab_workload.sh TAG ROUNDS WORKLOAD "VAR=a" "VAR=b" ...
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
TAG=$1; ROUNDS=$2; WL=$3; shift 3
for i in $(seq 1 $ROUNDS); do
  for e in "$@"; do
    env $e timeout -k 10 600 python3 bench.py --workload $WL --no-cpu-baseline > $OUT/envwl_$TAG.tmp 2>> $OUT/envwl_$TAG.err
    rc=$?; [ $rc -ne 0 ] && { tail -5 $OUT/envwl_$TAG.err; exit $rc; }
    python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(json.dumps({'env': sys.argv[2], 'round': int(sys.argv[3]), 'value': d['value'], 'ms': d['ms_per_step']}))" $OUT/envwl_$TAG.tmp "$e" $i | tee -a $OUT/envwl_$TAG.jsonl
  done
done
exit 0
