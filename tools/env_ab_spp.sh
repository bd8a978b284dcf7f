#!/bin/bash
# Interleaved A/B of MTX_* environment settings at several spp.
# Usage: tools/env_ab_spp.sh TAG ROUNDS "SPPS" "VAR=a" "VAR=b" ...
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
TAG=$1; ROUNDS=$2; SPPS=$3; shift 3
for i in $(seq 1 $ROUNDS); do
  for spp in $SPPS; do
    for e in "$@"; do
      env $e timeout -k 10 300 python3 bench.py --no-cpu-baseline --spp $spp --steps 5 --warmup 2 > $OUT/envspp_$TAG.tmp 2>> $OUT/envspp_$TAG.err
      rc=$?; [ $rc -ne 0 ] && { tail -5 $OUT/envspp_$TAG.err; exit $rc; }
      python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); k=d['kernels']; print(json.dumps({'env': sys.argv[2], 'spp': int(sys.argv[4]), 'round': int(sys.argv[3]), 'ms': d['ms_per_step'], 'closest': k['trace_closest']['ms_per_step'], 'shadow': k['trace_shadow']['ms_per_step'], 'shade': k['shade']['ms_per_step']}))" $OUT/envspp_$TAG.tmp "$e" $i $spp | tee -a $OUT/envspp_$TAG.jsonl
    done
  done
done
exit 0
