#!/bin/bash
# Interleaved A/B of MTX_* environment settings on one
# box: one compact line per run. Usage: tools/env_ab.sh TAG ROUNDS "BENCH ARGS" "VAR=a" "VAR=b VAR2=c" ...
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
TAG=$1; ROUNDS=$2; ARGS=$3; shift 3
for i in $(seq 1 $ROUNDS); do
  for e in "$@"; do
    env $e timeout -k 10 300 python3 bench.py --no-cpu-baseline $ARGS > $OUT/envab_$TAG.tmp 2>> $OUT/envab_$TAG.err
    rc=$?; [ $rc -ne 0 ] && { tail -5 $OUT/envab_$TAG.err; exit $rc; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); k=d.get('kernels',{}); g=lambda n: k.get(n,{}).get('ms_per_step'); print(json.dumps({'env': sys.argv[2], 'round': int(sys.argv[3]), 'value': d['value'], 'ms': d['ms_per_step'], 'closest': g('trace_closest'), 'shadow': g('trace_shadow'), 'shade': g('shade')}))" $OUT/envab_$TAG.tmp "$e" $i | tee -a $OUT/envab_$TAG.jsonl
  done
done
exit 0
