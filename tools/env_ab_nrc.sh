#!/bin/bash
# Interleaved A/B of MTX_* settings on the C5 NRC + radiance-cache line
# (bench.py --workload nrc, last line): value and the cache pass's encode /
# MLP times. Usage: tools/env_ab_nrc.sh TAG ROUNDS "VAR=a" "VAR=b VAR2=c" ...
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
TAG=$1; ROUNDS=$2; shift 2
for i in $(seq 1 $ROUNDS); do
  for e in "$@"; do
    env $e timeout -k 10 300 python3 bench.py --no-cpu-baseline --workload nrc --steps 5 --warmup 2 > $OUT/envnrc_$TAG.tmp 2>> $OUT/envnrc_$TAG.err
    rc=$?; [ $rc -ne 0 ] && { tail -5 $OUT/envnrc_$TAG.err; exit $rc; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); c=d['config']; print(json.dumps({'env': sys.argv[2], 'round': int(sys.argv[3]), 'value': d['value'], 'ms': d['ms_per_step'], 'encode_ms': c.get('cache_encode_ms'), 'mlp_ms': c.get('cache_mlp_ms'), 'queries': c.get('cache_queries_per_step')}))" $OUT/envnrc_$TAG.tmp "$e" $i | tee -a $OUT/envnrc_$TAG.jsonl
  done
done
exit 0
