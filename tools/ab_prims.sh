#!/bin/bash
# Interleaved A/B of source trees on the primitive workloads (bench.py
# --workload prims: prefix_sum, hash grid, scatter_reduce), one compact line
# per workload and run. Usage: tools/ab_prims.sh TAG ROUNDS name1 name2 ...  ("." = working tree)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
TAG=$1; ROUNDS=$2; shift 2
for i in $(seq 1 $ROUNDS); do
  for t in "$@"; do
    if [ "$t" = . ]; then D=$R; else D=$R/_ab/$t; fi
    (cd $D && timeout -k 10 300 python3 bench.py --workload prims --steps 5 --no-cpu-baseline) > $OUT/abp_$TAG.tmp 2>> $OUT/abp_$TAG.err
    rc=$?; [ $rc -ne 0 ] && { tail -5 $OUT/abp_$TAG.err; exit $rc; }
    python3 -c "
import json,sys
for l in open(sys.argv[1]):
    l=l.strip()
    if not l.startswith('{'): continue
    d=json.loads(l); r=d.get('roofline') or {}
    print(json.dumps({'tree': sys.argv[2], 'round': int(sys.argv[3]), 'metric': d['metric'][:40], 'value': d['value'], 'ms': d['ms_per_step'], 'frac': r.get('frac')}))" $OUT/abp_$TAG.tmp "$t" $i | tee -a $OUT/abp_$TAG.jsonl
  done
done
exit 0
