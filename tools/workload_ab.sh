#!/bin/bash
# Interleaved A/B of environment settings (e.g. MTX_LIB_VARIANT) on the
# secondary workloads: one compact line per run (value, ms and the kernel
# times bench.py reports). Usage:
#   tools/workload_ab.sh TAG ROUNDS "WORKLOADS" "VAR=a" "VAR=b" ...
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
TAG=$1; ROUNDS=$2; WL=$3; shift 3
for i in $(seq 1 $ROUNDS); do
  for w in $WL; do
    for e in "$@"; do
      env $e timeout -k 10 300 python3 bench.py --workload $w --steps 1 --no-cpu-baseline > $OUT/wlab_$TAG.tmp 2>> $OUT/wlab_$TAG.err
      rc=$?; [ $rc -ne 0 ] && { tail -5 $OUT/wlab_$TAG.err; exit $rc; }
      python3 -c "
import json, sys
for line in open(sys.argv[1]).read().strip().splitlines():  # one line per metric (prims: several)
    d = json.loads(line)
    k = {n: v.get('ms_per_step') for n, v in (d.get('kernels') or {}).items() if isinstance(v, dict)}
    print(json.dumps({'workload': sys.argv[4], 'env': sys.argv[2], 'round': int(sys.argv[3]), 'metric': d['metric'][:40],
                      'value': d['value'], 'unit': d['unit'], 'ms': d['ms_per_step'], 'kernels': k}))" $OUT/wlab_$TAG.tmp "$e" $i $w | tee -a $OUT/wlab_$TAG.jsonl
    done
  done
done
exit 0
