#!/bin/bash
# Bench under different MTX_* environment settings (no CPU baseline), one
# line per setting. Usage: tools/env_sweep.sh TAG "BENCH ARGS" "VAR=a VAR2=b" "VAR=c" ...
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
TAG=$1; shift
ARGS=$1; shift
mkdir -p $OUT
cd $R
for e in "$@"; do
  echo "== $e"
  env $e timeout -k 10 300 python3 bench.py --no-cpu-baseline $ARGS > $OUT/envsweep_$TAG.tmp 2>> $OUT/envsweep_$TAG.err
  rc=$?
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); d['env']=sys.argv[2]; print(json.dumps(d))" $OUT/envsweep_$TAG.tmp "$e" >> $OUT/envsweep_$TAG.jsonl
  tail -1 $OUT/envsweep_$TAG.jsonl | cut -c1-300; [ $rc -ne 0 ] && { tail -5 $OUT/envsweep_$TAG.err; exit $rc; }
done
exit 0
