#!/bin/bash
# Interleaved A/B of environment settings (e.g. MTX_LIB_VARIANT=x) on the C4
# per-rank band probe (tools/restir_band_probe.py), after the ReSTIR GPU tests
# under each setting. Usage: tools/ab_band_env.sh TAG ROUNDS "ENV1" "ENV2" ...
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
TAG=$1; ROUNDS=$2; shift 2
for e in "$@"; do
  env $e timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "restir" > $OUT/pytest_$TAG.log 2>&1 || { tail -20 $OUT/pytest_$TAG.log; exit 1; }
  echo "$e: $(tail -1 $OUT/pytest_$TAG.log)"
done
for i in $(seq 1 $ROUNDS); do
  for e in "$@"; do
    env $e timeout -k 10 300 python3 tools/restir_band_probe.py > $OUT/abb_$TAG.tmp 2>> $OUT/abb_$TAG.err || { tail -5 $OUT/abb_$TAG.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(json.dumps({'env': sys.argv[2], 'round': int(sys.argv[3]), 'full_ms': d['full_frame_ms'], 'band_ms': d['band_frame_ms'], 'ratio': d['full_over_band'], 'band_kernels_ms': d.get('band_kernels_ms')}))" $OUT/abb_$TAG.tmp "$e" $i | tee -a $OUT/abb_$TAG.jsonl
  done
done
exit 0
