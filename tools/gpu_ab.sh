#!/bin/bash
# Parity (pytest -m gpu, optional -k filter) then an interleaved A/B of
# library variants on one box. Usage: tools/gpu_ab.sh TAG ROUNDS "K" v1 v2 ...
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
TAG=$1; ROUNDS=$2; K=$3; shift 3
echo "== pytest"
if [ -n "$K" ]; then
  timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$K" > $OUT/pytest_$TAG.log 2>&1
else
  timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_$TAG.log 2>&1
fi
rc=$?; tail -2 $OUT/pytest_$TAG.log; [ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" $OUT/pytest_$TAG.log | head -20; exit $rc; }
echo "== ab"; bash tools/ab_variants.sh $TAG $ROUNDS "--steps 3 --warmup 1" "$@"
