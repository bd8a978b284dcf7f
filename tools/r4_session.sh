#!/bin/bash
# Round-4 GPU session: the GPU tests of the given files (or all), an
# interleaved A/B of source trees (tools/ab_trees.sh), and the C4 per-rank
# band probe. Every GPU step has its own time limit; the first failure ends it.
# Usage: tools/r4_session.sh TAG "TEST FILES|all|none" ROUNDS "trees..." [probe]
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
TAG=$1; FILES=$2; ROUNDS=$3; TREES=$4; PROBE=${5:-}
if [ "$FILES" != none ]; then
  [ "$FILES" = all ] && FILES=tests
  echo "== pytest $FILES"
  timeout -k 10 660 python3 -u -m pytest $FILES -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_$TAG.log 2>&1
  rc=$?; tail -3 $OUT/pytest_$TAG.log; [ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" $OUT/pytest_$TAG.log | head -20; exit $rc; }
fi
if [ "$ROUNDS" != 0 ]; then
  echo "== ab $TREES"
  bash tools/ab_trees.sh $TAG $ROUNDS "--steps 3 --warmup 1" $TREES || exit 1
fi
if [ -n "$PROBE" ]; then
  echo "== restir band probe"
  timeout -k 10 300 python3 tools/restir_band_probe.py > $OUT/${TAG}_restir_band_probe.jsonl 2> $OUT/${TAG}_probe.err || { tail -5 $OUT/${TAG}_probe.err; exit 1; }
  cut -c1-400 $OUT/${TAG}_restir_band_probe.jsonl
fi
exit 0
