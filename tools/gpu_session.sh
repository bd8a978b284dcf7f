#!/bin/bash
# GPU session: GPU tests of the given files under each library
# variant (MTX_LIB_VARIANT), then an interleaved A/B of environment settings
# (tools/env_ab.sh). Every GPU step has its own time limit; the first failure
# ends the session.
# Usage: tools/gpu_session.sh TAG "TEST FILES|none" "VARIANTS (e.g. '- m1')" ROUNDS "ENV1" "ENV2" ...
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
TAG=$1; FILES=$2; VARS=$3; ROUNDS=$4; shift 4
if [ "$FILES" != none ]; then
  for v in $VARS; do
    [ "$v" = - ] && v=""
    echo "== pytest $FILES variant '$v'"
    MTX_LIB_VARIANT=$v timeout -k 10 500 python3 -u -m pytest $FILES -m gpu -x -q --timeout 240 --timeout-method thread > $OUT/pytest_${TAG}_$v.log 2>&1
    rc=$?; tail -3 $OUT/pytest_${TAG}_$v.log; [ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" $OUT/pytest_${TAG}_$v.log | head -20; exit $rc; }
  done
fi
if [ "$ROUNDS" != 0 ]; then
  echo "== env ab"
  bash tools/env_ab.sh $TAG $ROUNDS "--steps 3 --warmup 1" "$@" || exit 1
fi
exit 0
