#!/bin/bash
# GPU parity tests (optional -k filter), then an interleaved A/B of MTX_*
# environment settings at several spp; stops at a crash / timeout of the tests.
# Usage: tools/tests_then_envab.sh TAG ROUNDS "K" "SPPS" "VAR=a" "VAR=b" ...
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
TAG=$1; ROUNDS=$2; K=$3; SPPS=$4; shift 4
if [ -n "$K" ]; then KK=(-k "$K"); else KK=(); fi
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread "${KK[@]}" > $OUT/pytest_$TAG.log 2>&1
rc=$?; tail -2 $OUT/pytest_$TAG.log
[ $rc -gt 1 ] && { echo "pytest rc=$rc: stopping"; exit $rc; }
[ $rc -eq 1 ] && { grep -E "^FAILED|Error" $OUT/pytest_$TAG.log | head -10; exit 1; }
bash tools/env_ab_spp.sh $TAG $ROUNDS "$SPPS" "$@"
