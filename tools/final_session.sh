#!/bin/bash
# Round-end measurement set, part 1: every GPU test, then the headline
# profile set (tools/profile_round.sh: bench line, rocprofv3 kernel trace +
# stats, PMC traffic and unit counters). Usage: tools/final_session.sh TAG
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out; TAG=$1; mkdir -p $OUT; cd $R
echo "== pytest"
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_$TAG.log 2>&1
rc=$?; tail -3 $OUT/pytest_$TAG.log; [ $rc -ne 0 ] && { grep -E "FAIL|Error" $OUT/pytest_$TAG.log | head -20; exit $rc; }
bash tools/profile_round.sh $TAG
