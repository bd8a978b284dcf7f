#!/bin/bash
# Round-end set on one box: smoke, pytest -m gpu, every workload line, kernel
# traces of the secondary configurations, headline bench + trace + PMC traffic.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out; TAG=${1:-r2e}; mkdir -p $OUT; cd $R
echo "== smoke"; timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke_$TAG.log 2>&1 || { tail -5 $OUT/smoke_$TAG.log; exit 1; }
echo "== pytest"; timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_$TAG.log 2>&1; rc=$?; tail -2 $OUT/pytest_$TAG.log; [ $rc -ne 0 ] && exit $rc
bash tools/workload_session.sh $TAG nrc restir pssmlt pssmltpath prims field nerad || exit 1
bash tools/profile_round.sh $TAG
