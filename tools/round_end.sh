#!/bin/bash
# Round-end measurement set (each GPU step time-limited; the first failure
# ends the call). Usage: tools/round_end.sh TAG PART
#   PART = main:      every GPU test, then the headline profile set
#                     (tools/profile_round.sh: bench line, rocprofv3 kernel
#                     trace + stats, PMC traffic and unit counters) and the
#                     per-rank strong-scaling probe (tools/scaling_probe.sh)
#   PART = workloads: PMC of the secondary workloads (tools/profile_workloads.sh),
#                     copied into profiles/ of this snapshot so that the bench
#                     lines that follow attach them; the headline bench line and
#                     one line per workload (tools/workload_session.sh)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out; TAG=$1; PART=${2:-main}; mkdir -p $OUT; cd $R
if [ "$PART" = main ]; then
  echo "== pytest"
  timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_$TAG.log 2>&1
  rc=$?; tail -3 $OUT/pytest_$TAG.log; [ $rc -ne 0 ] && { grep -E "FAIL|Error" $OUT/pytest_$TAG.log | head -20; exit $rc; }
  bash tools/profile_round.sh $TAG || exit 1
  bash tools/scaling_probe.sh $TAG
else
  bash tools/profile_workloads.sh $TAG restir nrc pssmlt || exit 1
  cp $OUT/${TAG}_*_pmc_traffic.json $OUT/${TAG}_*_pmc_units.json profiles/ || exit 1
  echo "== bench"
  timeout -k 10 400 python3 bench.py --steps 5 --warmup 2 > $OUT/bench2_$TAG.json 2> $OUT/bench2_$TAG.err || { tail -5 $OUT/bench2_$TAG.err; exit 1; }
  cut -c1-300 $OUT/bench2_$TAG.json
  bash tools/workload_session.sh $TAG nrc restir prims pssmlt
fi
