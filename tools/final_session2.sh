#!/bin/bash
# Round-end measurement set, part 2: PMC traffic + unit counters of the
# secondary workloads (tools/profile_workloads.sh), copied into profiles/ of
# this snapshot so that the bench lines that follow attach them; then the
# headline bench line (with part 1's committed PMC) and one line per
# workload (tools/workload_session.sh). Usage: tools/final_session2.sh TAG
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out; TAG=$1; mkdir -p $OUT; cd $R
bash tools/profile_workloads.sh $TAG restir nrc pssmlt || exit 1
cp $OUT/${TAG}_*_pmc_traffic.json $OUT/${TAG}_*_pmc_units.json profiles/ || exit 1
echo "== bench"
timeout -k 10 400 python3 bench.py --steps 5 --warmup 2 > $OUT/bench2_$TAG.json 2> $OUT/bench2_$TAG.err || { tail -5 $OUT/bench2_$TAG.err; exit 1; }
cut -c1-300 $OUT/bench2_$TAG.json
bash tools/workload_session.sh $TAG nrc restir prims pssmlt
