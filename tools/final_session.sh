#!/bin/bash
# End-of-round measurement set: every §8 workload line (bench.py --workload,
# with its CPU baseline), kernel-trace stats of the C3/C4/C5 and primitive
# runs, then the headline bench + kernel trace + PMC traffic
# (tools/profile_round.sh). Usage: tools/final_session.sh TAG
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out; TAG=${1:-r2d}; mkdir -p $OUT; cd $R
bash tools/workload_session.sh $TAG nrc restir pssmlt pssmltpath prims field nerad || exit 1
cd /tmp && export TMPDIR=/tmp
for w in restir nrc prims pssmlt; do
  echo "== trace $w"
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/wprof_${TAG}_$w -o t --output-format csv -- python3 $R/bench.py --workload $w --steps 1 --no-cpu-baseline > $OUT/wprof_${TAG}_$w.log 2>&1 || { echo "trace $w failed"; tail -5 $OUT/wprof_${TAG}_$w.log; exit 1; }
done
cd $R
bash tools/profile_round.sh $TAG
