set -u
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out; TAG=r2d; cd /tmp && export TMPDIR=/tmp
for w in restir nrc prims pssmlt; do
  echo "== trace $w"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/wprof_${TAG}_$w -o t --output-format csv -- python3 $R/bench.py --workload $w --steps 1 --cpu-seconds 1 > $OUT/wprof_${TAG}_$w.log 2>&1 || { echo "trace $w failed"; tail -5 $OUT/wprof_${TAG}_$w.log; exit 1; }
done
cd $R && bash tools/profile_round.sh $TAG
