#!/bin/bash
# Headline measurement set for one build: bench line, rocprofv3 kernel trace
# + stats of the same command, then the HBM counters in separate --pmc passes
# (FETCH_SIZE, WRITE_SIZE), summarised with the build's source hash and the
# bench key (tools/pmc_summary.py) so that bench.py attaches the traffic.
# Usage: tools/profile_round.sh TAG
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
TAG=${1:-r2}
BARGS="--steps 1 --warmup 0 --no-cpu-baseline"
mkdir -p $OUT
cd $R
echo "== bench"; timeout -k 10 400 python3 bench.py --steps 5 --warmup 2 > $OUT/bench_$TAG.json 2> $OUT/bench_$TAG.err
rc=$?; cut -c1-300 $OUT/bench_$TAG.json; [ $rc -ne 0 ] && { tail -5 $OUT/bench_$TAG.err; exit $rc; }
cd /tmp && export TMPDIR=/tmp
echo "== kernel trace"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof_$TAG -o trace --output-format csv -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $OUT/prof_${TAG}_trace.log 2>&1
rc=$?; [ $rc -ne 0 ] && { echo "trace rc=$rc"; tail -5 $OUT/prof_${TAG}_trace.log; exit $rc; }
tail -1 $OUT/prof_${TAG}_trace.log | cut -c1-200
for c in FETCH_SIZE WRITE_SIZE; do
  echo "== pmc $c"
  timeout -s KILL 300 rocprofv3 --pmc $c -d $OUT/prof_${TAG}_$c -o pmc --output-format csv -- python3 $R/bench.py $BARGS > $OUT/prof_${TAG}_$c.log 2>&1
  rc=$?; [ $rc -ne 0 ] && { echo "pmc rc=$rc"; tail -5 $OUT/prof_${TAG}_$c.log; exit $rc; }
done
UNITS="GRBM_GUI_ACTIVE TA_TA_BUSY_sum TCP_TCC_READ_REQ_sum SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"
echo "== pmc units"
timeout -s KILL 300 rocprofv3 --pmc $UNITS -d $OUT/prof_${TAG}_units -o pmc --output-format csv -- python3 $R/bench.py $BARGS > $OUT/prof_${TAG}_units.log 2>&1
rc=$?; [ $rc -ne 0 ] && { echo "pmc units rc=$rc"; tail -5 $OUT/prof_${TAG}_units.log; exit $rc; }
cd $R
python3 tools/pmc_summary.py $OUT/prof_${TAG}_FETCH_SIZE $OUT/prof_${TAG}_WRITE_SIZE $OUT/${TAG}_pmc_traffic.json "$BARGS"
python3 tools/pmc_units.py $OUT/prof_${TAG}_units $OUT/${TAG}_pmc_units.json "$BARGS"
find $OUT/prof_$TAG -name "*stats*"
exit 0
