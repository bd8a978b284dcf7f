#!/bin/bash
# rocprofv3 passes over a short bench run: kernel trace + stats, then the
# HBM counters (FETCH_SIZE, WRITE_SIZE: separate passes, they do not fit one)
# and SQ wave-state counters. Counter passes use --pmc with nothing else.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
TAG=${1:-r1}
BARGS=${2:-"--steps 1 --warmup 0 --no-cpu-baseline"}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
echo "== kernel trace"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof_$TAG -o trace --output-format csv -- python3 $R/bench.py $BARGS > $OUT/prof_${TAG}_trace.log 2>&1 || { echo "trace rc=$?"; tail -5 $OUT/prof_${TAG}_trace.log; exit 1; }
tail -1 $OUT/prof_${TAG}_trace.log | cut -c1-200
for pass in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM"; do
  name=$(echo $pass | cut -d' ' -f1)
  echo "== pmc $pass"
  timeout -k 10 600 rocprofv3 --pmc $pass -d $OUT/prof_${TAG}_$name -o pmc --output-format csv -- python3 $R/bench.py $BARGS > $OUT/prof_${TAG}_$name.log 2>&1 || { echo "pmc rc=$?"; tail -5 $OUT/prof_${TAG}_$name.log; exit 1; }
done
find $OUT/prof_$TAG* -name "*.csv" | head -20
exit 0
