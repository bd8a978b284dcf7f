#!/bin/bash
# rocprofv3 --pmc passes (one per argument: space-separated counters) over a
# short bench run; counters only, no tracing domains in the same pass.
# Usage: tools/pmc.sh TAG "BENCH ARGS" "C1 C2 ..." ["C3 ..." ...]
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
TAG=$1; BARGS=$2; shift 2
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
i=0
for pass in "$@"; do
  i=$((i+1))
  echo "== pmc[$i] $pass"
  timeout -k 10 600 rocprofv3 --pmc $pass -d $OUT/pmc_${TAG}_$i -o pmc --output-format csv -- python3 $R/bench.py $BARGS > $OUT/pmc_${TAG}_$i.log 2>&1 || { echo "pmc rc=$?"; tail -5 $OUT/pmc_${TAG}_$i.log; exit 1; }
done
exit 0
