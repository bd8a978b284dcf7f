#!/bin/bash
# L2 hit / miss counts per kernel for the default build and the MTX_NT_STREAM=0 variant
# (libmtx_nt0.so): one --pmc pass each. Usage: tools/pmc_l2_hits.sh
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for v in nt0 default; do
  lib=""; [ $v = nt0 ] && lib=nt0
  for c in "TCC_HIT_sum TCC_MISS_sum" "FETCH_SIZE" "WRITE_SIZE"; do
    n=$(echo $c | cut -d' ' -f1)
    MTX_LIB_VARIANT=$lib timeout -s KILL 120 rocprofv3 --pmc $c -d $OUT/pmc_nt_${v}_$n -o p --output-format csv -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline > $OUT/pmc_nt_${v}_$n.log 2>&1 || { echo "pmc $v $n failed"; tail -3 $OUT/pmc_nt_${v}_$n.log; exit 1; }
  done
done
exit 0
