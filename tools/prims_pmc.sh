#!/bin/bash
# Kernel trace + PMC passes of tools/prims_probe.py (group-by primitives).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/pp_${1:-a}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/trace -o t --output-format csv -- python3 $R/tools/prims_probe.py > $OUT/trace.log 2>&1 || { tail $OUT/trace.log; exit 1; }
grep ms $OUT/trace.log
i=0
for c in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT" "SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM_WR SQ_LDS_IDX_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $c -d $OUT/pmc$i -o p --output-format csv -- python3 $R/tools/prims_probe.py --reps 1 > $OUT/pmc$i.log 2>&1 || { echo "pmc $i failed"; tail -3 $OUT/pmc$i.log; exit 1; }
done
exit 0
