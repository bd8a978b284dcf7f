#!/bin/bash
# Diagnostic SQ counter passes over one headline step (stall breakdown per
# kernel: wave cycles split into active / waiting-on-memory / issue-stalled,
# instruction mix). Counters absent from `rocprofv3 -L` are dropped from a
# pass before it runs. Usage: tools/pmc_diag.sh TAG ["BENCH ARGS"]
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/diag_${1:-a}
BARGS=${2:-"--steps 1 --warmup 0 --no-cpu-baseline"}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > $OUT/counters.txt 2>&1 || { echo "rocprofv3 -L failed"; tail -3 $OUT/counters.txt; exit 1; }
i=0
for pass in \
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM" \
  "SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_IFETCH" \
  "SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR SQ_WAIT_INST_LDS SQ_ACTIVE_INST_MISC SQ_INSTS_BRANCH SQ_ACTIVE_INST_FLAT SQ_INSTS_FLAT SQ_INSTS_SMEM" \
  "TA_TA_BUSY_sum TA_BUFFER_WAVEFRONTS_sum TCP_TOTAL_CACHE_ACCESS_sum TCP_TCC_READ_REQ_sum" \
  "SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_ANY SQ_WAVE_CYCLES"; do
  i=$((i+1))
  keep=""
  for c in $pass; do
    base=${c%_sum}
    if grep -qw "$base" $OUT/counters.txt; then keep="$keep $c"; else echo "drop $c"; fi
  done
  [ -z "$keep" ] && continue
  echo "== pass $i:$keep"
  timeout -s KILL 150 rocprofv3 --pmc $keep -d $OUT/p$i -o p --output-format csv -- python3 $R/bench.py $BARGS > $OUT/p$i.log 2>&1 || { echo "pass $i rc=$?"; tail -3 $OUT/p$i.log; exit 1; }
done
cd $R
python3 tools/pmc_dispatch.py $OUT/p* > $OUT/table.txt 2>&1
head -40 $OUT/table.txt
exit 0
