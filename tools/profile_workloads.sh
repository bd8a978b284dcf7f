#!/bin/bash
# PMC traffic + unit counters of the closest-hit launches of the secondary
# workload lines (C3 PSSMLT, C4 ReSTIR, C5 NRC), in separate --pmc passes,
# summarised with the build's source hash and each workload's bench key
# (bench.traffic_key) so that tools/bench_workloads.py attaches them to a
# line of the same build and workload (the headline's roofline definition).
# Usage: tools/profile_workloads.sh TAG workload [workload ...]
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out; TAG=$1; shift; mkdir -p $OUT
UNITS="GRBM_GUI_ACTIVE TA_TA_BUSY_sum TCP_TCC_READ_REQ_sum SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"
for w in "$@"; do
  case $w in
    pssmlt|pssmltpath) BARGS="--workload $w --steps 1 --iterations 200 --no-cpu-baseline" ;;
    restir) BARGS="--workload $w --frames 3 --warmup 1 --no-cpu-baseline" ;;
    *) BARGS="--workload $w --steps 1 --no-cpu-baseline" ;;
  esac
  cd /tmp && export TMPDIR=/tmp
  for c in FETCH_SIZE WRITE_SIZE "$UNITS"; do
    n=$(echo $c | cut -d' ' -f1)
    echo "== $w pmc $n"
    timeout -s KILL 300 rocprofv3 --pmc $c -d $OUT/wl_${TAG}_${w}_$n -o pmc --output-format csv -- python3 $R/bench.py $BARGS > $OUT/wl_${TAG}_${w}_$n.log 2>&1
    rc=$?; [ $rc -ne 0 ] && { echo "pmc rc=$rc"; tail -5 $OUT/wl_${TAG}_${w}_$n.log; exit $rc; }
  done
  cd $R
  python3 tools/pmc_summary.py $OUT/wl_${TAG}_${w}_FETCH_SIZE $OUT/wl_${TAG}_${w}_WRITE_SIZE $OUT/${TAG}_${w}_pmc_traffic.json "$BARGS"
  python3 tools/pmc_units.py $OUT/wl_${TAG}_${w}_GRBM_GUI_ACTIVE $OUT/${TAG}_${w}_pmc_units.json "$BARGS"
done
exit 0
