#!/bin/bash
# Parity of the 256-thread trace-block variant, its A/B, and the counter list.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
MTX_LIB_VARIANT=tb256 timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "fullsize or render_film_bit_exact or trace" > $OUT/pytest_tb256.log 2>&1
rc=$?; tail -2 $OUT/pytest_tb256.log; [ $rc -ne 0 ] && { grep -E "^FAILED|Error" $OUT/pytest_tb256.log | head; exit $rc; }
bash tools/ab_variants.sh tb256 3 "--steps 3 --warmup 1" base tb256 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > $OUT/rocprof_counters.txt 2>&1
echo "counters rc=$?"
