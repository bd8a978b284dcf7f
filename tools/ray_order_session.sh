#!/bin/bash
# Ray-order experiment (tools/ray_order_experiment.py) under a kernel trace.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out; TAG=${1:-ro}; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace -d $OUT/ro_${TAG} -o t --output-format csv -- python3 $R/tools/ray_order_experiment.py ${2:-} > $OUT/ro_${TAG}.log 2>&1 || { tail -20 $OUT/ro_${TAG}.log; exit 1; }
cd $R && python3 tools/ray_order_summary.py $(ls $OUT/ro_${TAG}/*kernel_trace.csv | head -1) $OUT/ro_${TAG}.log $OUT/ro_${TAG}.jsonl
