#!/bin/bash
# Parity with the per-lane tail kernel forced early, then timing of tail
# thresholds at the per-rank size of an 8-GPU run (spp 32) and at spp 256.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
MTX_TAIL=1000000000 timeout -k 10 500 python3 -m pytest tests -q -m gpu -x -k "film or golden or fullsize or restir or sample" --timeout 300 > $OUT/pytest_tail.log 2>&1; rc=$?; tail -2 $OUT/pytest_tail.log; [ $rc -ne 0 ] && { grep -E "FAIL|assert" $OUT/pytest_tail.log | head; exit 1; }
bash tools/env_ab.sh tail32 2 "--spp 32 --steps 5 --warmup 2" "MTX_TAIL=0" "MTX_TAIL=1000000" "MTX_TAIL=4000000" "MTX_TAIL=16000000" || exit 1
bash tools/env_ab.sh tail256 2 "--steps 3 --warmup 1" "MTX_TAIL=0" "MTX_TAIL=4000000" "MTX_TAIL=16000000"
