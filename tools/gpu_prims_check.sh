#!/bin/bash
# Group-by primitives on the GPU: parity tests, then the kernel trace + PMC
# passes of tools/prims_probe.py (tools/prims_pmc.sh TAG).
set -u
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_prims_edges.py tests/test_gpu_parity.py -k "hashgrid or scatter or prims or prefix" > gpurun_out/t1.log 2>&1 || { tail -40 gpurun_out/t1.log; exit 1; }
tail -3 gpurun_out/t1.log
bash tools/prims_pmc.sh ${1:-b}
