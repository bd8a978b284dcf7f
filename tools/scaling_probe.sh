#!/bin/bash
# Per-rank workload of the strong-scaling curve on ONE GPU: bench.py at the
# spp one rank of N traces (256/N), plus a kernel trace of the N=8 share, to
# see what does not shrink with the work (launch tails, film, fixed costs).
# Usage: tools/scaling_probe.sh TAG
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out; TAG=${1:-sp}; mkdir -p $OUT; cd $R
for spp in 256 128 64 32; do
  timeout -k 10 300 python3 bench.py --spp $spp --steps 5 --warmup 2 --no-cpu-baseline > $OUT/scal_${TAG}_$spp.json 2> $OUT/scal_${TAG}_$spp.err || { tail -5 $OUT/scal_${TAG}_$spp.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); k=d['kernels']; print(json.dumps({'spp': int(sys.argv[2]), 'ms': d['ms_per_step'], 'closest': k['trace_closest']['ms_per_step'], 'shadow': k['trace_shadow']['ms_per_step'], 'shade': k['shade']['ms_per_step'], 'other': k['other_ms_per_step']}))" $OUT/scal_${TAG}_$spp.json $spp | tee -a $OUT/scal_${TAG}.jsonl
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/scal_${TAG}_prof -o t --output-format csv -- python3 $R/bench.py --spp 32 --steps 2 --warmup 1 --no-cpu-baseline > $OUT/scal_${TAG}_prof.log 2>&1
