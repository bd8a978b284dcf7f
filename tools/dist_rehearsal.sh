#!/bin/bash
# 1-GPU rehearsal of the N>1 workload lines: 2 ranks sharing cuda:0 over
# gloo (host-staged device tensors), one torchrun per workload, each step
# time-limited; stops at the first failure.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
TAG=${1:-r1}
shift
W=${@:-"path_mis restir pssmlt"}
mkdir -p $OUT
cd $R
port=29531
for w in $W; do
  echo "== rehearsal $w x2 (gloo)"
  timeout -k 10 600 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port $port bench.py --workload $w --gpus 2 --backend gloo --steps 1 --frames 3 --spp 64 --no-cpu-baseline \
    >> $OUT/rehearsal_$TAG.jsonl 2>> $OUT/rehearsal_$TAG.err
  rc=$?; tail -1 $OUT/rehearsal_$TAG.jsonl | cut -c1-400; [ $rc -ne 0 ] && { tail -8 $OUT/rehearsal_$TAG.err; exit $rc; }
  port=$((port + 1))
done
exit 0
