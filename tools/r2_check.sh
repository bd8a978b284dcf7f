#!/bin/bash
# Round-2 check session: smoke, pytest -m gpu, headline bench N=1, then the
# N=2 strong-scaling rehearsal (two gloo ranks sharing the box's one GPU).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
TAG=${1:-r2}
K=${2:-""}   # optional pytest -k filter
mkdir -p $OUT
cd $R
echo "== smoke"; timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke_$TAG.log 2>&1
rc=$?; tail -2 $OUT/smoke_$TAG.log; [ $rc -ne 0 ] && { echo "smoke rc=$rc"; exit $rc; }
echo "== pytest -m gpu"
if [ -n "$K" ]; then
  timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "$K" > $OUT/pytest_gpu_$TAG.log 2>&1
else
  timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu_$TAG.log 2>&1
fi
rc=$?; grep -E "passed|failed|error" $OUT/pytest_gpu_$TAG.log | tail -3; [ $rc -ne 0 ] && { tail -40 $OUT/pytest_gpu_$TAG.log; echo "pytest rc=$rc"; exit $rc; }
echo "== bench N=1"; timeout -k 10 400 python3 bench.py --steps 5 --warmup 2 > $OUT/bench_$TAG.json 2> $OUT/bench_$TAG.err
rc=$?; cut -c1-600 $OUT/bench_$TAG.json; [ $rc -ne 0 ] && { tail -5 $OUT/bench_$TAG.err; echo "bench rc=$rc"; exit $rc; }
echo "== bench N=2 gloo rehearsal"; timeout -k 10 400 python3 bench.py --gpus 2 --backend gloo --steps 2 --warmup 1 > $OUT/bench2_$TAG.json 2> $OUT/bench2_$TAG.err
rc=$?; cut -c1-400 $OUT/bench2_$TAG.json; [ $rc -ne 0 ] && { tail -5 $OUT/bench2_$TAG.err; echo "bench2 rc=$rc"; exit $rc; }
exit 0
