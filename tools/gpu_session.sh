#!/bin/bash
# One GPU session: smoke -> parity tests -> bench -> rocprofv3 kernel trace.
# Each GPU step has its own time limit; the session stops at the first crash.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
TAG=${1:-r1}
MODE=${2:-all}
mkdir -p $OUT
cd $R
echo "== smoke"; timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke_$TAG.log 2>&1
rc=$?; tail -3 $OUT/smoke_$TAG.log; [ $rc -ne 0 ] && { echo "smoke rc=$rc"; exit $rc; }
echo "== pytest -m gpu"; timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu_$TAG.log 2>&1
rc=$?; tail -15 $OUT/pytest_gpu_$TAG.log; [ $rc -gt 1 ] && { echo "pytest rc=$rc"; exit $rc; }
[ "$MODE" = "tests" ] && exit 0
echo "== bench"; timeout -k 10 600 python3 bench.py --steps 3 --warmup 1 > $OUT/bench_$TAG.json 2> $OUT/bench_$TAG.err
rc=$?; cat $OUT/bench_$TAG.json; tail -5 $OUT/bench_$TAG.err; [ $rc -ne 0 ] && { echo "bench rc=$rc"; exit $rc; }
echo "== rocprofv3"; cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof_$TAG -o bench --output-format csv -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $OUT/prof_$TAG.log 2>&1
rc=$?; tail -3 $OUT/prof_$TAG.log; echo "rocprof rc=$rc"
find $OUT/prof_$TAG -name "*stats*" | head
exit $rc
