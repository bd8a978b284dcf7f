#!/bin/bash
# C4 per-rank band probe (tools/restir_band_probe.py) after the ReSTIR GPU
# tests: default build, then each "VAR=value" environment given, then a
# rocprofv3 kernel trace of the default. Usage: tools/band_profile.sh TAG [VAR=value ...]
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out; TAG=${1:-band}; shift; mkdir -p $OUT; cd $R
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "restir or occlusion" > $OUT/pytest_$TAG.log 2>&1 || { tail -20 $OUT/pytest_$TAG.log; exit 1; }
tail -2 $OUT/pytest_$TAG.log
for v in default "$@"; do
  if [ $v = default ]; then E=""; else E="$v"; fi
  env $E timeout -k 10 300 python3 tools/restir_band_probe.py > $OUT/${TAG}_probe_tmp.jsonl 2> $OUT/${TAG}_probe.err || { tail -5 $OUT/${TAG}_probe.err; exit 1; }
  sed "s/^{/{\"env\": \"$v\", /" $OUT/${TAG}_probe_tmp.jsonl >> $OUT/${TAG}_probe.jsonl
  cut -c1-330 $OUT/${TAG}_probe_tmp.jsonl
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/prof_$TAG -o kt --output-format csv -- python3 $R/tools/restir_band_probe.py --frames 5 --warmup 2 > $OUT/prof_$TAG.log 2>&1 || { tail -5 $OUT/prof_$TAG.log; exit 1; }
exit 0
