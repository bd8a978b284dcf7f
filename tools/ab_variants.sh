#!/bin/bash
# A/B of library variants on one box, interleaved (A B A B ...) to cancel
# drift: one bench line per run with the variant name attached.
# Usage: tools/ab_variants.sh TAG ROUNDS "BENCH ARGS" variant1 variant2 ...
#   variant "base" = libmtx.so; others = libmtx_<name>.so (MTX_LIB_VARIANT)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
TAG=$1; ROUNDS=$2; ARGS=$3; shift 3
mkdir -p $OUT
cd $R
for i in $(seq 1 $ROUNDS); do
  for v in "$@"; do
    if [ "$v" = base ]; then V=""; else V=$v; fi
    MTX_LIB_VARIANT=$V timeout -k 10 300 python3 bench.py --no-cpu-baseline $ARGS > $OUT/ab_$TAG.tmp 2>> $OUT/ab_$TAG.err
    rc=$?
    [ $rc -ne 0 ] && { tail -5 $OUT/ab_$TAG.err; exit $rc; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); k=d['kernels']; print(json.dumps({'variant': sys.argv[2], 'round': int(sys.argv[3]), 'value': d['value'], 'ms': d['ms_per_step'], 'closest': k['trace_closest']['ms_per_step'], 'shadow': k['trace_shadow']['ms_per_step'], 'shade': k['shade']['ms_per_step'], 'other': k['other_ms_per_step'], 'nodes_per_ray': d['roofline']['node_visits_per_ray'], 'tris_per_ray': d['roofline']['tri_visits_per_ray'], 'rays': d['roofline'].get('rays_per_step'), 'shadow_rays': k['trace_shadow'].get('rays_per_step')}))" $OUT/ab_$TAG.tmp "$v" $i | tee -a $OUT/ab_$TAG.jsonl
  done
done
exit 0
