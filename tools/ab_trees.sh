#!/bin/bash
# Interleaved A/B of two source trees on one box: the working tree and a
# baseline snapshot (git archive of a commit into _ab/<name>, built in place;
# _ab/ is git-ignored but travels to the GPU box). One compact line per run.
# Usage: tools/ab_trees.sh TAG ROUNDS "BENCH ARGS" name1 name2 ...  (name "." = the working tree;
# "name@VAR=val,VAR2=val" adds environment settings)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
TAG=$1; ROUNDS=$2; ARGS=$3; shift 3
for i in $(seq 1 $ROUNDS); do
  for t in "$@"; do
    # "tree@VAR=val,VAR2=val" runs the tree with those environment settings
    tr=${t%%@*}; ENVS=""; [ "$tr" != "$t" ] && ENVS=$(echo ${t#*@} | tr ',' ' ')
    if [ "$tr" = . ]; then D=$R; else D=$R/_ab/$tr; fi
    (cd $D && env $ENVS timeout -k 10 300 python3 bench.py --no-cpu-baseline $ARGS) > $OUT/abt_$TAG.tmp 2>> $OUT/abt_$TAG.err
    rc=$?; [ $rc -ne 0 ] && { tail -5 $OUT/abt_$TAG.err; exit $rc; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); k=d['kernels']; g=lambda n: k.get(n,{}).get('ms_per_step'); r=d['roofline']; print(json.dumps({'tree': sys.argv[2], 'round': int(sys.argv[3]), 'value': d['value'], 'ms': d['ms_per_step'], 'closest': g('trace_closest'), 'shadow': g('trace_shadow'), 'shade': g('shade'), 'other': k.get('other_ms_per_step'), 'nodes_per_ray': r.get('node_visits_per_ray'), 'tris_per_ray': r.get('tri_visits_per_ray'), 'shadow_nodes': k['trace_shadow'].get('node_visits_per_ray'), 'shadow_tris': k['trace_shadow'].get('tri_visits_per_ray')}))" $OUT/abt_$TAG.tmp "$t" $i | tee -a $OUT/abt_$TAG.jsonl
  done
done
exit 0
