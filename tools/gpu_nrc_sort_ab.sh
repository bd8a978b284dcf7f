cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_field.py -m gpu > gpurun_out/tf.log 2>&1 || { tail -30 gpurun_out/tf.log; exit 1; }
tail -3 gpurun_out/tf.log
for f in 0 1 0 1; do MTX_CACHE_SORT=$f timeout -k 10 300 python bench.py --workload nrc --no-cpu-baseline > gpurun_out/nrc_$f.jsonl 2> gpurun_out/nrc_$f.err || exit 1; python3 -c "
import json,sys
for l in open('gpurun_out/nrc_$f.jsonl'):
    d=json.loads(l); print('sort=$f', d['metric'][:40], d['value'], d['config'].get('cache_encode_ms'), d['config'].get('cache_mlp_ms'), d['config'].get('extra_ms_per_step'))
"; done
