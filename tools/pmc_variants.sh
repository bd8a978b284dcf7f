#!/bin/bash
# SQ instruction/stall counters of the traversal kernels for library variants
# (one headline step per pass), summed per kernel over the step's launches.
# Usage: tools/pmc_variants.sh TAG variant1 variant2 ...   ("base" = libmtx.so)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out/pmcv_$1; shift; mkdir -p $OUT
BARGS="--steps 1 --warmup 0 --no-cpu-baseline"
cd /tmp && export TMPDIR=/tmp
for v in "$@"; do
  V=$v; [ "$v" = base ] && V=""
  i=0
  for pass in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD" "SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU TA_TA_BUSY_sum"; do
    i=$((i+1))
    MTX_LIB_VARIANT=$V timeout -s KILL 150 rocprofv3 --pmc $pass -d $OUT/${v}_p$i -o p --output-format csv -- python3 $R/bench.py $BARGS > $OUT/${v}_p$i.log 2>&1 || { echo "pmc $v $i failed"; tail -3 $OUT/${v}_p$i.log; exit 1; }
  done
done
cd $R
python3 - "$OUT" "$@" <<'PY'
import collections, csv, glob, json, os, sys
out, variants = sys.argv[1], sys.argv[2:]
res = {}
for v in variants:
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    for f in glob.glob(os.path.join(out, f"{v}_p*", "*counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0].replace("void ", "")
            if "trace_closest<false>" in k or "trace_shadow<false>" in k or "k_shade<2>" in k:
                agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
    res[v] = {k: dict(c) for k, c in agg.items()}
json.dump(res, open(os.path.join(out, "summary.json"), "w"), indent=1)
for v, ks in res.items():
    for k, c in ks.items():
        print(v, k, " ".join(f"{n}={c[n]:.3e}" for n in sorted(c)))
PY
exit 0
