#!/bin/bash
# One PMC pass for LDS bank conflicts per kernel of a workload (default: the
# primitives): conflict cycles / (LDS active - conflict) as rocprofv3's
# LdsBankConflict, LDS utilisation as LdsUtil. Usage: tools/pmc_lds.sh TAG [WORKLOAD]
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out; TAG=${1:-lds}; WL=${2:-prims}; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_LDS_ADDR_CONFLICT SQ_WAVE_CYCLES -d $OUT/lds_$TAG -o pmc --output-format csv -- python3 $R/bench.py --workload $WL --steps 1 --no-cpu-baseline > $OUT/lds_$TAG.log 2>&1
rc=$?; [ $rc -ne 0 ] && { echo "pmc rc=$rc"; tail -5 $OUT/lds_$TAG.log; exit $rc; }
cd $R
python3 - $OUT/lds_$TAG <<'PY'
import collections, csv, glob, os, sys
tot = collections.defaultdict(lambda: collections.defaultdict(float)); disp = collections.defaultdict(set)
for f in glob.glob(os.path.join(sys.argv[1], "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "")
        tot[k][r["Counter_Name"]] += float(r["Counter_Value"]); disp[k].add(r["Dispatch_Id"])
for k, c in sorted(tot.items()):
    act, bc = c.get("SQ_LDS_IDX_ACTIVE", 0), c.get("SQ_LDS_BANK_CONFLICT", 0)
    if c.get("SQ_INSTS_LDS", 0) == 0: continue
    cyc = c.get("GRBM_GUI_ACTIVE", 0) / 8  # per-XCD sum (MI355X_MICROARCH.md)
    print(f"{k[:48]:48s} n={len(disp[k]):3d} lds_insts={c['SQ_INSTS_LDS']/len(disp[k]):12.0f} "
          f"bank_conflict={bc/max(act-bc,1):.3f} addr_conflict={c.get('SQ_LDS_ADDR_CONFLICT',0)/max(act,1):.3f} "
          f"lds_util={act/max(cyc*256,1):.3f}")
PY
