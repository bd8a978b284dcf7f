#!/bin/bash
# One PMC pass for memory latency and wait states per kernel (one bench step):
# SQ_INST_LEVEL_VMEM / (SQ_INSTS_VMEM_RD + _WR) = average cycles a VMEM
# instruction is in flight; SQ_WAIT_ANY / SQ_WAVE_CYCLES = share of wave time
# waiting on a counter. Usage: tools/pmc_latency.sh TAG
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out; TAG=${1:-lat}; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INST_LEVEL_LDS -d $OUT/lat_$TAG -o pmc --output-format csv -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline > $OUT/lat_$TAG.log 2>&1
rc=$?; [ $rc -ne 0 ] && { echo "pmc rc=$rc"; tail -5 $OUT/lat_$TAG.log; exit $rc; }
cd $R
python3 - $OUT/lat_$TAG <<'PY'
import collections, csv, glob, os, sys
tot = collections.defaultdict(lambda: collections.defaultdict(float)); disp = collections.defaultdict(set)
for f in glob.glob(os.path.join(sys.argv[1], "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "")
        tot[k][r["Counter_Name"]] += float(r["Counter_Value"]); disp[k].add(r["Dispatch_Id"])
for k, c in sorted(tot.items()):
    if c.get("GRBM_GUI_ACTIVE", 0) / 8 / len(disp[k]) < 1e5: continue
    vm = c.get("SQ_INSTS_VMEM_RD", 0) + c.get("SQ_INSTS_VMEM_WR", 0)
    print(f"{k[:36]:36s} n={len(disp[k]):3d} vmem_lat={c.get('SQ_INST_LEVEL_VMEM',0)/max(vm,1):8.1f} "
          f"wait={c.get('SQ_WAIT_ANY',0)/max(c.get('SQ_WAVE_CYCLES',1),1):.3f} "
          f"wait_inst={c.get('SQ_WAIT_INST_ANY',0)/max(c.get('SQ_WAVE_CYCLES',1),1):.3f} "
          f"active={c.get('SQ_ACTIVE_INST_ANY',0)/max(c.get('SQ_WAVE_CYCLES',1),1):.3f} "
          f"vmem_wr_frac={c.get('SQ_INSTS_VMEM_WR',0)/max(vm,1):.3f}")
PY
