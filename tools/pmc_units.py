"""Per-kernel unit occupancy from one rocprofv3 --pmc pass (tools/profile_round.sh):

    GRBM_GUI_ACTIVE TA_TA_BUSY_sum TCP_TCC_READ_REQ_sum SQ_BUSY_CYCLES
    SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR

Per launch (a kernel's counters summed over its dispatches / dispatches, so a
kernel that also runs in bench.py's untimed counter step is not counted twice):
  cycles      GRBM_GUI_ACTIVE / 8 (rocprofv3 sums the 8 XCDs; MI355X_MICROARCH.md)
  ta_busy     TA_TA_BUSY_sum / 256 CUs / cycles: the vector-memory address
              path (TA/TCP) of a CU, busy fraction
  valu_busy   SQ_INSTS_VALU x 2 / (4 SIMDs x 256 CUs) / cycles: a wave64 VALU
              instruction occupies a 32-lane gfx950 SIMD for 2 cycles
  salu_busy   SQ_INSTS_SALU / (4 x 256) / cycles (one scalar issue per SIMD-cycle)
  l1_l2_read_bytes  TCP_TCC_READ_REQ_sum x 128 B (a request per 128-B line)
  ta_cycles_per_vmem  TA busy cycles per VMEM wave-instruction

    python tools/pmc_units.py PASS_DIR OUT.json ["BENCH ARGS"]

The JSON records the source hash of the profiled build and the bench key (as
tools/pmc_summary.py), so bench.py attaches it only to the same build and run.
"""
import collections
import csv
import glob
import json
import os
import sys

N_CU, N_XCD, SIMDS = 256, 8, 4


def per_kernel(d):
    tot = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0].replace("void ", "")
            tot[k][r["Counter_Name"]] += float(r["Counter_Value"])
            disp[k].add(r["Dispatch_Id"])
    return tot, {k: len(v) for k, v in disp.items()}


def units(c, n):
    cyc = c.get("GRBM_GUI_ACTIVE", 0.0) / N_XCD / max(1, n)
    if cyc <= 0:
        return None
    per = {k: v / max(1, n) for k, v in c.items()}
    vmem = per.get("SQ_INSTS_VMEM_RD", 0.0) + per.get("SQ_INSTS_VMEM_WR", 0.0)
    ta = per.get("TA_TA_BUSY_sum", 0.0) / N_CU
    return {
        "launches": n,
        "cycles_per_launch": round(cyc),
        "ta_busy": round(ta / cyc, 4),
        "valu_busy": round(per.get("SQ_INSTS_VALU", 0.0) * 2 / (SIMDS * N_CU) / cyc, 4),
        "salu_busy": round(per.get("SQ_INSTS_SALU", 0.0) / (SIMDS * N_CU) / cyc, 4),
        "l1_l2_read_bytes_per_launch": round(per.get("TCP_TCC_READ_REQ_sum", 0.0) * 128),
        "vmem_insts_per_launch": round(vmem),
        "ta_cycles_per_vmem": round(per.get("TA_TA_BUSY_sum", 0.0) / max(1.0, vmem), 2),
        "raw_per_launch": {k: round(v) for k, v in sorted(per.items())},
    }


def main(pass_dir, out, bench_args=""):
    tot, n = per_kernel(pass_dir)
    res = {k: u for k in sorted(tot) if (u := units(tot[k], n[k])) is not None}
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench

    sys.argv = ["bench.py"] + bench_args.split()
    key = bench.traffic_key(bench.parse())
    json.dump({"source": pass_dir, "src_sha": bench.src_sha(), "bench_args": bench_args, "bench_key": key,
               "definition": __doc__.split("\n\n")[1].strip(), "kernels": res}, open(out, "w"), indent=1)
    for k, v in res.items():
        if v["cycles_per_launch"] > 1e5:
            print(f"{k[:40]:40s} n={v['launches']:3d} ta={v['ta_busy']:.3f} valu={v['valu_busy']:.3f} "
                  f"salu={v['salu_busy']:.3f} ta/vmem={v['ta_cycles_per_vmem']:.1f}")


if __name__ == "__main__":
    main(*sys.argv[1:4])
