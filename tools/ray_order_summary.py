"""Pairs the k_trace_raw launches of a rocprofv3 kernel trace with the launch
tags tools/ray_order_experiment.py printed; prints min / median ms per order.
Usage: ray_order_summary.py KERNEL_TRACE_CSV EXPERIMENT_LOG [OUT.jsonl]"""
import csv
import json
import sys
from collections import defaultdict


def main(trace_csv, log, out=None):
    rows = [r for r in csv.DictReader(open(trace_csv)) if "k_trace_raw" in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    tags = [json.loads(l) for l in open(log) if l.startswith('{"launch"')]
    assert len(rows) == len(tags), (len(rows), len(tags))
    ms = defaultdict(list)
    for r, t in zip(rows, tags):
        ms[t["launch"]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6)
    lines = []
    for k, v in ms.items():
        v.sort()
        lines.append({"order": k, "ms_min": round(v[0], 3), "ms_med": round(v[len(v) // 2], 3), "n": len(v)})
    base = {l["order"]: l["ms_min"] for l in lines}
    for l in lines:
        kind = l["order"].split("_")[0]
        ref = base.get(kind + "_natural", base.get(kind + "_scanline"))
        if ref:
            l["vs_natural"] = round(l["ms_min"] / ref, 3)
        print(json.dumps(l))
    if out:
        with open(out, "a") as f:
            for l in lines:
                f.write(json.dumps(l) + "\n")


if __name__ == "__main__":
    main(*sys.argv[1:])
