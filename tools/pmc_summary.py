"""Summarise rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes per kernel.

FETCH_SIZE / WRITE_SIZE are kilobytes of L2 <-> fabric traffic (Infinity-
Cache hits included). On gfx950 FETCH_SIZE reports half of the bytes of wide
coalesced reads, so it is doubled (/opt/skills/guides/MI355X_MICROARCH.md,
HBM section); WRITE_SIZE is taken as is.

    python tools/pmc_summary.py FETCH_DIR WRITE_DIR OUT.json ["BENCH ARGS"]

The JSON records the source hash of the profiled build (bench.src_sha()) and
the bench key of the profiled command (bench.traffic_key of BENCH ARGS), so
bench.py attaches the traffic only to a run of the same build and config.
"""
import collections
import csv
import glob
import json
import os
import sys


def per_kernel(d, counter):
    tot = collections.defaultdict(float)
    n = collections.Counter()
    for f in glob.glob(os.path.join(d, "*counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != counter:
                continue
            k = r["Kernel_Name"].split("(")[0].replace("void ", "")
            tot[k] += float(r["Counter_Value"]) * 1024.0
            n[k] += 1
    return tot, n


def main(fetch_dir, write_dir, out, bench_args=""):
    f, nf = per_kernel(fetch_dir, "FETCH_SIZE")
    w, _ = per_kernel(write_dir, "WRITE_SIZE")
    res = {}
    for k in sorted(f):
        res[k] = {"launches": nf[k], "fetch_bytes_raw": f[k], "fetch_bytes_x2": 2 * f[k], "write_bytes": w.get(k, 0.0),
                  "hbm_bytes_per_launch": (2 * f[k] + w.get(k, 0.0)) / max(1, nf[k])}
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench

    sys.argv = ["bench.py"] + bench_args.split()
    key = bench.traffic_key(bench.parse())
    json.dump({"source": [fetch_dir, write_dir], "correction": "FETCH_SIZE x2 (gfx950), KB -> bytes",
               "src_sha": bench.src_sha(), "bench_args": bench_args, "bench_key": key,
               "kernels": res}, open(out, "w"), indent=1)
    for k, v in res.items():
        print(f"{k:45s} n={v['launches']:4d} HBM/launch={v['hbm_bytes_per_launch'] / 1e9:8.3f} GB")


if __name__ == "__main__":
    main(*sys.argv[1:5])
