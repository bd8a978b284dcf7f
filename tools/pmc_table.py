"""Per-kernel table of rocprofv3 --pmc counter_collection CSVs (sum over the
dispatches of each kernel name, divided by their count): usage
pmc_table.py DIR [DIR ...]"""
import collections
import csv
import glob
import re
import sys

acc = collections.defaultdict(lambda: collections.defaultdict(float))
cnt = collections.defaultdict(set)
for d in sys.argv[1:]:
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            m = re.search(r"(k_\w+(<[^>]*>)?)", r["Kernel_Name"])
            k = m.group(1) if m else r["Kernel_Name"][:40]
            acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
            cnt[(k, r["Counter_Name"])].add(r["Dispatch_Id"])
for k, cs in acc.items():
    print(k)
    for c, v in sorted(cs.items()):
        nd = len(cnt[(k, c)])
        print(f"    {c:28s} {v / nd:16.4g}   (x{nd})")
