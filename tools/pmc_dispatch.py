"""Per-dispatch table of rocprofv3 --pmc passes (one directory per pass),
matched by Dispatch_Id (the passes run the same deterministic program).

    python tools/pmc_dispatch.py DIR1 DIR2 ... [--filter SUBSTR]
FETCH_SIZE is doubled (gfx950, MI355X_MICROARCH.md HBM section) and shown
in GB with WRITE_SIZE; the other counters are printed raw."""
import collections
import csv
import glob
import os
import sys


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    flt = None
    if "--filter" in sys.argv:
        flt = sys.argv[sys.argv.index("--filter") + 1]
        args.remove(flt)
    rows = collections.OrderedDict()
    names = []
    for d in args:
        for f in glob.glob(os.path.join(d, "*counter_collection.csv")):
            for r in csv.DictReader(open(f)):
                k = int(r["Dispatch_Id"])
                e = rows.setdefault(k, {"kernel": r["Kernel_Name"].split("(")[0].replace("void ", ""),
                                        "ms": (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6})
                c = r["Counter_Name"]
                v = float(r["Counter_Value"])
                if c == "FETCH_SIZE":
                    c, v = "fetch_GB", 2 * v * 1024 / 1e9
                elif c == "WRITE_SIZE":
                    c, v = "write_GB", v * 1024 / 1e9
                e[c] = e.get(c, 0.0) + v
                if c not in names:
                    names.append(c)
    print("id  kernel                            ms  " + "  ".join(f"{n[:22]:>22s}" for n in names))
    for k in sorted(rows):
        e = rows[k]
        if flt and flt not in e["kernel"]:
            continue
        vals = "  ".join(f"{e.get(n, float('nan')):22.4g}" for n in names)
        print(f"{k:<4d}{e['kernel'][:30]:30s}{e['ms']:8.3f}  {vals}")


if __name__ == "__main__":
    main()
