"""bench.py's PMC attachment (CPU): a committed profile is used only for the
build (source hash) and bench arguments it measured."""
import json
import os
import sys

from conftest import ROOT

sys.path.insert(0, ROOT)


def _write(d, name, sha, key, kernels):
    os.makedirs(os.path.join(d, "profiles"), exist_ok=True)
    with open(os.path.join(d, "profiles", name), "w") as f:
        json.dump({"src_sha": sha, "bench_key": key, "kernels": kernels}, f)


def test_units_and_traffic_match_build_and_args(tmp_path, monkeypatch):
    import bench

    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    monkeypatch.setattr(sys, "argv", ["bench.py"])
    args = bench.parse()
    key, sha = bench.traffic_key(args), bench.src_sha()
    k = "mtxd::k_trace_closest<false>"
    u = {"ta_busy": 0.8, "valu_busy": 0.5, "salu_busy": 0.1, "l1_l2_read_bytes_per_launch": 1,
         "ta_cycles_per_vmem": 20.0, "raw_per_launch": {}}
    _write(tmp_path, "a_pmc_units.json", sha, key, {k: u})
    got, src = bench.measured_units([k, "other"], key)
    assert src == os.path.join("profiles", "a_pmc_units.json")
    assert got[k]["ta_busy"] == 0.8 and got["other"] is None and "raw_per_launch" not in got[k]
    # another build: not attached
    _write(tmp_path, "a_pmc_units.json", "0" * 16, key, {k: u})
    got, src = bench.measured_units([k], key)
    assert got[k] is None and src.startswith("stale")
    # other bench arguments: not attached
    _write(tmp_path, "b_pmc_traffic.json", sha, key + " x", {k: {"hbm_bytes_per_launch": 5}})
    got, src = bench.measured_traffic([k], key)
    assert got[k] is None and "differ" in src
    _write(tmp_path, "b_pmc_traffic.json", sha, key, {k: {"hbm_bytes_per_launch": 5}})
    got, _ = bench.measured_traffic([k], key)
    assert got[k] == 5


def test_vmem_peak_from_probe():
    """The roofline peak is the probe's byte rate of the vector-memory path
    (1 KiB per 16.9 CU-cycles, profiles/r3_ta_rate.txt) x 256 CUs x 2.4 GHz."""
    import bench

    line = [x for x in open(os.path.join(ROOT, "profiles", "r3_ta_rate.txt")) if x.startswith("x16 coalesced")
            and "L1" in x][0]
    cyc = float(line.split()[-1])
    assert abs(cyc - 16.9) < 0.1
    assert abs(bench.VMEM_PEAK_GBS / (1024 / cyc * 256 * 2.4) - 1) < 0.005


def test_pmc_kernel_names_exist_in_the_latest_profile():
    """The kernel names bench.py looks up (PMC_KERNELS) are the ones the
    newest committed rocprofv3 kernel trace of the headline bench reports: a
    kernel's template signature changing without a new profile would leave
    the bench line's traffic / units empty."""
    import csv
    import glob
    import re

    import bench

    def rnd(path):
        m = re.match(r"r(\d+)", os.path.basename(path))
        return (int(m.group(1)) if m else -1, os.path.basename(path))

    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_bench_kernel_stats.csv")), key=rnd)
    assert files
    names = set()
    with open(files[-1]) as f:
        for row in csv.DictReader(f):
            n = row.get("Name") or row.get("KernelName") or ""
            names.add(re.sub(r"^void ", "", n).split("(")[0])
    for k in bench.PMC_KERNELS.values():
        assert k in names, (k, os.path.basename(files[-1]))
