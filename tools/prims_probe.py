"""Minimal driver for profiling the group-by primitives (no CPU baseline):
hashgrid 2^24 points (n_cells = n) and scatter_reduce add 2^24 -> 2^20,
`--reps` calls each; prints the device time of every call."""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mitsuba3-experiments_amd"))

from mtx import primitives  # noqa: E402
from mtx._lib import context, lib  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--reps", type=int, default=3)
ap.add_argument("--what", default="hashgrid,scatter")
a = ap.parse_args()
ctx = context(0)
rng = np.random.default_rng(0)
n = 1 << 24
if "hashgrid" in a.what:
    p = rng.random((3, n), dtype=np.float32)
    for _ in range(a.reps):
        primitives.HashGrid(p, 100, n)
        print("hashgrid ms", round(lib().mtx_last_device_ms(ctx.handle), 4), flush=True)
if "scatter" in a.what:
    nt = 1 << 20
    idx = rng.integers(0, nt, n, dtype=np.uint32)
    val = rng.random(n, dtype=np.float32)
    tgt = np.zeros(nt, np.float32)
    for _ in range(a.reps):
        primitives.scatter_reduce_with("add", tgt, val, idx)
        print("scatter ms", round(lib().mtx_last_device_ms(ctx.handle), 4), flush=True)
