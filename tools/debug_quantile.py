"""Debug aid: dq_quantile_summary / dq_quantile_summaries on the 2e7-row device-resident t(3) column of
tests/test_gpu_quantiles.py against the oracle's order statistics; prints the mismatching ranks."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np

from deequ_amd import engine
from deequ_amd.table import Table
from oracle import oracle as O

rng = np.random.default_rng(9)
n = int(float(sys.argv[1])) if len(sys.argv) > 1 else 20_000_000
x = rng.standard_t(3, n)
valid = rng.random(n) > 0.01
t = Table.from_arrays({"x": x}, validity={"x": valid})
s = O.java_sorted_doubles(t, "x")
for dev in (False, True):
    if dev:
        t.to_device(0)
    for name, got in (("single", engine.ctx().quantile_summary(t["x"].native(), t.nrows, 0.01)),
                      ("batched", engine.ctx().quantile_summaries([([t["x"].native()], 0.01)])[0])):
        vals, ranks, cnt = got
        exp = s[ranks - 1]
        bad = np.nonzero(vals.view(np.uint64) != exp.view(np.uint64))[0]
        print(dev, name, "n", cnt, len(s), "samples", len(vals), "bad", len(bad), flush=True)
        for i in bad[:8]:
            lo, hi = np.searchsorted(s, vals[i], "left"), np.searchsorted(s, vals[i], "right")
            print("   rank %d got %r (ranks %d..%d) exp %r" % (ranks[i], vals[i], lo + 1, hi, exp[i]), flush=True)
