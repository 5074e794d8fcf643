"""Standard deviation of integral values 1e12 + small noise through the striped (StandardDeviation alone) and the
heavy (with ApproxCountDistinct) kernels, against the exact value (small-sized scratch experiment)."""
import sys
import numpy as np
import deequ_amd as D
import deequ_amd.native as N
from deequ_amd.table import Column, Table, pack_validity

for n in (1_000_003, 20_000_000):
    rng = np.random.default_rng(77)
    v = (10 ** 12 + rng.integers(-50, 50, n)).astype(np.int64)
    valid = rng.random(n) >= 0.03
    t = Table([Column("o", N.TYPE_LONG, v, pack_validity(valid))]).to_device()
    x = (v[valid] - 10 ** 12).astype(np.float64)
    exact = float(np.sqrt(np.mean((x - x.mean()) ** 2)))
    for extra in ([], [D.ApproxCountDistinct("o")]):
        a = D.StandardDeviation("o")
        r = D.AnalysisRunner.onData(t).addAnalyzers([a] + extra).run().metric(a).value.get()
        print(sys.argv[1], n, "heavy" if extra else "striped", "rel err %.3e" % (abs(r - exact) / exact), flush=True)
