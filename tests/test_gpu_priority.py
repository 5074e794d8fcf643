"""dq_set_priority (r06): a context's work moved to a high- or low-priority stream gives the same results, its cached
scratch stays usable across the stream change, and runAsync(priority=1) equals run()."""
import numpy as np
import pytest

import deequ_amd as D
from deequ_amd import engine
from deequ_amd import native as N
from deequ_amd.table import Table

pytestmark = pytest.mark.gpu


def _table():
    rng = np.random.default_rng(11)
    n = 200_000
    s = [None if rng.random() < 0.05 else "p%d" % int(v) for v in rng.integers(0, 20_000, n)]
    x = [float(v) for v in rng.normal(size=n)]
    return Table.from_pydict({"s": s, "x": x}, types={"s": "string", "x": "double"}).to_device()


def test_priorities_give_identical_results():
    t = _table()
    an = [D.Size(), D.Mean("x"), D.StandardDeviation("x"), D.ApproxCountDistinct("s"), D.Uniqueness(["s"]),
          D.Entropy("s"), D.ApproxQuantile("x", 0.5)]
    want = D.AnalysisRunner.onData(t).addAnalyzers(an).run()
    ctx = N.Context(engine.device())
    try:
        for p in (1, -1, 0, 1):
            ctx.set_priority(p)  # the second change re-tags scratch cached by the first runs
            with engine.using_context(ctx):
                got = D.AnalysisRunner.onData(t).addAnalyzers(an).run()
            for a in an:
                assert got.metric(a).value.get() == want.metric(a).value.get(), (p, a)
    finally:
        ctx.close()
    with pytest.raises(N.NativeError):
        N.Context(engine.device()).set_priority(2)


def test_run_async_with_priority_equals_run():
    t = _table()
    an = [D.Uniqueness(["s"]), D.Entropy("s"), D.ApproxQuantile("x", 0.25)]
    want = D.AnalysisRunner.onData(t).addAnalyzers(an).run()
    h = D.AnalysisRunner.onData(t).addAnalyzers(an).runAsync(priority=1)
    D.AnalysisRunner.onData(t).addAnalyzers([D.Mean("x")]).run()  # the caller's own work meanwhile
    got = h.result()
    for a in an:
        assert got.metric(a).value.get() == want.metric(a).value.get(), a
