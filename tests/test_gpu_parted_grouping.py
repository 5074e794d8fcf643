"""Groupings over a two-chunk ChunkedTable read both chunks in place (dq_frequencies_parts): every group, count,
Histogram bin and grouping metric equals the build over the concatenated column (R/AnalysisRunner.scala:385-460
merges chunk states; the whole-shard grouping replaces that merge for a shard held as two row chunks)."""
import numpy as np
import pytest

import deequ_amd as D
from deequ_amd import engine
from deequ_amd.table import PartedColumn, Table

pytestmark = pytest.mark.gpu


def _close(a, b):
    return a == b or abs(a - b) <= 1e-12 * max(1.0, abs(b))


def _data(n, seed):
    rng = np.random.default_rng(seed)
    long_tail = "x" * 40  # keys past the packed-tuple width (the long-tuple build)
    s = []
    for v in rng.integers(0, 5000, n):
        u = rng.random()
        s.append(None if u < 0.04 else "" if u < 0.06 else (long_tail + str(int(v))) if u < 0.1 else "v%d" % int(v))
    k = [None if rng.random() < 0.02 else int(v) for v in rng.integers(0, 40, n)]
    return {"s": s, "k": k}, {"s": "string", "k": "long"}


def _tables(data, types, cut):
    n = len(data["s"])
    full = Table.from_pydict(data, types=types).to_device()
    chunks = [Table.from_pydict({c: v[a:b] for c, v in data.items()}, types=types).to_device()
              for a, b in ((0, cut), (cut, n))]
    return full, D.ChunkedTable(chunks)


@pytest.mark.parametrize("n,cut", [(50_000, 20_000), (50_000, 1), (50_000, 49_999), (3_000, 0), (3_000, 3_000),
                                   (400_000, 150_000)])
def test_parted_frequencies_equal_the_concatenated_build(n, cut):
    data, types = _data(n, seed=n + cut)
    full, ct = _tables(data, types, cut)
    view = ct.grouping_view(["s", "k"])
    assert all(isinstance(view[c], PartedColumn) for c in ("s", "k"))
    for keys, nulls in ((["s"], False), (["s"], True), (["s", "k"], False), (["k", "s"], True)):
        got = engine.frequencies(view, keys, include_nulls=nulls)
        want = engine.frequencies(full, keys, include_nulls=nulls)
        assert got.summary() == want.summary(), (keys, nulls)
        assert got.to_dict() == want.to_dict(), (keys, nulls)
        gt, wt = got.top(25), want.top(25)
        assert sorted(c for _, c in gt) == sorted(c for _, c in wt)


def test_parted_run_equals_concat_and_whole_table_runs(monkeypatch):
    data, types = _data(120_000, seed=5)
    full, ct = _tables(data, types, 70_001)
    an = [D.Size(), D.Uniqueness(["s"]), D.Distinctness(["s"]), D.UniqueValueRatio(["s"]), D.CountDistinct(["s"]),
          D.Entropy("s"), D.CountDistinct(["s", "k"]), D.MutualInformation(["s", "k"]), D.Histogram("s"),
          D.Histogram("s", maxDetailBins=10), D.Histogram("k")]
    want = D.AnalysisRunner.onData(full).addAnalyzers(an).run()
    got = D.AnalysisRunner.onData(ct).addAnalyzers(an).run()
    monkeypatch.setenv("DQ_GROUP_CONCAT", "1")
    cat = D.AnalysisRunner.onData(ct).addAnalyzers(an).run()
    for a in an:
        w, g, c = (r.metric(a).value.get() for r in (want, got, cat))
        if isinstance(w, float):
            assert _close(g, w) and _close(c, w), (a, g, c, w)
        else:
            assert g == w and c == w, a


def test_fixed_width_keys_keep_the_concatenated_fast_build():
    data, types = _data(10_000, seed=9)
    _, ct = _tables(data, types, 4_000)
    assert not isinstance(ct.grouping_view(["k"])["k"], PartedColumn)
    assert isinstance(ct.grouping_view(["s", "k"])["k"], PartedColumn)
