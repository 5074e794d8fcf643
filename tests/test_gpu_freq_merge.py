"""Frequency-state algebra on the GPU: FrequenciesAndNumRows.sum as a device merge of two tables
(dq_freq_merge: the null-safe full outer join of A/GroupingAnalyzers.scala:127-147), persisted frequency
states read back as canonical (key, count) pairs and merged on the device (aggregateWith), 64-bit counts,
and MutualInformation's marginals + sum on the device (A/MutualInformation.scala:35-97). Bars: exact
group counts and numRows; entropy / MutualInformation within 1e-12 of the exact (fsum) oracle."""
import math
import os
import time

import numpy as np
import pytest

import deequ_amd as D
import deequ_amd.native as N
from deequ_amd import engine
from deequ_amd.table import Table, Column
import oracle as O

pytestmark = pytest.mark.gpu


def _tables(rng, n, kind):
    if kind == "long":
        a = rng.integers(0, n // 3 + 1, n).astype(np.int64)
        b = rng.integers(n // 6, n // 2 + 1, n).astype(np.int64)
        return Table.from_arrays({"k": a}), Table.from_arrays({"k": b})
    vals = np.array([0.0, -0.0, np.nan, 1.5, -2.25, np.inf, 3.0], dtype=np.float64)
    a = np.where(rng.random(n) < 0.3, vals[rng.integers(0, len(vals), n)], rng.integers(0, 200, n) / 4.0)
    b = np.where(rng.random(n) < 0.3, vals[rng.integers(0, len(vals), n)], rng.integers(100, 300, n) / 4.0)
    return (Table.from_arrays({"k": a}, validity={"k": rng.random(n) > 0.05}),
            Table.from_arrays({"k": b}, validity={"k": rng.random(n) > 0.05}))


def _norm(d):
    return {tuple(O._group_key(v) for v in k): c for k, c in d.items()}


@pytest.mark.parametrize("kind", ["long", "double"])
def test_device_merge_equals_union(kind):
    rng = np.random.default_rng(3)
    ta, tb = _tables(rng, 50_000, kind)
    an = D.CountDistinct(["k"])
    sa, sb = an.computeStateFrom(ta), an.computeStateFrom(tb)
    merged = sa.sum(sb)
    assert isinstance(merged.frequencies, engine.FrequencyTable)  # merged on the device, not as a dict
    fa, na = O.frequencies(ta, ["k"])
    fb, nb = O.frequencies(tb, ["k"])
    exp = dict(fa)
    for k, c in fb.items():
        exp[k] = exp.get(k, 0) + c
    assert merged.numRows == na + nb
    assert _norm(merged.as_dict()) == exp
    s = merged.summary(None)
    e = O.grouping_summary(exp, na + nb)
    assert (s["num_groups"], s["num_unique"]) == (e["num_groups"], e["num_unique"])
    assert abs(s["entropy"] - e["entropy"]) <= 1e-12 * e["entropy"]
    for a in (D.Uniqueness(["k"]), D.Distinctness(["k"]), D.CountDistinct(["k"]), D.UniqueValueRatio(["k"]),
              D.Entropy("k")):
        got = a.computeMetricFrom(merged).value.get()
        union = a.computeMetricFrom(a.computeStateFrom(Table([Column("k", ta["k"].spark_type,
                                                                         np.concatenate([ta["k"].values,
                                                                                         tb["k"].values]),
                                                                         _cat_validity(ta["k"], tb["k"]))])))
        want = union.value.get()
        assert got == want or abs(got - want) <= 1e-12 * abs(want), (a, got, want)


def _cat_validity(a, b):
    from deequ_amd.table import unpack_validity, pack_validity
    va = unpack_validity(a.validity, a.length) if a.validity is not None else np.ones(a.length, bool)
    vb = unpack_validity(b.validity, b.length) if b.validity is not None else np.ones(b.length, bool)
    return pack_validity(np.concatenate([va, vb]))


def test_aggregate_with_persisted_state_merges_on_device(tmp_path):
    """runner: the state of table A persisted, then table B run with aggregateWith = that provider -> the
    metrics of A u B (A/Analyzer.scala:107-128); the loaded state is canonical pairs, merged by dq_freq_merge."""
    rng = np.random.default_rng(9)
    ta, tb = _tables(rng, 40_000, "double")
    analyzers = [D.Uniqueness(["k"]), D.Distinctness(["k"]), D.Entropy("k"), D.CountDistinct(["k"]),
                 D.Histogram("k", None, 50)]
    prov = D.HdfsStateProvider(None, str(tmp_path / "s"))
    D.AnalysisRunner.onData(ta).addAnalyzers(analyzers).saveStatesWith(prov).run()
    loaded = prov.load(analyzers[0])
    assert isinstance(loaded.frequencies, engine.PairFrequencies)
    got = D.AnalysisRunner.onData(tb).addAnalyzers(analyzers).aggregateWith(prov).run()
    union = Table([Column("k", N.TYPE_DOUBLE, np.concatenate([ta["k"].values, tb["k"].values]),
                          _cat_validity(ta["k"], tb["k"]))])
    want = D.AnalysisRunner.onData(union).addAnalyzers(analyzers).run()
    for a in analyzers:
        g, w = got.metric(a).value.get(), want.metric(a).value.get()
        if isinstance(a, D.Histogram):
            assert g.numberOfBins == w.numberOfBins
            assert sorted(v.absolute for v in g.values.values()) == sorted(v.absolute for v in w.values.values())
        else:
            assert g == w or abs(g - w) <= 1e-12 * abs(w), (a, g, w)


def test_sixty_four_bit_counts():
    """Spark counts with Long: a group seen >= 2^32 times (here through pre-aggregated pairs) stays exact."""
    keys = np.array([7, 7, 11, 13, 7], dtype=np.int64)
    counts = np.array([3_000_000_000, 2_000_000_000, 1, 4_294_967_296, 5], dtype=np.int64)
    t = engine.FrequencyTable.from_pairs(N.TYPE_LONG, keys, counts, int(counts.sum()))
    d = t.to_dict()
    assert d == {(7,): 5_000_000_005, (11,): 1, (13,): 4_294_967_296}
    s = t.summary(None)
    assert s["num_groups"] == 3 and s["num_unique"] == 1 and s["max_count"] == 5_000_000_005
    assert t.top(2) == [((7,), 5_000_000_005), ((13,), 4_294_967_296)]


@pytest.mark.parametrize("kinds", [("long", "long"), ("string", "double"), ("string", "string")])
def test_mutual_information_on_device(kinds):
    rng = np.random.default_rng(21)
    n = 30_000
    x = rng.integers(0, 40, n)
    y = (x * 7 + rng.integers(0, 5, n)) % 53
    cols = {}
    for name, kind, v in (("x", kinds[0], x), ("y", kinds[1], y)):
        valid = rng.random(n) > 0.07
        if kind == "long":
            cols[name] = Column(name, N.TYPE_LONG, v.astype(np.int64), _pack(valid))
        elif kind == "double":
            cols[name] = Column(name, N.TYPE_DOUBLE, v.astype(np.float64) / 2, _pack(valid))
        else:
            from deequ_amd.table import _column_from_pylist
            cols[name] = _column_from_pylist(name, "string", ["v%d" % a if m else None for a, m in zip(v, valid)])
    t = Table([cols["x"], cols["y"]])
    a = D.MutualInformation(["x", "y"])
    state = a.computeStateFrom(t)
    assert isinstance(state.frequencies, engine.FrequencyTable)
    got = a.computeMetricFrom(state).value.get()
    freq, nrows = O.frequencies(t, ["x", "y"])
    px, py = {}, {}
    for (u, w), c in freq.items():
        px[u] = px.get(u, 0) + c
        py[w] = py.get(w, 0) + c
    exp = math.fsum((c / nrows) * math.log((c / nrows) / ((px[u] / nrows) * (py[w] / nrows)))
                    for (u, w), c in freq.items() if u is not None and w is not None)
    assert abs(got - exp) <= 1e-12 * abs(exp), (got, exp)


def _pack(mask):
    from deequ_amd.table import pack_validity
    return pack_validity(mask)


def test_c4_size_merge_and_mutual_information_under_a_second():
    """aggregateWith over two ~1e8-group tables and MutualInformation on a C4-size joint
    table each in < 1 s. The C4 keys (1e9 rows, exactly 1e8 distinct) split into two halves merge to the
    closed-form table; MI(k, k) = H(k) in closed form. DQ_C4_ROWS scales it down."""
    import torch
    R = int(float(os.environ.get("DQ_C4_ROWS", "1e9")))
    Dn = R // 10
    ctx = engine.ctx()
    keys = torch.empty(R, dtype=torch.int64, device="cuda")
    ctx.synth_freq_keys(R, Dn, 0, R, keys.data_ptr())
    ctx.synchronize()
    half = R // 2
    ca = Column("k", N.TYPE_LONG, None, None, length=half)
    ca.device = {"values": keys[:half]}
    cb = Column("k", N.TYPE_LONG, None, None, length=R - half)
    cb.device = {"values": keys[half:]}
    an = D.Uniqueness(["k"])
    sa, sb = an.computeStateFrom(Table([ca])), an.computeStateFrom(Table([cb]))
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    merged = sa.sum(sb)
    s = merged.summary(None)
    merge_s = time.perf_counter() - t0
    big = (R - Dn // 2) / (Dn // 2)
    exp_ent = math.fsum([-(Dn // 2) * (big / R) * math.log(big / R), -(Dn // 2) * (1 / R) * math.log(1 / R)])
    assert (s["num_rows"], s["num_groups"], s["num_unique"]) == (R, Dn, Dn // 2)
    assert abs(s["entropy"] - exp_ent) <= 1e-12 * exp_ent
    del sa, sb, merged
    ck = Column("k", N.TYPE_LONG, None, None, length=R)
    ck.device = {"values": keys}
    ck2 = Column("k2", N.TYPE_LONG, None, None, length=R)
    ck2.device = {"values": keys}
    t = Table([ck, ck2])
    mi = D.MutualInformation(["k", "k2"])
    state = mi.computeStateFrom(t)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    got = mi.computeMetricFrom(state).value.get()
    mi_s = time.perf_counter() - t0
    assert abs(got - exp_ent) <= 1e-12 * exp_ent, (got, exp_ent)
    print("merge %.3f s, MI %.3f s" % (merge_s, mi_s))
    assert merge_s < 1.0 and mi_s < 1.0, (merge_s, mi_s)
