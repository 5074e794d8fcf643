"""GPU parity of the fused scan (libdq.so HIP kernels) against the oracle and the reference KATs.

Bars (BASELINE.json north_star): bit-exact for counts, integral sums, min/max and HLL registers;
fp64 mean / stddev / correlation within 1e-12 relative of the exact (long double) oracle.
"""
import math

import numpy as np
import pytest

import deequ_amd as D
import deequ_amd.native as N
from deequ_amd import engine
from deequ_amd.table import Table, Column, pack_validity
import oracle as O
from helpers import analyzer_from_spec, check_metric, table_from_fixture

pytestmark = pytest.mark.gpu

SCAN = {"Size", "Completeness", "Compliance", "Mean", "Sum", "Minimum", "Maximum", "StandardDeviation",
        "Correlation", "ApproxCountDistinct", "MinLength", "MaxLength", "DataType", "ApproxQuantile", "PatternMatch"}
REL = 1e-12


def scan_kats(kats):
    return [k for k in kats["kats"] if k["analyzer"][0] in SCAN]


def test_scan_kats_one_by_one(kats):
    for k in scan_kats(kats):
        t = table_from_fixture(kats["fixtures"][k["fixture"]])
        a = analyzer_from_spec(k["analyzer"])
        m = a.calculate(t)
        # PatternMatch over a double column included (AnalyzerTests.scala:664-668: 0.75 through Double.toString)
        check_metric(m, k["expected"], rel=1e-15 if k["analyzer"][0] == "StandardDeviation" else 0.0)


def test_scan_kats_fused_in_one_run(kats):
    # All shareable analyzers of a fixture in ONE AnalysisRunner run -> ONE fused scan call (dq_scan_launch_count
    # counts calls). HBM passes are not counted here: columns that a `where` / non-fused Compliance predicate reads
    # are read once more by the predicate pass (predicate_kernel), the scan reads every column once.
    by_fixture = {}
    for k in scan_kats(kats):
        by_fixture.setdefault(k["fixture"], []).append(k)
    for fx, ks in by_fixture.items():
        t = table_from_fixture(kats["fixtures"][fx])
        analyzers, exps = [], []
        for k in ks:
            a = analyzer_from_spec(k["analyzer"])
            if isinstance(k["expected"], dict) and k["expected"].get("failure") == "*":
                continue  # an unresolvable predicate fails the whole batch (R/AnalysisRunner.scala:320-323)
            analyzers.append(a)
            exps.append(k["expected"])
        before = engine.ctx().scan_launch_count()
        ctx = D.AnalysisRunner.onData(t).addAnalyzers(analyzers).run()
        after = engine.ctx().scan_launch_count()
        assert after - before <= 1, fx
        for a, e in zip(analyzers, exps):
            check_metric(ctx.metric(a), e, rel=1e-15 if isinstance(a, D.StandardDeviation) else 0.0)


def test_unresolvable_predicate_fails_the_whole_batch(kats):
    t = table_from_fixture(kats["fixtures"]["dfWithNumericValues"])
    bad = D.Compliance("rule1", "attNoSuchColumn > 3")
    good = D.Mean("att1")
    ctx = D.AnalysisRunner.onData(t).addAnalyzer(bad).addAnalyzer(good).run()
    assert ctx.metric(bad).value.isFailure and ctx.metric(good).value.isFailure


def test_empty_state_message():
    # T/analyzers/NullHandlingTests.scala:130-140
    t = Table.from_rows([(None,)] * 8, ["numericCol"], ["double"])
    m = D.Mean("numericCol").calculate(t)
    assert m.value.isFailure
    assert str(m.value.failed) == "Empty state for analyzer Mean(numericCol,None), all input values were NULL."


def test_incremental_states_merge(kats):
    inc = kats["incremental"]
    a, b = table_from_fixture(inc["initial"]), table_from_fixture(inc["delta"])
    for spec, va, vb, vm, src in inc["cases"]:
        an = analyzer_from_spec(spec)
        if type(an).__name__ not in SCAN:
            continue
        sa, sb = an.computeStateFrom(a), an.computeStateFrom(b)
        assert an.computeMetricFrom(sa).value.get() == va, src
        assert an.computeMetricFrom(sb).value.get() == vb, src
        assert an.computeMetricFrom(D.analyzers.merge(sa, sb)).value.get() == vm, src


# ---- randomized parity against the oracle -------------------------------------------------------
def random_table(rng, n, null_frac=0.1, with_nan=False):
    cols = []
    specs = [("d", "double"), ("f", "float"), ("l", "long"), ("i", "int"), ("s", "short"), ("b", "byte"),
             ("dec", "decimal"), ("k", "long"), ("g", "double")]
    for name, t in specs:
        valid = rng.random(n) >= null_frac
        if t == "double":
            v = rng.normal(50.0, 20.0, n)
            if with_nan:
                v[rng.random(n) < 0.01] = np.nan
        elif t == "float":
            v = rng.normal(0, 3, n).astype(np.float32)
        elif t == "long":
            v = rng.integers(-2 ** 62, 2 ** 62, n, dtype=np.int64) if name == "l" else rng.integers(0, 50, n)
        elif t == "int":
            v = rng.integers(-2 ** 31, 2 ** 31, n, dtype=np.int64).astype(np.int32)
        elif t == "short":
            v = rng.integers(-2 ** 15, 2 ** 15, n).astype(np.int16)
        elif t == "byte":
            v = rng.integers(-128, 128, n).astype(np.int8)
        else:  # decimal(18, 2): unscaled int64
            v = rng.integers(-10 ** 9, 10 ** 9, n, dtype=np.int64)
        from deequ_amd.table import NUMPY_OF, spark_type_of
        st = spark_type_of(t)
        c = Column(name, st, np.ascontiguousarray(v.astype(NUMPY_OF[st])),
                   None if valid.all() else pack_validity(valid),
                   decimal_precision=18 if t == "decimal" else 0, decimal_scale=2 if t == "decimal" else 0)
        cols.append(c)
    return Table(cols)


def _close(a, b, rel=REL):
    if math.isnan(a) or math.isnan(b):
        return math.isnan(a) and math.isnan(b)
    return a == b or abs(a - b) <= rel * max(abs(a), abs(b))


def assert_state_parity(table, analyzer, got):
    exp = O.expected_state(table, analyzer, exact=True)
    name = type(analyzer).__name__
    if exp is None or got is None:
        assert exp is None and got is None, (analyzer, exp, got)
        return
    if name in ("Size", "Completeness", "Compliance"):
        assert (got.numMatches, got.count if hasattr(got, "count") else 0) == \
               (exp.numMatches, exp.count if hasattr(exp, "count") else 0), analyzer
    elif name == "Mean":
        assert got.count == exp.count, analyzer
        assert _close(got.sum_, exp.sum_), (analyzer, got, exp)
    elif name == "Sum":
        assert _close(got.sum_, exp.sum_), (analyzer, got, exp)
    elif name in ("Minimum", "Maximum"):
        g = got.minValue if name == "Minimum" else got.maxValue
        e = exp.minValue if name == "Minimum" else exp.maxValue
        assert (math.isnan(g) and math.isnan(e)) or g == e, (analyzer, g, e)
    elif name == "StandardDeviation":
        assert got.n == exp.n and _close(got.avg, exp.avg) and _close(got.m2, exp.m2), (analyzer, got, exp)
    elif name == "Correlation":
        # all six CorrelationState fields within 1e-12 of the exact oracle: xMk / yMk relative, the averages
        # relative to max(|avg|, standard deviation) and ck relative to sqrt(xMk * yMk); the metric to 1e-12
        assert got.n == exp.n, analyzer
        sx, sy = math.sqrt(abs(exp.xMk) / exp.n), math.sqrt(abs(exp.yMk) / exp.n)
        scale_ck = math.sqrt(abs(exp.xMk * exp.yMk))
        for g, e, sc in [(got.xAvg, exp.xAvg, max(abs(exp.xAvg), sx)), (got.yAvg, exp.yAvg, max(abs(exp.yAvg), sy)),
                         (got.ck, exp.ck, scale_ck), (got.xMk, exp.xMk, abs(exp.xMk)), (got.yMk, exp.yMk, abs(exp.yMk))]:
            assert (math.isnan(g) and math.isnan(e)) or g == e or abs(g - e) <= REL * sc, (analyzer, got, exp)
        gm, em = got.metricValue(), exp.metricValue()
        assert (math.isnan(gm) and math.isnan(em)) or abs(gm - em) <= REL, (analyzer, gm, em)
    elif name == "ApproxCountDistinct":
        assert got.words == exp.words, analyzer
    else:
        raise AssertionError(name)


def all_analyzers(table, where=None):
    out = [D.Size(where)]
    for c in table.columns:
        out += [D.Completeness(c, where), D.Mean(c, where), D.Sum(c, where), D.Minimum(c, where),
                D.Maximum(c, where), D.StandardDeviation(c, where), D.ApproxCountDistinct(c, where)]
    out += [D.Correlation("d", "g", where), D.Correlation("l", "i", where), D.Correlation("f", "d", where),
            D.Correlation("g", "d", where), D.Compliance("c1", "d > 50", where), D.Compliance("c2", "k = 3 OR i < 0", where)]
    return out


@pytest.mark.parametrize("n", [0, 1, 63, 2047, 2048, 2049, 100003])
def test_random_parity_all_types(n):
    rng = np.random.default_rng(n + 11)
    t = random_table(rng, n, with_nan=(n % 2 == 1))
    analyzers = all_analyzers(t)
    batch = D.ScanBatch(t)
    offsets = [a.addOps(batch) for a in analyzers]
    states = batch.run()
    for a, ops in zip(analyzers, offsets):
        assert_state_parity(t, a, a.fromAggregationResult(states, ops))


@pytest.mark.parametrize("where", ["k < 25", "d > 40 AND i IS NOT NULL", "s < 0 OR b > 10", "k IN (1, 2, 3)"])
def test_random_parity_with_where(where):
    rng = np.random.default_rng(5)
    t = random_table(rng, 50001)
    analyzers = all_analyzers(t, where)
    batch = D.ScanBatch(t)
    offsets = [a.addOps(batch) for a in analyzers]
    states = batch.run()
    for a, ops in zip(analyzers, offsets):
        assert_state_parity(t, a, a.fromAggregationResult(states, ops))


def test_device_resident_matches_host_staged():
    rng = np.random.default_rng(9)
    t = random_table(rng, 300000)
    analyzers = all_analyzers(t)
    host = D.AnalysisRunner.onData(t).addAnalyzers(analyzers).run()
    t.to_device()
    dev = D.AnalysisRunner.onData(t).addAnalyzers(analyzers).run()
    for a in analyzers:
        assert host.metric(a) == dev.metric(a), a


def test_run_to_run_bitwise_reproducible():
    rng = np.random.default_rng(4)
    t = random_table(rng, 200000).to_device()
    analyzers = all_analyzers(t)
    r1 = D.AnalysisRunner.onData(t).addAnalyzers(analyzers).run()
    r2 = D.AnalysisRunner.onData(t).addAnalyzers(analyzers).run()
    for a in analyzers:
        assert r1.metric(a) == r2.metric(a), a


def test_nan_and_signed_zero_semantics():
    # Spark orders NaN above every double: max = NaN if any NaN; min ignores NaN unless all are NaN.
    t = Table.from_arrays({"x": np.array([1.0, np.nan, -3.0, 2.0]), "y": np.array([np.nan, np.nan, np.nan, np.nan])})
    st = D.ScanBatch(t)
    ops = [D.Maximum("x").addOps(st), D.Minimum("x").addOps(st), D.Minimum("y").addOps(st), D.Sum("x").addOps(st)]
    res = st.run()
    assert math.isnan(D.Maximum("x").fromAggregationResult(res, ops[0]).maxValue)
    assert D.Minimum("x").fromAggregationResult(res, ops[1]).minValue == -3.0
    assert math.isnan(D.Minimum("y").fromAggregationResult(res, ops[2]).minValue)
    assert math.isnan(D.Sum("x").fromAggregationResult(res, ops[3]).sum_)


def test_synthetic_generators_match_oracle_bitwise():
    import torch
    ctx = engine.ctx()
    n = 1 << 16
    for kind, seed, dt in [(1, 0x5EED0000, torch.float64), (2, 0x5EED0002, torch.float64),
                           (3, 0x5EED0003, torch.float64), (4, 0x5EED0004, torch.int64),
                           (5, 0x5EED0005, torch.int64), (6, 0x5EED0006, torch.float64)]:
        buf = torch.empty(n, dtype=dt, device="cuda")
        ctx.synth_column(kind, seed, 1000, n, buf.data_ptr())
        torch.cuda.synchronize()
        ctx.synchronize()
        got = buf.cpu().numpy()
        exp = O.synth_column(kind, seed, 1000, n)
        assert np.array_equal(got.view(np.uint64), exp.view(np.uint64)), kind
    vb = torch.zeros(n // 8, dtype=torch.uint8, device="cuda")
    ctx.synth_validity(0x5EED0100, 0, n, 10, vb.data_ptr())
    ctx.synchronize()
    from deequ_amd.table import unpack_validity
    assert np.array_equal(unpack_validity(vb.cpu().numpy(), n), O.synth_validity(0x5EED0100, 0, n, 10))


@pytest.mark.parametrize("chunk", [2048, 65536])
def test_streamed_host_scan_equals_staged_scan(chunk):
    """dq_scan_streamed: host columns copied through HBM in row chunks (copy of chunk i + 1 overlapping the scan of
    chunk i), chunk states folded in row order: the same states as one staged scan (exact for counts, Long sums,
    min / max, HLL registers; fp sums / moments within 1e-12 of the exact oracle)."""
    rng = np.random.default_rng(chunk)
    t = random_table(rng, 250_001, with_nan=True)
    analyzers = all_analyzers(t, "k < 30")
    batch = D.ScanBatch(t)
    offsets = [a.addOps(batch) for a in analyzers]
    got = D.runners.ScanResult(engine.ctx().scan_streamed(batch.native_columns(), t.nrows, batch.ops,
                                                          [p.to_native() for p in batch.preds], chunk))
    for a, ops in zip(analyzers, offsets):
        assert_state_parity(t, a, a.fromAggregationResult(got, ops))
