"""ApproxQuantile(s) host logic on the CPU: the restated Spark QuantileSummaries (merge / compress /
query / PercentileDigest serialization) over zero-uncertainty summaries built from the oracle's exact
order statistics, the reference's KATs (T/analyzers/AnalyzerTests.scala:568-635) and the rank bound
(BASELINE.json: ApproxQuantile is judged by its declared relativeError rank bound; the values of
Spark's own GK sketch are parity-unpinned — the reference tests only bounds)."""
import math

import numpy as np
import pytest

import deequ_amd as D
from deequ_amd.quantiles import PercentileDigest, QuantileSummaries, Stats
from deequ_amd.table import Table
import oracle as O


def digest_of(values, rel, valid=None):
    t = Table.from_arrays({"x": np.asarray(values)}, validity=None if valid is None else {"x": valid})
    s = O.java_sorted_doubles(t, "x")
    ranks = O.summary_ranks(len(s), rel)
    return PercentileDigest.from_order_statistics(rel, s[ranks - 1], ranks, len(s)), s


def within_rank_bound(sorted_vals, q, rel, got):
    """QuantileSummaries' guarantee for query(q): the rank of the answer is within
    ceil(rel * n) (+1 for the 2.2 minRank bookkeeping) of ceil(q * n)."""
    n = len(sorted_vals)
    lo, hi = O.rank_interval(sorted_vals, got)
    target = max(1, math.ceil(q * n))
    slack = math.ceil(rel * n) + 1
    return lo - slack <= target <= hi + slack


def spark_digest_of(values, rel):
    t = Table.from_arrays({"x": np.asarray(values)})
    return PercentileDigest.spark_single_partition(rel, O.java_sorted_doubles(t, "x"))


def test_reference_kats_range_minus_1000_1000():
    # T/analyzers/AnalyzerTests.scala:568-601: sparkContext.range(-1000, 1000) under master "local"
    # (one partition, T/SparkContextSpec.scala:77), i.e. Spark's single-partition digest
    dg = spark_digest_of(np.arange(-1000, 1000, dtype=np.int64), 0.01)
    assert -20 < dg.getPercentiles([0.5])[0] < 20
    assert -520 < dg.getPercentiles([0.25])[0] < -480
    assert 480 < dg.getPercentiles([0.75])[0] < 520


@pytest.mark.parametrize("rel", [0.0, 0.001, 0.01, 0.1, 0.5, 1.0])
def test_rank_bound_random(rel):
    rng = np.random.default_rng(int(rel * 1000) + 1)
    x = np.concatenate([rng.normal(size=3000), rng.integers(-5, 5, 1000).astype(float), [np.nan, -0.0, 0.0]])
    dg, s = digest_of(x, rel)
    for q in np.linspace(0, 1, 41):
        got = dg.getPercentiles([float(q)])[0]
        assert within_rank_bound(s, q, rel, got), (rel, q, got)


def test_spark_single_partition_digest_hand_computed():
    # n = 2000, rel = 0.01 -> first sample, then Stats(v, 1, floor(0.02 i)) compressed with threshold 40:
    # the median query returns -19 (the value Spark 2.2 gives for this input in one partition)
    dg = spark_digest_of(np.arange(-1000, 1000, dtype=np.int64), 0.01)
    s = dg.quantileSummaries.sampled
    assert (s[0].value, s[0].g, s[0].delta) == (-1000.0, 1, 0)
    assert (s[-1].value, s[-1].g, s[-1].delta) == (999.0, 39, 0)
    assert dg.getPercentiles([0.5, 0.25, 0.75]) == [-19.0, -501.0, 487.0]
    assert sum(x.g for x in s) == 2000


@pytest.mark.parametrize("rel", [0.0, 0.01, 0.1])
def test_spark_single_partition_rank_bound(rel):
    rng = np.random.default_rng(3)
    x = rng.normal(size=4000)
    dg = spark_digest_of(x, rel)
    s = np.sort(x)
    for q in np.linspace(0, 1, 21):
        got = dg.getPercentiles([float(q)])[0]
        n = len(s)
        lo, hi = O.rank_interval(s, got)
        assert lo - 2 * math.ceil(rel * n) - 1 <= math.ceil(q * n) <= hi + 2 * math.ceil(rel * n) + 1


def test_exact_when_relative_error_zero():
    x = np.array([5.0, 1.0, 3.0, 2.0, 4.0])
    dg, s = digest_of(x, 0.0)
    assert [st.g for st in dg.quantileSummaries.sampled] == [1] * 5
    assert dg.getPercentiles([0.0, 1.0]) == [1.0, 5.0]


def test_merge_keeps_rank_bound():
    rng = np.random.default_rng(7)
    a, b = rng.normal(size=5000), rng.exponential(size=3000)
    da, _ = digest_of(a, 0.01)
    db, _ = digest_of(b, 0.01)
    m = da.merge(db)
    s = np.sort(np.concatenate([a, b]))
    assert m.quantileSummaries.count == 8000
    for q in (0.01, 0.1, 0.25, 0.5, 0.75, 0.9, 0.99):
        got = m.getPercentiles([q])[0]
        # merged summaries keep g + delta <= 2 * rel * n, so the bound doubles at most
        n = len(s)
        lo, hi = O.rank_interval(s, got)
        assert lo - 2 * math.ceil(0.01 * n) - 1 <= math.ceil(q * n) <= hi + 2 * math.ceil(0.01 * n) + 1, (q, got)


def test_compress_and_merge_against_hand_computed_summary():
    # QuantileSummaries.merge with threshold 2 * rel * count(left): (count=10, rel=0.1) -> 2.0
    a = QuantileSummaries(10000, 0.1, [Stats(1, 1, 0), Stats(3, 1, 0), Stats(5, 8, 0)], 10)
    b = QuantileSummaries(10000, 0.1, [Stats(2, 1, 0), Stats(4, 9, 0)], 10)
    m = a.merge(b)
    assert m.count == 20
    # sorted: 1(1),2(1),3(1),4(9),5(8); from the back: head=5; 4: 9+8 >= 2 keep; 3: 1+9 >= 2 keep;
    # 2: 1+1+0 = 2 not < 2 keep -> [2,3,4,5] + min 1
    assert [(s.value, s.g) for s in m.sampled] == [(1, 1), (2, 1), (3, 1), (4, 9), (5, 8)]
    c = QuantileSummaries(10000, 0.5, [Stats(1, 1, 0), Stats(2, 1, 0), Stats(3, 1, 0), Stats(4, 1, 0)], 4)
    m2 = c.merge(QuantileSummaries(10000, 0.5, [Stats(5, 1, 0)], 1))
    # threshold 2*0.5*4 = 4: head=5; 4: 1+1 < 4 merge (g=2); 3: 1+2 < 4 merge (g=3); 2: 1+3 = 4 keep
    assert [(s.value, s.g) for s in m2.sampled] == [(1, 1), (2, 1), (5, 3)]


def test_serialization_round_trip():
    dg, _ = digest_of(np.arange(100, dtype=float), 0.05)
    raw = dg.serialize()
    assert len(raw) == 20 + 16 * len(dg.quantileSummaries.sampled)
    back = PercentileDigest.deserialize(raw)
    assert back.quantileSummaries.sampled == dg.quantileSummaries.sampled
    assert back.quantileSummaries.count == 100 and back.quantileSummaries.relativeError == 0.05


def test_parameter_checks_messages():
    t = Table.from_arrays({"att1": np.arange(10, dtype=np.int64)})
    m = D.ApproxQuantile("att1", 0.5, relativeError=1.1).calculate(t)
    assert str(m.value.failed) == ("Relative error parameter must be in the closed interval [0, 1]. "
                                   "Currently, the value is: 1.1!")
    m = D.ApproxQuantile("att1", -0.1).calculate(t)
    assert str(m.value.failed) == ("Quantile parameter must be in the closed interval [0, 1]. "
                                   "Currently, the value is: -0.1!")
    m = D.ApproxQuantiles("att1", [0.5, 1.1]).calculate(t)
    assert m.value.isFailure and "1.1" in str(m.value.failed)


def test_java_order_of_oracle():
    t = Table.from_arrays({"x": np.array([np.nan, 0.0, -0.0, -np.inf, 1.0])})
    s = O.java_sorted_doubles(t, "x")
    assert math.isinf(s[0]) and math.copysign(1, s[1]) < 0 and math.copysign(1, s[2]) > 0 and math.isnan(s[4])


def test_java_double_order_puts_negative_zero_between_negatives_and_zero():
    """Double.compare order: every negative < -0.0 < 0.0 < positives < NaN (a -0.0 mapped to -0.5 misordered
    (-0.5, 0) values before)."""
    from deequ_amd.quantiles import _java_double_key
    from deequ_amd.kll import _order_key
    vals = [float("nan"), 0.25, 0.0, -0.0, -0.05, -0.7, float("-inf"), float("inf")]
    for key in (_java_double_key, _order_key):
        got = sorted(vals, key=key)
        assert [repr(v) for v in got] == ["-inf", "-0.7", "-0.05", "-0.0", "0.0", "0.25", "inf", "nan"]
