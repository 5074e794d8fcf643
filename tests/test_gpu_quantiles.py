"""GPU parity of dq_quantile_summary (quantile.hip: splitter histogram + compaction + rocPRIM sort)
against the oracle's exact order statistics (numpy sort in java.lang.Double.compare order), and
the ApproxQuantile(s) analyzers end to end. Bar: bit-exact values at every summary rank (integer /
ordering work); the analyzers' answers are Spark's own single-partition digest below 50000 rows and
within the declared relativeError rank bound above."""
import math

import numpy as np
import pytest

import deequ_amd as D
from deequ_amd import engine
from deequ_amd.table import Table, Column, pack_validity
import oracle as O

pytestmark = pytest.mark.gpu


def summary(t, col, rel):
    return engine.ctx().quantile_summary(t[col].native(), t.nrows, rel)


def check_exact(t, col, rel):
    vals, ranks, n = summary(t, col, rel)
    s = O.java_sorted_doubles(t, col)
    assert n == len(s)
    exp_r = O.summary_ranks(n, rel)
    assert np.array_equal(ranks, exp_r)
    exp = s[exp_r - 1] if n else s[:0]
    assert np.array_equal(vals.view(np.uint64), exp.view(np.uint64)), (col, rel)
    return vals, ranks, n


@pytest.mark.parametrize("dist", ["normal", "uniform01", "lognormal", "ints", "dups", "const", "specials"])
def test_summary_exact_f64(dist):
    rng = np.random.default_rng(hash(dist) & 0xFFFF)
    n = 300_000
    if dist == "normal":
        x = rng.normal(size=n)
    elif dist == "uniform01":
        x = rng.random(n)  # exponents pile up: the splitters must stay equi-depth
    elif dist == "lognormal":
        x = rng.lognormal(0, 5, n)
    elif dist == "ints":
        x = rng.integers(-50, 50, n).astype(np.float64)
    elif dist == "dups":
        x = np.where(rng.random(n) < 0.5, 0.0, rng.normal(size=n))
    elif dist == "const":
        x = np.full(n, 3.25)
    else:
        x = rng.normal(size=n)
        k = rng.integers(0, n, 2000)
        x[k[:500]] = np.nan
        x[k[500:1000]] = -0.0
        x[k[1000:1500]] = 0.0
        x[k[1500:1750]] = np.inf
        x[k[1750:]] = -np.inf
    valid = rng.random(n) > 0.03
    t = Table.from_arrays({"x": x}, validity={"x": valid})
    for rel in (0.01, 0.001, 0.25):
        check_exact(t, "x", rel)


@pytest.mark.parametrize("dtype", [np.int8, np.int16, np.int32, np.int64, np.float32])
def test_summary_exact_types(dtype):
    rng = np.random.default_rng(5)
    n = 120_001
    if dtype == np.float32:
        x = rng.normal(size=n).astype(np.float32)
    elif dtype == np.int64:
        x = rng.integers(-(2 ** 62), 2 ** 62, n, dtype=np.int64)  # cast to double rounds: ties are exercised
        x[:10] = [np.iinfo(np.int64).min, np.iinfo(np.int64).max, 0, -1, 1, 2 ** 53 + 1, 2 ** 53, -(2 ** 53) - 1, 7, 7]
    else:
        info = np.iinfo(dtype)
        x = rng.integers(info.min, info.max, n, dtype=dtype, endpoint=True)
    t = Table.from_arrays({"x": x})
    check_exact(t, "x", 0.01)


def test_summary_decimal():
    rng = np.random.default_rng(11)
    n = 80_000
    c = Column("d", "DecimalType", rng.integers(-10 ** 9, 10 ** 9, n, dtype=np.int64), decimal_precision=12,
               decimal_scale=3)
    t = Table([c])
    check_exact(t, "d", 0.01)


def test_summary_small_rel_zero_is_full_sort():
    rng = np.random.default_rng(2)
    x = rng.normal(size=4097)
    t = Table.from_arrays({"x": x})
    vals, ranks, n = check_exact(t, "x", 0.0)
    assert n == 4097 and len(vals) == 4097


def test_summary_empty_and_all_null():
    t = Table.from_arrays({"x": np.arange(100, dtype=np.float64)}, validity={"x": np.zeros(100, dtype=bool)})
    vals, ranks, n = summary(t, "x", 0.01)
    assert n == 0 and len(vals) == 0
    t0 = Table.from_arrays({"x": np.zeros(0, dtype=np.float64)})
    vals, ranks, n = summary(t0, "x", 0.01)
    assert n == 0 and len(vals) == 0


def test_summary_device_resident_large():
    rng = np.random.default_rng(9)
    n = 20_000_000
    x = rng.standard_t(3, n)
    valid = rng.random(n) > 0.01
    t = Table.from_arrays({"x": x}, validity={"x": valid})
    t.to_device(0)
    check_exact(t, "x", 0.01)


def test_approx_quantile_reference_kats():
    # T/analyzers/AnalyzerTests.scala:568-601 (master "local": one partition)
    t = Table.from_arrays({"att1": np.arange(-1000, 1000, dtype=np.int64)})
    got = [D.ApproxQuantile("att1", q).calculate(t).value.get() for q in (0.5, 0.25, 0.75)]
    assert -20 < got[0] < 20 and -520 < got[1] < -480 and 480 < got[2] < 520
    assert got == [-19.0, -501.0, 487.0]  # Spark 2.2's single-partition digest, restated
    m = D.ApproxQuantiles("att1", [0.25, 0.5, 0.75]).calculate(t)
    assert m.value.get() == {"0.25": -501.0, "0.5": -19.0, "0.75": 487.0}


def test_approx_quantile_all_null_and_fused_run():
    x = np.arange(10, dtype=np.float64)
    t = Table.from_arrays({"x": x, "y": x}, validity={"x": np.zeros(10, dtype=bool)})
    m = D.ApproxQuantile("x", 0.5).calculate(t)
    assert m.value.isFailure and type(m.value.failed).__name__ == "EmptyStateException"
    m = D.ApproxQuantiles("x", [0.5]).calculate(t)
    assert m.value.isSuccess and m.value.get() == {}
    ctx = D.AnalysisRunner.onData(t).addAnalyzers(
        [D.Size(), D.ApproxQuantile("y", 0.5), D.ApproxQuantile("y", 0.9), D.Mean("y")]).run()
    assert ctx.metric(D.ApproxQuantile("y", 0.5)).value.get() == 4.0
    assert ctx.metric(D.Mean("y")).value.get() == 4.5


def test_approx_quantile_large_within_rank_bound():
    rng = np.random.default_rng(4)
    n = 2_000_000
    x = rng.exponential(size=n)
    t = Table.from_arrays({"x": x})
    s = np.sort(x)
    for rel in (0.01, 0.001):
        for q in (0.0, 0.01, 0.1, 0.5, 0.9, 0.999, 1.0):
            got = D.ApproxQuantile("x", q, rel).calculate(t).value.get()
            lo, hi = O.rank_interval(s, got)
            target = max(1, math.ceil(q * n))
            slack = math.ceil(rel * n) + 1
            assert lo - slack <= target <= hi + slack, (rel, q, got)


def _split(col, cuts):
    """Column -> consecutive row-range parts at `cuts` (host buffers sliced, validity re-packed per part)."""
    from deequ_amd.table import unpack_validity
    valid = unpack_validity(col.validity, col.length)
    out, lo = [], 0
    for hi in list(cuts) + [col.length]:
        v = valid[lo:hi]
        out.append(Column(col.name, col.spark_type, np.ascontiguousarray(col.values[lo:hi]),
                          None if v.all() else pack_validity(v), decimal_precision=col.decimal_precision,
                          decimal_scale=col.decimal_scale, length=hi - lo))
        lo = hi
    return out


def _batched_table():
    rng = np.random.default_rng(21)
    n = 250_003
    x = rng.normal(size=n)
    k = rng.integers(0, n, 3000)
    x[k[:700]] = np.nan
    x[k[700:1400]] = -0.0
    x[k[1400:2100]] = 0.0
    x[k[2100:2500]] = np.inf
    x[k[2500:]] = -np.inf
    cols = {"f64": x, "i64": rng.integers(-(2 ** 62), 2 ** 62, n, dtype=np.int64),
            "f32": rng.lognormal(0, 3, n).astype(np.float32), "i8": rng.integers(-128, 128, n).astype(np.int8),
            "dup": np.where(rng.random(n) < 0.6, 1.5, rng.random(n))}
    valid = {c: rng.random(n) > 0.05 for c in cols}
    valid["i8"] = np.ones(n, dtype=bool)
    t = Table.from_arrays(cols, validity=valid)
    dec = Column("dec", "DecimalType", rng.integers(-10 ** 12, 10 ** 12, n, dtype=np.int64), decimal_precision=15,
                 decimal_scale=4)
    return Table(list(t.columns.values()) + [dec])


@pytest.mark.parametrize("device", [False, True])
def test_summaries_batched_parts_exact(device):
    """dq_quantile_summaries over several columns, each in parts (an empty part included), in one call: every
    request's samples equal the oracle's order statistics of the parts concatenated, bit for bit."""
    t = _batched_table()
    n = t.nrows
    cuts = [77_777, 77_777, 190_001]
    reqs, expect, keep = [], [], []
    for i, (name, rel) in enumerate([("f64", 0.01), ("i64", 0.001), ("f32", 0.25), ("i8", 0.01), ("dup", 0.01),
                                     ("dec", 0.002), ("f64", 0.05)]):
        parts = _split(t[name], cuts if i % 2 == 0 else cuts[2:])
        if device:
            for p in parts:
                Table([p]).to_device(0)
        keep.append(parts)  # the part buffers stay alive through the call
        reqs.append(([p.native() for p in parts], rel))
        expect.append((name, rel))
    got = engine.ctx().quantile_summaries(reqs)
    for (name, rel), (vals, ranks, cnt) in zip(expect, got):
        s = O.java_sorted_doubles(t, name)
        assert cnt == len(s)
        exp_r = O.summary_ranks(cnt, rel)
        assert np.array_equal(ranks, exp_r), name
        assert np.array_equal(vals.view(np.uint64), s[exp_r - 1].view(np.uint64)), (name, rel)
    assert n == 250_003


def test_summaries_batched_sort_path_and_empty():
    """relative_error 0 (every rank: the sort path) beside a selected request and an all-NULL one."""
    rng = np.random.default_rng(8)
    x = rng.normal(size=9000)
    y = rng.integers(0, 50, 9000).astype(np.float64)
    t = Table.from_arrays({"x": x, "y": y, "z": x}, validity={"z": np.zeros(9000, dtype=bool)})
    px, py, pz = _split(t["x"], [3000]), _split(t["y"], [1, 8999]), _split(t["z"], [4500])
    got = engine.ctx().quantile_summaries([([p.native() for p in px], 0.0), ([p.native() for p in py], 0.01),
                                           ([p.native() for p in pz], 0.01)])
    for name, rel, (vals, ranks, cnt) in [("x", 0.0, got[0]), ("y", 0.01, got[1])]:
        s = O.java_sorted_doubles(t, name)
        exp_r = O.summary_ranks(cnt, rel)
        assert cnt == 9000 and np.array_equal(ranks, exp_r)
        assert np.array_equal(vals.view(np.uint64), s[exp_r - 1].view(np.uint64)), name
    assert got[2][2] == 0 and len(got[2][0]) == 0


def test_approx_quantile_chunked_equals_whole():
    """ApproxQuantile(s) over a ChunkedTable read the chunks as parts: the same digest, so the same answers, as one
    run over the whole table (above the 50000-row head size)."""
    from deequ_amd.table import ChunkedTable
    t = _batched_table()
    cuts = [60_000, 150_000]
    pf, pi, pd = (_split(t[c], cuts) for c in ("f64", "i64", "dec"))
    ct = ChunkedTable([Table([pf[i], pi[i], pd[i]]) for i in range(3)])
    an = [D.ApproxQuantile("f64", 0.5), D.ApproxQuantile("i64", 0.9, 0.001), D.ApproxQuantiles("dec", [0.1, 0.5]),
          D.Size()]
    whole = D.AnalysisRunner.onData(t).addAnalyzers(an).run()
    parted = D.AnalysisRunner.onData(ct).addAnalyzers(an).run()
    for a in an:
        assert parted.metric(a).value.get() == whole.metric(a).value.get(), a
