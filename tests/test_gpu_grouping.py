"""GPU parity of the frequency tables (grouping analyzers + Histogram) against the oracle and the
reference KATs. Bars: bit-exact group counts / numRows / distinct counts / histograms; entropy within
1e-12 relative of the exact (fsum) oracle."""
import math

import numpy as np
import pytest

import deequ_amd as D
import deequ_amd.native as N
from deequ_amd.native import NativeError
from deequ_amd import engine
from deequ_amd.table import Table, Column, pack_validity
import oracle as O
from helpers import analyzer_from_spec, check_metric, table_from_fixture

pytestmark = pytest.mark.gpu

GROUPING = {"Uniqueness", "Distinctness", "UniqueValueRatio", "Entropy", "CountDistinct", "MutualInformation",
            "Histogram"}


def test_grouping_kats(kats):
    for k in kats["kats"]:
        if k["analyzer"][0] not in GROUPING:
            continue
        t = table_from_fixture(kats["fixtures"][k["fixture"]])
        a = analyzer_from_spec(k["analyzer"])
        check_metric(a.calculate(t), k["expected"], rel=1e-15)


def test_grouping_kats_through_runner(kats):
    # several grouping analyzers on the same columns share one frequency table
    t = table_from_fixture(kats["fixtures"]["dfFull"])
    analyzers = [D.Uniqueness(["att1"]), D.Distinctness(["att1"]), D.Entropy("att1"), D.CountDistinct(["att1"]),
                 D.UniqueValueRatio(["att1"]), D.Size()]
    ctx = D.AnalysisRunner.onData(t).addAnalyzers(analyzers).run()
    assert ctx.metric(D.Uniqueness(["att1"])).value.get() == 0.25
    assert ctx.metric(D.Distinctness(["att1"])).value.get() == 0.5
    ent = -(0.75 * math.log(0.75) + 0.25 * math.log(0.25))
    assert abs(ctx.metric(D.Entropy("att1")).value.get() - ent) < 1e-15
    assert ctx.metric(D.CountDistinct(["att1"])).value.get() == 2.0
    assert ctx.metric(D.UniqueValueRatio(["att1"])).value.get() == 0.5
    assert ctx.metric(D.Size()).value.get() == 4.0


def test_incremental_grouping_merges(kats):
    inc = kats["incremental"]
    a, b = table_from_fixture(inc["initial"]), table_from_fixture(inc["delta"])
    for spec, va, vb, vm, src in inc["cases"]:
        an = analyzer_from_spec(spec)
        if type(an).__name__ not in GROUPING:
            continue
        sa, sb = an.computeStateFrom(a), an.computeStateFrom(b)
        assert an.computeMetricFrom(sa).value.get() == va, src
        assert an.computeMetricFrom(sb).value.get() == vb, src
        assert an.computeMetricFrom(sa.sum(sb)).value.get() == vm, src


def _summary_vs_oracle(table, cols, include_nulls=False):
    ft = engine.frequencies(table, cols, include_nulls=include_nulls)
    s = ft.summary(None)
    freq, n = O.frequencies(table, cols, include_nulls=include_nulls)
    exp = O.grouping_summary(freq, n)
    assert s["num_rows"] == n
    assert s["num_groups"] == exp["num_groups"]
    assert s["num_unique"] == exp["num_unique"]
    assert abs(s["entropy"] - exp["entropy"]) <= 1e-12 * max(1.0, exp["entropy"])
    got = ft.to_dict()
    norm = {tuple(O._group_key(v) for v in k): c for k, c in got.items()}
    assert norm == freq
    return ft, freq


@pytest.mark.parametrize("n", [0, 1, 1000, 65537])
def test_fixed_width_keys_parity(n):
    rng = np.random.default_rng(n)
    valid = rng.random(n) > 0.1
    cols = {
        "l": rng.integers(-50, 50, n).astype(np.int64),
        "i": rng.integers(-3, 3, n).astype(np.int32),
        "d": np.where(rng.random(n) < 0.05, np.nan, rng.integers(0, 20, n) / 4.0),
        "f": (rng.integers(0, 7, n) / 2.0).astype(np.float32),
        "b": rng.integers(0, 2, n).astype(np.bool_),
        "u": rng.permutation(n).astype(np.int64),
    }
    t = Table.from_arrays(cols, validity={"l": valid, "d": valid})
    for c in cols:
        _summary_vs_oracle(t, [c])
        _summary_vs_oracle(t, [c], include_nulls=True)


def test_signed_zero_and_nan_grouping():
    x = np.array([0.0, -0.0, np.nan, float(np.frombuffer(np.uint64(0x7ff8000000000001).tobytes(), np.float64)[0]),
                  1.0, 1.0])
    t = Table.from_arrays({"x": x})
    ft, freq = _summary_vs_oracle(t, ["x"])
    assert ft.summary()["num_groups"] == 4  # 0.0, -0.0, NaN (canonical), 1.0


def test_all_ones_key_is_counted():
    # int64 -1 has every bit set: the fast path must not confuse it with an empty slot
    t = Table.from_arrays({"k": np.array([-1, -1, 5, -1, 0], dtype=np.int64)})
    _summary_vs_oracle(t, ["k"])


def test_string_and_multicolumn_keys_parity():
    rng = np.random.default_rng(3)
    n = 20000
    words = ["", "a", "bb", "ccc", "ü", "NullValue", "x" * 40, "long string " * 5]
    s1 = [None if rng.random() < 0.1 else words[rng.integers(0, len(words))] for _ in range(n)]
    s2 = [None if rng.random() < 0.3 else str(rng.integers(0, 30)) for _ in range(n)]
    i1 = [None if rng.random() < 0.2 else int(rng.integers(0, 4)) for _ in range(n)]
    t = Table.from_pydict({"s1": s1, "s2": s2, "i1": i1}, types={"s1": "string", "s2": "string", "i1": "int"})
    _summary_vs_oracle(t, ["s1"])
    _summary_vs_oracle(t, ["s1", "s2"])
    _summary_vs_oracle(t, ["s2", "i1"])
    _summary_vs_oracle(t, ["s1", "s2", "i1"])


def test_histogram_string_null_merges_with_literal_nullvalue():
    # Histogram casts to string and fills NULL with "NullValue" (A/Histogram.scala:60-63)
    t = Table.from_pydict({"s": ["NullValue", None, "a", None]}, types={"s": "string"})
    m = D.Histogram("s").calculate(t)
    dist = m.value.get()
    assert dist.numberOfBins == 2
    assert dist["NullValue"].absolute == 3 and dist["a"].absolute == 1


def test_histogram_topn_and_ratios():
    rng = np.random.default_rng(8)
    n = 50000
    vals = rng.zipf(1.6, n) % 3000
    valid = rng.random(n) > 0.02
    t = Table.from_arrays({"v": vals.astype(np.int64)}, validity={"v": valid})
    m = D.Histogram("v", None, 100).calculate(t)
    dist = m.value.get()
    freq, _ = O.frequencies(t, ["v"], include_nulls=True)
    assert dist.numberOfBins == len(freq)
    top = sorted(freq.values(), reverse=True)[:100]
    assert sorted((v.absolute for v in dist.values.values()), reverse=True) == top
    for key, v in dist.values.items():
        okey = None if key == "NullValue" else int(key)
        assert freq[(okey,)] == v.absolute
        assert v.ratio == v.absolute / n


def test_c4_closed_form_at_reduced_scale():
    # exactly D distinct keys, D/2 of them 19 times and D/2 once.
    total, distinct = 10_000_000, 1_000_000
    import torch
    keys = torch.empty(total, dtype=torch.int64, device="cuda")
    engine.ctx().synth_freq_keys(total, distinct, 0, total, keys.data_ptr())
    engine.ctx().synchronize()
    col = Column("k", N.TYPE_LONG, None, None, length=total)
    col.device = {"values": keys}
    t = Table([col])
    analyzers = [D.Uniqueness(["k"]), D.Distinctness(["k"]), D.UniqueValueRatio(["k"]), D.CountDistinct(["k"]),
                 D.Entropy("k")]
    ctx = D.AnalysisRunner.onData(t).addAnalyzers(analyzers).run()
    half = distinct // 2
    assert ctx.metric(analyzers[0]).value.get() == half / total
    assert ctx.metric(analyzers[1]).value.get() == distinct / total
    assert ctx.metric(analyzers[2]).value.get() == 0.5
    assert ctx.metric(analyzers[3]).value.get() == float(distinct)
    big = (total - half) / half  # occurrences of the repeated keys
    exact = math.fsum([-half * (big / total) * math.log(big / total), -half * (1 / total) * math.log(1 / total)])
    assert abs(ctx.metric(analyzers[4]).value.get() - exact) <= 1e-12 * exact
    # device generator == oracle generator on a slice
    sl = keys[123456:123456 + 4096].cpu().numpy()
    assert np.array_equal(sl, O.synth_freq_keys(total, distinct, 123456, 4096))


def _value_mixing_to_all_ones():
    """The int64 whose splitmix64 finalizer is 2^64 - 1 (the inverse finalizer of all ones)."""
    m = (1 << 64) - 1

    def inv(a):
        x = a
        for _ in range(6):
            x = (x * (2 - a * x)) & m
        return x

    def unxorshift(z, k):
        r = z
        for _ in range(64 // k + 1):
            r = z ^ (r >> k)
        return r & m
    z = m
    z = unxorshift(z, 31)
    z = (z * inv(0x94D049BB133111EB)) & m
    z = unxorshift(z, 27)
    z = (z * inv(0xBF58476D1CE4E5B9)) & m
    z = unxorshift(z, 30)
    return z - (1 << 64) if z >= 1 << 63 else z


def _sorted_pairs(ft):
    k, c = ft.export_pairs()
    o = np.lexsort((c, k))
    return k[o], c[o]


@pytest.mark.parametrize("case", ["uniform", "repeats", "heavy_hitter", "nulls_nan_sentinel", "narrow_window",
                                  "narrow_outlier", "int32", "float32"])
def test_fast_build_equals_exact_build(case, monkeypatch):
    """The fast build (fixed-capacity buckets, atomically reserved runs, no count pass; >= 2^24 rows) against the
    exactly-counted build on the same keys: identical groups, counts and summary. A heavy hitter overflows a
    bucket and must take the exact path by itself. Narrow keys (32-bit offsets in the partition buffers): 8-byte
    keys inside a sampled window (negative, far from zero), a key outside the window on a row the sample skips
    (the build restarts with 64-bit keys), and 4-byte keys (always narrow)."""
    import torch
    n = 40_000_000
    rng = np.random.default_rng(7)
    if case == "narrow_window":
        v = rng.integers(-5_000_000_000 - 2_000_000, -5_000_000_000, n, dtype=np.int64)
    elif case == "narrow_outlier":
        v = rng.integers(0, 2_000_000, n, dtype=np.int64)
        v[12345] = 1 << 40  # not on the sample's stride (n / 65536 = 610)
        v[777777] = -(1 << 40)
    elif case == "int32":
        v = rng.integers(-2 ** 31, 2 ** 31, n, dtype=np.int64).astype(np.int32)
        v[::7] = rng.integers(-1000, 1000, len(v[::7]), dtype=np.int32)
    elif case == "float32":
        v = (rng.integers(-3_000_000, 3_000_000, n) / 4.0).astype(np.float32)
        v[rng.random(n) < 0.01] = np.nan
        v[rng.random(n) < 0.01] = -0.0
    elif case == "uniform":
        v = rng.integers(0, 2 ** 62, n, dtype=np.int64)
        v[::1_000_003] = _value_mixing_to_all_ones()  # its mixed key is the EMPTY slot marker
    elif case == "repeats":
        v = rng.integers(0, n // 19, n, dtype=np.int64)
    elif case == "heavy_hitter":
        v = np.where(rng.random(n) < 0.3, 12345, rng.integers(0, 10 ** 6, n)).astype(np.int64)
    else:
        v = rng.integers(-500_000, 500_000, n).astype(np.float64) / 8.0
        v[rng.random(n) < 0.01] = np.nan
        v[rng.random(n) < 0.01] = -0.0
    valid = rng.random(n) > 0.02 if case in ("nulls_nan_sentinel", "narrow_window") else None
    col = Column("k", {np.dtype(np.float64): N.TYPE_DOUBLE, np.dtype(np.int64): N.TYPE_LONG,
                       np.dtype(np.int32): N.TYPE_INT, np.dtype(np.float32): N.TYPE_FLOAT}[v.dtype], None, None,
                 length=n)
    col.device = {"values": torch.from_numpy(v).cuda()}
    if valid is not None:
        col.device["validity"] = torch.from_numpy(pack_validity(valid)).cuda()
    t = Table([col])
    for include_nulls in ((False, True) if valid is not None else (False,)):
        fast = engine.frequencies(t, ["k"], include_nulls)
        monkeypatch.setenv("DQ_FREQ_EXACT", "1")
        exact = engine.frequencies(t, ["k"], include_nulls)
        monkeypatch.delenv("DQ_FREQ_EXACT")
        sf, se = fast.summary(None), exact.summary(None)
        for key in ("num_rows", "num_groups", "num_unique", "max_count", "null_count"):
            assert sf[key] == se[key], (case, key, sf, se)
        assert abs(sf["entropy"] - se["entropy"]) <= 1e-12 * se["entropy"]
        kf, cf = _sorted_pairs(fast)
        ke, ce = _sorted_pairs(exact)
        assert np.array_equal(kf, ke) and np.array_equal(cf, ce), case
        assert [c for _, c in fast.top(5)] == [c for _, c in exact.top(5)]
        del fast, exact


def _freq_dict(t, cols, include_nulls=False, env=None):
    import os
    old = {k: os.environ.get(k) for k in (env or {})}
    os.environ.update(env or {})
    try:
        ft = engine.frequencies(t, cols, include_nulls=include_nulls)
        return ft.to_dict(), ft.summary(None)
    finally:
        for k, v in old.items():
            if v is None:
                del os.environ[k]
            else:
                os.environ[k] = v


@pytest.mark.parametrize("device", [False, True])
def test_small_table_path_equals_the_regular_path(device):
    """Small general-path tables (<= ~2600 distinct string / multi-column keys) take the fused one-pass build
    (small_build_kernel + small_check_kernel); its groups, counts, NULL handling (Histogram's "NullValue") and
    summary equal the regular extract / build / verify path (DQ_FREQ_NO_SMALL=1) and the oracle, over 3e5 rows in
    many workgroups (groups seen by several workgroups, representatives merged to the smallest row)."""
    rng = np.random.default_rng(17)
    n = 300_001
    words = np.array(["w%d" % i for i in range(700)] + ["", "NullValue", "ü" * 3, "x" * 60], dtype=object)
    s = [None if rng.random() < 0.05 else words[rng.integers(0, len(words))] for _ in range(n)]
    k = [None if rng.random() < 0.1 else int(rng.integers(0, 3)) for _ in range(n)]
    t = Table.from_pydict({"s": s, "k": k}, types={"s": "string", "k": "int"})
    if device:
        t.to_device(0)
    for cols, nulls in ((["s"], True), (["s"], False), (["s", "k"], False), (["s", "k"], True)):
        small, ssum = _freq_dict(t, cols, nulls)
        regular, rsum = _freq_dict(t, cols, nulls, {"DQ_FREQ_NO_SMALL": "1"})
        assert small == regular, cols
        assert ssum == rsum, (cols, ssum, rsum)
    _summary_vs_oracle(t, ["s", "k"])


@pytest.mark.parametrize("distinct", [60, 3000, 1_000_000])
def test_optimistic_small_build_equals_the_sized_path(distinct):
    """General keys with >= 2^22 rows first try the one-pass small build without the sizing pass: it must equal the
    sized path (DQ_FREQ_NO_OPTIMISTIC=1) when it succeeds (60 distinct strings), when the union of the workgroup
    tables overflows the one region (3000) and when every workgroup's LDS table fills at once (1e6 distinct)."""
    import pyarrow as pa
    rng = np.random.default_rng(distinct)
    n = 5_000_000
    words = np.array(["v%07d" % i for i in range(distinct)], dtype=object)
    idx = rng.integers(0, distinct, n)
    valid = rng.random(n) > 0.03
    arr = pa.array(words[idx], type=pa.string(), mask=~valid)
    t = Table.from_arrow(pa.table({"s": arr, "k": pa.array(rng.integers(0, 2, n))}))
    t.to_device(0)
    for cols, nulls in ((["s"], True), (["s", "k"], False)):
        opt, osum = _freq_dict(t, cols, nulls)
        sized, ssum = _freq_dict(t, cols, nulls, {"DQ_FREQ_NO_OPTIMISTIC": "1"})
        assert opt == sized, (distinct, cols)
        assert osum == ssum, (distinct, cols, osum, ssum)


def test_fingerprint_collisions_are_never_merged():
    """Fingerprints narrowed to 4 bits (DQ_FREQ_FP_MASK) collide on every seed: both the small path and the regular
    path detect the collisions against the representatives and fail the build instead of merging groups."""
    words = ["w%d" % i for i in range(40)]
    t = Table.from_pydict({"s": [words[i % 40] for i in range(5000)]}, types={"s": "string"})
    for extra in ({}, {"DQ_FREQ_NO_SMALL": "1"}):
        with pytest.raises(NativeError):
            _freq_dict(t, ["s"], False, dict(extra, DQ_FREQ_FP_MASK="0xF"))


def test_histogram_binning_udf_per_distinct_value(kats):
    """Histogram(column, binningUdf) (A/Histogram.scala:59-65: the UDF over the column, its result cast to string,
    NULL filled with "NullValue", then the group-by): the reference's own case (AnalyzerTests.scala:227-245, a/b ->
    Value1, the rest -> Value2 over dfMissing.att1) and a 2e6-row LONG column against the oracle's per-row binning. The
    UDF runs once per distinct value (+ once for NULL), not once per row."""
    t = table_from_fixture(kats["fixtures"]["dfMissing"])
    calls = []

    def binner(v):
        calls.append(v)
        return "Value1" if v in ("a", "b") else "Value2"
    h = D.Histogram("att1", binner).calculate(t).value.get()
    assert h.numberOfBins == 2 and set(h.values) == {"Value1", "Value2"}
    rng = np.random.default_rng(4)
    n = 2_000_000
    v = rng.integers(0, 1000, n).astype(np.int64)
    valid = rng.random(n) > 0.02
    t = Table.from_arrays({"v": v}, validity={"v": valid})
    calls.clear()

    def bin2(x):
        calls.append(x)
        if x is None:
            return None  # -> "NullValue"
        return "lo" if x < 300 else (7 if x < 900 else None)
    h = D.Histogram("v", bin2, 10).calculate(t).value.get()
    assert len(calls) <= 1001
    want = {}
    for x, ok in zip(v.tolist(), valid.tolist()):
        lab = bin2(x if ok else None)
        lab = "NullValue" if lab is None else str(lab)
        want[lab] = want.get(lab, 0) + 1
    assert h.numberOfBins == len(want)
    assert {k: d.absolute for k, d in h.values.items()} == want
    for k, d in h.values.items():
        assert d.ratio == want[k] / n


def test_histogram_binning_udf_string_input():
    """Histogram(..., udfInputAsString=True): the UDF sees the Spark string form of a non-string column's values (as a
    Scala UDF declared over String does through Spark's implicit cast) -- a first-character binning of DOUBLE values
    counts "1.0", "1.5", "10.25" together."""
    vals = [1.0, 1.5, 10.25, 2.0, None, 2.5, 1.0]
    t = Table.from_pydict({"x": vals}, types={"x": "double"})
    seen = []

    def first(s):
        seen.append(s)
        return None if s is None else s[:1]
    h = D.Histogram("x", first, udfInputAsString=True).calculate(t).value.get()
    assert {k: d.absolute for k, d in h.values.items()} == {"1": 4, "2": 2, "NullValue": 1}
    assert all(v is None or isinstance(v, str) for v in seen)
    assert "1.0" in seen and "10.25" in seen
