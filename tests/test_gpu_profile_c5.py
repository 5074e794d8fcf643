"""Reduced BASELINE config C5: the full 3-pass ColumnProfiler over a 20-column mixed
numeric / string table (5 fp64 + 5 int64 + 10 UTF-8 strings: 3 low-cardinality, 3 numeric-looking,
4 free text 1-20 characters; 5 % nulls) at 1e6 rows, checked against the oracle's own restatement of
the profiler (oracle.expected_profile: M/profiles/ColumnProfiler.scala:91-208, 357-606):
  pass 1  completeness exact, approximateNumDistinctValues = HLL++ estimate of the oracle registers
          (bit-exact), DataType class counts + determineType exact;
  pass 2  string columns inferred Integral / Fractional cast with Spark's casts; minimum / maximum /
          Long sums exact, mean / fp64 sum / stdDev within 1e-12 relative of the exact values;
  pass 3  exact histograms of the columns with <= 120 approximate distinct values (keys formatted as
          Spark's Cast to string, NULL as "NullValue", ratio = count / rows).
DQ_C5_ROWS overrides the row count."""
import math
import os

import numpy as np
import pytest

import deequ_amd as D
from deequ_amd.table import Table
import oracle as O

pytestmark = pytest.mark.gpu

ROWS = int(float(os.environ.get("DQ_C5_ROWS", "1e6")))


def c5_table(n, seed=5):
    return Table.from_arrow(c5_arrow(n, seed))


def c5_arrow(n, seed=5):
    import pyarrow as pa
    rng = np.random.default_rng(seed)

    def nulls():
        return rng.random(n) < 0.05

    arrays, names = [], []

    def add(name, values, mask):
        arrays.append(pa.array(values, mask=mask))
        names.append(name)

    add("d_norm", rng.normal(0.0, 1.0, n), nulls())
    add("d_unif", rng.random(n), nulls())
    add("d_dyad", rng.integers(-256, 257, n) / 256.0, nulls())
    add("d_n100", 100.0 + 15.0 * rng.normal(0.0, 1.0, n), nulls())
    add("d_lowc", rng.integers(0, 30, n) * 0.5 - 3.0, nulls())                  # 30 values -> pass-3 histogram
    add("l_wide", rng.integers(-2 ** 40, 2 ** 40, n, dtype=np.int64), nulls())
    add("l_lowc", rng.integers(0, 61, n, dtype=np.int64), nulls())             # 61 values -> histogram
    add("l_i32", rng.integers(-2 ** 31, 2 ** 31, n, dtype=np.int64), nulls())
    add("l_small", rng.integers(0, 1000, n, dtype=np.int64), nulls())
    add("l_neg", -rng.integers(0, 2 ** 62, n, dtype=np.int64), nulls())

    def strings(vals, mask):
        return [None if m else v for v, m in zip(vals, mask)]

    cats = np.array(["cat_%d" % i for i in range(50)], dtype=object)
    add("s_cat50", strings(cats[rng.integers(0, 50, n)], nulls()), None)
    add("s_bool", strings(np.array(["true", "false"], dtype=object)[rng.integers(0, 2, n)], nulls()), None)
    v100 = np.array(["v%02d" % i for i in range(100)], dtype=object)
    add("s_cat100", strings(v100[rng.integers(0, 100, n)], nulls()), None)
    add("s_int", strings([str(int(x)) for x in rng.integers(-10 ** 6, 10 ** 6, n)], nulls()), None)
    add("s_dec", strings(["%.2f" % x for x in rng.random(n) * 1000.0], nulls()), None)
    mix = [str(int(x)) if r < 0.7 else "%.3f" % (x / 7.0) for x, r in zip(rng.integers(-5000, 5000, n), rng.random(n))]
    add("s_mixnum", strings(mix, nulls()), None)
    letters = np.frombuffer(b"abcdefghijklmnopqrstuvwxyz0123456789 ", dtype=np.uint8)
    for k in range(4):
        lens = rng.integers(1, 21, n)
        pool = letters[rng.integers(0, len(letters), int(lens.sum()))].tobytes().decode()
        offs = np.concatenate([[0], np.cumsum(lens)])
        txt = [pool[offs[i]:offs[i + 1]] for i in range(n)]
        if k == 3:  # some multi-byte UTF-8 (characters, not bytes, count for lengths; HLL hashes the bytes)
            txt = [t + "é" if i % 17 == 0 else t for i, t in enumerate(txt)]
        add("s_text%d" % k, strings(txt, nulls()), None)
    return pa.Table.from_arrays(arrays, names=names)


def _close(a, b, rel=1e-12):
    return a == b or abs(a - b) <= rel * max(abs(a), abs(b))


def test_c5_reduced_column_profile_against_oracle():
    t = c5_table(ROWS)
    assert len(t.columns) == 20
    exp = O.expected_profile(t)
    t.to_device()
    _check_profile(t, D.ColumnProfiler.profile(t), exp)


def test_c5_chunked_column_profile_against_oracle():
    """The same table as 3 row chunks (ChunkedTable: how a shard whose string bytes exceed int32 offsets is held):
    each pass runs per chunk and the chunk states merge with the reference's State.sum (HLL registers max, moments
    Chan-merged, KLL sketches merged, DataType / histogram counts added) -- equal to the oracle over the whole
    table, HLL estimates bit-exact."""
    pat = c5_arrow(ROWS)
    full = Table.from_arrow(pat)
    exp = O.expected_profile(full)
    cut = [0, ROWS // 3, ROWS // 3 + ROWS // 4 + 7, ROWS]
    chunks = [Table.from_arrow(pat.slice(a, b - a)).to_device() for a, b in zip(cut, cut[1:])]
    ct = D.ChunkedTable(chunks)
    assert ct.nrows == ROWS
    _check_profile(full, D.ColumnProfiler.profile(ct), exp)
    # AnalysisRunner over the chunks equals the single-table run (scan, grouping and KLL analyzers)
    an = [D.Size(), D.Completeness("s_int"), D.Mean("d_n100"), D.Sum("l_wide"), D.Maximum("l_neg"),
          D.StandardDeviation("d_norm"), D.ApproxCountDistinct("s_text0"), D.Uniqueness(["s_cat50", "l_lowc"]),
          D.Entropy("s_cat100"), D.Correlation("d_norm", "d_unif"), D.KLLSketch("d_unif")]
    full.to_device()
    want = D.AnalysisRunner.onData(full).addAnalyzers(an).run()
    got = D.AnalysisRunner.onData(ct).addAnalyzers(an).run()
    for a in an:
        w, g = want.metric(a).value.get(), got.metric(a).value.get()
        if isinstance(a, D.KLLSketch):
            assert sum(b.count for b in g.buckets) == sum(b.count for b in w.buckets), a
        else:
            assert _close(g, w), (a, g, w)


def _check_profile(t, prof, exp):
    assert prof.numRecords == ROWS
    seen_hist = seen_numeric_string = 0
    for name, e in exp.items():
        p = prof.profiles[name]
        assert p.completeness == e["completeness"], name
        assert p.approximateNumDistinctValues == e["approx_distinct"], name
        assert p.dataType == e["dataType"], (name, p.dataType, e["dataType"])
        assert p.isDataTypeInferred == e["inferred"], name
        assert p.typeCounts == e["typeCounts"], (name, p.typeCounts, e["typeCounts"])
        if e["dataType"] in ("Integral", "Fractional"):
            assert isinstance(p, D.NumericColumnProfile), name
            st = e["numeric"]
            assert (p.minimum, p.maximum) == (st["min"], st["max"]), name
            if e["dataType"] == "Integral":
                assert p.sum == st["sum"], name
            else:
                assert _close(p.sum, st["sum"]), (name, p.sum, st["sum"])
            assert _close(p.mean, st["mean"]), (name, p.mean, st["mean"])
            assert _close(p.stdDev, st["stdDev"]), (name, p.stdDev, st["stdDev"])
            assert sum(b.count for b in p.kll.buckets) == st["n"], name
            seen_numeric_string += t[name].spark_type == O.T_STRING
        if e["histogram"] is None:
            assert p.histogram is None, name
        else:
            seen_hist += 1
            got = {k: v.absolute for k, v in p.histogram.values.items()}
            assert got == e["histogram"], name
            assert p.histogram.numberOfBins == len(e["histogram"])
            for k, v in p.histogram.values.items():
                assert v.ratio == e["histogram"][k] / ROWS
    assert seen_hist >= 5 and seen_numeric_string == 3


def test_chunked_run_with_an_all_null_chunk_equals_the_whole_table():
    """A column that is NULL on every row of one chunk: that chunk's empty states are no failure -- the merged state
    decides (as Spark's partial aggregates do); a column NULL everywhere fails on both sides the same way."""
    rng = np.random.default_rng(5)
    n = 30_000
    x = [None if (i < 12_000 or rng.random() < 0.1) else float(rng.normal()) for i in range(n)]
    k = [int(v) for v in rng.integers(0, 50, n)]
    z = [None] * n
    data = {"x": x, "k": k, "z": z}
    types = {"x": "double", "k": "long", "z": "double"}
    full = Table.from_pydict(data, types=types).to_device()
    cuts = [0, 12_000, 20_000, n]
    chunks = [Table.from_pydict({c: v[a:b] for c, v in data.items()}, types=types).to_device()
              for a, b in zip(cuts, cuts[1:])]
    ct = D.ChunkedTable(chunks)
    an = [D.Mean("x"), D.Minimum("x"), D.StandardDeviation("x"), D.Completeness("x"), D.ApproxCountDistinct("x"),
          D.Uniqueness(["x"]), D.KLLSketch("x"), D.Mean("z"), D.Sum("k"), D.Size()]
    want = D.AnalysisRunner.onData(full).addAnalyzers(an).run()
    got = D.AnalysisRunner.onData(ct).addAnalyzers(an).run()
    for a in an:
        w, g = want.metric(a).value, got.metric(a).value
        assert w.isSuccess == g.isSuccess, (a, w, g)
        if not w.isSuccess:
            continue
        if isinstance(a, D.KLLSketch):
            assert sum(b.count for b in g.get().buckets) == sum(b.count for b in w.get().buckets), a
        else:
            assert _close(g.get(), w.get()), (a, g.get(), w.get())


def test_c5_chunked_shard_at_scale_against_oracle():
    """The 2.5e8-row C5 shard bench.py times (two 1.25e8-row chunks, ChunkedTable) profiled by the full ColumnProfiler,
    checked against the oracle at that size (it was checked only by the bench's property asserts).
    The 10 numeric columns are regenerated row by row by the oracle's streamed suite (same counter-based generators
    and validity): completeness and min / max exact, integral sums exact, fp64 sum / mean / stdDev within 1e-12 of the
    exact values, approximateNumDistinctValues from bit-exact HLL registers, KLL bucket weights = non-NULL count. The
    10 string columns: completeness exact and the HLL estimate from the oracle's XXH64 registers over the device bytes."""
    import torch
    import bench
    import deequ_amd.native as N
    from deequ_amd import engine
    rows = 250_000_000
    t, _ = bench.c5_shard(torch, N, engine.ctx(), torch.device("cuda", 0), rows)
    assert len(t.chunks) == 2
    prof = D.ColumnProfiler.profile(t)
    assert prof.numRecords == rows
    specs = []
    for j, (name, kind) in enumerate(bench.C5_NUMERIC):
        specs.append(dict(name=name, kind=kind, spark_type=O.T_DOUBLE if kind in (1, 2, 3, 6, 7) else O.T_LONG,
                          seed=0xC5000000 + j, vseed=0xC5200000 + j, permille=50, hll=1))
    cols, _ = O.generated_suite(specs, 0, rows)
    for sp, o in zip(specs, cols):
        p = prof.profiles[sp["name"]]
        n = o["n"]
        assert p.completeness == n / rows, sp["name"]
        assert p.approximateNumDistinctValues == int(O.hll_count(o["words"])), sp["name"]
        assert isinstance(p, D.NumericColumnProfile), sp["name"]
        if sp["spark_type"] == O.T_LONG:
            assert (p.minimum, p.maximum) == (float(o["imin"]), float(o["imax"])), sp["name"]
            assert p.sum == float(o["isum"]), sp["name"]
        else:
            assert (p.minimum, p.maximum) == (o["dmin"], o["dmax"]), sp["name"]
            if sp["kind"] == 1:  # dyadic values: every partial sum is exact
                assert p.sum == o["ex_sum"], sp["name"]
            else:
                assert _close(p.sum, o["ex_sum"]), (sp["name"], p.sum, o["ex_sum"])
        sigma = math.sqrt(o["ex_m2"] / n)
        # the mean against max(|mean|, sigma), as the C2 bars (a zero-mean column has no relative scale of its own)
        assert abs(p.mean - o["ex_mean"]) <= 1e-12 * max(abs(o["ex_mean"]), sigma), (sp["name"], p.mean, o["ex_mean"])
        assert _close(p.stdDev, sigma), (sp["name"], p.stdDev, sigma)
        assert sum(b.count for b in p.kll.buckets) == n, sp["name"]
    # string columns: completeness and HLL registers over the device bytes, chunk by chunk
    for name, _ in bench.C5_STRINGS:
        regs = np.zeros(512, dtype=np.uint8)
        valid_total = 0
        for ch in t.chunks:
            c = ch[name]
            off = c.device["offsets"].cpu().numpy()
            data = c.device["values"].cpu().numpy()
            bits = c.device["validity"].cpu().numpy()
            mask = np.unpackbits(bits, bitorder="little")[:c.length].astype(np.uint8)
            valid_total += int(mask.sum())
            O.lib().oracle_hll_strings(data.ctypes.data, off.ctypes.data, mask.ctypes.data, c.length, regs.ctypes.data)
            del data, off
        p = prof.profiles[name]
        assert p.completeness == valid_total / rows, name
        words = np.zeros(52, dtype=np.int64)
        O.lib().oracle_hll_pack(regs.ctypes.data, words.ctypes.data)
        assert p.approximateNumDistinctValues == int(O.hll_count([int(w) for w in words])), name


def _check_c5_extras(full, ctx, extras):
    """ApproxQuantile(0.5) inside the GK rank bound of the exact order statistics (relativeError 0.01; a merged
    summary of several partitions keeps the bound, QuantileSummaries.merge), Uniqueness / Entropy against the oracle's
    exact grouping (A/ApproxQuantile.scala:28-103, A/Uniqueness.scala:29-36, A/Entropy.scala:28-42)."""
    for a in extras:
        m = ctx.metric(a).value
        assert m.isSuccess, (a, m)
        if isinstance(a, D.ApproxQuantile):
            s = O.java_sorted_doubles(full, a.column)
            n = len(s)
            lo, hi = O.rank_interval(s, m.get())
            target = max(1, math.ceil(0.5 * n))
            slack = math.ceil(0.01 * n) + 1
            assert lo - slack <= target <= hi + slack, (a, m.get(), lo, hi, target)
        else:
            col = a.columns[0] if isinstance(a, D.Uniqueness) else a.column
            freq, n = O.frequencies(full, [col])
            exp = O.grouping_summary(freq, n)
            want = exp["num_unique"] / n if isinstance(a, D.Uniqueness) else exp["entropy"]
            assert _close(m.get(), want), (a, m.get(), want)


def test_c5_quantiles_and_grouping_against_oracle():
    """The part of BASELINE config C5 beside the ColumnProfiler (`ApproxQuantile(0.5)` on numerics; the
    grouping analyzers): the analyzer list bench.py's C5 line times, on the reduced table, whole and as 3 row chunks."""
    import bench
    pat = c5_arrow(ROWS)
    full = Table.from_arrow(pat)
    extras = [D.ApproxQuantile(c, 0.5) for c in pat.column_names[:10]]
    extras += [D.Uniqueness(["s_cat100"]), D.Entropy("s_cat100"), D.Uniqueness(["s_text0"]), D.Entropy("s_text0")]
    assert len(bench.c5_extra_analyzers(D)) == len(extras)  # the bench's list has the same shape
    dev = Table.from_arrow(pat).to_device()
    _check_c5_extras(full, D.AnalysisRunner.onData(dev).addAnalyzers(extras).run(), extras)
    cut = [0, ROWS // 3, ROWS // 3 + ROWS // 4 + 7, ROWS]
    ct = D.ChunkedTable([Table.from_arrow(pat.slice(a, b - a)).to_device() for a, b in zip(cut, cut[1:])])
    _check_c5_extras(full, D.AnalysisRunner.onData(ct).addAnalyzers(extras).run(), extras)


def test_c5_step_runs_the_extras_beside_the_profiler(monkeypatch):
    """bench.py's C5 step submits the extra analyzers with runAsync (a helper context) and profiles meanwhile: the
    extras' metrics pass the oracle checks and the profile equals the one the sequential step computes."""
    import bench
    pat = c5_arrow(ROWS)
    full = Table.from_arrow(pat)
    cut = [0, ROWS // 2 + 11, ROWS]
    ct = D.ChunkedTable([Table.from_arrow(pat.slice(a, b - a)).to_device() for a, b in zip(cut, cut[1:])])
    extras = [D.ApproxQuantile(c, 0.5) for c in pat.column_names[:10]]
    extras += [D.Uniqueness(["s_cat100"]), D.Entropy("s_cat100"), D.Uniqueness(["s_text0"]), D.Entropy("s_text0")]
    monkeypatch.delenv("DQ_C5_SEQUENTIAL", raising=False)
    prof, actx = bench.c5_step(D, ct, extras)
    _check_c5_extras(full, actx, extras)
    monkeypatch.setenv("DQ_C5_SEQUENTIAL", "1")
    prof2, actx2 = bench.c5_step(D, ct, extras)
    for a in extras:
        assert actx.metric(a).value.get() == actx2.metric(a).value.get(), a
    assert prof.numRecords == prof2.numRecords == ROWS
    for name, p in prof2.profiles.items():
        q = prof.profiles[name]
        assert (q.completeness, q.approximateNumDistinctValues, q.dataType) == \
            (p.completeness, p.approximateNumDistinctValues, p.dataType), name
        if isinstance(p, D.NumericColumnProfile):
            assert (q.minimum, q.maximum, q.sum, q.mean, q.stdDev) == (p.minimum, p.maximum, p.sum, p.mean, p.stdDev)
        assert (q.histogram is None) == (p.histogram is None), name
        if p.histogram is not None:
            assert q.histogram == p.histogram, name
