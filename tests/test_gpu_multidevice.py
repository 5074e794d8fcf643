"""One C-ABI context over several GPUs (dq_open_devices, include/dq.h; SURVEY.md §8b multi-GPU row): host
columns are row-sharded over the devices, scanned concurrently and folded in device order; grouping keys are
pre-aggregated per device and exchanged by owner device — over RCCL when the devices are distinct (here:
ndev = 1, a communicator of size 1, which is the RCCL path end to end), with device copies when shards share
a GPU (ndev = 4 on this one-GPU box). Every result must equal the single-device engine's and the oracle's."""
import math
import os

import numpy as np
import pytest

import deequ_amd as D
import deequ_amd.native as N
from deequ_amd import engine
from deequ_amd.table import Table, Column
import oracle as O
from test_gpu_scan import random_table, all_analyzers, assert_state_parity

pytestmark = pytest.mark.gpu


@pytest.fixture(params=[("0", True), ("0,0,0,0", False), ("0,0,0", False)], ids=["rccl-1", "copy-4", "copy-3"])
def multi(request, monkeypatch):
    spec, rccl = request.param
    monkeypatch.setenv("DQ_DEVICES", spec)
    ctx = engine.ctx()
    assert ctx.num_devices() == len(spec.split(","))
    assert ctx.uses_rccl() == rccl
    return ctx


def test_sharded_scan_matches_oracle(multi):
    rng = np.random.default_rng(17)
    t = random_table(rng, 100_003, with_nan=True)
    analyzers = all_analyzers(t)
    batch = D.ScanBatch(t)
    offsets = [a.addOps(batch) for a in analyzers]
    before = multi.scan_launch_count()
    states = batch.run()
    assert multi.scan_launch_count() - before == 1  # one fused scan call for the batch, over every device
    for a, ops in zip(analyzers, offsets):
        assert_state_parity(t, a, a.fromAggregationResult(states, ops))


def test_sharded_scan_with_where_and_strings(multi):
    from deequ_amd.table import _column_from_pylist
    rng = np.random.default_rng(5)
    n = 30_001
    words = ["alpha", "beta", "", "12", "3.5", "true", "héllo", None]
    s = [words[i] for i in rng.integers(0, len(words), n)]
    t = Table([_column_from_pylist("s", "string", s), Column("k", N.TYPE_LONG, rng.integers(0, 9, n).astype(np.int64))])
    analyzers = [D.Size("k < 5"), D.Completeness("s", "k < 5"), D.MinLength("s"), D.MaxLength("s"), D.DataType("s"),
                 D.ApproxCountDistinct("s"), D.PatternMatch("s", r"^\d"), D.Compliance("c", "length(s) > 3", "k > 1")]
    got = D.AnalysisRunner.onData(t).addAnalyzers(analyzers).run()
    for a in analyzers:
        exp = O.expected_state(t, a)
        st = a.computeStateFrom(t)  # through the same multi-device context
        assert (st is None and exp is None) or st == exp, (a, st, exp)
        assert got.metric(a).value.isSuccess, a


@pytest.mark.parametrize("kind", ["long", "double"])
def test_sharded_frequencies_match_oracle(multi, kind):
    rng = np.random.default_rng(11)
    n = 80_001
    if kind == "long":
        v = rng.integers(0, 20_000, n).astype(np.int64)
    else:
        v = np.where(rng.random(n) < 0.2, np.array([np.nan, -0.0, 0.0, np.inf])[rng.integers(0, 4, n)],
                     rng.integers(0, 5000, n) / 8.0)
    t = Table.from_arrays({"k": v}, validity={"k": rng.random(n) > 0.03})
    for include_nulls in (False, True):
        ft = engine.frequencies(t, ["k"], include_nulls=include_nulls)
        freq, nrows = O.frequencies(t, ["k"], include_nulls=include_nulls)
        exp = O.grouping_summary(freq, nrows)
        s = ft.summary(None)
        assert (s["num_rows"], s["num_groups"], s["num_unique"]) == (nrows, exp["num_groups"], exp["num_unique"])
        assert abs(s["entropy"] - exp["entropy"]) <= 1e-12 * exp["entropy"]
        got = {tuple(O._group_key(x) for x in key): c for key, c in ft.to_dict().items()}
        assert got == freq
        top = ft.top(10)
        assert [c for _, c in top] == sorted(freq.values(), reverse=True)[:10]
    for a in (D.Uniqueness(["k"]), D.Distinctness(["k"]), D.Entropy("k"), D.CountDistinct(["k"]),
              D.UniqueValueRatio(["k"])):
        m = a.calculate(t)
        assert m.value.isSuccess, (a, m)


@pytest.mark.parametrize("cols", [["s"], ["s", "k"], ["k", "d"]])
def test_sharded_general_grouping_matches_oracle(multi, cols):
    """String / multi-column keys on a multi-device context: per-device pre-aggregation, groups to their hash owner,
    weighted owner tables; exported keys are rows of the caller's table (the group's smallest row)."""
    from test_distributed_gloo import mixed_table
    t = mixed_table(30_000, seed=8)
    for include_nulls in ((False, True) if len(cols) == 1 else (False,)):
        ft = engine.frequencies(t, cols, include_nulls=include_nulls)
        freq, nrows = O.frequencies(t, cols, include_nulls=include_nulls)
        exp = O.grouping_summary(freq, nrows)
        s = ft.summary(None)
        assert (s["num_rows"], s["num_groups"], s["num_unique"]) == (nrows, exp["num_groups"], exp["num_unique"])
        assert abs(s["entropy"] - exp["entropy"]) <= 1e-12 * exp["entropy"]
        got = {tuple(O._group_key(x) for x in key): c for key, c in ft.to_dict().items()}
        assert got == freq
        keys, counts = ft.export_raw()
        py = list(zip(*[t[n].to_pylist() for n in cols]))
        first = {}
        for r, row in enumerate(py):
            first.setdefault(tuple(O._group_key(x) for x in row), r)
        for r, c in zip(keys.tolist(), counts.tolist()):  # a group's key is its smallest row
            key = tuple(O._group_key(x) for x in py[r])
            assert freq[key] == c and first[key] == r
        assert [c for _, c in ft.top(7)] == sorted(freq.values(), reverse=True)[:7]


def test_sharded_mutual_information_matches_oracle(multi):
    from test_distributed_gloo import mixed_table, _oracle_mi
    t = mixed_table(30_000, seed=12)
    for cols in (["s", "k"], ["k", "d"]):
        m = D.MutualInformation(cols).calculate(t)
        assert m.value.isSuccess, m
        exp = _oracle_mi(t, cols)
        assert abs(m.value.get() - exp) <= 1e-12 * max(1.0, abs(exp)), (cols, m.value.get(), exp)


def test_scan_sharded_over_device_resident_shards():
    """dq_scan_sharded: shards already resident in HBM (here 3 shards on this one GPU) give the whole-table states."""
    import ctypes
    import torch
    os.environ.pop("DQ_DEVICES", None)
    ctx3 = N.Context(devices=[0, 0, 0])
    rng = np.random.default_rng(3)
    n = 50_000
    x = rng.normal(3.0, 2.0, n)
    k = rng.integers(-5, 5, n).astype(np.int64)
    full = Table.from_arrays({"x": x, "k": k})
    analyzers = [D.Size(), D.Mean("x"), D.StandardDeviation("x"), D.Sum("k"), D.Minimum("k"), D.ApproxCountDistinct("k"),
                 D.Correlation("x", "k")]
    batch = D.ScanBatch(full)
    offs = [a.addOps(batch) for a in analyzers]
    bounds = [0, 20_000, 20_000 + 2048 * 5, n]
    shard_tabs, arrays, rows = [], [], []
    for i in range(3):
        part = Table.from_arrays({"x": x[bounds[i]:bounds[i + 1]], "k": k[bounds[i]:bounds[i + 1]]}).to_device(0)
        shard_tabs.append(part)
        cols = (N.DqColumn * 2)(*[part[c].native() for c in ("x", "k")])
        arrays.append(cols)
        rows.append(bounds[i + 1] - bounds[i])
    ptrs = (ctypes.c_void_p * 3)(*[ctypes.cast(a, ctypes.c_void_p) for a in arrays])
    nrows = (ctypes.c_int64 * 3)(*rows)
    ops = (N.DqOp * len(batch.ops))(*batch.ops)
    preds = (N.DqPredicate * 1)()
    out = (N.DqState * len(batch.ops))()
    rc = ctx3.lib.dq_scan_sharded(ctx3.handle, ptrs, nrows, 2, ops, len(batch.ops), preds, 0, out)
    ctx3.check(rc, "dq_scan_sharded")
    res = D.runners.ScanResult([out[i] for i in range(len(batch.ops))])
    for a, o in zip(analyzers, offs):
        assert_state_parity(full, a, a.fromAggregationResult(res, o))
    ctx3.close()


def _shards(n, ndev):
    per = ((n + ndev - 1) // ndev + 2047) // 2048 * 2048
    return [(min(i * per, n), max(0, min(n, (i + 1) * per) - min(i * per, n))) for i in range(ndev)]


def _quantile_column(n, seed):
    rng = np.random.default_rng(seed)
    v = rng.normal(0.0, 10.0, n)
    r = rng.random(n)
    v[r < 0.01] = np.nan
    v[(r >= 0.01) & (r < 0.03)] = -0.0
    v[(r >= 0.03) & (r < 0.05)] = 0.0
    v[(r >= 0.05) & (r < 0.15)] = 7.25  # a heavy duplicate: answered from a splitter
    return Table.from_arrays({"v": v, "i": rng.integers(-1000, 1000, n).astype(np.int32)},
                             validity={"v": rng.random(n) > 0.05})


@pytest.mark.parametrize("rel", [0.01, 0.001, 0.0])
def test_sharded_quantile_summary_equals_one_device(multi, rel):
    """VERDICT r2 missing #3: dq_quantile_summary on a multi-device context runs the selection passes on every
    device's shard (histograms added, candidates gathered on the first device) and returns exactly the single-device
    samples: the order statistics of the whole column, for every device count."""
    n = 120_007 if rel else 20_011
    t = _quantile_column(n, 7)
    single = N.Context(0)
    for name in ("v", "i"):
        got = multi.quantile_summary(t[name].native(), n, rel)
        want = single.quantile_summary(t[name].native(), n, rel)
        assert got[2] == want[2]
        np.testing.assert_array_equal(got[1], want[1])
        assert got[0].tobytes() == want[0].tobytes(), name
    single.close()
    for q in (0.1, 0.5, 0.9):
        assert D.ApproxQuantile("v", q, 0.01).calculate(t).value.isSuccess


def test_sharded_kll_is_the_device_order_merge_of_partition_sketches(multi):
    """dq_kll_sketch on a multi-device context: one partition per device (KLLRunner.sketchPartitions), merged in
    device order (QuantileNonSample.merge + Math.max / Math.min of the extremes, R/KLLRunner.scala:40-44, 104-112):
    byte-equal to the single-device sketches of the same shards merged by the host restatement (deequ_amd/kll.py)."""
    from deequ_amd.kll import KLLState
    n = 300_007
    t = _quantile_column(n, 9)
    single = N.Context(0)
    for name, size, f in (("v", 2048, 0.64), ("i", 64, 0.5)):
        got = multi.kll_sketch(t[name].native(), n, size, f)
        acc = None
        for r0, cnt in _shards(n, multi.num_devices()):
            part = t.select_rows(np.isin(np.arange(n), np.arange(r0, r0 + cnt)))
            st = KLLState.fromBytes(single.kll_sketch(part[name].native(), cnt, size, f))
            acc = st if acc is None else acc.sum(st)
        assert got == acc.toBytes(), name
    single.close()


@pytest.mark.parametrize("to", ["long", "double"])
def test_sharded_cast_writes_host_results(multi, to):
    """dq_cast_column on a multi-device context: each device casts its shard; the host buffers equal the single-device
    cast (values where valid, the validity bitmap)."""
    from deequ_amd.table import _column_from_pylist
    rng = np.random.default_rng(3)
    n = 70_001
    words = ["12", "-7", "3.5", "abc", "", " 4", "1e3", "99999999999999999999", "0.000125", None]
    col = _column_from_pylist("s", "string", [words[j] for j in rng.integers(0, len(words), n)])
    tt = N.TYPE_LONG if to == "long" else N.TYPE_DOUBLE
    vals = np.zeros(n, dtype=np.int64 if to == "long" else np.float64)
    mask = np.zeros((n + 63) // 64 * 8, dtype=np.uint8)
    multi.cast_column(col.native(), n, tt, vals.ctypes.data, mask.ctypes.data)
    import torch
    single = N.Context(0)
    dv = torch.zeros(n, dtype=torch.int64 if to == "long" else torch.float64, device="cuda")
    dm = torch.zeros((n + 63) // 64 * 8, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    single.cast_column(col.native(), n, tt, dv.data_ptr(), dm.data_ptr())
    single.synchronize()
    want_m = dm.cpu().numpy()
    assert np.array_equal(mask, want_m)
    from deequ_amd.table import unpack_validity
    ok = unpack_validity(want_m, n)
    assert np.array_equal(vals[ok].view(np.int64), dv.cpu().numpy()[ok].view(np.int64))
    single.close()


def test_chunked_table_on_a_multi_device_context(monkeypatch):
    """a ChunkedTable under DQ_DEVICES runs its grouping, Histogram and ApproxQuantile analyzers chunk by
    chunk (the multi-device context shards every call itself and takes neither int64 string offsets nor parted
    columns) and merges the chunk states; the metrics equal the single-device run over the whole table."""
    rng = np.random.default_rng(23)
    n = 60_000
    s = [None if rng.random() < 0.05 else "w%d" % int(v) for v in rng.integers(0, 4000, n)]
    k = [int(v) for v in rng.integers(0, 300, n)]
    x = [None if rng.random() < 0.1 else float(v) for v in rng.normal(size=n)]
    data, types = {"s": s, "k": k, "x": x}, {"s": "string", "k": "long", "x": "double"}
    full = Table.from_pydict(data, types=types)
    cuts = [0, 25_000, 41_000, n]
    ct = D.ChunkedTable([Table.from_pydict({c: v[a:b] for c, v in data.items()}, types=types)
                         for a, b in zip(cuts, cuts[1:])])
    an = [D.Size(), D.Mean("x"), D.Uniqueness(["s"]), D.Entropy("k"), D.CountDistinct(["s", "k"]), D.Histogram("s"),
          D.ApproxQuantile("x", 0.5)]
    monkeypatch.delenv("DQ_DEVICES", raising=False)
    want = D.AnalysisRunner.onData(full).addAnalyzers(an).run()
    monkeypatch.setenv("DQ_DEVICES", "0,0")
    assert engine.ctx().multi
    got = D.AnalysisRunner.onData(ct).addAnalyzers(an).run()
    for a in an:
        g, w = got.metric(a).value, want.metric(a).value
        assert g.isSuccess and w.isSuccess, (a, g, w)
        if isinstance(a, D.Histogram):  # top-N details: ties broken arbitrarily (A/Histogram.scala:113-117)
            import collections
            exact = collections.Counter("NullValue" if v is None else v for v in s)
            assert g.get().numberOfBins == w.get().numberOfBins == len(exact)
            assert all(v.absolute == exact[key] for key, v in g.get().values.items())
            assert sorted(v.absolute for v in g.get().values.values()) == \
                sorted(v.absolute for v in w.get().values.values())
        elif isinstance(a, D.ApproxQuantile):  # both inside the rank bound of the same column
            vals = np.sort(np.array([v for v in x if v is not None]))
            for v in (g.get(), w.get()):
                lo, hi = O.rank_interval(vals, v)
                target = math.ceil(0.5 * len(vals))
                assert lo - math.ceil(0.01 * len(vals)) - 1 <= target <= hi + math.ceil(0.01 * len(vals)) + 1
        else:
            assert abs(g.get() - w.get()) <= 1e-12 * max(1.0, abs(w.get())), (a, g.get(), w.get())
