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
