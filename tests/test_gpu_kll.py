"""GPU parity of dq_kll_sketch (kll.hip: host count-automaton schedule + per-level LDS bitonic
compactions) against the oracle's sequential QuantileNonSample restatement (oracle.kll_state_bytes).
Bar: the KLLState bytes are identical (integer / ordering work: every compactor buffer, offset,
compression count, size field and min / max). At the bench scale (no sequential oracle in seconds),
size-independent properties: total weight = n, exact min / max, rank error of the sketch quantiles."""
import json
import math
import os

import numpy as np
import pytest

import deequ_amd as D
from deequ_amd import engine
from deequ_amd.kll import KLLState, BucketValue
from deequ_amd.native import NativeError
from deequ_amd.table import Table
import oracle as O

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def gpu_bytes(t, col, size=2048, f=0.64):
    return engine.ctx().kll_sketch(t[col].native(), t.nrows, size, f)


def non_null(x, valid):
    x = np.asarray(x)
    return x if valid is None else x[valid]


def check(x, valid=None, size=2048, f=0.64, device=False):
    t = Table.from_arrays({"x": x}, validity={"x": valid} if valid is not None else None)
    if device:
        t.to_device(0)
    got = gpu_bytes(t, "x", size, f)
    exp = O.kll_state_bytes(non_null(x, valid).astype(np.float64), size, f)
    if got != exp:
        g, e = KLLState.fromBytes(got), KLLState.fromBytes(exp)
        for h, (a, b) in enumerate(zip(g.qSketch.compactors, e.qSketch.compactors)):
            assert (a.numOfCompress, a.offset) == (b.numOfCompress, b.offset), h
            assert np.array_equal(np.array(a.buffer).view(np.uint64), np.array(b.buffer).view(np.uint64)), h
        assert (g.globalMin, g.globalMax) == (e.globalMin, e.globalMax)
        assert got == exp
    return got


def test_reference_kll_kats():
    with open(os.path.join(HERE, "golden", "kll_kats.json")) as f:
        kats = json.load(f)
    for case in kats:
        size, fac, nb = case["params"]
        vals = case["values"] + [0] * case["nulls"]
        valid = np.array([True] * len(case["values"]) + [False] * case["nulls"])
        dt = np.int16 if case["type"] == "short" else np.float64
        t = Table.from_arrays({"att1": np.array(vals, dtype=dt)}, validity={"att1": valid})
        ctx = D.AnalysisRunner.onData(t).addAnalyzer(D.KLLSketch("att1", D.KLLParameters(size, fac, nb))).run()
        bd = ctx.metric(D.KLLSketch("att1", D.KLLParameters(size, fac, nb))).value.get()
        assert bd.buckets == [BucketValue(*b) for b in case["buckets"]], case["name"]
        assert bd.parameters == case["parameters"] and bd.data == case["data"], case["name"]


@pytest.mark.parametrize("n", [0, 1, 2, 5, 2050, 2051, 3199, 100_000, 1_000_003])
def test_sketch_bytes_f64_no_nulls(n):
    x = np.random.default_rng(n).normal(size=n)
    check(x)


@pytest.mark.parametrize("size,f", [(2, 0.64), (16, 0.5), (64, 0.64), (100, 0.9), (2048, 0.64), (4096, 0.64),
                                    (5000, 0.3)])
def test_sketch_bytes_parameters(size, f):
    rng = np.random.default_rng(size)
    x = rng.normal(size=300_000)
    valid = rng.random(300_000) > 0.05
    check(x, valid, size, f)


@pytest.mark.parametrize("dtype", [np.int8, np.int16, np.int32, np.int64, np.float32])
def test_sketch_bytes_types(dtype):
    rng = np.random.default_rng(7)
    n = 200_001
    if dtype == np.float32:
        x = rng.normal(size=n).astype(np.float32)
    elif dtype == np.int64:
        x = rng.integers(-(2 ** 62), 2 ** 62, n, dtype=np.int64)  # Long.toDouble rounds
        x[:6] = [np.iinfo(np.int64).min, np.iinfo(np.int64).max, 2 ** 53 + 1, 2 ** 53, -(2 ** 53) - 1, 0]
    else:
        info = np.iinfo(dtype)
        x = rng.integers(info.min, info.max, n, dtype=dtype, endpoint=True)
    valid = rng.random(n) > 0.02
    check(x, valid)
    check(x)


def test_sketch_specials_and_device_columns():
    rng = np.random.default_rng(21)
    n = 500_000
    x = rng.integers(-3, 3, n).astype(np.float64)  # heavy duplicates
    k = rng.integers(0, n, 4000)
    x[k[:1000]] = np.nan
    x[k[1000:2000]] = -0.0
    x[k[2000:3000]] = np.inf
    x[k[3000:]] = -np.inf
    check(x)
    valid = rng.random(n) > 0.3
    check(x, valid, device=True)
    check(rng.normal(size=n), None, device=True)


@pytest.mark.parametrize("shape", ["ascending", "descending", "sawtooth", "few_values", "normal"])
@pytest.mark.parametrize("size,f", [(2048, 0.64), (64, 0.64), (16, 0.5)])
def test_sketch_run_shapes(shape, size, f, monkeypatch):
    """Compactions above level 0 merge the natural runs of their range (kll.hip kll_natural_sort, <= 4 runs) and fall
    back to the full sort beyond that: inputs whose level-0 ranges are already sorted / reversed / periodic / mostly
    ties give every run count, against the oracle; the natural path equals the full sort (DQ_KLL_NO_RUNS)."""
    n = 400_003
    rng = np.random.default_rng(len(shape) * 1000 + size)
    x = {"ascending": np.arange(n, dtype=np.float64),
         "descending": -np.arange(n, dtype=np.float64),
         "sawtooth": (np.arange(n) % 3001).astype(np.float64),
         "few_values": rng.integers(0, 4, n).astype(np.float64),
         "normal": rng.normal(size=n)}[shape]
    got = check(x, None, size, f)
    valid = rng.random(n) > 0.1
    check(x, valid, size, f, device=True)
    monkeypatch.setenv("DQ_KLL_NO_RUNS", "1")  # read at every compaction launch
    assert got == check(x, None, size, f)


@pytest.mark.parametrize("case", ["signed_zeros", "denormals", "nan_heavy", "mostly_nan", "extremes"])
def test_level0_fp64_sort_equals_the_order_key_sort(case, monkeypatch):
    """Level-0 compactions sort doubles with fp64 min / max (kll.hip kll_compact_xf_kernel) and restore Java's
    Double.compare order by position: NaN above +inf, -0.0 below +0.0. Inputs made of exactly those ties (signed zeros
    among negatives and denormals, NaN / inf heavy ranges) give the oracle's bytes and the order-key sort's
    (DQ_KLL_NO_F64=1), from host and device columns, with NULLs."""
    rng = np.random.default_rng(len(case))
    n = 300_007
    tiny = 5e-324
    if case == "signed_zeros":
        x = rng.choice(np.array([-0.0, 0.0, -1.0, 1.0, -tiny, tiny, -0.0, -0.0]), n)
    elif case == "denormals":
        x = rng.integers(-40, 40, n).astype(np.float64) * tiny
    elif case == "nan_heavy":
        x = rng.normal(size=n)
        x[rng.random(n) < 0.3] = np.nan
        x[rng.random(n) < 0.05] = np.inf
        x[rng.random(n) < 0.05] = -np.inf
    elif case == "mostly_nan":
        x = np.full(n, np.nan)
        x[rng.integers(0, n, 500)] = -0.0
        x[rng.integers(0, n, 500)] = 0.0
    else:
        x = rng.choice(np.array([np.finfo(np.float64).max, -np.finfo(np.float64).max, np.inf, -np.inf, 1e-308,
                                 -1e-308, 0.0, -0.0]), n)
    valid = rng.random(n) > 0.1
    got = check(x)
    got_v = check(x, valid, device=True)
    monkeypatch.setenv("DQ_KLL_NO_F64", "1")  # read at every compaction launch
    assert got == check(x) and got_v == check(x, valid, device=True)


def test_sketch_all_null_and_min_max_quirk():
    x = np.arange(100, dtype=np.float64)
    raw = check(x, np.zeros(100, dtype=bool))
    st = KLLState.fromBytes(raw)
    assert st.globalMin == 2147483647.0 and st.globalMax == -2147483648.0
    st = KLLState.fromBytes(check(np.array([3e9, 5e9, 4e9])))
    assert st.globalMin == 2147483647.0 and st.globalMax == 5e9


def test_sketch_too_large_parameters_fail_loudly():
    t = Table.from_arrays({"x": np.random.default_rng(1).normal(size=100_000)})
    with pytest.raises(NativeError):
        gpu_bytes(t, "x", 20000, 0.64)


def test_kll_decimal_column_fails_the_run():
    from deequ_amd.table import Column
    t = Table([Column("d", "DecimalType", np.arange(10, dtype=np.int64), decimal_precision=10, decimal_scale=2)])
    with pytest.raises(ValueError):
        D.AnalysisRunner.onData(t).addAnalyzer(D.KLLSketch("d")).run()


def test_kll_with_other_analyzers_and_state_merge():
    rng = np.random.default_rng(31)
    x = rng.normal(size=200_000)
    t = Table.from_arrays({"x": x, "y": x * 2})
    ctx = D.AnalysisRunner.onData(t).addAnalyzers([D.Size(), D.KLLSketch("x"), D.Mean("y"),
                                                   D.KLLSketch("y", D.KLLParameters(512, 0.64, 10))]).run()
    assert ctx.metric(D.Size()).value.get() == 200_000
    bx = ctx.metric(D.KLLSketch("x")).value.get()
    assert len(bx.buckets) == 100 and sum(b.count for b in bx.buckets) == 200_000
    by = ctx.metric(D.KLLSketch("y", D.KLLParameters(512, 0.64, 10))).value.get()
    assert len(by.buckets) == 10 and sum(b.count for b in by.buckets) == 200_000
    # two partitions merged on the host (KLLRunner's treeReduce) keep every item's weight
    a = KLLState.fromBytes(gpu_bytes(Table.from_arrays({"x": x[:120_000]}), "x"))
    b = KLLState.fromBytes(gpu_bytes(Table.from_arrays({"x": x[120_000:]}), "x"))
    sk = a.sum(b).qSketch
    assert sum(len(c.buffer) << i for i, c in enumerate(sk.compactors)) == 200_000


def test_sketch_large_properties():
    import torch
    n = 100_000_000
    ctx = engine.ctx()
    buf = torch.empty(n, dtype=torch.float64, device="cuda")
    ctx.synth_column(3, 0x5EED0003, 0, n, buf.data_ptr())  # N(100, 15^2), SURVEY.md §8d column c3
    from deequ_amd.table import Column
    col = Column("x", "DoubleType", None, length=n)
    col.device = {"values": buf}
    raw = engine.ctx().kll_sketch(col.native(), n, 2048, 0.64)
    st = KLLState.fromBytes(raw)
    sk = st.qSketch
    assert sum(len(c.buffer) << i for i, c in enumerate(sk.compactors)) == n
    assert st.globalMin == float(buf.min()) and st.globalMax == float(buf.max())
    srt = torch.sort(buf).values
    qs = sk.quantiles(100)
    for i in (0, 9, 49, 89, 98):
        r = int(torch.searchsorted(srt, torch.tensor([qs[i]], dtype=torch.float64, device="cuda"))) / n
        assert abs(r - (i + 1) / 100) < 0.005


@pytest.mark.parametrize("device", [False, True])
def test_kll_sketch_columns_equals_per_column_sketches(device):
    """dq_kll_sketch_columns (one call, parallel host schedules, one round trip) gives every column exactly the bytes
    of its own dq_kll_sketch, and of the oracle: six columns of different types, null shares and lengths of their
    non-NULL streams (0, a few, 1e5, 3e5 items)."""
    n = 300_001
    rng = np.random.default_rng(21)
    cols = {"d": rng.normal(100.0, 15.0, n), "f": rng.random(n).astype(np.float32),
            "l": rng.integers(-2 ** 50, 2 ** 50, n, dtype=np.int64), "i": rng.integers(-1000, 1000, n).astype(np.int32),
            "none": rng.random(n), "few": rng.random(n)}
    valid = {"d": rng.random(n) > 0.05, "f": None, "l": rng.random(n) > 0.5, "i": rng.random(n) > 0.9,
             "none": np.zeros(n, dtype=bool), "few": rng.random(n) < 3e-5}
    t = Table.from_arrays(cols, validity={k: v for k, v in valid.items() if v is not None})
    if device:
        t.to_device(0)
    names = list(cols)
    batch = engine.ctx().kll_sketch_columns([t[c].native() for c in names], t.nrows, 2048, 0.64)
    for c, raw in zip(names, batch):
        assert raw == gpu_bytes(t, c), c
        assert raw == O.kll_state_bytes(non_null(cols[c], valid[c]).astype(np.float64), 2048, 0.64), c


@pytest.mark.parametrize("null_share", [0.0, 0.05, 0.99])
def test_level0_in_place_equals_the_dense_stream(null_share, monkeypatch):
    """Level-0 compactions reading the raw column in place (the default: the range's row span located from the
    NULL-compaction tile offsets, its non-NULL values staged in dense order) instead of the written-out dense stream
    (DQ_KLL_DENSE=1): the KLLState bytes are equal for an int64 column, a float column and a double column with NULLs,
    including a 99 %-NULL column whose compactions span many staging chunks; the small case also equals the oracle."""
    rng = np.random.default_rng(int(null_share * 100) + 7)
    n = 3_000_000
    cols = {"l": rng.integers(-10 ** 9, 10 ** 9, n), "f": rng.normal(size=n).astype(np.float32),
            "d": rng.normal(size=n)}
    valid = {c: rng.random(n) >= null_share for c in cols}
    t = Table.from_arrays(cols, validity=valid)
    t.to_device(0)
    names = list(cols)
    inplace = engine.ctx().kll_sketch_columns([t[c].native() for c in names], t.nrows, 2048, 0.64)
    monkeypatch.setenv("DQ_KLL_DENSE", "1")
    dense = engine.ctx().kll_sketch_columns([t[c].native() for c in names], t.nrows, 2048, 0.64)
    monkeypatch.delenv("DQ_KLL_DENSE")
    assert inplace == dense
    small = Table.from_arrays({c: v[:200_000] for c, v in cols.items()}, validity={c: v[:200_000] for c, v in valid.items()})
    for c in names:
        got = gpu_bytes(small, c)
        exp = O.kll_state_bytes(non_null(np.asarray(cols[c][:200_000]), valid[c][:200_000]).astype(np.float64), 2048, 0.64)
        assert got == exp, c
