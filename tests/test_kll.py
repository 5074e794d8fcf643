"""KLLSketch host logic and oracle (CPU): the oracle's sequential QuantileNonSample restatement against
the reference's KLL known answers (T/KLL/KLLProfileTest.scala via tests/golden/kll_kats.json), the host
state algebra (KLLState bytes, QuantileNonSample.merge / quantiles, bucket metric) against the same
answers and the oracle, and the analyzer's preconditions."""
import json
import math
import os

import numpy as np
import pytest

import deequ_amd as D
from deequ_amd.kll import QuantileNonSample, KLLState, bucket_distribution, BucketValue
from deequ_amd.table import Table
import oracle as O

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def kll_kats():
    with open(os.path.join(HERE, "golden", "kll_kats.json")) as f:
        return json.load(f)


def test_oracle_matches_reference_kll_kats(kll_kats):
    for case in kll_kats:
        size, f, nb = case["params"]
        sk = O.kll_sketch_sequential(case["values"], size, f)
        assert [c[2] for c in sk["compactors"]] == case["data"], case["name"]
        st = KLLState.fromBytes(O.kll_state_bytes(case["values"], size, f))
        bd = bucket_distribution(st, nb)
        assert bd.buckets == [BucketValue(*b) for b in case["buckets"]], case["name"]
        assert bd.parameters == case["parameters"]
        assert bd.data == case["data"]


@pytest.mark.parametrize("n,size,f", [(0, 2048, 0.64), (1, 2048, 0.64), (7, 2, 0.64), (5000, 16, 0.5),
                                      (20000, 64, 0.64), (50000, 2048, 0.64), (30000, 100, 0.9)])
def test_host_update_matches_oracle(n, size, f):
    rng = np.random.default_rng(n + size)
    v = rng.normal(size=n)
    q = QuantileNonSample(size, f)
    for x in v:
        q.update(x)
    raw = O.kll_state_bytes(v, size, f)
    assert KLLState.fromBytes(raw).qSketch.serialize() == q.serialize()
    assert KLLState.fromBytes(raw).toBytes() == raw


def test_kll_weights_and_min_max_quirk():
    # UntypedQuantileNonSample starts min/max at Int.MaxValue/Int.MinValue (R/KLLRunner.scala:27-28)
    st = KLLState.fromBytes(O.kll_state_bytes([3e9, 4e9], 2048, 0.64))
    assert st.globalMin == 2147483647.0 and st.globalMax == 4e9
    st = KLLState.fromBytes(O.kll_state_bytes([], 2048, 0.64))
    assert st.globalMin == 2147483647.0 and st.globalMax == -2147483648.0
    st = KLLState.fromBytes(O.kll_state_bytes([1.0, float("nan"), 2.0], 2048, 0.64))
    assert math.isnan(st.globalMin) and math.isnan(st.globalMax)
    v = np.random.default_rng(3).random(123457)
    sk = KLLState.fromBytes(O.kll_state_bytes(v, 256, 0.64)).qSketch
    assert sum(len(c.buffer) << i for i, c in enumerate(sk.compactors)) == len(v)


def test_merge_conserves_weight_and_capacity():
    rng = np.random.default_rng(8)
    a, b = rng.normal(size=40000), rng.normal(size=25000)
    sa = KLLState.fromBytes(O.kll_state_bytes(a, 128, 0.64))
    sb = KLLState.fromBytes(O.kll_state_bytes(b, 128, 0.64))
    m = sa.sum(sb)
    sk = m.qSketch
    assert sum(len(c.buffer) << i for i, c in enumerate(sk.compactors)) == len(a) + len(b)
    assert sk.compactorActualSize == sk.getCompactorItemsCount() < sk.compactorTotalSize
    assert m.globalMin == min(2147483647.0, a.min(), b.min()) and m.globalMax == max(a.max(), b.max())
    # merging did not mutate the inputs (the Scala merge mutates `this`; states here stay values)
    assert KLLState.fromBytes(O.kll_state_bytes(a, 128, 0.64)) == sa


@pytest.mark.parametrize("seed", range(8))
def test_library_merge_equals_the_restated_merge(seed):
    """KLLState.sum goes through the library (dq_kll_merge_states, host only): byte-equal to the Python
    QuantileNonSample.merge + condense restatement over sketches of unequal depth, NaN / +-0.0 / ties and small
    sketch sizes (many condense rounds), in both argument orders."""
    rng = np.random.default_rng(seed)
    size, f = [(2048, 0.64), (64, 0.64), (16, 0.5), (128, 0.9)][seed % 4]
    pool = np.concatenate([rng.normal(0, 10, 40), [0.0, -0.0, np.nan, np.inf, -np.inf, 1.5, 1.5]])
    na, nb = [(50_000, 3_000), (0, 7), (20_000, 20_000), (1, 1)][seed // 2 % 4]
    a = rng.choice(pool, na) if seed % 3 else rng.normal(size=na)
    b = rng.choice(pool, nb)
    sa = KLLState.fromBytes(O.kll_state_bytes(a, size, f))
    sb = KLLState.fromBytes(O.kll_state_bytes(b, size, f))
    for x, y in ((sa, sb), (sb, sa)):
        got = x.sum(y).toBytes()
        exp = KLLState.fromBytes(x.toBytes()).sum_restated(KLLState.fromBytes(y.toBytes())).toBytes()
        assert got == exp


def test_quantiles_rank_error_is_small():
    rng = np.random.default_rng(12)
    v = rng.random(200000)
    sk = KLLState.fromBytes(O.kll_state_bytes(v, 2048, 0.64)).qSketch
    qs = sk.quantiles(100)
    srt = np.sort(v)
    for i, q in enumerate(qs):
        r = np.searchsorted(srt, q) / len(v)
        assert abs(r - (i + 1) / 100) < 0.01


def test_kll_preconditions_and_metric_shape():
    t = Table.from_rows([("a", 1.0), ("b", 2.0)], ["s", "x"], ["string", "double"])
    m = D.KLLSketch("x", D.KLLParameters(2, 0.64, 101)).calculate(t)
    assert m.value.isFailure and type(m.value.failed).__name__ == "IllegalAnalyzerParameterException"
    m = D.KLLSketch("s").calculate(t)
    assert m.value.isFailure and type(m.value.failed).__name__ == "WrongColumnTypeException"
    m = D.KLLSketch("nope").calculate(t)
    assert m.value.isFailure and type(m.value.failed).__name__ == "NoSuchColumnException"
    assert repr(D.KLLSketch("x")) == "KLLSketch(x,None)"
    st = KLLState.fromBytes(O.kll_state_bytes([1.0, 2.0, 3.0, 4.0, 5.0, 6.0], 2, 0.64))
    metric = D.KLLSketch("x", D.KLLParameters(2, 0.64, 2)).computeMetricFrom(st)
    flat = metric.flatten()
    assert [d.name for d in flat] == ["KLL.buckets"] + ["KLL.low", "KLL.high", "KLL.count"] * 2
    assert flat[0].value.get() == 2.0 and flat[3].value.get() == 4.0


def _slow_quantiles(sk, q):
    """The reference's quantiles loop (A/QuantileNonSample.scala:249-281) over (item, weight) pairs."""
    import math
    out = []
    for i, c in enumerate(sk.compactors[:sk.curNumOfCompactors]):
        out.extend((v, 1 << i) for v in c.buffer)
    if not out:
        return []

    def key(v):
        if v != v:
            return (2, 0.0, 0)
        return (0, v, 0 if math.copysign(1.0, v) < 0 else 1)  # Double.compare: -0.0 < 0.0
    items = sorted(out, key=lambda p: key(p[0]))
    total = sum(w for _, w in items)
    nt, curq, i, so_far = total // q, 1, 0, 0
    res = [items[0][0]] * (q - 1)
    while i < len(items) and curq < q:
        while so_far < nt:
            so_far += items[i][1]
            i += 1
        res[curq - 1] = items[min(i, len(items) - 1)][0]
        curq += 1
        nt = curq * total // q
    return res


def _slow_rank(sk, x, exclusive):
    r = 0
    for i, c in enumerate(sk.compactors[:sk.curNumOfCompactors]):
        for v in c.buffer:
            if (v < x) if exclusive else not (v > x):
                r += 1 << i
    return r


@pytest.mark.parametrize("seed", range(6))
def test_vectorised_quantiles_and_ranks_match_the_reference_loops(seed):
    rng = np.random.default_rng(seed)
    sk = QuantileNonSample(64 if seed % 2 else 2048, 0.64)
    n = [0, 1, 3, 50, 5000, 40000][seed]
    pool = np.concatenate([rng.normal(0, 10, 50), [0.0, -0.0, np.nan, np.inf, -np.inf, 1.5, 1.5]])
    for v in rng.choice(pool, n) if n else []:
        sk.update(float(v))
    for q in (2, 7, 100, 1000):
        got, exp = sk.quantiles(q), _slow_quantiles(sk, q)
        assert len(got) == len(exp)
        assert all((a == b and math.copysign(1, a) == math.copysign(1, b)) or (a != a and b != b)
                   for a, b in zip(got, exp)), (q, got[:5], exp[:5])
    probes = [float(x) for x in pool[:20]] + [0.0, -0.0, float("nan"), float("inf"), -1e300]
    for ex in (True, False):
        got = sk.getRanks(probes, exclusive=ex)
        assert [int(g) for g in got] == [_slow_rank(sk, x, ex) for x in probes]
