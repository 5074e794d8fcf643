"""The simple-predicate kernel (pred_simple_kernel: leaves `column <op> constant` / `column IS [NOT] NULL` / IN lists,
combined by AND / OR / NOT on a per-lane bit stack) against the general predicate VM (DQ_PRED_VM=1, same process)
and the oracle: `where` filters and non-fused Compliance predicates over every fixed-width numeric type with NULLs,
NaN, +-inf, -0.0, and SQL three-valued logic."""
import os

import numpy as np
import pytest

import deequ_amd as D
import deequ_amd.native as N
from deequ_amd.table import Column, Table, pack_validity

from test_gpu_scan import assert_state_parity

pytestmark = pytest.mark.gpu


def typed_table(n, seed):
    rng = np.random.default_rng(seed)
    d = rng.normal(0.0, 3.0, n)
    r = rng.random(n)
    d[r < 0.01] = np.nan
    d[(r >= 0.01) & (r < 0.015)] = np.inf
    d[(r >= 0.015) & (r < 0.02)] = -np.inf
    d[(r >= 0.02) & (r < 0.05)] = -0.0
    d[(r >= 0.05) & (r < 0.08)] = 0.0
    cols = [
        ("d", N.TYPE_DOUBLE, d),
        ("f", N.TYPE_FLOAT, d.astype(np.float32)),
        ("l", N.TYPE_LONG, rng.integers(-5, 6, n).astype(np.int64)),
        ("i", N.TYPE_INT, rng.integers(-2 ** 31, 2 ** 31, n).astype(np.int32)),
        ("s", N.TYPE_SHORT, rng.integers(-3, 4, n).astype(np.int16)),
        ("b", N.TYPE_BYTE, rng.integers(-128, 128, n).astype(np.int8)),
        ("z", N.TYPE_BOOLEAN, (rng.random(n) < 0.4).astype(np.uint8)),
    ]
    out = []
    for j, (name, ty, v) in enumerate(cols):
        valid = rng.random(n) >= (0.1 if j % 2 == 0 else 0.0)
        out.append(Column(name, ty, np.ascontiguousarray(v), pack_validity(valid)))
    return Table(out)


PREDICATES = [
    "d > 0", "0 < d", "d = 0", "d != 0", "d <= 2.5", "d >= -1", "f < 0.5", "f = 0",
    "l >= 0", "l < 3", "3 > l", "l = 2", "l != 2", "l > 1.5", "i > 0", "s <= 0", "b < -100", "z = true", "z != 1",
    "l IN (1, 2, 3)", "d IN (0.0, 1.5)", "d IS NULL", "d IS NOT NULL", "l IS NULL",
    "NOT (d > 1)", "NOT d > 1 AND l < 0", "d > 1 AND l < 0", "d > 1 OR l IS NULL", "(l = 1 OR l = 2) AND NOT d < 0",
    "d > 0 OR f > 0 OR l > 0 OR i > 0", "NOT (d > 0 AND d < 1) OR l IN (4, 5)",
]


def analyzers_for(pred):
    return [D.Size(pred), D.Completeness("l", pred), D.Mean("d", pred), D.Sum("l", pred),
            D.Compliance("c", "(%s) OR l = 99" % pred)]


def _run(t, analyzers, vm):
    old = os.environ.get("DQ_PRED_VM")
    os.environ["DQ_PRED_VM"] = "1" if vm else "0"
    try:
        batch = D.ScanBatch(t)
        offsets = [a.addOps(batch) for a in analyzers]
        states = batch.run()
        return [a.fromAggregationResult(states, o) for a, o in zip(analyzers, offsets)]
    finally:
        if old is None:
            del os.environ["DQ_PRED_VM"]
        else:
            os.environ["DQ_PRED_VM"] = old


def _key(s):
    return None if s is None else repr(s)


def _same(a, x, y):
    """Fast path vs VM: bit-exact, except fp64 sums of a DOUBLE column (MeanState.sum_), whose summation order
    follows the kernel shape that ran (a `where` produced by the filter column's own scan folds in another order
    than the VM's bitmaps) -- those within the north star's 1e-12 relative bar."""
    if isinstance(a, D.Mean) and x is not None and y is not None:
        if x.count != y.count:
            return False
        if x.sum_ == y.sum_ or (x.sum_ != x.sum_ and y.sum_ != y.sum_):
            return True
        return abs(x.sum_ - y.sum_) <= 1e-12 * abs(y.sum_)
    return _key(x) == _key(y)


@pytest.mark.parametrize("n", [1, 130, 70001])
def test_simple_predicates_match_vm_and_oracle(n):
    t = typed_table(n, n)
    for pred in PREDICATES:
        an = analyzers_for(pred)
        fast = _run(t, an, vm=False)
        vm = _run(t, an, vm=True)
        for a, x, y in zip(an, fast, vm):
            assert _same(a, x, y), (pred, a, x, y)
            assert_state_parity(t, a, x)


def test_simple_predicate_rate_1e8():
    """1e8 rows: the simple kernel equals the VM on a compound `where` (the VM is the slow reference here)."""
    n = 100_000_000
    rng = np.random.default_rng(5)
    v = rng.integers(-1000, 1000, n).astype(np.int64)
    t = Table([Column("l", N.TYPE_LONG, v, pack_validity(rng.random(n) >= 0.01))]).to_device()
    an = [D.Size("l < 0 OR l IN (5, 7)"), D.Sum("l", "l > 10 AND NOT l >= 500")]
    fast = _run(t, an, vm=False)
    vm = _run(t, an, vm=True)
    assert [_key(x) for x in fast] == [_key(y) for y in vm]
