"""`where` filters evaluated inside the scan (WhereOut, deequ_amd/csrc/dq_internal.h; A/Analyzer.scala:409-432):
a simple filter over one 8-byte column scanned under it is evaluated by that column's own scan (scan_heavy8_kernel
with the where producer), any other simple filter by where_masks_kernel; both write one mask (valid & where TRUE)
per consumer column and count conditionalCount. Checked against the oracle over every column type, ragged tails,
NULL / NaN filters, bits and string slots that still read the filter's bitmaps, several filters in one batch, and the
fall-back to the bitmap pass; the launch counters prove which producer ran."""
import os

import numpy as np
import pytest

import deequ_amd as D
import deequ_amd.native as N
from deequ_amd import engine
from deequ_amd.table import Column, Table, pack_validity

from test_gpu_scan import all_analyzers, assert_state_parity, random_table

pytestmark = pytest.mark.gpu

# all_analyzers reads d, g and l inside Correlation pair slots: only k has a one-column 8-byte slot of its own
FUSED = ["k < 25", "NOT (k = 3) OR k IS NULL", "k IN (1, 2, 3) AND k IS NOT NULL"]
STANDALONE = ["s < 0 OR b > 10", "i > 0", "d > 40 AND k < 10", "f IS NULL", "l >= 0", "d > 40 AND d IS NOT NULL",
              "g IN (1.5, 2.5) OR g > 60"]


def _run(t, analyzers, masks=True):
    old = os.environ.get("DQ_WHERE_MASKS")
    os.environ["DQ_WHERE_MASKS"] = "1" if masks else "0"
    try:
        before = engine.ctx().kernel_launches()
        batch = D.ScanBatch(t)
        offsets = [a.addOps(batch) for a in analyzers]
        states = batch.run()
        after = engine.ctx().kernel_launches()
        return [a.fromAggregationResult(states, o) for a, o in zip(analyzers, offsets)], \
            {k: after[k] - before[k] for k in after if after[k] != before[k]}
    finally:
        if old is None:
            del os.environ["DQ_WHERE_MASKS"]
        else:
            os.environ["DQ_WHERE_MASKS"] = old


@pytest.mark.parametrize("n", [0, 1, 2047, 2049, 50001])
@pytest.mark.parametrize("where", FUSED + STANDALONE)
def test_where_masks_match_the_oracle(where, n):
    rng = np.random.default_rng(n + 3)
    t = random_table(rng, n, with_nan=True)
    analyzers = all_analyzers(t, where)
    got, launches = _run(t, analyzers)
    for a, s in zip(analyzers, got):
        assert_state_parity(t, a, s)
    if where in FUSED:
        assert launches.get("where_fused") == 1 and "where_masks" not in launches, launches
    else:
        assert launches.get("where_masks") == 1 and "where_fused" not in launches, launches
    # the bitmap pass (DQ_WHERE_MASKS=0) gives the same states for every slot the filter does not produce from
    old, old_launches = _run(t, analyzers, masks=False)
    assert "where_fused" not in old_launches and "where_masks" not in old_launches
    for a, x, y in zip(analyzers, got, old):
        if type(a).__name__ in ("Size", "Completeness", "Compliance", "ApproxCountDistinct"):
            assert repr(x) == repr(y), (where, a, x, y)


@pytest.mark.parametrize("where", ["d > 0.5 OR d = 0", "d IS NULL OR d < -1", "NOT d > 0", "d IN (0.0, 2.0)"])
def test_double_column_producer(where):
    """The filter's own DOUBLE column produces it (scan_heavy8_kernel<1, true, ...> with the where producer): NaN
    (greater than every number, equal to itself), -0.0 = 0.0, +-inf, NULLs; ragged tail."""
    n = 70001
    rng = np.random.default_rng(4)
    d = rng.normal(0.0, 2.0, n)
    r = rng.random(n)
    d[r < 0.02] = np.nan
    d[(r >= 0.02) & (r < 0.03)] = np.inf
    d[(r >= 0.03) & (r < 0.04)] = -np.inf
    d[(r >= 0.04) & (r < 0.06)] = -0.0
    d[(r >= 0.06) & (r < 0.08)] = 0.0
    t = Table([Column("d", N.TYPE_DOUBLE, d, pack_validity(rng.random(n) > 0.1)),
               Column("l", N.TYPE_LONG, rng.integers(-2 ** 40, 2 ** 40, n).astype(np.int64), None),
               Column("x", N.TYPE_DOUBLE, rng.normal(5.0, 1.0, n), pack_validity(rng.random(n) > 0.2))])
    an = [D.Size(where), D.Completeness("d", where), D.Mean("d", where), D.Maximum("d", where), D.Minimum("d", where),
          D.Sum("l", where), D.StandardDeviation("l", where), D.Mean("x", where), D.StandardDeviation("x", where),
          D.Completeness("x", where), D.Correlation("l", "x", where)]
    got, launches = _run(t, an)
    assert launches.get("where_fused") == 1, launches
    for a, s in zip(an, got):
        assert_state_parity(t, a, s)


def test_bits_and_string_slots_read_the_producers_bitmaps():
    """Completeness of a column no value slot reads, a Compliance the scan cannot fuse and MinLength / MaxLength /
    DataType over a string column, all under a filter the int64 column's scan produces: the producer also writes
    the filter's TRUE / NOT-NULL bitmaps for them."""
    n = 30011
    rng = np.random.default_rng(7)
    k = rng.integers(0, 50, n).astype(np.int64)
    words = ["", "a", "bb", "ccc", "12", "3.5", "true", "héllo"]
    strs = [words[j] for j in rng.integers(0, len(words), n)]
    t = Table([Column("k", N.TYPE_LONG, k, pack_validity(rng.random(n) > 0.1)),
               Column("u", N.TYPE_LONG, rng.integers(-9, 9, n).astype(np.int64), pack_validity(rng.random(n) > 0.3)),
               D.Table.from_pydict({"s": strs}).columns["s"]])
    w = "k < 20"
    an = [D.Size(w), D.Mean("k", w), D.Completeness("u", w), D.Compliance("cu", "u > 0 OR u IS NULL", w),
          D.MinLength("s", w), D.MaxLength("s", w), D.DataType("s", w), D.Completeness("s", w)]
    got, launches = _run(t, an)
    assert launches.get("where_fused") == 1, launches
    old, _ = _run(t, an, masks=False)
    for a, x, y in zip(an, got, old):
        assert repr(x) == repr(y) or type(a).__name__ == "Mean", (a, x, y)
    for a, s in zip(an[:4], got[:4]):
        assert_state_parity(t, a, s)


def test_several_filters_and_unfiltered_ops_in_one_scan():
    rng = np.random.default_rng(11)
    t = random_table(rng, 40009)
    an = all_analyzers(t, "k < 10") + all_analyzers(t, "d > 55") + all_analyzers(t, "s < 0 OR b > 10") + \
        all_analyzers(t)
    got, launches = _run(t, an)
    assert launches.get("where_fused") == 1 and launches.get("where_masks") == 2, launches
    for a, s in zip(an, got):
        assert_state_parity(t, a, s)


def test_more_consumers_than_masks_fall_back_to_the_bitmap_pass():
    """A filter read by more than kWhereMasks (32) columns keeps the bitmap pass (pred_simple_kernel)."""
    n = 5003
    rng = np.random.default_rng(2)
    cols = [Column("x%d" % j, N.TYPE_LONG, rng.integers(-100, 100, n).astype(np.int64),
                   pack_validity(rng.random(n) > 0.05)) for j in range(40)]
    t = Table(cols)
    w = "x0 > 0"
    an = [D.Sum("x%d" % j, w) for j in range(40)] + [D.Size(w)]
    got, launches = _run(t, an)
    assert "where_fused" not in launches and launches.get("pred_simple") == 1, launches
    for a, s in zip(an, got):
        assert_state_parity(t, a, s)


def test_all_null_filter_and_empty_selection():
    """A filter that is NULL on every row: Size(where) / Mean(where) are None (conditionalCount is a NULL sum); a
    filter that is FALSE on every row: counts 0, value states None."""
    n = 4099
    t = Table([Column("k", N.TYPE_LONG, np.arange(n, dtype=np.int64), pack_validity(np.zeros(n, dtype=bool))),
               Column("v", N.TYPE_DOUBLE, np.ones(n), None)])
    an = [D.Size("k > 0"), D.Mean("v", "k > 0"), D.Sum("k", "k > 0"), D.Completeness("v", "k > 0")]
    got, launches = _run(t, an)
    assert launches.get("where_fused") == 1, launches
    for a, s in zip(an, got):
        assert_state_parity(t, a, s)
    t2 = Table([Column("k", N.TYPE_LONG, np.arange(n, dtype=np.int64), None), Column("v", N.TYPE_DOUBLE, np.ones(n), None)])
    an2 = [D.Size("k < 0"), D.Mean("v", "k < 0"), D.Completeness("v", "k < 0")]
    got2, _ = _run(t2, an2)
    for a, s in zip(an2, got2):
        assert_state_parity(t2, a, s)
