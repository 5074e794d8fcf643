"""The lean HEAVY scan kernel for 8-byte columns (scan_heavy8_kernel, incl. its branch-free FULL variant) against the
oracle on edge data: NaN / +-inf / -0.0 / signalling-NaN bits among valid rows, NaN and inf garbage in NULL slots,
integers beyond 2^53 (exact min / max fallback), Long overflow, ragged tails, fused compares whose `0 <op> c` holds,
a NaN constant (generic compare path), and `where` filters."""
import math

import numpy as np
import pytest

import deequ_amd as D
from deequ_amd.table import Column, Table, pack_validity
import deequ_amd.native as N

from test_gpu_scan import assert_state_parity

pytestmark = pytest.mark.gpu


def edge_table(n, seed):
    rng = np.random.default_rng(seed)
    cols = []
    # doubles: normals with NaN, +-inf, -0.0, a signalling NaN bit pattern; NULL slots hold NaN / inf garbage
    for name in ("a", "b"):
        v = rng.normal(3.0, 7.0, n)
        r = rng.random(n)
        v[r < 0.004] = np.nan
        v[(r >= 0.004) & (r < 0.006)] = np.inf
        v[(r >= 0.006) & (r < 0.008)] = -np.inf
        v[(r >= 0.008) & (r < 0.02)] = -0.0
        bits = v.view(np.uint64)
        bits[(r >= 0.02) & (r < 0.021)] = np.uint64(0x7FF0000000000001)  # signalling NaN
        valid = rng.random(n) >= 0.05
        garbage = rng.random(n)
        v[~valid & (garbage < 0.5)] = np.nan
        v[~valid & (garbage >= 0.5)] = np.inf
        cols.append(Column(name, N.TYPE_DOUBLE, v, pack_validity(valid)))
    # longs: one beyond 2^53 (exact min / max fallback, Long wrap-around of the sum), one small
    big = rng.integers(-2 ** 63, 2 ** 63 - 1, n, dtype=np.int64, endpoint=True)
    big[:3] = [np.iinfo(np.int64).max, np.iinfo(np.int64).min, 2 ** 53 + 1][:min(3, n)]
    small = rng.integers(-40, 40, n).astype(np.int64)
    for name, v in (("l", big), ("k", small)):
        valid = rng.random(n) >= 0.05
        cols.append(Column(name, N.TYPE_LONG, np.ascontiguousarray(v), pack_validity(valid)))
    return Table(cols)


def full_suite(where=None):
    out = [D.Size(where)]
    for c, pred in (("a", "a > 0"), ("b", "b <= 2.5"), ("l", "l >= 0"), ("k", "k < 3")):
        out += [D.Completeness(c, where), D.Mean(c, where), D.Sum(c, where), D.Minimum(c, where),
                D.Maximum(c, where), D.StandardDeviation(c, where), D.ApproxCountDistinct(c, where),
                D.Compliance("p_" + c, pred, where)]
    out += [D.Correlation("a", "b", where), D.Correlation("l", "k", where)]
    return out


def run_parity(t, analyzers):
    batch = D.ScanBatch(t)
    offsets = [a.addOps(batch) for a in analyzers]
    states = batch.run()
    for a, ops in zip(analyzers, offsets):
        assert_state_parity(t, a, a.fromAggregationResult(states, ops))


@pytest.mark.parametrize("n", [1, 2047, 2049, 65536 + 77, 400003])
def test_full_variant_edge_data(n):
    run_parity(edge_table(n, n), full_suite())


@pytest.mark.parametrize("where", ["k < 10", "a > 1 OR l IS NULL"])
def test_heavy_with_where(where):
    run_parity(edge_table(150001, 3), full_suite(where))


def test_heavy_generic_compares():
    # zero satisfies the compare (masked rows corrected), NaN constants (generic path), integral column vs a
    # fractional constant, HLL alone on a column (values read only by the hash)
    t = edge_table(90001, 8)
    analyzers = [D.Compliance("z1", "a >= -1"), D.Compliance("z2", "k != 7"), D.Compliance("nan1", "b < 'NaN'"),
                 D.Compliance("mix", "l > 0.5"), D.ApproxCountDistinct("a"), D.ApproxCountDistinct("l"),
                 D.Completeness("a"), D.Mean("b"), D.Maximum("k"), D.ApproxCountDistinct("b")]
    try:
        run_parity(t, analyzers)
    except Exception as e:  # a predicate form the SQL subset rejects is skipped, never silently wrong
        if "parse" in str(e).lower():
            pytest.skip(str(e))
        raise


def test_full_variant_run_to_run_reproducible():
    t = edge_table(300001, 21).to_device()
    a = full_suite()
    r1 = D.AnalysisRunner.onData(t).addAnalyzers(a).run()
    r2 = D.AnalysisRunner.onData(t).addAnalyzers(a).run()
    for x in a:
        m1, m2 = r1.metric(x).value, r2.metric(x).value
        assert (m1.isSuccess == m2.isSuccess) and (not m1.isSuccess or
                                                   (math.isnan(m1.get()) and math.isnan(m2.get())) or
                                                   m1.get() == m2.get()), x


@pytest.mark.parametrize("n", [2049, 300007])
def test_striped_kernel_edge_data(n):
    """The striped kernel (no HLL / compare / correlation): integral min / max tracked as doubles with the exact
    int64 fallback for batches beyond 2^53, Long sums, NaN / inf / -0.0 rows and garbage in NULL slots."""
    t = edge_table(n, n + 5)
    analyzers = [D.Size()]
    for c in ("a", "b", "l", "k"):
        analyzers += [D.Completeness(c), D.Mean(c), D.Sum(c), D.Minimum(c), D.Maximum(c), D.StandardDeviation(c)]
    run_parity(t, analyzers)


def test_striped_moments_large_offset():
    """Shifted one-reciprocal moments on integral values 1e12 + noise in [-50, 50) (|mean| / sigma ~ 3e10): the lane's
    first batch is shifted by its own first value, later batches by the running mean. Any double accumulation of such
    data (Spark's per-row update included) carries ~ulp(1e12) / sigma relative error per value; the previous
    two-reciprocal merge measured 1.4e-9 - 4.1e-9, this one 1.0e-9 - 5.2e-9 (tools/offset_moments.py), so the bound is
    2e-8 relative on the metric (the 1e-12 state bar is for data whose offset does not dwarf the spread)."""
    n = 1_000_003
    rng = np.random.default_rng(77)
    v = (10 ** 12 + rng.integers(-50, 50, n)).astype(np.int64)
    valid = rng.random(n) >= 0.03
    t = Table([Column("o", N.TYPE_LONG, v, pack_validity(valid))])
    x = (v[valid] - 10 ** 12).astype(np.float64)
    exact = float(np.sqrt(np.mean((x - x.mean()) ** 2)))
    for extra in ([], [D.ApproxCountDistinct("o")]):  # striped kernel, heavy kernel
        a = D.StandardDeviation("o")
        r = D.AnalysisRunner.onData(t).addAnalyzers([a] + extra).run().metric(a).value.get()
        assert abs(r - exact) <= 2e-8 * exact, (extra, r, exact)
    run_parity(t, [D.Mean("o"), D.Minimum("o"), D.Maximum("o"), D.Sum("o")])
