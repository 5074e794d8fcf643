"""GPU parity of the BASELINE.json configurations at their own workload sizes:

  C2 + the north-star suite10   1e9 rows x 8 generated columns (c0, c1 dyadic; c2 U[0,1); c3 N(100, 15^2);
                                c4..c7 int64 U[-2^31, 2^31); 1 % nulls): Size + {Completeness, Mean, Sum,
                                Minimum, Maximum, StandardDeviation, Compliance(c > 0), ApproxCountDistinct}
                                per column + Correlation(c_2k, c_2k+1)
  C3                            1e9 rows: k = splitmix64 mod 2^30 (HLL), x ~ N(0, 1), y = 0.6 x + 0.8 e
                                (rho ~ 0.6), 1 % nulls; also row-sharded into 8 contiguous shards scanned
                                one by one and folded in rank order (the multi-GPU merge), which must give
                                the unsharded states

The columns are generated in HBM by dq_synth_column / dq_synth_validity; the oracle
(oracle/dq_oracle.c oracle_generated_suite) regenerates them row by row on the host and computes
every state exactly. Bars (BASELINE.json north_star):
  * bit-exact: counts, Long sums, min / max, Compliance counts, HLL registers, and the fp64 sums of the
    dyadic columns (their exact sum is representable);
  * within 1e-12: fp64 sums of the other columns (relative); moments and co-moments — m2 / xMk / yMk
    relative, the averages relative to max(|avg|, standard deviation) and ck relative to
    sqrt(xMk * yMk) (a mean or co-moment that is ~0 cannot carry a relative bound; these scales make
    the StandardDeviation and Correlation METRICS agree to 1e-12).
DQ_CONFIG_ROWS overrides the row count (default 1e9).
"""
import math
import os

import numpy as np
import pytest

import deequ_amd as D
import deequ_amd.native as N
from deequ_amd import engine
from deequ_amd.table import Table, Column
import oracle as O

pytestmark = pytest.mark.gpu

ROWS = int(float(os.environ.get("DQ_CONFIG_ROWS", "1e9")))
REL = 1e-12
C2_SEED = 0x5EED0000
C2_KINDS = [1, 1, 2, 3, 4, 4, 4, 4]


def _device_table(specs, rows, row0=0):
    import torch
    ctx = engine.ctx()
    cols = []
    for sp in specs:
        dt = torch.float64 if sp["spark_type"] == N.TYPE_DOUBLE else torch.int64
        v = torch.empty(max(rows, 1), dtype=dt, device="cuda")
        ctx.synth_column(sp["kind"], sp["seed"], row0, rows, v.data_ptr())
        c = Column(sp["name"], sp["spark_type"], None, None, length=rows)
        c.device = {"values": v}
        if sp.get("permille", -1) >= 0:
            m = torch.zeros(max((rows + 63) // 64 * 8, 8), dtype=torch.uint8, device="cuda")
            ctx.synth_validity(sp["vseed"], row0, rows, sp["permille"], m.data_ptr())
            c.device["validity"] = m
        cols.append(c)
    ctx.synchronize()
    torch.cuda.synchronize()
    return Table(cols)


def _states(table, analyzers):
    batch = D.ScanBatch(table)
    offsets = [a.addOps(batch) for a in analyzers]
    res = batch.run()
    return {a: a.fromAggregationResult(res, o) for a, o in zip(analyzers, offsets)}


def _rel(got, exp, scale=None, tol=REL):
    s = abs(exp) if scale is None else scale
    return got == exp or abs(got - exp) <= tol * s


def _check_column(st, name, sp, o, rows):
    dbl = sp["spark_type"] == N.TYPE_DOUBLE
    exact_sum = sp["kind"] == 1 or not dbl  # dyadic doubles and Long sums are exact
    exp_sum = o["ex_sum"] if dbl else float(o["isum"])
    comp = st[D.Completeness(name)]
    assert (comp.numMatches, comp.count) == (o["n"], rows), name
    mean = st[D.Mean(name)]
    assert mean.count == o["n"], name
    assert (mean.sum_ == exp_sum) if exact_sum else _rel(mean.sum_, exp_sum), (name, mean.sum_, exp_sum)
    s = st[D.Sum(name)].sum_
    assert (s == exp_sum) if exact_sum else _rel(s, exp_sum), (name, s, exp_sum)
    mn, mx = st[D.Minimum(name)].minValue, st[D.Maximum(name)].maxValue
    assert mn == (o["dmin"] if dbl else float(o["imin"])), (name, mn)
    assert mx == (o["dmax"] if dbl else float(o["imax"])), (name, mx)
    sd = st[D.StandardDeviation(name)]
    sigma = math.sqrt(o["ex_m2"] / o["n"])
    assert sd.n == o["n"], name
    assert _rel(sd.avg, o["ex_mean"], max(abs(o["ex_mean"]), sigma)), (name, sd.avg, o["ex_mean"])
    assert _rel(sd.m2, o["ex_m2"]), (name, sd.m2, o["ex_m2"], (sd.m2 - o["ex_m2"]) / o["ex_m2"])
    comp = st[D.Compliance("pos_" + name, "%s > 0" % name)]
    assert (comp.numMatches, comp.count) == (o["pred_true"], rows), name
    assert st[D.ApproxCountDistinct(name)].words == o["words"], name


def _check_corr(state, o, name):
    assert state.n == o["n"], name
    sx, sy = math.sqrt(o["x_mk"] / o["n"]), math.sqrt(o["y_mk"] / o["n"])
    assert _rel(state.xAvg, o["x_avg"], max(abs(o["x_avg"]), sx)), (name, state.xAvg, o["x_avg"])
    assert _rel(state.yAvg, o["y_avg"], max(abs(o["y_avg"]), sy)), (name, state.yAvg, o["y_avg"])
    assert _rel(state.ck, o["ck"], math.sqrt(o["x_mk"] * o["y_mk"])), (name, state.ck, o["ck"])
    assert _rel(state.xMk, o["x_mk"]), (name, state.xMk, o["x_mk"])
    assert _rel(state.yMk, o["y_mk"]), (name, state.yMk, o["y_mk"])
    exp_corr = o["ck"] / math.sqrt(o["x_mk"] * o["y_mk"])
    assert abs(state.metricValue() - exp_corr) <= REL, (name, state.metricValue(), exp_corr)


def c2_specs():
    specs = []
    for c, kind in enumerate(C2_KINDS):
        specs.append(dict(name="c%d" % c, kind=kind, spark_type=N.TYPE_DOUBLE if kind in (1, 2, 3) else N.TYPE_LONG,
                          seed=C2_SEED + c, vseed=C2_SEED + 0x100 + c, permille=10, hll=1, pred_gt0=1))
    return specs


def suite10(names):
    out = [D.Size()]
    for c in names:
        out += [D.Completeness(c), D.Mean(c), D.Sum(c), D.Minimum(c), D.Maximum(c), D.StandardDeviation(c)]
    out += [D.Compliance("pos_%s" % c, "%s > 0" % c) for c in names]
    out += [D.ApproxCountDistinct(c) for c in names]
    out += [D.Correlation(names[2 * i], names[2 * i + 1]) for i in range(len(names) // 2)]
    return out


def test_c2_suite10_parity_at_scale():
    specs = c2_specs()
    names = [s["name"] for s in specs]
    table = _device_table(specs, ROWS)
    analyzers = suite10(names)
    st = _states(table, analyzers)
    del table
    pairs = [(2 * i, 2 * i + 1) for i in range(4)]
    cols, corrs = O.generated_suite(specs, 0, ROWS, pairs)
    assert st[D.Size()].numMatches == ROWS
    for sp, o in zip(specs, cols):
        _check_column(st, sp["name"], sp, o, ROWS)
    for (x, y), o in zip(pairs, corrs):
        _check_corr(st[D.Correlation(names[x], names[y])], o, (names[x], names[y]))


def c2_ops(names, where=None):
    """BASELINE C2's 49 ops (bench.py c2_analyzers), optionally all under one `where`."""
    out = [D.Size(where)]
    for c in names:
        out += [D.Completeness(c, where), D.Mean(c, where), D.Sum(c, where), D.Minimum(c, where),
                D.Maximum(c, where), D.StandardDeviation(c, where)]
    return out


def _check_c2_column(st, name, sp, o, count, where=None):
    """Bars of BASELINE.json north_star: bit-exact counts, Long sums, min / max and dyadic double sums; 1e-12 for the
    other double sums and the moments (mean against max(|mean|, sigma))."""
    dbl = sp["spark_type"] == N.TYPE_DOUBLE
    exact_sum = sp["kind"] == 1 or not dbl
    exp_sum = o["ex_sum"] if dbl else float(o["isum"])
    comp = st[D.Completeness(name, where)]
    assert (comp.numMatches, comp.count) == (o["n"], count), name
    mean = st[D.Mean(name, where)]
    assert mean.count == o["n"], name
    assert (mean.sum_ == exp_sum) if exact_sum else _rel(mean.sum_, exp_sum), (name, mean.sum_, exp_sum)
    s = st[D.Sum(name, where)].sum_
    assert (s == exp_sum) if exact_sum else _rel(s, exp_sum), (name, s, exp_sum)
    assert st[D.Minimum(name, where)].minValue == (o["dmin"] if dbl else float(o["imin"])), name
    assert st[D.Maximum(name, where)].maxValue == (o["dmax"] if dbl else float(o["imax"])), name
    sd = st[D.StandardDeviation(name, where)]
    sigma = math.sqrt(o["ex_m2"] / o["n"])
    assert sd.n == o["n"], name
    assert _rel(sd.avg, o["ex_mean"], max(abs(o["ex_mean"]), sigma)), (name, sd.avg, o["ex_mean"])
    assert _rel(sd.m2, o["ex_m2"]), (name, sd.m2, o["ex_m2"], (sd.m2 - o["ex_m2"]) / o["ex_m2"])
    # the reference's own arithmetic order (64 sequential partitions merged in order) against the same exact value
    return {"col": name, "gpu_m2_rel": (sd.m2 - o["ex_m2"]) / o["ex_m2"],
            "spark_m2_rel": (o["sp_m2"] - o["ex_m2"]) / o["ex_m2"],
            "gpu_mean_err": (sd.avg - o["ex_mean"]) / max(abs(o["ex_mean"]), sigma),
            "spark_mean_err": (o["sp_mean"] - o["ex_mean"]) / max(abs(o["ex_mean"]), sigma),
            "gpu_sum_rel": (s - exp_sum) / abs(exp_sum) if exp_sum else 0.0,
            "spark_sum_rel": (o["sp_sum"] - exp_sum) / abs(exp_sum) if exp_sum else 0.0}


def _launch_delta(before):
    after = engine.ctx().kernel_launches()
    return {k: after[k] - before[k] for k in after if after[k] != before[k]}


def _report(tag, rows):
    print("\n%s: relative error vs the exact oracle (GPU | Spark-order restatement)" % tag)
    for r in rows:
        print("  %-3s m2 %+.2e | %+.2e   mean %+.2e | %+.2e   sum %+.2e | %+.2e" % (
            r["col"], r["gpu_m2_rel"], r["spark_m2_rel"], r["gpu_mean_err"], r["spark_mean_err"], r["gpu_sum_rel"],
            r["spark_sum_rel"]))


def test_c2_headline_shape_parity_at_scale():
    """the exact 49-op C2 list bench.py times (no HLL / compare, so every column runs on the striped
    scan_values_kernel: one launch for the 4 fp64 slots, one for the 4 int64 slots) over the 1e9-row generator, against
    the exact streamed oracle; the launch counters prove which kernel evaluated it."""
    specs = c2_specs()
    names = [s["name"] for s in specs]
    table = _device_table(specs, ROWS)
    before = engine.ctx().kernel_launches()
    st = _states(table, c2_ops(names))
    assert _launch_delta(before) == {"striped": 2}
    del table
    cols, _ = O.generated_suite(specs, 0, ROWS)
    assert st[D.Size()].numMatches == ROWS
    _report("C2 %d rows" % ROWS, [_check_c2_column(st, sp["name"], sp, o, ROWS) for sp, o in zip(specs, cols)])


WHERE_ROWS = int(float(os.environ.get("DQ_WHERE_ROWS", "2e8")))


def test_c2_under_where_parity_at_scale():
    """The C2 suite with every analyzer under `where c4 < 0` (conditionalSelection / conditionalCount,
    A/Analyzer.scala:409-432; c4 is int64 with 1 % nulls, so the filter is NULL on those rows) against the oracle's
    where-aware generated suite: Size(where) = rows with c4 < 0, every Completeness count the same, every aggregate over
    the selected rows only."""
    specs = c2_specs()
    names = [s["name"] for s in specs]
    w = "c4 < 0"
    table = _device_table(specs, WHERE_ROWS)
    before = engine.ctx().kernel_launches()
    st = _states(table, c2_ops(names, w))
    launches = _launch_delta(before)
    del table
    cols, _, cnt = O.generated_suite(specs, 0, WHERE_ROWS, where=("and", [(4, "<", 0)]))
    # the shape bench.py's c2_where line times: c4's own scan evaluates the filter and writes every consumer's mask
    # (the fused producer), the other columns run the striped kernel on those masks; no predicate kernel
    assert launches == {"striped": 2, "where_fused": 1}, launches
    assert st[D.Size(w)].numMatches == cnt["where_true"]
    assert 0.45 * WHERE_ROWS < cnt["where_true"] < 0.55 * WHERE_ROWS
    _report("C2 under %s, %d rows" % (w, WHERE_ROWS),
            [_check_c2_column(st, sp["name"], sp, o, cnt["where_true"], w) for sp, o in zip(specs, cols)])


def test_compound_compliance_parity_at_scale():
    """Compliance("c4 < 0 OR c5 > 1") (A/Compliance.scala:37-53: sum(cast(pred AS int)), a NULL predicate counts 0;
    SQL OR: TRUE if either side is TRUE, NULL if neither is TRUE and one is NULL) and the same under a compound
    `where c0 > 0 AND c6 >= 0` with a Mean, at >= 1e8 rows against the oracle."""
    specs = c2_specs()
    table = _device_table(specs, WHERE_ROWS)
    comp = D.Compliance("neg_or_big", "c4 < 0 OR c5 > 1")
    w = "c0 > 0 AND c6 >= 0"
    compw = D.Compliance("neg_or_big_w", "c4 < 0 OR c5 > 1", w)
    mean_w = D.Mean("c3", w)
    before = engine.ctx().kernel_launches()
    st = _states(table, [comp, compw, mean_w, D.Size(w)])
    launches = _launch_delta(before)
    # one fused pass: the compound Compliance predicates run as simple predicates (`pred_simple`), the compound
    # `where` as consumer masks (`where_masks`), Mean(c3) on the striped kernel and Size(where) on the bitmap kernel
    assert launches == {"striped": 1, "bits": 1, "pred_simple": 1, "where_masks": 1}, launches
    del table
    pred = ("or", [(4, "<", 0), (5, ">", 1)])
    cols, _, cnt = O.generated_suite(specs, 0, WHERE_ROWS, preds=[pred])
    t, nn = cnt["preds"][0]
    assert (st[comp].numMatches, st[comp].count) == (t, WHERE_ROWS)
    assert nn < WHERE_ROWS  # rows where both sides are NULL or FALSE/NULL exist: the NULL rule is exercised
    cols, _, cntw = O.generated_suite(specs, 0, WHERE_ROWS, where=("and", [(0, ">", 0.0), (6, ">=", 0)]), preds=[pred])
    tw, _ = cntw["preds"][0]
    assert (st[compw].numMatches, st[compw].count) == (tw, cntw["where_true"])
    assert st[D.Size(w)].numMatches == cntw["where_true"]
    o = cols[3]
    assert st[mean_w].count == o["n"] and _rel(st[mean_w].sum_, o["ex_sum"]), (st[mean_w].sum_, o["ex_sum"])


def c3_specs():
    return [dict(name="k", kind=N.SYNTH_KEY30, spark_type=N.TYPE_LONG, seed=0xC3000001, vseed=0xC3000101, permille=10,
                 hll=1),
            dict(name="x", kind=N.SYNTH_GAUSS01, spark_type=N.TYPE_DOUBLE, seed=0xC3000002, vseed=0xC3000102,
                 permille=10),
            dict(name="y", kind=N.SYNTH_GAUSS_CORR, spark_type=N.TYPE_DOUBLE, seed=0xC3000002, vseed=0xC3000103,
                 permille=10)]


def test_c3_hll_and_correlation_at_scale_sharded():
    specs = c3_specs()
    analyzers = [D.ApproxCountDistinct("k"), D.Correlation("x", "y"), D.Completeness("k")]
    table = _device_table(specs, ROWS)
    full = _states(table, analyzers)
    del table
    cols, corrs = O.generated_suite(specs, 0, ROWS, [(1, 2)])
    assert full[analyzers[0]].words == cols[0]["words"]
    _check_corr(full[analyzers[1]], corrs[0], "C3")
    assert 0.55 < full[analyzers[1]].metricValue() < 0.65
    assert full[analyzers[2]].numMatches == cols[0]["n"]
    # 8 contiguous 2048-aligned row shards (the 8-GPU layout of bench.py / distributed.py), each scanned
    # on its own, states folded in rank order with the reference merges (dq_state_fold)
    G = 8
    per = ((ROWS + G - 1) // G + 2047) // 2048 * 2048
    parts, offs = [], None
    for r in range(G):
        row0 = min(r * per, ROWS)
        n = max(0, min(ROWS, row0 + per) - row0)
        shard = _device_table(specs, n, row0)
        batch = D.ScanBatch(shard)
        offs = [a.addOps(batch) for a in analyzers]
        res = batch.run()
        parts.append(b"".join(bytes(s) for s in res))
        del shard
    nops = len(parts[0]) // N.STATE_SIZE
    folded = D.runners.ScanResult(N.fold_states(np.frombuffer(b"".join(parts), dtype=np.uint8), G, nops))
    sh = {a: a.fromAggregationResult(folded, o) for a, o in zip(analyzers, offs)}
    assert sh[analyzers[0]].words == cols[0]["words"]
    _check_corr(sh[analyzers[1]], corrs[0], "C3 sharded")
    assert (sh[analyzers[2]].numMatches, sh[analyzers[2]].count) == (cols[0]["n"], ROWS)


def test_c4_full_scale_closed_forms_histogram_and_null_variant(monkeypatch):
    """BASELINE C4 at full size: 1e9 int64 keys, exactly 1e8 distinct (5e7 x 19 + 5e7 x 1).
    Closed forms exact (entropy within 1e-12 of the fsum value), Histogram with 1e8 bins whose top-1000 counts are
    all 19 (a multiset: ties), ratio = 19 / 1e9. The 1 %-null variant has no closed form: its fast build (fixed
    buckets, atomically reserved runs) must equal the exactly-counted build -- the path pinned against the oracle at
    smaller sizes -- in the summary, the top-1000 and order-free checksums of the whole export."""
    import torch
    R = ROWS
    Dn = R // 10
    ctx = engine.ctx()
    keys = torch.empty(R, dtype=torch.int64, device="cuda")
    ctx.synth_freq_keys(R, Dn, 0, R, keys.data_ptr())
    ctx.synchronize()
    col = Column("k", N.TYPE_LONG, None, None, length=R)
    col.device = {"values": keys}
    t = Table([col])
    ft = engine.frequencies(t, ["k"])
    s = ft.summary(None)
    half = Dn // 2
    big = (R - half) / half
    ent = math.fsum([-half * (big / R) * math.log(big / R), -half * (1 / R) * math.log(1 / R)])
    assert (s["num_rows"], s["num_groups"], s["num_unique"], s["max_count"]) == (R, Dn, half, int(big))
    assert abs(s["entropy"] - ent) <= 1e-12 * ent
    del ft
    h = D.Histogram("k", None, 1000).calculate(t).value.get()
    assert h.numberOfBins == Dn and len(h.values) == 1000
    assert all(v.absolute == int(big) and v.ratio == big / R for v in h.values.values())
    valid = torch.zeros((R + 63) // 64 * 8, dtype=torch.uint8, device="cuda")
    ctx.synth_validity(0x5EED0C4, 0, R, 10, valid.data_ptr())
    ctx.synchronize()
    col.device["validity"] = valid
    got = []
    for exact in (False, True):
        if exact:
            monkeypatch.setenv("DQ_FREQ_EXACT", "1")
        ft = engine.frequencies(t, ["k"])
        sm = ft.summary(None)
        k, c = ft.export_raw()
        ku = k.view(np.uint64)
        cu = c.astype(np.uint64)
        with np.errstate(over="ignore"):
            chk = (int(ku.sum(dtype=np.uint64)), int((ku * cu).sum(dtype=np.uint64)), int((ku ^ (cu << np.uint64(40))).sum(dtype=np.uint64)))
        got.append(((sm["num_rows"], sm["num_groups"], sm["num_unique"], sm["max_count"]), sm["entropy"],
                    sorted(x for _, x in ft.top(1000)), chk, int(c.sum()), len(k)))
        del ft, k, c
    monkeypatch.delenv("DQ_FREQ_EXACT")
    (a, ea, ta, ca, na, ga), (b, eb, tb, cb, nb, gb) = got
    assert a == b and ta == tb and ca == cb and na == nb == a[0] and ga == gb == a[1]
    assert abs(ea - eb) <= 1e-12 * eb
    assert 0.985 * R < a[0] < 0.995 * R  # ~1 % nulls dropped
