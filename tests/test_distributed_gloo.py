"""Multi-rank runner on CPU: world_size 2 (and 3) over gloo. The per-rank compute is a CPU test double
(oracle states, dict-based group tables) so this covers the collective choreography — state all-gather +
rank-ordered fold, the owner shuffle of pre-aggregated groups (fixed-width, string and multi-column keys),
global numRows / entropy, the two-owner MutualInformation, the sharded ColumnProfiler — while the GPU compute
of each piece is covered by the -m gpu tests."""
import math
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import deequ_amd as D
import deequ_amd.native as N
from deequ_amd.states import state_to_native
from deequ_amd.table import Table, unpack_validity


class OracleLocal:
    def scan_states(self, batch):
        import oracle as O
        raw = bytearray()
        for op in batch.ops:
            a = op_to_analyzer(batch, op)
            st = O.expected_state(batch.data, a, exact=False)
            if st is not None:  # the oracle's own state -> the product's State of the same reference class
                st = getattr(D, type(st).__name__)(*st.key())
                col = batch.data[a.column] if op.kind in (N.OP_MEAN, N.OP_SUM) else None
                if col is not None and col.spark_type in (N.TYPE_BYTE, N.TYPE_SHORT, N.TYPE_INT, N.TYPE_LONG):
                    # the shard's exact Long partial, as the GPU scan reports it (merged with wrap-around)
                    wt, _ = O._where(batch.data, a.where)
                    vals = np.asarray(col.values).astype(np.int64)[O._valid(col) & wt]
                    with np.errstate(over="ignore"):
                        st.exact = int(vals.sum(dtype=np.int64))
            raw += bytes(state_to_native(op.kind, st))
        digests = []
        for column, rel in batch.quantile_reqs:  # the runner's digest policy over oracle order statistics
            from deequ_amd.quantiles import PercentileDigest, DEFAULT_HEAD_SIZE
            s = O.java_sorted_doubles(batch.data, column)
            if batch.data.nrows < DEFAULT_HEAD_SIZE:
                digests.append(PercentileDigest.spark_single_partition(rel, s))
            else:
                r = O.summary_ranks(len(s), rel)
                digests.append(PercentileDigest.from_order_statistics(rel, s[r - 1], r, len(s)))
        return torch.frombuffer(bytearray(raw or b"\0"), dtype=torch.uint8)[:len(raw)], digests

    def kll_state(self, shard, column, sketch_size, shrinking_factor):
        import oracle as O
        c = shard[column]
        vals = np.asarray(c.values, dtype=np.float64)[unpack_validity(c.validity, c.length)]
        return O.kll_state_bytes(vals, sketch_size, shrinking_factor)

    def cast_column(self, shard, name, to_type):
        """ColumnProfiler.castColumn with the oracle's Spark string -> long / double casts."""
        import oracle as O
        from deequ_amd.table import _column_from_pylist
        c = shard[name]
        if c.spark_type == N.TYPE_STRING:
            conv = O.spark_string_to_long if to_type == N.TYPE_LONG else O.java_parse_double
            vals = [None if v is None else conv(v) for v in c.to_pylist()]
        else:
            vals = c.to_pylist()
        return _column_from_pylist(name, to_type, vals)

    # ---- grouping: dict-based stand-ins for the per-rank frequency tables ----------------------------------
    def group_block(self, shard, cols, include_nulls):
        import oracle as O
        freq, nrows = O.frequencies(shard, cols, include_nulls=include_nulls)
        nulls = freq.pop((None,) * len(cols), 0) if include_nulls else 0
        return _block(list(freq.items()), [(c, shard[c].spark_type) for c in cols], nrows - nulls, nulls)

    def owned_table(self, block, include_nulls):
        d = {}
        for key, c in zip(block.keys(), block.counts.tolist()):
            d[key] = d.get(key, 0) + c
        return d

    def table_summary(self, table, n):
        counts = list(table.values())
        # the device summary's contract: each term rounded once to 2^-104 fixed point, the integers added
        fx = sum(N.fx_of(-(c / n) * math.log(c / n)) for c in counts) if counts and n else 0
        return {"num_groups": len(counts), "num_unique": sum(1 for c in counts if c == 1),
                "entropy": N.fx_to_float(fx), "entropy_fx": fx, "num_rows": sum(counts)}

    def top_block(self, table, block, k):
        items = sorted(table.items(), key=lambda kv: -kv[1])[:k]
        return _block(items, [(c.name, c.spark_type) for c in block.columns])

    def merged_block(self, table, block):
        return _block(list(table.items()), [(c.name, c.spark_type) for c in block.columns])

    def row_counts(self, block, cols):
        idx = [block.names.index(c) for c in cols]
        sub = [tuple(k[i] for i in idx) for k in block.keys()]
        tot = {}
        for key, c in zip(sub, block.counts.tolist()):
            tot[key] = tot.get(key, 0) + c
        return np.array([0 if all(v is None for v in key) else tot[key] for key in sub], dtype=np.int64)


def _plain(v):
    """oracle group key component -> a plain value for a column (NaN / -0.0 markers undone)."""
    if isinstance(v, tuple):
        return float("nan") if v == ("nan",) else -0.0
    return float(v) if isinstance(v, float) else v


def _block(items, schema, num_rows=0, null_rows=0):
    from deequ_amd.groups import GroupBlock
    from deequ_amd.table import _column_from_pylist
    cols = [_column_from_pylist(name, t, [_plain(k[i]) for k, _ in items]) for i, (name, t) in enumerate(schema)]
    return GroupBlock(cols, np.array([c for _, c in items], dtype=np.int64), num_rows, null_rows)


def op_to_analyzer(batch, op):
    names = batch.names
    where = None
    for text, idx in batch.pred_index.items():
        if idx == op.where:
            where = text
    c0 = names[op.column[0]] if op.column[0] >= 0 else None
    c1 = names[op.column[1]] if op.column[1] >= 0 else None
    k = op.kind
    if k == N.OP_SIZE:
        return D.Size(where)
    if k == N.OP_COMPLIANCE:
        pred = [t for t, i in batch.pred_index.items() if i == op.predicate][0]
        return D.Compliance("c", pred, where)
    if k == N.OP_CORRELATION:
        return D.Correlation(c0, c1, where)
    if k == N.OP_DATATYPE:
        return D.DataType(c0, where)
    cls = {N.OP_COMPLETENESS: D.Completeness, N.OP_MEAN: D.Mean, N.OP_SUM: D.Sum, N.OP_MINIMUM: D.Minimum,
           N.OP_MAXIMUM: D.Maximum, N.OP_STANDARD_DEVIATION: D.StandardDeviation,
           N.OP_APPROX_COUNT_DISTINCT: D.ApproxCountDistinct}[k]
    return cls(c0, where)


def full_table(n=3000, seed=0):
    rng = np.random.default_rng(seed)
    return Table.from_arrays(
        {"x": rng.normal(5.0, 2.0, n), "y": rng.normal(0.0, 1.0, n), "k": rng.integers(0, 200, n).astype(np.int64),
         "d": (rng.integers(0, 40, n) / 4.0)},
        validity={"x": rng.random(n) > 0.1, "k": rng.random(n) > 0.05})


class _BinK:
    """A binning UDF over the LONG column k (NULL rows included, as a Scala UDF over an object type sees them):
    strings, an int (cast to "1") and None (filled with "NullValue")."""

    def __call__(self, v):
        if v is None:
            return "missing"
        return "low" if v < 50 else (1 if v < 100 else None)

    def __repr__(self):
        return "binK"


BIN_K = _BinK()  # one instance per process: the analyzer's identity (Histogram equality compares the UDF object)


def analyzers():
    return [D.Size(), D.Completeness("x"), D.Mean("x"), D.Sum("k"), D.Minimum("y"), D.Maximum("k"),
            D.StandardDeviation("x"), D.Correlation("x", "y"), D.ApproxCountDistinct("k"),
            D.Compliance("big", "x > 5", "k < 150"), D.Mean("y", "k > 20"),
            D.Uniqueness(["k"]), D.Distinctness(["k"]), D.Entropy("k"), D.CountDistinct(["k"]),
            D.UniqueValueRatio(["k"]), D.Histogram("d", None, 10), D.Uniqueness(["d"]), D.Histogram("k", BIN_K, 10),
            D.ApproxQuantile("x", 0.5), D.ApproxQuantile("y", 0.9, 0.05), D.ApproxQuantiles("y", [0.1, 0.5]),
            D.KLLSketch("x", D.KLLParameters(64, 0.64, 10)), D.KLLSketch("k")]


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        t = full_table()
        n = t.nrows
        per = (n + world - 1) // world
        mask = np.zeros(n, dtype=bool)
        mask[rank * per:min(n, (rank + 1) * per)] = True
        shard = t.select_rows(mask)
        runner = D.distributed.DistributedAnalysisRunner(local=OracleLocal())
        ctx = runner.run(shard, analyzers())
        out = {}
        for a in analyzers():
            m = ctx.metric(a)
            if isinstance(a, D.Histogram):
                d = m.value.get()
                out[repr(a)] = (d.numberOfBins, sorted((k, v.absolute) for k, v in d.values.items()))
            elif isinstance(a, D.ApproxQuantiles):
                out[repr(a)] = dict(m.value.get())
            elif isinstance(a, D.KLLSketch):
                bd = m.value.get()
                out[repr(a)] = ([(b.lowValue, b.highValue, b.count) for b in bd.buckets], bd.data)
            else:
                out[repr(a)] = m.value.get()
        q.put((rank, out))
    finally:
        dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("world", [2, 3])
def test_distributed_runner_matches_single_table_oracle(world):
    import oracle as O
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = dict(q.get(timeout=240) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # every rank returns the same metrics
    for r in range(1, world):
        assert results[r].keys() == results[0].keys()
        for k in results[0]:
            a, b = results[0][k], results[r][k]
            assert a == b or (isinstance(a, float) and math.isnan(a) and math.isnan(b)), k
    got = results[0]
    t = full_table()
    for a in analyzers():
        name = type(a).__name__
        g = got[repr(a)]
        if name == "Histogram" and a.binningUdf is not None:
            # A/Histogram.scala:59-65: the UDF over every row of the whole table, its result cast to string
            bins = {}
            for (v,), c in O.frequencies(t, [a.column], include_nulls=True)[0].items():
                lab = a.binningUdf(v)
                lab = "NullValue" if lab is None else str(lab)
                bins[lab] = bins.get(lab, 0) + c
            assert g == (len(bins), sorted(bins.items())), (g, bins)
            continue
        if name == "Histogram":
            freq, _ = O.frequencies(t, [a.column], include_nulls=True)
            assert g[0] == len(freq)
            top = sorted(freq.values(), reverse=True)[:10]
            assert sorted((c for _, c in g[1]), reverse=True) == top
            continue
        if name in ("ApproxQuantile", "ApproxQuantiles"):
            # per-rank Spark digests merged in rank order: within the merged summary's rank bound
            srt = O.java_sorted_doubles(t, a.column)
            n = len(srt)
            qs = [a.quantile] if name == "ApproxQuantile" else a.quantiles
            vals = [g] if name == "ApproxQuantile" else [g[repr(q)] for q in qs]
            for q, v in zip(qs, vals):
                lo, hi = O.rank_interval(srt, v)
                slack = 2 * math.ceil(a.relativeError * n) + world
                assert lo - slack <= math.ceil(q * n) <= hi + slack, (a, q, v)
            continue
        if name in ("Uniqueness", "Distinctness", "Entropy", "CountDistinct", "UniqueValueRatio"):
            freq, nrows = O.frequencies(t, a.columns)
            s = O.grouping_summary(freq, nrows)
            exp = {"Uniqueness": s["num_unique"] / nrows, "Distinctness": s["num_groups"] / nrows,
                   "Entropy": s["entropy"], "CountDistinct": float(s["num_groups"]),
                   "UniqueValueRatio": s["num_unique"] / s["num_groups"]}[name]
            assert abs(g - exp) <= 1e-12 * max(1.0, abs(exp)), (a, g, exp)
            continue
        if name == "KLLSketch":
            # partition sketches (the sequential oracle per rank shard) merged in rank order
            from deequ_amd.kll import KLLState, bucket_distribution
            c = t[a.column]
            valid = unpack_validity(c.validity, c.length)
            per = (t.nrows + world - 1) // world
            acc = None
            for r in range(world):
                seg = np.asarray(c.values, dtype=np.float64)[r * per:(r + 1) * per][valid[r * per:(r + 1) * per]]
                st = KLLState.fromBytes(O.kll_state_bytes(seg, a.sketchSize, a.shrinkingFactor))
                acc = st if acc is None else acc.sum(st)
            bd = bucket_distribution(acc, a.numberOfBuckets)
            assert g[0] == [(b.lowValue, b.highValue, b.count) for b in bd.buckets], a
            assert g[1] == bd.data and sum(b[2] for b in g[0]) == int(valid.sum()), a
            continue
        st = O.expected_state(t, a, exact=True)
        exp = O.hll_count(st.words) if name == "ApproxCountDistinct" else st.metricValue()
        if name in ("Size", "Completeness", "Compliance", "Sum", "Maximum", "Minimum", "ApproxCountDistinct"):
            assert g == exp, (a, g, exp)
        else:
            assert abs(g - exp) <= 1e-12 * max(1.0, abs(exp)), (a, g, exp)


class FailingOnRankOne(OracleLocal):
    """Rank 1 fails locally in the scan, the KLL sketch and the key partitioning (a local failure
    must not leave the other ranks blocked in a collective)."""

    def __init__(self, rank):
        self.rank = rank

    def scan_states(self, batch):
        if self.rank == 1:
            raise RuntimeError("regex backtracking limit exceeded")
        return super().scan_states(batch)

    def kll_state(self, shard, column, sketch_size, shrinking_factor):
        if self.rank == 1:
            raise MemoryError("out of device memory")
        return super().kll_state(shard, column, sketch_size, shrinking_factor)

    def group_block(self, shard, cols, include_nulls):
        if self.rank == 1:
            raise RuntimeError("partition failed")
        return super().group_block(shard, cols, include_nulls)


def _failing_worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        t = full_table(600)
        per = (t.nrows + world - 1) // world
        mask = np.zeros(t.nrows, dtype=bool)
        mask[rank * per:min(t.nrows, (rank + 1) * per)] = True
        runner = D.distributed.DistributedAnalysisRunner(local=FailingOnRankOne(rank))
        analyzers = [D.Size(), D.Mean("x"), D.KLLSketch("x"), D.Uniqueness(["k"]),
                     D.Histogram("d", lambda v: None if v is None else str(int(v)))]
        ctx = runner.run(t.select_rows(mask), analyzers)
        out = {(repr(a) if a.__class__.__name__ != "Histogram" else "Histogram"):
               (ctx.metric(a).value.isFailure, str(ctx.metric(a).value.failed) if ctx.metric(a).value.isFailure else None)
               for a in analyzers}
        q.put((rank, out))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_one_failing_rank_fails_every_rank_without_hanging(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_failing_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = dict(q.get(timeout=180) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in range(world):
        assert results[r] == results[0]  # identical failure metrics on every rank
    got = results[0]
    assert got["Size(None)"][0] and "rank 1 failed" in got["Size(None)"][1]
    assert got["Mean(x,None)"][0]
    assert any(k.startswith("KLLSketch") and v[0] and "rank 1 failed" in v[1] for k, v in got.items())
    assert got["Uniqueness(List(k))"][0] and "rank 1 failed" in got["Uniqueness(List(k))"][1]
    hist = got["Histogram"]
    assert hist[0] and "rank 1 failed" in hist[1]


def mixed_table(n=2400, seed=3):
    from deequ_amd.table import _column_from_pylist
    rng = np.random.default_rng(seed)
    words = ["a", "b", "", "ccc", "dd", "héllo", "12", "x y"]
    s = [None if rng.random() < 0.1 else words[i] for i in rng.integers(0, len(words), n)]
    k = [None if rng.random() < 0.07 else int(v) for v in rng.integers(0, 30, n)]
    special = [float("nan"), -0.0, 0.0, 1.5]
    d = [None if rng.random() < 0.05 else (special[int(v) % 4] if v < 8 else float(v) / 4.0)
         for v in rng.integers(0, 60, n)]
    return Table([_column_from_pylist("s", "string", s), _column_from_pylist("k", N.TYPE_LONG, k),
                  _column_from_pylist("d", N.TYPE_DOUBLE, d)])


def grouping_analyzers():
    return [D.Uniqueness(["s"]), D.Uniqueness(["s", "k"]), D.Distinctness(["k", "d"]), D.CountDistinct(["s", "d"]),
            D.Entropy("s"), D.UniqueValueRatio(["s", "k", "d"]), D.Histogram("s"), D.Histogram("d", None, 5),
            D.MutualInformation(["s", "k"]), D.MutualInformation(["k", "d"])]


def _grouping_worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        t = mixed_table()
        per = (t.nrows + world - 1) // world
        mask = np.zeros(t.nrows, dtype=bool)
        mask[rank * per:min(t.nrows, (rank + 1) * per)] = True
        ctx = D.distributed.DistributedAnalysisRunner(local=OracleLocal()).run(t.select_rows(mask),
                                                                               grouping_analyzers())
        out = {}
        for a in grouping_analyzers():
            v = ctx.metric(a).value
            assert v.isSuccess, (a, v)
            if isinstance(a, D.Histogram):
                d = v.get()
                out[repr(a)] = (d.numberOfBins, sorted((k, x.absolute, x.ratio) for k, x in d.values.items()))
            else:
                out[repr(a)] = v.get()
        q.put((rank, out))
    finally:
        dist.destroy_process_group()


def _run_workers(target, world, timeout=240):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=target, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = dict(q.get(timeout=timeout) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in range(1, world):
        assert results[r] == results[0]
    return results[0]


def _oracle_mi(t, cols):
    import oracle as O
    freq, nrows = O.frequencies(t, cols)
    px, py = {}, {}
    for (u, w), c in freq.items():
        px[u] = px.get(u, 0) + c
        py[w] = py.get(w, 0) + c
    return math.fsum((c / nrows) * math.log((c / nrows) / ((px[u] / nrows) * (py[w] / nrows)))
                     for (u, w), c in freq.items() if u is not None and w is not None)


@pytest.mark.parametrize("world", [2, 3])
def test_distributed_string_and_multicolumn_grouping_and_mutual_information(world):
    """string / multi-column keys and MutualInformation over row shards equal the single-table
    oracle (A/GroupingAnalyzers.scala:53-79, A/MutualInformation.scala:35-97, A/Histogram.scala:66-96)."""
    import oracle as O
    from deequ_amd.analyzers import _hist_key
    got = _run_workers(_grouping_worker, world)
    t = mixed_table()
    for a in grouping_analyzers():
        name = type(a).__name__
        g = got[repr(a)]
        if name == "Histogram":
            freq, n = O.frequencies(t, [a.column], include_nulls=True)
            assert g[0] == len(freq)
            exp = sorted(freq.values(), reverse=True)[:a.maxDetailBins]
            assert sorted((c for _, c, _ in g[1]), reverse=True) == exp
            for key, c, ratio in g[1]:
                assert ratio == c / n
            if a.column == "s":  # every group shown: the keys themselves
                want = {(_hist_key(k[0]) if k[0] is not None else "NullValue"): c for k, c in freq.items()}
                assert {k: c for k, c, _ in g[1]} == want
            continue
        if name == "MutualInformation":
            exp = _oracle_mi(t, a.columns)
            assert abs(g - exp) <= 1e-12 * max(1.0, abs(exp)), (a, g, exp)
            continue
        freq, nrows = O.frequencies(t, a.columns)
        s = O.grouping_summary(freq, nrows)
        exp = {"Uniqueness": s["num_unique"] / nrows, "Distinctness": s["num_groups"] / nrows,
               "Entropy": s["entropy"], "CountDistinct": float(s["num_groups"]),
               "UniqueValueRatio": s["num_unique"] / s["num_groups"]}[name]
        assert abs(g - exp) <= 1e-12 * max(1.0, abs(exp)), (a, g, exp)


def test_group_block_pack_roundtrip_and_owner_hash():
    """The exchange format: pack / unpack is lossless (strings, NULLs, NaN / -0.0 bit patterns) and the owner of a
    key does not depend on which rank's block (or which position) it comes from."""
    from deequ_amd import groups as G
    t = mixed_table(500, seed=9)
    items = [((s, k, d), 1) for s, k, d in zip(t["s"].to_pylist(), t["k"].to_pylist(), t["d"].to_pylist())]
    blk = _block(items, [("s", N.TYPE_STRING), ("k", N.TYPE_LONG), ("d", N.TYPE_DOUBLE)])
    back = G.unpack(G.pack(blk), blk.schema())
    assert back.keys() == blk.keys() and back.counts.tolist() == blk.counts.tolist()
    rev = blk.subset(np.arange(blk.size)[::-1])
    o1, o2 = G.owners(blk, 5), G.owners(rev, 5)
    assert (o1 == o2[::-1]).all() and set(o1.tolist()) == set(range(5))
    assert (G.owners(blk, 3, key_columns=["k"]) == G.owners(_block([((k,), 1) for k in t["k"].to_pylist()],
                                                                    [("k", N.TYPE_LONG)]), 3)).all()
    sub = G.concat([blk.subset(np.arange(0, 200)), blk.subset(np.arange(200, blk.size))], blk.schema())
    assert sub.keys() == blk.keys()


def test_string_hashes_do_not_depend_on_the_slice_size():
    """groups.string_hashes runs its prefix sums over bounded byte slices (host memory ~24 B per key
    byte of the whole block otherwise); every slice size gives the same hashes, empty strings included."""
    from deequ_amd import groups as G
    rng = np.random.default_rng(5)
    lens = rng.integers(0, 50, 3000)
    offs = np.concatenate([[0], np.cumsum(lens)]).astype(np.int32)
    vals = rng.integers(0, 256, int(offs[-1])).astype(np.uint8)
    ref = G.string_hashes(vals, offs, slice_bytes=1 << 30)
    for sb in (1, 7, 64, 4096):
        assert np.array_equal(G.string_hashes(vals, offs, slice_bytes=sb), ref)
    same = G.string_hashes(np.frombuffer(b"abcabc", np.uint8), np.array([0, 3, 6], np.int32), slice_bytes=2)
    assert same[0] == same[1]


def test_pair_exchange_owner_balance_for_integer_valued_float_keys():
    """The device pair path routes canonical keys by (mix64(key) >> 32) % world: integer-valued DOUBLE
    keys (all-zero low bits) and FLOAT keys (zero high bits) spread over every rank like any other keys, and the
    owner equals the host group exchange's mix64 routing."""
    from deequ_amd import engine, groups as G
    from deequ_amd.distributed import owner_ranks
    for spark_type, vals in ((N.TYPE_DOUBLE, np.arange(-20000, 20000, dtype=np.float64)),
                             (N.TYPE_FLOAT, np.arange(0, 40000, dtype=np.float32)),
                             (N.TYPE_DOUBLE, np.arange(1, 40001) * 0.5),
                             (N.TYPE_LONG, np.arange(40000, dtype=np.int64) << 40)):
        keys = engine.canonical_keys(spark_type, vals)
        for world in (2, 4, 8):
            own = owner_ranks(torch, torch.from_numpy(keys.copy()), world).numpy()
            ref = (G.mix64(keys.view(np.uint64)) >> np.uint64(32)) % np.uint64(world)
            assert np.array_equal(own, ref.astype(np.int64))
            share = np.bincount(own, minlength=world) / len(keys)
            assert share.min() > 0.8 / world and share.max() < 1.2 / world, (spark_type, world, share)


def _profile_worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from test_gpu_profile_c5 import c5_table
        t = c5_table(3000)
        per = (t.nrows + world - 1) // world
        mask = np.zeros(t.nrows, dtype=bool)
        mask[rank * per:min(t.nrows, (rank + 1) * per)] = True
        prof = D.distributed.DistributedAnalysisRunner(local=OracleLocal()).profile(t.select_rows(mask))
        out = {"numRecords": prof.numRecords}
        for name, p in prof.profiles.items():
            d = {"completeness": p.completeness, "approx": p.approximateNumDistinctValues, "type": p.dataType,
                 "inferred": p.isDataTypeInferred, "typeCounts": p.typeCounts,
                 "hist": None if p.histogram is None else
                 ({k: (v.absolute, v.ratio) for k, v in p.histogram.values.items()}, p.histogram.numberOfBins)}
            if isinstance(p, D.NumericColumnProfile):
                d.update(minimum=p.minimum, maximum=p.maximum, sum=p.sum, mean=p.mean, stdDev=p.stdDev,
                         kll_n=sum(b.count for b in p.kll.buckets))
            out[name] = d
        q.put((rank, out))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_distributed_column_profiler_matches_single_table_oracle(world):
    """the 3-pass ColumnProfiler over row shards (reduced C5 table: 20 mixed columns) equals the
    oracle's restatement of the profiler on the whole table (M/profiles/ColumnProfiler.scala:91-208, 357-606)."""
    import oracle as O
    from test_gpu_profile_c5 import c5_table
    got = _run_workers(_profile_worker, world, timeout=300)
    t = c5_table(3000)
    exp = O.expected_profile(t)
    assert got["numRecords"] == t.nrows
    hist = 0
    for name, e in exp.items():
        p = got[name]
        assert (p["completeness"], p["approx"], p["type"], p["inferred"], p["typeCounts"]) == \
            (e["completeness"], e["approx_distinct"], e["dataType"], e["inferred"], e["typeCounts"]), name
        if e["dataType"] in ("Integral", "Fractional"):
            st = e["numeric"]
            assert (p["minimum"], p["maximum"]) == (st["min"], st["max"]), name
            for key in ("sum", "mean", "stdDev"):
                ok = p[key] == st[key] if (key == "sum" and e["dataType"] == "Integral") else \
                    abs(p[key] - st[key]) <= 1e-12 * max(abs(st[key]), 1e-300)
                assert ok, (name, key, p[key], st[key])
            assert p["kll_n"] == st["n"], name
        if e["histogram"] is None:
            assert p["hist"] is None, name
        else:
            hist += 1
            values, nbins = p["hist"]
            assert {k: v[0] for k, v in values.items()} == e["histogram"] and nbins == len(e["histogram"]), name
            assert all(v[1] == v[0] / t.nrows for v in values.values()), name
    assert hist >= 5
