"""Multi-rank runner on CPU: world_size 2 (and 3) over gloo. The per-rank compute is a CPU test double
(oracle states, numpy key partitioning) so this covers the collective choreography — state
all-gather + rank-ordered fold, hash-partitioned all-to-all of keys, global numRows / entropy — while
the GPU compute of each piece is covered by the -m gpu tests."""
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


def mix64(z):
    z = np.uint64(z)
    with np.errstate(over="ignore"):
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def canonical_keys(col):
    v = np.asarray(col.values)
    if col.spark_type == N.TYPE_DOUBLE:
        b = v.view(np.uint64).copy()
        b[np.isnan(v)] = np.uint64(0x7FF8000000000000)
        return b
    return v.astype(np.int64).view(np.uint64)


class OracleTable:
    """Stand-in for the local frequency table over owned canonical keys."""

    def __init__(self, keys):
        self.u, self.c = np.unique(np.asarray(keys, dtype=np.uint64), return_counts=True)
        self.num_rows = int(self.c.sum())

    def summary(self, n=None):
        n = n or self.num_rows
        ent = math.fsum(float(-(c / n) * math.log(c / n)) for c in self.c)
        return {"num_groups": len(self.c), "num_unique": int((self.c == 1).sum()), "entropy": ent,
                "num_rows": self.num_rows}

    def top(self, k):
        order = np.argsort(-self.c, kind="stable")[:k]
        return [((int(self.u[i].astype(np.int64)),), int(self.c[i])) for i in order]


class OracleLocal:
    def scan_states(self, batch):
        import oracle as O
        raw = bytearray()
        for op in batch.ops:
            a = op_to_analyzer(batch, op)
            st = O.expected_state(batch.data, a, exact=False)
            if st is not None:  # the oracle's own state -> the product's State of the same reference class
                st = getattr(D, type(st).__name__)(*st.key())
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

    def partition(self, column, world):
        valid = unpack_validity(column.validity, column.length)
        keys = canonical_keys(column)[valid]
        owner = np.array([int(mix64(k) >> np.uint64(32)) % world for k in keys], dtype=np.int64)
        order = np.argsort(owner, kind="stable")
        counts = [int((owner == r).sum()) for r in range(world)]
        return torch.from_numpy(keys[order].view(np.int64).copy()), counts, int((~valid).sum())

    def frequencies_of_keys(self, keys):
        return OracleTable(keys.numpy().view(np.uint64))


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


def analyzers():
    return [D.Size(), D.Completeness("x"), D.Mean("x"), D.Sum("k"), D.Minimum("y"), D.Maximum("k"),
            D.StandardDeviation("x"), D.Correlation("x", "y"), D.ApproxCountDistinct("k"),
            D.Compliance("big", "x > 5", "k < 150"), D.Mean("y", "k > 20"),
            D.Uniqueness(["k"]), D.Distinctness(["k"]), D.Entropy("k"), D.CountDistinct(["k"]),
            D.UniqueValueRatio(["k"]), D.Histogram("d", None, 10), D.Uniqueness(["d"]),
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

    def partition(self, column, world):
        if self.rank == 1:
            raise RuntimeError("partition failed")
        return super().partition(column, world)


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
                     D.Histogram("d", lambda s: s[:1])]
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
    assert hist[0] and "binningUdf" in hist[1]
