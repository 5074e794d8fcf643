"""The multi-GPU runner's GPU pieces on the one-GPU test box: world_size 2 processes sharing cuda:0
with gloo collectives (RCCL needs one GPU per rank; the 8-GPU RCCL run is the driver's bench), so
dq_scan per shard, the per-rank group tables and the weighted per-owner tables all run on the GPU."""
import math
import os
import socket

import numpy as np
import deequ_amd.native as N
import pytest
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _table(n=200_003, seed=1):
    from deequ_amd.table import Table
    rng = np.random.default_rng(seed)
    return Table.from_arrays(
        {"x": rng.normal(5.0, 2.0, n), "y": rng.normal(0.0, 1.0, n), "k": rng.integers(0, 5000, n).astype(np.int64),
         "d": (rng.integers(0, 40, n) / 4.0)},
        validity={"x": rng.random(n) > 0.1, "k": rng.random(n) > 0.05})


def _analyzers():
    import deequ_amd as D
    return [D.Size(), D.Completeness("x"), D.Mean("x"), D.Sum("k"), D.Minimum("y"), D.Maximum("k"),
            D.StandardDeviation("x"), D.Correlation("x", "y"), D.ApproxCountDistinct("k"),
            D.Compliance("big", "x > 5", "k < 150"), D.Uniqueness(["k"]), D.Distinctness(["k"]), D.Entropy("k"),
            D.CountDistinct(["k"]), D.UniqueValueRatio(["k"]), D.Histogram("d", None, 10), D.KLLSketch("x")]


def _worker(rank, world, port, q, backend="gloo"):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch
    import torch.distributed as dist
    if backend == "nccl":
        torch.cuda.set_device(0)
    dist.init_process_group(backend, rank=rank, world_size=world)
    try:
        import deequ_amd as D
        t = _table()
        n = t.nrows
        per = (n + world - 1) // world
        mask = np.zeros(n, dtype=bool)
        mask[rank * per:min(n, (rank + 1) * per)] = True
        shard = t.select_rows(mask).to_device(0)
        ctx = D.distributed.DistributedAnalysisRunner().run(shard, _analyzers())
        out = {}
        for a in _analyzers():
            m = ctx.metric(a)
            if isinstance(a, D.Histogram):
                d = m.value.get()
                out[repr(a)] = (d.numberOfBins, sorted((k, v.absolute) for k, v in d.values.items()))
            elif isinstance(a, D.KLLSketch):
                bd = m.value.get()
                out[repr(a)] = ([(b.lowValue, b.highValue, b.count) for b in bd.buckets], bd.data)
            else:
                out[repr(a)] = m.value.get()
        q.put((rank, out))
    finally:
        dist.destroy_process_group()


def test_two_ranks_on_one_gpu_match_single_gpu_run():
    import deequ_amd as D
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=100) for _ in range(2))
    for p in procs:
        p.join(timeout=30)
        assert p.exitcode == 0
    single = D.AnalysisRunner.onData(_table()).addAnalyzers(_analyzers()).run()
    for a in _analyzers():
        g = res[0][repr(a)]
        assert g == res[1][repr(a)], a
        m = single.metric(a).value.get()
        if isinstance(a, D.KLLSketch):
            # two partition sketches merged in rank order (KLLRunner's treeReduce)
            from deequ_amd.kll import bucket_distribution
            t = _table()
            per = (t.nrows + 1) // 2
            halves = []
            for r in range(2):
                mask = np.zeros(t.nrows, dtype=bool)
                mask[r * per:(r + 1) * per] = True
                halves.append(D.runners.KLLRunner.sketch_column(t.select_rows(mask), "x", 2048, 0.64))
            bd = bucket_distribution(halves[0].sum(halves[1]), 100)
            assert g[0] == [(b.lowValue, b.highValue, b.count) for b in bd.buckets] and g[1] == bd.data
            assert sum(b[2] for b in g[0]) == sum(b.count for b in m.buckets)
            continue
        if isinstance(a, D.Histogram):
            assert g[0] == m.numberOfBins
            assert sorted(c for _, c in g[1]) == sorted(v.absolute for v in m.values.values())
        elif isinstance(a, (D.Mean, D.StandardDeviation, D.Correlation, D.Entropy)):
            assert abs(g - m) <= 1e-12 * max(1.0, abs(m)), (a, g, m)
        else:
            assert g == m, (a, g, m)


def _grouping_gpu_worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import deequ_amd as D
        from test_distributed_gloo import mixed_table, grouping_analyzers
        from test_gpu_profile_c5 import c5_table
        t = mixed_table(40_000, seed=4)
        per = (t.nrows + world - 1) // world
        mask = np.zeros(t.nrows, dtype=bool)
        mask[rank * per:min(t.nrows, (rank + 1) * per)] = True
        runner = D.distributed.DistributedAnalysisRunner()
        ctx = runner.run(t.select_rows(mask), grouping_analyzers())
        out = {}
        for a in grouping_analyzers():
            v = ctx.metric(a).value
            assert v.isSuccess, (a, v)
            if isinstance(a, D.Histogram):
                d = v.get()
                out[repr(a)] = (d.numberOfBins, sorted((k, x.absolute) for k, x in d.values.items()))
            else:
                out[repr(a)] = v.get()
        c5 = c5_table(60_000)
        per = (c5.nrows + world - 1) // world
        mask = np.zeros(c5.nrows, dtype=bool)
        mask[rank * per:min(c5.nrows, (rank + 1) * per)] = True
        prof = runner.profile(c5.select_rows(mask).to_device(0))
        pr = {}
        for name, p in prof.profiles.items():
            d = {"completeness": p.completeness, "approx": p.approximateNumDistinctValues, "type": p.dataType,
                 "typeCounts": p.typeCounts,
                 "hist": None if p.histogram is None else {k: v.absolute for k, v in p.histogram.values.items()}}
            if isinstance(p, D.NumericColumnProfile):
                d.update(minimum=p.minimum, maximum=p.maximum, sum=p.sum, mean=p.mean, stdDev=p.stdDev)
            pr[name] = d
        q.put((rank, (out, pr)))
    finally:
        dist.destroy_process_group()


def test_two_ranks_string_multicolumn_grouping_mi_and_profiler_on_gpu():
    """The sharded runner's GPU pieces for VERDICT r1 item 7 (group blocks from dq_frequencies, weighted owner
    tables, dq_freq_row_counts for MutualInformation's marginals, the 3-pass profiler) — 2 ranks on one GPU over
    gloo — against the single-table oracle."""
    import oracle as O
    from test_distributed_gloo import mixed_table, grouping_analyzers, _oracle_mi
    from test_gpu_profile_c5 import c5_table
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_grouping_gpu_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=110) for _ in range(2))
    for p in procs:
        p.join(timeout=30)
        assert p.exitcode == 0
    assert res[0] == res[1]
    got, prof = res[0]
    t = mixed_table(40_000, seed=4)
    for a in grouping_analyzers():
        name = type(a).__name__
        g = got[repr(a)]
        if name == "Histogram":
            freq, n = O.frequencies(t, [a.column], include_nulls=True)
            assert g[0] == len(freq)
            assert sorted((c for _, c in g[1]), reverse=True) == sorted(freq.values(), reverse=True)[:a.maxDetailBins]
        elif name == "MutualInformation":
            exp = _oracle_mi(t, a.columns)
            assert abs(g - exp) <= 1e-12 * max(1.0, abs(exp)), (a, g, exp)
        else:
            freq, nrows = O.frequencies(t, a.columns)
            sm = O.grouping_summary(freq, nrows)
            exp = {"Uniqueness": sm["num_unique"] / nrows, "Distinctness": sm["num_groups"] / nrows,
                   "Entropy": sm["entropy"], "CountDistinct": float(sm["num_groups"]),
                   "UniqueValueRatio": sm["num_unique"] / sm["num_groups"]}[name]
            assert abs(g - exp) <= 1e-12 * max(1.0, abs(exp)), (a, g, exp)
    c5 = c5_table(60_000)
    exp = O.expected_profile(c5)
    for name, e in exp.items():
        p = prof[name]
        assert (p["completeness"], p["approx"], p["type"], p["typeCounts"]) == \
            (e["completeness"], e["approx_distinct"], e["dataType"], e["typeCounts"]), name
        if e["dataType"] in ("Integral", "Fractional"):
            st = e["numeric"]
            assert (p["minimum"], p["maximum"]) == (st["min"], st["max"]), name
            if e["dataType"] == "Integral":
                assert p["sum"] == st["sum"], name
            for key in ("mean", "stdDev"):
                assert abs(p[key] - st[key]) <= 1e-12 * abs(st[key]), (name, key, p[key], st[key])
        assert p["hist"] == e["histogram"], name


def test_row_counts_join_rows_with_their_groups():
    """dq_freq_row_counts: every row gets its group's (weighted) count; rows outside the grouping get 0."""
    from deequ_amd import engine
    from deequ_amd.table import Table, _column_from_pylist
    rng = np.random.default_rng(2)
    n = 50_000
    words = ["a", "bb", "", "ccc", None]
    s = [words[i] for i in rng.integers(0, len(words), n)]
    k = [None if rng.random() < 0.1 else int(v) for v in rng.integers(0, 50, n)]
    w = rng.integers(1, 5, n).astype(np.int64)
    t = Table([_column_from_pylist("s", "string", s), _column_from_pylist("k", N.TYPE_LONG, k)])
    for cols in (["s"], ["k"], ["s", "k"]):
        rc = engine.frequencies(t, cols, weights=w).row_counts()
        keys = list(zip(*[t[c].to_pylist() for c in cols]))
        tot = {}
        for key, x in zip(keys, w.tolist()):
            tot[key] = tot.get(key, 0) + x
        want = [0 if all(v is None for v in key) else tot[key] for key in keys]
        assert rc.tolist() == want, cols


def test_rccl_backend_one_rank_matches_single_gpu_run():
    """The RCCL (nccl) backend's collectives with device tensors -- all_gather_into_tensor of the scan states, the
    device (key, count) pairs through all_to_all_single, the all-gathered KLL / digest / group blobs -- on a real
    communicator (world size 1: RCCL needs one GPU per rank, and this box has one). Before r06 every GPU test of the
    sharded runner used gloo; the metrics equal the single-GPU run."""
    import deequ_amd as D
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_worker, args=(0, 1, port, q, "nccl"))
    p.start()
    rank, got = q.get(timeout=200)
    p.join(timeout=60)
    assert p.exitcode == 0
    single = D.AnalysisRunner.onData(_table()).addAnalyzers(_analyzers()).run()
    for a in _analyzers():
        g, m = got[repr(a)], single.metric(a).value.get()
        if isinstance(a, D.KLLSketch):
            assert g[0] == [(b.lowValue, b.highValue, b.count) for b in m.buckets] and g[1] == m.data
        elif isinstance(a, D.Histogram):
            assert g[0] == m.numberOfBins
            assert sorted(c for _, c in g[1]) == sorted(v.absolute for v in m.values.values())
        elif isinstance(a, (D.Mean, D.StandardDeviation, D.Correlation, D.Entropy)):
            assert abs(g - m) <= 1e-12 * max(1.0, abs(m)), (a, g, m)
        else:
            assert g == m, (a, g, m)
