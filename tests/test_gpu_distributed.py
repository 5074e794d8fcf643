"""The multi-GPU runner's GPU pieces on the one-GPU test box: world_size 2 processes sharing cuda:0
with gloo collectives (RCCL needs one GPU per rank; the 8-GPU RCCL run is the driver's bench), so
dq_scan per shard, dq_partition_keys and the per-owner device tables all run on the GPU."""
import math
import os
import socket

import numpy as np
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


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
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
