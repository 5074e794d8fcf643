"""Benchmark: the fused analyzer suite of BASELINE config C2 on device-resident synthetic columns.

One step = one AnalysisRunner scan pass of the suite over the rank's row shard (49 ops: Size +
{Completeness, Mean, Sum, Minimum, Maximum, StandardDeviation} over 8 columns: 4 fp64 + 4 int64,
1 % nulls), the RCCL all-gather of the per-rank states (N > 1) and the rank-ordered
semigroup fold of those states on the host. BASELINE's configuration is one synthetic 1B-row table at 1/2/4/8 GPUs
(Spark partitions of one table feeding one `data.agg`, R/AnalysisRunner.scala:313), so the default is strong
scaling: the 1e9 rows are split into contiguous 2048-row-aligned shards over the N ranks and `value` = 1e9 rows /
the max-over-ranks step time (`--scaling weak` gives every rank its own --rows-row shard of an N x --rows table).
Inputs are generated in HBM by the counter-based splitmix64 generators before timing.

`--gpus N` without a launcher starts N rank processes itself (spawn_ranks); under torch.distributed.run the
ranks come from RANK / LOCAL_RANK / WORLD_SIZE. N > 1 runs on RCCL (nccl); `--dist-backend gloo
--device-override 0` rehearses N ranks on one GPU.

The same JSON line carries `secondary` measurements of the other BASELINE workloads, each timed the
same way (its own steps, HIP events on the scan stream, its own roofline):
  suite10  the north-star 10-analyzer suite over the same 8 columns (C2 ops + Compliance(c > 0) +
           ApproxCountDistinct + Correlation(c_2k, c_2k+1): 69 ops), every rank count;
  c3       ApproxCountDistinct(k) + Correlation(x, y) + Completeness(k), 1e9 rows sharded over the ranks;
  c4       the grouping analyzers' frequency table (computeFrequencies + the fused table aggregation) on
           1e9 int64 keys with exactly 1e8 distinct, closed forms checked (N = 1; N > 1: row shards, device
           (key, count) pairs exchanged by RCCL all-to-all, owner tables);
  c2_host_streamed  the C2 suite over pinned host columns streamed through HBM (dq_scan_streamed): the
           end-to-end rate including the host link, never the headline value (N = 1).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--rows R] [--scaling weak|strong] [--no-secondary]
"""
import argparse
import ctypes
import json
import math
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
os.environ.setdefault("GPU_MAX_HW_QUEUES", "8")  # before any HIP call: see deequ_amd/native.py

PEAK_HBM_GBPS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md, chip-level parameters)
SEED = 0x5EED0000
# C2 column kinds: c0, c1 dyadic (exact sums); c2 U[0,1); c3 N(100, 15^2); c4..c7 int64 U[-2^31, 2^31)
C2_KINDS = [1, 1, 2, 3, 4, 4, 4, 4]


def c2_analyzers(D, names):
    out = [D.Size()]
    for c in names:
        out += [D.Completeness(c), D.Mean(c), D.Sum(c), D.Minimum(c), D.Maximum(c), D.StandardDeviation(c)]
    return out


def suite10_analyzers(D, names):
    """The north star's 10 analyzer kinds over the C2 columns."""
    out = c2_analyzers(D, names)
    out += [D.Compliance("pos_%s" % c, "%s > 0" % c) for c in names]
    out += [D.ApproxCountDistinct(c) for c in names]
    out += [D.Correlation(names[2 * i], names[2 * i + 1]) for i in range(len(names) // 2)]
    return out


class ScanWorkload:
    """One fused dq_scan step over `table` for `analyzers` (+ the RCCL all-gather and rank-ordered fold when
    world > 1), timed with HIP events on `stream`."""

    def __init__(self, torch, N, D, ctx, table, analyzers, stream, dev, world, backend):
        import torch.distributed as dist
        self.torch, self.N, self.ctx, self.stream, self.world, self.dist = torch, N, ctx, stream, world, dist
        self.backend = backend
        self.batch = D.ScanBatch(table)
        self.offsets = [a.addOps(self.batch) for a in analyzers]
        self.nops = len(self.batch.ops)
        self.out = torch.empty(self.nops * N.STATE_SIZE, dtype=torch.uint8, device=dev)
        coll_dev = dev if backend == "nccl" else torch.device("cpu")
        self.gathered = torch.empty(world * self.nops * N.STATE_SIZE, dtype=torch.uint8, device=coll_dev)
        self.host = torch.empty(world * self.nops * N.STATE_SIZE, dtype=torch.uint8, pin_memory=True)
        self.host_np = self.host.numpy()
        self.cols = self.batch.native_columns()
        self.preds = [p.to_native() for p in self.batch.preds]
        self.nrows = table.nrows

    def step(self, ev=None):
        if ev is not None:
            ev[0].record(self.stream)
        self.ctx.scan(self.cols, self.nrows, self.batch.ops, self.preds, out_device_ptr=self.out.data_ptr())
        if ev is not None:
            ev[1].record(self.stream)
        if self.world > 1:
            src_t = self.out if self.backend == "nccl" else self.out.cpu()
            self.dist.all_gather_into_tensor(self.gathered, src_t)  # RCCL over xGMI
            src = self.gathered
        else:
            src = self.out
        self.host[:src.numel()].copy_(src, non_blocking=True)
        self.stream.synchronize()
        # rank-ordered fold with the reference semigroup merges (State.sum), one C-ABI call
        return self.N.fold_states(self.host_np, self.world, self.nops)


def timed(torch, dist, world, steps, warmup, stream, step):
    """W untimed steps, then K steps bracketed by barrier + synchronize; max wall time over ranks and the
    mean HIP-event time of the kernels each step brackets."""
    for _ in range(warmup):
        step(None)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
    t0 = time.perf_counter()
    res = None
    for i in range(steps):
        res = step(ev[i])
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda" if dist.get_backend() == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    kernel_ms = float(np.mean([a.elapsed_time(b) for a, b in ev]))
    return elapsed, kernel_ms, res


def shard_plan(rows, world, rank, scaling):
    """(total rows of the job, first row of this rank's shard, rows of the shard): strong scaling splits `rows` over
    the ranks, weak scaling gives every rank `rows` of a world x rows table; contiguous shards aligned to the
    2048-row tile."""
    if scaling == "weak":
        return int(rows) * world, rank * int(rows), int(rows)
    total = int(rows)
    per = (total + world - 1) // world
    per = (per + 2047) // 2048 * 2048
    row0 = min(rank * per, total)
    return total, row0, max(0, min(total, row0 + per) - row0)


def build_shard(torch, N, ctx, row0, nrows, dev):
    from deequ_amd.table import Table, Column
    cols = []
    for c, kind in enumerate(C2_KINDS):
        dt = torch.float64 if kind in (1, 2, 3, 6) else torch.int64
        vals = torch.empty(max(nrows, 1), dtype=dt, device=dev)
        valid = torch.zeros(max((nrows + 63) // 64 * 8, 8), dtype=torch.uint8, device=dev)
        ctx.synth_column(kind, SEED + c, row0, nrows, vals.data_ptr())
        ctx.synth_validity(SEED + 0x100 + c, row0, nrows, 10, valid.data_ptr())
        spark_type = N.TYPE_DOUBLE if dt == torch.float64 else N.TYPE_LONG
        col = Column("c%d" % c, spark_type, None, None, length=nrows)
        col.device = {"values": vals, "validity": valid}
        cols.append(col)
    ctx.synchronize()
    return Table(cols)


def bench_c3(torch, N, D, ctx, stream, dev, total, steps, dist=None, world=1, rank=0, backend="nccl"):
    """BASELINE config C3: k = splitmix64 mod 2^30 (HLL), x ~ N(0, 1), y = 0.6 x + 0.8 e, 1 % nulls, rows sharded
    contiguously over the ranks (2048-row aligned); per step the fused scan of the shard, the RCCL all-gather of the
    states and their rank-ordered fold (HLL registers max-merged, CorrelationState Chan-merged)."""
    from deequ_amd.table import Table, Column
    _, row0, nrows = shard_plan(total, world, rank, "strong")
    cols = []
    for name, kind, seed, vseed, st in (("k", N.SYNTH_KEY30, 0xC3000001, 0xC3000101, N.TYPE_LONG),
                                        ("x", N.SYNTH_GAUSS01, 0xC3000002, 0xC3000102, N.TYPE_DOUBLE),
                                        ("y", N.SYNTH_GAUSS_CORR, 0xC3000002, 0xC3000103, N.TYPE_DOUBLE)):
        v = torch.empty(max(nrows, 1), dtype=torch.int64 if st == N.TYPE_LONG else torch.float64, device=dev)
        m = torch.zeros(max((nrows + 63) // 64 * 8, 8), dtype=torch.uint8, device=dev)
        ctx.synth_column(kind, seed, row0, nrows, v.data_ptr())
        ctx.synth_validity(vseed, row0, nrows, 10, m.data_ptr())
        c = Column(name, st, None, None, length=nrows)
        c.device = {"values": v, "validity": m}
        cols.append(c)
    ctx.synchronize()
    t = Table(cols)
    w = ScanWorkload(torch, N, D, ctx, t, [D.ApproxCountDistinct("k"), D.Correlation("x", "y"), D.Completeness("k")],
                     stream, dev, world, backend)
    el, kms, _ = timed(torch, dist, world, steps, 1, stream, w.step)
    bpr = 3 * (8 + 1 / 8)
    ach = bpr * nrows / (kms * 1e-3) / 1e9
    c3_traffic = committed_json("c3_traffic_*.json", nrows, need="traffic_bytes_per_call") if world == 1 else None
    return {"workload": "C3: ApproxCountDistinct(k) + Correlation(x, y) + Completeness(k), 3 cols x %d rows, 1%% nulls, "
                        "rows sharded over %d GPU(s), states all-gathered (RCCL) and folded in rank order"
                        % (total, world),
            "value": total / (el / steps), "unit": "rows/s", "ms_per_step": el / steps * 1e3,
            "roofline": {"bound": "hbm", "achieved": ach, "peak": PEAK_HBM_GBPS, "unit": "GB/s",
                         "frac": ach / PEAK_HBM_GBPS,
                         "traffic": c3_traffic[0]["traffic_bytes_per_call"] / 1e9 if c3_traffic else None,
                         "traffic_unit": "GB per dq_scan call (rocprofv3 PMC, %s)" % (c3_traffic[1] if c3_traffic
                                                                                      else "not measured"),
                         "kernel": "dq_scan avg %.3f ms (HIP events, this rank), %.3f B/row x %d rows per GPU"
                                   % (kms, bpr, nrows)}}


def bench_c4(torch, N, D, ctx, stream, dev, total, steps):
    """BASELINE config C4 on one GPU: the frequency table of 1e9 int64 keys with exactly 1e8 distinct
    (5e7 x 19 + 5e7 x 1) and the grouping analyzers' table aggregation, closed forms checked."""
    import math
    from deequ_amd import engine
    from deequ_amd.table import Table, Column
    distinct = total // 10
    keys = torch.empty(total, dtype=torch.int64, device=dev)
    ctx.synth_freq_keys(total, distinct, 0, total, keys.data_ptr())
    ctx.synchronize()
    c = Column("k", N.TYPE_LONG, None, None, length=total)
    c.device = {"values": keys}
    t = Table([c])
    out = {}

    def step(ev):
        if ev is not None:
            ev[0].record(stream)
        ft = engine.frequencies(t, ["k"])
        s = ft.summary(None)
        if ev is not None:
            ev[1].record(stream)
        out["s"] = s
        del ft
        return s

    el, kms, _ = timed(torch, None, 1, steps, 1, stream, step)
    s = out["s"]
    half = distinct // 2
    big = (total - half) / half
    ent = math.fsum([-half * (big / total) * math.log(big / total), -half * (1 / total) * math.log(1 / total)])
    ok = (s["num_rows"], s["num_groups"], s["num_unique"]) == (total, distinct, half) and \
        abs(s["entropy"] - ent) <= 1e-12 * ent
    assert ok, (s, ent)
    bpr = 8.0
    table_bytes = 2 * 16 * distinct  # write + read of the 16-B slots of each group
    ach = (bpr * total + table_bytes) / (el / steps) / 1e9
    traffic = None
    found = committed_json("c4_traffic_*.json", total, need="traffic_bytes_per_call")
    if found:
        traffic = (found[0]["traffic_bytes_per_call"] / 1e9, found[1])
    else:  # the round-2 layout
        found = committed_json("c4_traffic_*.json", total, need="total_GB_per_call")
        if found:
            traffic = (found[0]["total_GB_per_call"], found[1])
    return {"workload": "C4: computeFrequencies + Uniqueness/Distinctness/UniqueValueRatio/CountDistinct/Entropy "
                        "aggregation, 1e9 int64 keys, 1e8 distinct; closed forms exact",
            "value": total / (el / steps), "unit": "rows/s", "ms_per_step": el / steps * 1e3,
            "roofline": {"bound": "hbm", "achieved": ach, "peak": PEAK_HBM_GBPS, "unit": "GB/s",
                         "frac": ach / PEAK_HBM_GBPS, "traffic": traffic[0] if traffic else None,
                         "traffic_unit": "GB per build (HBM FETCH+WRITE from rocprofv3 PMC, %s)"
                                         % (traffic[1] if traffic else "not measured at this size"),
                         "kernel": "end-to-end build + summary, wall clock per step (fast grouping: partition1_fast "
                                   "-> scatter2_fast -> build, DESIGN.md §3); algorithmic %.1f GB (keys read once + "
                                   "the groups' slots written and read once)" % ((bpr * total + table_bytes) / 1e9)}}


def bench_c4_dist(torch, N, D, dev, total, steps, dist, world, rank):
    """BASELINE config C4 over `world` GPUs: each rank holds a contiguous shard of the 1e9 keys (1e8 distinct) and the
    DistributedAnalysisRunner computes Uniqueness / Distinctness / UniqueValueRatio / CountDistinct / Entropy: local
    tables -> device (key, count) pairs -> RCCL all-to-all to the key's owner -> owner tables -> all-reduced summary.
    Closed forms checked on every rank."""
    import math
    from deequ_amd import engine
    from deequ_amd.distributed import DistributedAnalysisRunner
    from deequ_amd.table import Table, Column
    distinct = total // 10
    _, row0, nrows = shard_plan(total, world, rank, "strong")
    ctx = engine.ctx()
    keys = torch.empty(max(nrows, 1), dtype=torch.int64, device=dev)
    ctx.synth_freq_keys(total, distinct, row0, nrows, keys.data_ptr())
    ctx.synchronize()
    c = Column("k", N.TYPE_LONG, None, None, length=nrows)
    c.device = {"values": keys}
    t = Table([c])
    analyzers = [D.Uniqueness(["k"]), D.Distinctness(["k"]), D.UniqueValueRatio(["k"]), D.CountDistinct(["k"]),
                 D.Entropy("k")]
    runner = DistributedAnalysisRunner()
    out = {}

    stream = torch.cuda.current_stream()

    def step(ev):
        if ev is not None:
            ev[0].record(stream)
        out["r"] = runner.run(t, analyzers)
        if ev is not None:
            ev[1].record(stream)

    el, _, _ = timed(torch, dist, world, steps, 1, stream, step)
    r = out["r"]
    half = distinct // 2
    big = (total - half) / half
    ent = math.fsum([-half * (big / total) * math.log(big / total), -half * (1 / total) * math.log(1 / total)])
    got = [r.metric(a).value.get() for a in analyzers]
    exp = [half / total, distinct / total, half / distinct, float(distinct), ent]
    assert all(abs(g - e) <= 1e-12 * abs(e) for g, e in zip(got, exp)), (got, exp)
    bpr = 8.0
    ach = (bpr * nrows + 2 * 16 * distinct / world) / (el / steps) / 1e9
    return {"workload": "C4 over %d GPUs: DistributedAnalysisRunner grouping analyzers on 1e9 int64 keys (1e8 distinct), "
                        "device (key, count) pairs exchanged by RCCL all-to-all to their owner rank; closed forms exact"
                        % world,
            "value": total / (el / steps), "unit": "rows/s", "ms_per_step": el / steps * 1e3,
            "roofline": {"bound": "hbm", "achieved": ach, "peak": PEAK_HBM_GBPS, "unit": "GB/s",
                         "frac": ach / PEAK_HBM_GBPS, "traffic": None,
                         "kernel": "end-to-end step per rank (local build + exchange + owner build + summary)"}}


C5_NUMERIC = [("d_dyad", 1), ("d_unif", 2), ("d_n100", 3), ("d_gauss", 6), ("d_corr", 7),
              ("l_i32a", 4), ("l_key30a", 5), ("l_i32b", 4), ("l_key30b", 5), ("l_i32c", 4)]
C5_STRINGS = [("s_cat50", 101), ("s_bool", 102), ("s_cat100", 103), ("s_int", 104), ("s_dec", 105), ("s_mixnum", 106),
              ("s_text0", 107), ("s_text1", 107), ("s_text2", 107), ("s_text3", 107)]


def c5_shard(torch, N, ctx, dev, rows, chunk_rows=125_000_000, only=None):
    """One GPU's shard of BASELINE config C5 generated in HBM: 5 fp64 + 5 int64 columns (the C2 generators) and 10
    UTF-8 string columns (3 low-cardinality, 3 numeric-looking, 4 free text 1-20 characters), 5 % nulls each. A
    shard above `chunk_rows` rows is held as row chunks (ChunkedTable): one string column's bytes of the 2.5e8-row
    shard exceed its int32 Arrow offsets. `only`: generate just these columns (same values and validity)."""
    from deequ_amd.table import ChunkedTable, Table, Column
    chunks, nbytes = [], 0
    for r0 in range(0, rows, chunk_rows):
        n = min(chunk_rows, rows - r0)
        cols = []
        for j, (name, kind) in enumerate(C5_NUMERIC):
            if only is not None and name not in only:
                continue
            dt = torch.float64 if kind in (1, 2, 3, 6, 7) else torch.int64
            v = torch.empty(n, dtype=dt, device=dev)
            ctx.synth_column(kind, 0xC5000000 + j, r0, n, v.data_ptr())
            c = Column(name, N.TYPE_DOUBLE if dt == torch.float64 else N.TYPE_LONG, None, None, length=n)
            c.device = {"values": v}
            cols.append(c)
            nbytes += 8 * n
        for j, (name, kind) in enumerate(C5_STRINGS):
            if only is not None and name not in only:
                continue
            off = torch.empty(n + 1, dtype=torch.int32, device=dev)
            total = ctx.synth_strings(kind, 0xC5100000 + j, r0, n, off.data_ptr())
            data = torch.zeros(total + 16, dtype=torch.uint8, device=dev)
            ctx.synth_strings(kind, 0xC5100000 + j, r0, n, off.data_ptr(), data.data_ptr())
            c = Column(name, N.TYPE_STRING, None, None, length=n)
            c.device = {"values": data, "offsets": off}
            cols.append(c)
            nbytes += total + 4 * n
        index = {name: j for j, (name, _) in enumerate(C5_NUMERIC + C5_STRINGS)}
        for c in cols:
            m = torch.zeros((n + 63) // 64 * 8, dtype=torch.uint8, device=dev)
            ctx.synth_validity(0xC5200000 + index[c.name], r0, n, 50, m.data_ptr())
            c.device["validity"] = m
            nbytes += n / 8
        chunks.append(Table(cols))
    ctx.synchronize()
    return (chunks[0] if len(chunks) == 1 else ChunkedTable(chunks)), nbytes


def c5_extra_analyzers(D):
    """The rest of BASELINE config C5 / SURVEY §8d beside the ColumnProfiler's passes: ApproxQuantile(0.5) on every
    numeric column and the grouping analyzers (Uniqueness, Entropy) on a low-cardinality and a free-text column."""
    out = [D.ApproxQuantile(name, 0.5) for name, _ in C5_NUMERIC]
    for col in ("s_cat100", "s_text0"):
        out += [D.Uniqueness([col]), D.Entropy(col)]
    return out


def c5_step(D, t, extras):
    """One C5 step: the 3-pass ColumnProfiler + one AnalysisRunner run of the extra analyzers, the run submitted on a
    helper context (runAsync) so it overlaps the profiler's passes (DQ_C5_SEQUENTIAL=1: one after the other). The
    extras' chain (the text grouping's LDS-heavy partition / build kernels, then the quantiles) is the longer one and
    its kernels are starved of CUs by the profiler's: its stream gets high priority (DQ_C5_ASYNC_PRIORITY, default 1:
    136-141 ms a step on most boxes against 153-174 ms at normal priority). Before the helper contexts kept 48 GB of idle
    scratch (native.AUX_IDLE_SCRATCH_BYTES), about one box in five ran the overlapped step at 340-560 ms at either
    priority (profiles/r06/c5_priority_risk_r06bg.txt)."""
    if os.environ.get("DQ_C5_SEQUENTIAL"):
        prof = D.ColumnProfiler.profile(t)
        return prof, D.AnalysisRunner.onData(t).addAnalyzers(extras).run()
    main_prio = os.environ.get("DQ_C5_MAIN_PRIORITY")
    if main_prio is not None:  # A/B: the profiler's own context at another stream priority
        from deequ_amd import engine
        engine.ctx().set_priority(int(main_prio))
    pending = D.AnalysisRunner.onData(t).addAnalyzers(extras).runAsync(int(os.environ.get("DQ_C5_ASYNC_PRIORITY", 1)))
    try:
        prof = D.ColumnProfiler.profile(t)
    finally:
        pending.join()
    return prof, pending.result()


def bench_c5(torch, N, D, ctx, dev, rows, steps):
    """BASELINE config C5 at one GPU's shard size: the full 3-pass ColumnProfiler (generic statistics, numeric
    statistics + KLL over the numeric and numeric-looking string columns after Spark's casts, exact histograms of
    the low-cardinality columns) plus ApproxQuantile(0.5) on the numeric columns and Uniqueness / Entropy on a
    low-cardinality and a free-text column, over a 20-column mixed table in HBM. Wall time per step, sanity-checked."""
    t, nbytes = c5_shard(torch, N, ctx, dev, rows)
    extras = c5_extra_analyzers(D)
    prof = None
    for _ in range(2):  # warm-up: every context's scratch cache holds its working set before the timed steps
        c5_step(D, t, extras)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        prof, actx = c5_step(D, t, extras)
    torch.cuda.synchronize()
    el = (time.perf_counter() - t0) / steps
    # the profiler alone (the r02-r04 C5 line), for comparison
    t0 = time.perf_counter()
    for _ in range(steps):
        D.ColumnProfiler.profile(t)
    torch.cuda.synchronize()
    el_profile = (time.perf_counter() - t0) / steps
    assert prof.numRecords == rows
    for a in extras:
        assert actx.metric(a).value.isSuccess, (a, actx.metric(a).value)
    for name, _ in C5_NUMERIC:  # the median of a column the profiler also summarised lies inside its range
        p = prof.profiles[name]
        assert p.minimum <= actx.metric(D.ApproxQuantile(name, 0.5)).value.get() <= p.maximum, name
    assert 0.0 < actx.metric(D.Entropy("s_cat100")).value.get() <= math.log(100) + 1e-12
    for name, p in prof.profiles.items():
        assert 0.94 < p.completeness < 0.96, (name, p.completeness)
    hist = {n: p.histogram for n, p in prof.profiles.items() if p.histogram is not None}
    assert hist["s_bool"].numberOfBins == 3 and hist["s_cat50"].numberOfBins == 51, hist.keys()
    assert sum(v.absolute for v in hist["s_cat100"].values.values()) == rows
    types = {n: p.dataType for n, p in prof.profiles.items()}
    assert types["s_int"] == "Integral" and types["s_dec"] == "Fractional" and types["s_text0"] == "String", types
    ach = nbytes / el / 1e9
    c5_traffic = committed_json("c5_traffic_*.json", rows, need="traffic_bytes_per_call")
    passes = c5_pass_times(torch, D, t)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    D.AnalysisRunner.onData(t).addAnalyzers(extras).run()
    torch.cuda.synchronize()
    passes["extras_quantiles_grouping"] = round((time.perf_counter() - t0) * 1e3, 2)
    return {"workload": "C5 shard: ColumnProfiler passes 1-3 (Completeness, ApproxCountDistinct, DataType; Min / Max / "
                        "Mean / StdDev / Sum / KLL on 13 numeric and cast numeric-string columns; exact histograms of "
                        "%d low-cardinality columns) + ApproxQuantile(0.5) x 10 numeric columns + Uniqueness / Entropy "
                        "of s_cat100 and s_text0, over %d rows x 20 columns (5 fp64, 5 int64, 10 UTF-8), 5%% nulls, "
                        "held as %d row chunk(s) (one GPU's share of the 8-GPU 2e9-row table)"
                        % (len(hist), rows, len(getattr(t, "chunks", [t]))),
            "value": rows / el, "unit": "rows/s", "ms_per_step": el * 1e3,
            "profile_only_ms": el_profile * 1e3,
            "roofline": {"bound": "hbm", "achieved": ach, "peak": PEAK_HBM_GBPS, "unit": "GB/s",
                         "frac": ach / PEAK_HBM_GBPS,
                         "traffic": c5_traffic[0]["traffic_bytes_per_call"] / 1e9 if c5_traffic else None,
                         "traffic_unit": "GB per profile (rocprofv3 PMC, %s)" % (c5_traffic[1] if c5_traffic
                                                                                 else "not measured"),
                         "kernel": "end-to-end profile wall time; achieved = the table's bytes (%.1f GB: values, "
                                   "offsets, UTF-8 data, validity) once per profile" % (nbytes / 1e9)},
            "passes_ms": passes}


def c5_pass_times(torch, D, t):
    """Wall time of each ColumnProfiler pass of one extra (untimed) profile, the device synchronised at every pass
    boundary: pass 1 (Completeness, ApproxCountDistinct, DataType, Size), the pass-2 casts, pass 2 (numeric
    statistics scan + the KLL extra pass), pass 3 (histograms)."""
    from deequ_amd.profiles import LocalPasses

    class Timed(LocalPasses):
        def __init__(self):
            self.ms, self.runs = {}, 0

        def _t(self, key, fn):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            out = fn()
            torch.cuda.synchronize()
            self.ms[key] = self.ms.get(key, 0.0) + (time.perf_counter() - t0) * 1e3
            return out

        def run(self, data, analyzers):
            self.runs += 1
            return self._t("pass1_generic" if self.runs == 1 else "pass2_numeric_and_kll",
                           lambda: LocalPasses.run(self, data, analyzers))

        def cast(self, data, name, to_type):
            return self._t("pass2_casts", lambda: LocalPasses.cast(self, data, name, to_type))

        def histograms(self, data, targets):
            return self._t("pass3_histograms", lambda: LocalPasses.histograms(self, data, targets))

    p = Timed()
    D.ColumnProfiler.profile(t, passes=p)
    return {k: round(v, 2) for k, v in p.ms.items()}


def bench_host_streamed(torch, N, D, ctx, dev, rows, steps, chunk_rows=1 << 25):
    """The C2 suite over HOST-resident columns (pinned memory) streamed through HBM in row chunks
    (dq_scan_streamed: the copy of chunk i + 1 overlaps the scan of chunk i): the end-to-end rate, bound by the
    host link — reported apart from the HBM-resident headline."""
    from deequ_amd.table import Table, Column
    cols = []
    for c, kind in enumerate(C2_KINDS):
        dt = torch.float64 if kind in (1, 2, 3, 6) else torch.int64
        v = torch.empty(rows, dtype=dt, device=dev)
        m = torch.zeros((rows + 63) // 64 * 8, dtype=torch.uint8, device=dev)
        ctx.synth_column(kind, SEED + c, 0, rows, v.data_ptr())
        ctx.synth_validity(SEED + 0x100 + c, 0, rows, 10, m.data_ptr())
        ctx.synchronize()
        hv = torch.empty(rows, dtype=dt, pin_memory=True)
        hm = torch.empty(m.numel(), dtype=torch.uint8, pin_memory=True)
        hv.copy_(v)
        hm.copy_(m)
        del v, m
        col = Column("c%d" % c, N.TYPE_DOUBLE if dt == torch.float64 else N.TYPE_LONG, hv.numpy(), hm.numpy(),
                     length=rows)
        col._pinned = (hv, hm)
        cols.append(col)
    t = Table(cols)
    batch = D.ScanBatch(t)
    offs = [a.addOps(batch) for a in c2_analyzers(D, list(t.columns))]
    natives = batch.native_columns()
    preds = [p.to_native() for p in batch.preds]
    res = ctx.scan_streamed(natives, rows, batch.ops, preds, chunk_rows)  # warm-up
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        res = ctx.scan_streamed(natives, rows, batch.ops, preds, chunk_rows)
    el = (time.perf_counter() - t0) / steps
    from deequ_amd.states import state_from_native
    assert state_from_native(res[offs[0][0]]).numMatches == rows
    bpr = 8 * (8 + 1 / 8)
    return {"workload": "C2 suite over host-resident (pinned) columns, %d rows streamed through HBM in %d-row chunks "
                        "(copy of the next chunk overlapped with the scan)" % (rows, chunk_rows),
            "value": rows / el, "unit": "rows/s", "ms_per_step": el * 1e3,
            "host_link_GBps": bpr * rows / el / 1e9,
            "note": "end-to-end incl. host->device copies (PCIe); not comparable to the HBM-resident value"}


def cpu_baseline(seconds, sample_rows, threads=None):
    """The oracle's Spark-order restatement (oracle/dq_oracle.c oracle_scan_spark) over a bounded
    sample of the same synthetic columns, split into `threads` contiguous row partitions scanned
    concurrently (Spark local[N]'s one-task-per-partition shape; ctypes releases the GIL). Rows/s of
    the 8-column suite; the O(threads) state merge is not timed."""
    import threading
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    L = O.lib()
    L.oracle_scan_spark.restype = ctypes.c_int64
    L.oracle_scan_spark.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p]
    if threads is None:
        threads = min(16, int(os.environ.get("OMP_NUM_THREADS", 0)) or os.cpu_count() or 1)
    threads = max(1, min(int(threads), sample_rows))
    cols = []
    for c, kind in enumerate(C2_KINDS):
        v = O.synth_column(kind, SEED + c, 0, sample_rows)
        m = O.synth_validity(SEED + 0x100 + c, 0, sample_rows, 10).astype(np.uint8)
        cols.append((7 if kind in (1, 2, 3) else 5, v, m))
    bounds = [sample_rows * i // threads for i in range(threads + 1)]
    done = [0] * threads
    start = threading.Barrier(threads + 1)
    deadline = [0.0]

    def worker(i):
        lo, hi = bounds[i], bounds[i + 1]
        out = np.zeros(5)
        start.wait()
        while True:
            for st, v, m in cols:
                L.oracle_scan_spark(st, v[lo:].ctypes.data, m[lo:].ctypes.data, hi - lo, out.ctypes.data)
            done[i] += hi - lo
            if time.perf_counter() >= deadline[0]:
                break

    ts = [threading.Thread(target=worker, args=(i,)) for i in range(threads)]
    for t in ts:
        t.start()
    t0 = time.perf_counter()
    deadline[0] = t0 + seconds
    start.wait()
    for t in ts:
        t.join()
    el = time.perf_counter() - t0
    rows = sum(done)
    return {"value": rows / el, "unit": "rows/s", "cores": threads, "kind": "port",
            "sample": "oracle_scan_spark over a %d-row x 8-col sample of the C2 columns in %d row partitions "
                      "(one host thread each), %.1f sample passes in %.1f s (Spark-order count/sum/min/max/"
                      "Welford; not deequ/Spark itself)" % (sample_rows, threads, rows / sample_rows, el)}


def _timed_threads(seconds, threads, work):
    """Run work(i) -> rows in `threads` host threads (ctypes releases the GIL) until `seconds` have passed;
    (rows done, elapsed s)."""
    import threading
    done = [0] * threads
    start = threading.Barrier(threads + 1)
    deadline = [0.0]

    def worker(i):
        start.wait()
        while True:
            done[i] += work(i)
            if time.perf_counter() >= deadline[0]:
                break

    ts = [threading.Thread(target=worker, args=(i,)) for i in range(threads)]
    for t in ts:
        t.start()
    t0 = time.perf_counter()
    deadline[0] = t0 + seconds
    start.wait()
    for t in ts:
        t.join()
    return sum(done), time.perf_counter() - t0


def _cpu_threads(threads=None):
    if threads is None:
        threads = min(16, int(os.environ.get("OMP_NUM_THREADS", 0)) or os.cpu_count() or 1)
    return max(1, int(threads))


def cpu_baseline_suite10(seconds, sample_rows, threads=None):
    """CPU leg of the suite10 line: the oracle's Spark-order row loops (oracle_scan_suite10_col: count / Sum /
    Min / Max / CentralMomentAgg / Compliance(c > 0) / HLL++ update per column; oracle_corr_spark per pair) over a
    bounded sample of the C2 columns, one contiguous row partition per host thread."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    L = O.lib()
    L.oracle_scan_suite10_col.restype = ctypes.c_int64
    L.oracle_scan_suite10_col.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64,
                                          ctypes.c_void_p, ctypes.c_void_p]
    L.oracle_corr_spark.restype = ctypes.c_int64
    L.oracle_corr_spark.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p,
                                    ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p]
    threads = min(_cpu_threads(threads), sample_rows)
    cols = []
    for c, kind in enumerate(C2_KINDS):
        v = O.synth_column(kind, SEED + c, 0, sample_rows)
        m = O.synth_validity(SEED + 0x100 + c, 0, sample_rows, 10).astype(np.uint8)
        cols.append((7 if kind in (1, 2, 3) else 5, v, m))
    bounds = [sample_rows * i // threads for i in range(threads + 1)]
    regs = [np.zeros(512, dtype=np.uint8) for _ in range(threads)]
    outs = [np.zeros(6) for _ in range(threads)]

    def work(i):
        lo, hi = bounds[i], bounds[i + 1]
        for st, v, m in cols:
            L.oracle_scan_suite10_col(st, v[lo:].ctypes.data, m[lo:].ctypes.data, hi - lo, regs[i].ctypes.data,
                                      outs[i].ctypes.data)
        for k in range(4):
            (tx, x, mx), (ty, y, my) = cols[2 * k], cols[2 * k + 1]
            L.oracle_corr_spark(tx, x[lo:].ctypes.data, mx[lo:].ctypes.data, ty, y[lo:].ctypes.data, my[lo:].ctypes.data,
                                hi - lo, outs[i].ctypes.data)
        return hi - lo

    rows, el = _timed_threads(seconds, threads, work)
    return {"value": rows / el, "unit": "rows/s", "cores": threads, "kind": "port",
            "sample": "oracle_scan_suite10_col x 8 + oracle_corr_spark x 4 over a %d-row sample of the C2 columns in %d "
                      "row partitions (one host thread each), %.1f sample passes in %.1f s (Spark-order row updates "
                      "incl. XXH64 + HLL++; not deequ/Spark itself)" % (sample_rows, threads, rows / sample_rows, el)}


def cpu_baseline_c4(seconds, sample_rows, threads=None):
    """CPU leg of the C4 line: count(*) GROUP BY key as a per-partition open-addressing hash aggregate
    (oracle_count_keys) over a bounded sample of the C4 keys, one partition per host thread."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    L = O.lib()
    L.oracle_count_keys.restype = ctypes.c_int64
    L.oracle_count_keys.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64]
    threads = min(_cpu_threads(threads), sample_rows)
    keys = O.synth_freq_keys(1_000_000_000, 100_000_000, 0, sample_rows)
    bounds = [sample_rows * i // threads for i in range(threads + 1)]
    per = max(bounds[i + 1] - bounds[i] for i in range(threads))
    cap = 1 << max(4, int(per * 2 - 1).bit_length())
    tables = [np.zeros(2 * cap, dtype=np.int64) for _ in range(threads)]
    used = [np.zeros(cap, dtype=np.uint8) for _ in range(threads)]

    def work(i):
        lo, hi = bounds[i], bounds[i + 1]
        L.oracle_count_keys(keys[lo:].ctypes.data, hi - lo, tables[i].ctypes.data, used[i].ctypes.data, cap)
        return hi - lo

    rows, el = _timed_threads(seconds, threads, work)
    return {"value": rows / el, "unit": "rows/s", "cores": threads, "kind": "port",
            "sample": "oracle_count_keys (open-addressing count(*) GROUP BY key per partition) over the first %d C4 keys "
                      "in %d partitions (one host thread each), %.1f sample passes in %.1f s (partial tables only; "
                      "not deequ/Spark itself)" % (sample_rows, threads, rows / sample_rows, el)}


def committed_json(pattern, rows, need=None):
    """(content, path) of the last profiles/<round>/<pattern> whose "rows" equals `rows` (any when None) and that holds
    the key `need` (when given), or None."""
    import glob
    best = None
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "*", pattern))):
        try:
            d = json.load(open(path))
        except (OSError, ValueError):
            continue
        if (rows is None or int(d.get("rows", -1)) == rows) and (need is None or need in d):
            best = (d, os.path.relpath(path, ROOT))
    return best


def measured_traffic(rows_per_gpu):
    """HBM bytes per dq_scan call of this workload from the committed rocprofv3 PMC passes
    (tools/gpu_pmc.sh -> tools/pmc_traffic.py -> profiles/<round>/c2_traffic_*.json), in GB, or None
    when no PMC measurement of this exact shard size is committed."""
    found = committed_json("c2_traffic_*.json", rows_per_gpu, need="traffic_bytes_per_call")
    return (found[0]["traffic_bytes_per_call"] / 1e9, found[1]) if found else None


def spawn_ranks(args):
    """`--gpus N` without a launcher: start N rank processes of this script (RANK / LOCAL_RANK / WORLD_SIZE /
    MASTER_* set, rendezvous on 127.0.0.1), forward rank 0's stdout, and return the first failing exit status. The
    parent makes no GPU call (it never touches torch.cuda), so the children are fresh processes on their GPUs; if one
    rank fails the others are stopped (by PID) instead of waiting in a collective."""
    import socket
    import subprocess
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    procs = []
    for r in range(args.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(args.gpus),
                   LOCAL_WORLD_SIZE=str(args.gpus), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env,
                                      stdout=subprocess.PIPE if r == 0 else sys.stderr.fileno()))
    out0 = []
    import threading
    reader = threading.Thread(target=lambda: out0.extend(procs[0].stdout.read().decode().splitlines()))
    reader.start()
    rc = 0
    while any(p.poll() is None for p in procs):
        bad = [p.returncode for p in procs if p.returncode not in (None, 0)]
        if bad:
            rc = bad[0]
            for p in procs:
                if p.poll() is None:
                    p.kill()
            break
        time.sleep(0.2)
    for p in procs:
        p.wait()
        if p.returncode and not rc:
            rc = p.returncode
    reader.join()
    for line in out0:
        print(line, flush=True)
    return rc


def launch_check(args, world, rank):
    """--launch-check: the launcher plumbing without any GPU call (CPU tests): gloo rendezvous, one all-reduce, rank 0
    prints {"n_gpus": world, ...}."""
    import torch
    import torch.distributed as dist
    assert world == args.gpus, (world, args.gpus)
    if world > 1:
        dist.init_process_group("gloo", rank=rank, world_size=world)
        t = torch.tensor([rank + 1], dtype=torch.int64)
        dist.all_reduce(t)
        ranks_sum = int(t.item())
        dist.destroy_process_group()
    else:
        ranks_sum = 1
    total, _, nrows = shard_plan(args.rows, world, rank, args.scaling)
    if rank == 0:
        print(json.dumps({"launch_check": True, "n_gpus": world, "ranks_sum": ranks_sum,
                          "local_rank": int(os.environ.get("LOCAL_RANK", "0")),
                          "config": {"rows": total, "rows_per_gpu": nrows, "scaling": args.scaling}}), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--rows", type=float, default=1e9)
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--cpu-sample-rows", type=int, default=8_000_000)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-secondary", action="store_true", help="only the headline C2 line")
    ap.add_argument("--dist-backend", default="nccl", help="nccl (RCCL over xGMI) or gloo (rehearsal on one GPU)")
    ap.add_argument("--device-override", type=int, default=None, help="run every rank on this GPU (rehearsal)")
    ap.add_argument("--scaling", choices=("weak", "strong"), default="strong",
                    help="strong (default, BASELINE's 1B-row table at 1/2/4/8 GPUs): --rows split over the ranks; "
                         "weak: every rank scans its own --rows-row shard of a world x --rows table")
    ap.add_argument("--launch-check", action="store_true", help=argparse.SUPPRESS)
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(spawn_ranks(args))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.launch_check:
        return launch_check(args, world, rank)
    if world != args.gpus:
        sys.exit("bench.py: WORLD_SIZE=%d but --gpus %d" % (world, args.gpus))

    import torch
    import torch.distributed as dist
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group(args.dist_backend, rank=rank, world_size=world)
        assert dist.get_world_size() == args.gpus
        # the measured multi-GPU path is RCCL over xGMI; gloo only as an explicit one-GPU rehearsal
        assert dist.get_backend() == args.dist_backend and (args.dist_backend == "nccl" or
                                                             args.device_override is not None), \
            "multi-GPU bench runs on RCCL (nccl); gloo needs --device-override (rehearsal)"
    if args.device_override is not None:
        local = args.device_override
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    import deequ_amd as D
    import deequ_amd.native as N
    from deequ_amd import engine
    from deequ_amd.states import state_from_native
    engine.set_device(local)
    ctx = engine.ctx()
    # One explicit stream for the scan, the collectives and the copies (torch's default stream
    # reports handle 0, which dq_set_stream would map to the context's own stream).
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    ctx.set_stream(stream.cuda_stream)

    total, row0, nrows = shard_plan(args.rows, world, rank, args.scaling)
    table = build_shard(torch, N, ctx, row0, nrows, dev)
    names = list(table.columns)
    bytes_per_row = sum(8 + 1.0 / 8 for _ in names)  # values + validity bit, per column

    c2 = ScanWorkload(torch, N, D, ctx, table, c2_analyzers(D, names), stream, dev, world, args.dist_backend)
    elapsed, scan_ms, states = timed(torch, dist, world, args.steps, args.warmup, stream, c2.step)
    # sanity: the folded Size equals the table size
    size_state = state_from_native(states[c2.offsets[0][0]])
    assert size_state.numMatches == total, (size_state, total)

    alg_bytes = bytes_per_row * nrows
    achieved = alg_bytes / (scan_ms * 1e-3) / 1e9
    ms_per_step = elapsed / args.steps * 1e3
    value = total / (elapsed / args.steps)
    traffic = measured_traffic(nrows)
    result = {
        "metric": "rows/sec + HBM GB/s (% peak) for fused analyzer suite, 1B rows, 1/2/4/8 GPUs",
        "value": value,
        "unit": "rows/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        "scaling": args.scaling,
        "vs_baseline": None,
        "dtype": "f64+i64",
        "data": "synthetic (counter-based splitmix64 columns generated in HBM, SURVEY.md §8d)",
        "config": {"workload": "C2 fused scan suite: Size + {Completeness, Mean, Sum, Minimum, Maximum, "
                               "StandardDeviation} x 8 cols (4 fp64 + 4 int64, 1% nulls) = 49 ops",
                   "rows": total, "rows_per_gpu": nrows, "scaling": args.scaling, "columns": len(names), "ops": c2.nops,
                   "parallelism": "rows sharded dp%d + %s all-gather of states"
                                  % (world, "RCCL" if args.dist_backend == "nccl" else args.dist_backend),
                   "dist_backend": args.dist_backend if world > 1 else None},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": PEAK_HBM_GBPS, "unit": "GB/s",
                     "frac": achieved / PEAK_HBM_GBPS, "traffic": traffic[0] if traffic else None,
                     "traffic_unit": "GB per dq_scan call (HBM FETCH+WRITE from rocprofv3 PMC, %s)"
                                     % (traffic[1] if traffic else "not measured for this shard size"),
                     "kernel": "dq_scan fused pass (scan_values_kernel launches + partial folds), HIP events "
                               "on the scan stream, avg %.3f ms over %d steps; algorithmic bytes %.1f B/row x %d rows"
                               % (scan_ms, args.steps, bytes_per_row, nrows)},
    }
    del c2
    if not args.no_secondary:
        sec = {}
        s10 = ScanWorkload(torch, N, D, ctx, table, suite10_analyzers(D, names), stream, dev, world, args.dist_backend)
        el, kms, st = timed(torch, dist, world, max(3, args.steps // 4), 1, stream, s10.step)
        ach = alg_bytes / (kms * 1e-3) / 1e9
        s10_traffic = committed_json("suite10_traffic_*.json", nrows, need="traffic_bytes_per_call")
        s10_valu = committed_json("suite10_sq_counters_*.json", None, need="runs")
        valu = None
        if s10_valu is not None and world == 1 and nrows == 1_000_000_000:
            # VALU roofline of the (VALU-bound) heavy kernels: wave64 VALU instructions per call (rocprofv3 SQ_INSTS_VALU,
            # the last committed run) x 64 lanes / the measured scan time, against 256 CUs x 64 lanes x 2.4 GHz
            runs = s10_valu[0]["runs"]
            last = runs[sorted(runs)[-1]]
            insts = sum(k["SQ_INSTS_VALU"] for k in last.values())
            peak = 256 * 64 * 2.4e9 / 1e12
            a = insts * 64 / (kms * 1e-3) / 1e12
            valu = {"bound": "valu", "achieved": a, "peak": peak, "unit": "Tlane-op/s", "frac": a / peak,
                    "insts_per_call": insts, "source": s10_valu[1],
                    "note": "SQ_INSTS_VALU of the committed profile; the chip ran at ~2.0 GHz under this load "
                            "(SQ_BUSY_CYCLES), so frac against 2.4 GHz understates issue utilisation (~0.82)"}
        sec["suite10"] = {
            "workload": "north-star 10-analyzer suite: C2 ops + Compliance(c > 0) + ApproxCountDistinct x 8 cols + "
                        "Correlation(c_2k, c_2k+1) x 4 = %d ops, one fused pass" % s10.nops,
            "value": total / (el / max(3, args.steps // 4)), "unit": "rows/s", "ms_per_step": el / max(3, args.steps // 4) * 1e3,
            "roofline": {"bound": "hbm", "achieved": ach, "peak": PEAK_HBM_GBPS, "unit": "GB/s",
                         "frac": ach / PEAK_HBM_GBPS,
                         "traffic": s10_traffic[0]["traffic_bytes_per_call"] / 1e9 if s10_traffic else None,
                         "traffic_unit": "GB per dq_scan call (rocprofv3 PMC, %s)" % (s10_traffic[1] if s10_traffic
                                                                                      else "not measured"),
                         "kernel": "dq_scan avg %.3f ms (HIP events); VALU-bound: XXH64 + moments per value "
                                   "(DESIGN.md §3)" % kms},
            "valu_roofline": valu}
        del s10
        # C2 with every analyzer under `where c4 < 0` (conditionalSelection): the filter is evaluated by c4's own scan
        w = "c4 < 0"
        c2w_an = [D.Size(w)]
        for cn in names:
            c2w_an += [D.Completeness(cn, w), D.Mean(cn, w), D.Sum(cn, w), D.Minimum(cn, w), D.Maximum(cn, w),
                       D.StandardDeviation(cn, w)]
        c2w = ScanWorkload(torch, N, D, ctx, table, c2w_an, stream, dev, world, args.dist_backend)
        before = ctx.kernel_launches()
        el, kms, _ = timed(torch, dist, world, max(3, args.steps // 4), 1, stream, c2w.step)
        after = ctx.kernel_launches()
        ach = alg_bytes / (kms * 1e-3) / 1e9
        c2w_traffic = committed_json("c2where_traffic_*.json", nrows, need="traffic_bytes_per_call")
        sec["c2_where"] = {
            "workload": "C2's 49 ops, every one under `where %s` (int64 column, 1%% nulls: ~50%% of the rows selected)" % w,
            "value": total / (el / max(3, args.steps // 4)), "unit": "rows/s",
            "ms_per_step": el / max(3, args.steps // 4) * 1e3,
            "launches_per_step": {k: (after[k] - before[k]) / (max(3, args.steps // 4) + 1)
                                  for k in after if after[k] != before[k]},
            "roofline": {"bound": "hbm", "achieved": ach, "peak": PEAK_HBM_GBPS, "unit": "GB/s",
                         "frac": ach / PEAK_HBM_GBPS,
                         "traffic": c2w_traffic[0]["traffic_bytes_per_call"] / 1e9 if c2w_traffic else None,
                         "traffic_unit": "GB per dq_scan call (rocprofv3 PMC, %s)" % (c2w_traffic[1] if c2w_traffic
                                                                                      else "not measured"),
                         "kernel": "dq_scan avg %.3f ms (HIP events): the filter column's scan produces the valid & "
                                   "where masks the other columns' scans read; algorithmic %.1f B/row as C2"
                                   % (kms, bytes_per_row)}}
        del c2w
        del table
        torch.cuda.empty_cache()
        sec["c3"] = bench_c3(torch, N, D, ctx, stream, dev, total, max(3, args.steps // 4), dist, world, rank,
                             args.dist_backend)
        torch.cuda.empty_cache()
        if world > 1:
            sec["c4"] = bench_c4_dist(torch, N, D, dev, total, max(3, args.steps // 4), dist, world, rank)
            torch.cuda.empty_cache()
        if world == 1:
            sec["c4"] = bench_c4(torch, N, D, ctx, stream, dev, total, max(3, args.steps // 4))
            torch.cuda.empty_cache()
            sec["c2_host_streamed"] = bench_host_streamed(torch, N, D, ctx, dev, min(total, 200_000_000), 2)
            torch.cuda.empty_cache()
            sec["c5_shard"] = bench_c5(torch, N, D, ctx, dev, min(total, 250_000_000), 2)
            torch.cuda.empty_cache()
        result["secondary"] = sec
    if rank == 0 and world == 1 and not args.no_cpu:
        result["cpu_baseline"] = cpu_baseline(args.cpu_seconds, args.cpu_sample_rows)
        if "secondary" in result:
            sec = result["secondary"]
            sec["suite10"]["cpu_baseline"] = cpu_baseline_suite10(args.cpu_seconds / 2, args.cpu_sample_rows // 2)
            if "c4" in sec:
                sec["c4"]["cpu_baseline"] = cpu_baseline_c4(args.cpu_seconds / 2, 1 << 24)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
