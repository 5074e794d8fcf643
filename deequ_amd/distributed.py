"""Row-sharded multi-GPU AnalysisRunner: one process per GPU, torch.distributed
(backend "nccl" = RCCL over xGMI; "gloo" for CPU tests).

Scan-shareable analyzers: every rank runs the fused scan over its row shard, the fixed-size dq_state
records of all ranks are all-gathered in ONE collective, and every rank folds them in rank order
with the reference semigroup merges (dq_state_merge = State.sum, e.g. A/StandardDeviation.scala:37-44)
— deterministic and identical on every rank; a plain all-reduce cannot express the Chan merge.

Grouping analyzers (one fixed-width key column): every rank buckets the canonical keys of its
non-NULL rows by owner rank (dq_partition_keys), the buckets travel in one all-to-all, and each
owner builds the frequency table of the keys it owns, so group sets are disjoint across ranks. The
global numRows is an all-reduce; #groups / #unique are sums; entropy terms use the global numRows and
their per-rank sums are folded in rank order (A/GroupingAnalyzers.scala:53-79, R/AnalysisRunner.scala:480-548).

The per-rank compute is behind `GpuLocal` (libdq.so); the collective choreography is shared with the
CPU test double in tests/test_distributed_gloo.py.
"""
import ctypes
import math

import numpy as np

from . import native as N
from . import engine
from .analyzers import (ScanShareableAnalyzer, GroupingAnalyzer, ScanShareableFrequencyBasedAnalyzer, Histogram,
                        FrequenciesAndNumRows, Preconditions, metricFromFailure)
from .metrics import (HistogramMetric, Distribution, DistributionValue, Success, Failure, wrap_if_necessary,
                      MetricCalculationRuntimeException, UnsupportedOnDevice)
from .runners import AnalyzerContext, ScanBatch, ScanResult


def fold_states(raw, world, nops):
    """Rank-ordered semigroup fold of all-gathered dq_state records (rank-major bytes), in one
    dq_state_fold call."""
    raw = np.ascontiguousarray(np.asarray(raw, dtype=np.uint8))
    return N.fold_states(raw, world, nops)


def kahan_fold(values):
    s, c = 0.0, 0.0
    for v in values:
        y = v - c
        t = s + y
        c = (t - s) - y
        s = t
    return s


class Exchange:
    """The collectives the sharded runner needs, on the process group's device."""

    def __init__(self, group=None):
        import torch
        import torch.distributed as dist
        self.torch, self.dist, self.group = torch, dist, group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        backend = dist.get_backend(group)
        self.device = torch.device("cuda", torch.cuda.current_device()) if backend == "nccl" else torch.device("cpu")

    def all_gather_bytes(self, t):
        out = self.torch.empty(self.world * t.numel(), dtype=self.torch.uint8, device=self.device)
        self.dist.all_gather_into_tensor(out, t.to(self.device), group=self.group)
        return out

    def all_gather_blobs(self, blob):
        """Variable-size byte strings of every rank, in rank order (sizes first, then padded bytes)."""
        torch = self.torch
        n = torch.tensor([len(blob)], dtype=torch.int64, device=self.device)
        sizes = torch.empty(self.world, dtype=torch.int64, device=self.device)
        self.dist.all_gather_into_tensor(sizes, n, group=self.group)
        sizes = [int(v) for v in sizes.cpu().tolist()]
        width = max(max(sizes), 1)
        buf = torch.zeros(width, dtype=torch.uint8)
        if blob:
            buf[:len(blob)] = torch.frombuffer(bytearray(blob), dtype=torch.uint8)
        out = torch.empty(self.world * width, dtype=torch.uint8, device=self.device)
        self.dist.all_gather_into_tensor(out, buf.to(self.device), group=self.group)
        raw = out.cpu().numpy().tobytes()
        return [raw[r * width:r * width + sizes[r]] for r in range(self.world)]

    def all_reduce_i64(self, values):
        t = self.torch.tensor(values, dtype=self.torch.int64, device=self.device)
        self.dist.all_reduce(t, group=self.group)
        return [int(v) for v in t.cpu().tolist()]

    def all_gather_f64(self, value):
        t = self.torch.tensor([value], dtype=self.torch.float64, device=self.device)
        out = self.torch.empty(self.world, dtype=self.torch.float64, device=self.device)
        self.dist.all_gather_into_tensor(out, t, group=self.group)
        return out.cpu().tolist()

    def all_to_all_keys(self, keys, send_counts):
        """keys: int64 tensor bucketed by destination rank; returns the keys this rank owns."""
        torch = self.torch
        sc = torch.tensor(send_counts, dtype=torch.int64, device=self.device)
        rc = torch.empty_like(sc)
        self.dist.all_to_all_single(rc, sc, group=self.group)
        recv_counts = [int(v) for v in rc.cpu().tolist()]
        out = torch.empty(sum(recv_counts), dtype=torch.int64, device=self.device)
        self.dist.all_to_all_single(out, keys.to(self.device), output_split_sizes=recv_counts,
                                    input_split_sizes=list(send_counts), group=self.group)
        return out

    def all_gather_pairs(self, keys, counts, k):
        """Top-k candidates of every rank -> list of (key, count)."""
        torch = self.torch
        pad = torch.full((k,), -1, dtype=torch.int64)
        kk, cc = pad.clone(), pad.clone()
        n = len(keys)
        kk[:n] = torch.tensor(list(keys), dtype=torch.int64) if n else kk[:0]
        cc[:n] = torch.tensor(list(counts), dtype=torch.int64) if n else cc[:0]
        both = torch.cat([kk, cc]).to(self.device)
        out = torch.empty(self.world * 2 * k, dtype=torch.int64, device=self.device)
        self.dist.all_gather_into_tensor(out, both, group=self.group)
        arr = out.cpu().numpy().reshape(self.world, 2, k)
        pairs = []
        for r in range(self.world):
            for i in range(k):
                if arr[r, 1, i] >= 0:
                    pairs.append((int(arr[r, 0, i]), int(arr[r, 1, i])))
        return pairs


class GpuLocal:
    """Per-rank compute on this process's GPU through libdq.so."""

    def scan_states(self, batch):
        """This shard's dq_state records (device bytes) and its quantile digests."""
        import torch
        nops = len(batch.ops)
        out = torch.empty(max(nops, 1) * N.STATE_SIZE, dtype=torch.uint8, device="cuda")
        torch.cuda.current_stream().synchronize()  # `out` allocated on torch's stream
        ctx = engine.ctx()
        res = batch.run(out_device_ptr=out.data_ptr())
        ctx.synchronize()  # the scan runs on the context's stream; order it before torch reads `out`
        return out[:nops * N.STATE_SIZE], list(res.quantiles)

    def kll_state(self, shard, column, sketch_size, shrinking_factor):
        """This shard's KLLState bytes (one partition, rows in order)."""
        from .runners import KLLRunner
        return KLLRunner.sketch_column(shard, column, sketch_size, shrinking_factor).toBytes()

    def partition(self, column, world):
        import torch
        ctx = engine.ctx()
        keys = torch.empty(max(column.length, 1), dtype=torch.int64, device="cuda")
        counts = (ctypes.c_int64 * world)()
        nulls = ctypes.c_int64(0)
        rc = ctx.lib.dq_partition_keys(ctx.handle, ctypes.byref(column.native()), column.length, world,
                                       ctypes.c_void_p(keys.data_ptr()), counts, ctypes.byref(nulls))
        ctx.check(rc, "dq_partition_keys")
        send = [int(counts[i]) for i in range(world)]
        return keys[:sum(send)], send, int(nulls.value)

    def frequencies_of_keys(self, keys):
        """Local table over owned canonical keys (grouping on their 64-bit patterns)."""
        from .table import Table, Column
        col = Column("k", N.TYPE_LONG, None, None, length=int(keys.numel()))
        col.device = {"values": keys.to("cuda").contiguous()}
        return engine.frequencies(Table([col]), ["k"])


def _decode_canonical(spark_type, decimal_scale, k):
    u = np.uint64(k & 0xFFFFFFFFFFFFFFFF)
    if spark_type == N.TYPE_DOUBLE:
        return engine.GroupFloat(u.view(np.float64))
    if spark_type == N.TYPE_FLOAT:
        return engine.GroupFloat(np.uint32(int(u) & 0xFFFFFFFF).view(np.float32))
    i = int(u.view(np.int64))
    if spark_type == N.TYPE_BOOLEAN:
        return bool(i)
    if spark_type == N.TYPE_DECIMAL:
        from decimal import Decimal
        return Decimal(i).scaleb(-decimal_scale)
    return i


class DistributedFrequencies:
    """Global view of a hash-partitioned frequency table (the grouping state across ranks)."""

    def __init__(self, exchange, local_table, column, num_rows, null_rows):
        self.ex, self.local, self.column = exchange, local_table, column
        self.num_rows = num_rows  # global
        self.null_rows = null_rows  # global NULL rows (Histogram)
        self._summary = {}

    def summary(self, n=None):
        n = self.num_rows if n is None else n
        if n not in self._summary:
            s = self.local.summary(n)
            groups, unique = self.ex.all_reduce_i64([s["num_groups"], s["num_unique"]])
            ent = kahan_fold(self.ex.all_gather_f64(s["entropy"]))
            self._summary[n] = {"num_rows": self.num_rows, "num_groups": groups, "num_unique": unique,
                                "entropy": ent}
        return self._summary[n]

    @property
    def num_groups(self):
        return self.summary()["num_groups"] + (1 if self.null_rows else 0)

    def top(self, k):
        loc = self.local.top(k)
        keys = [int(np.int64(np.uint64(_canonical_key(key[0], self.column)))) for key, c in loc]
        pairs = self.ex.all_gather_pairs(keys, [c for _, c in loc], k)
        out = [((_decode_canonical(self.column.spark_type, self.column.decimal_scale, kk),), c) for kk, c in pairs]
        if self.null_rows:
            out.append(((None,), self.null_rows))
        out.sort(key=lambda kv: -kv[1])
        return out[:k]


def _canonical_key(v, column):
    """Inverse of the local table's decode (it grouped canonical bits as LONG)."""
    return int(v) & 0xFFFFFFFFFFFFFFFF


class DistributedAnalysisRunner:
    """AnalysisRunner over a row shard per rank; every rank returns the same AnalyzerContext.

    Failure protocol: every stage runs its local (per-rank) compute first, then every rank takes part in
    one agreement collective (`_agree`) before any data collective, so a rank that fails locally (a regex
    budget, an out-of-memory, a bad shard) never leaves its peers blocked in a collective it skips: all
    ranks learn the first failing rank's error and turn it into the same failure metrics."""

    def __init__(self, exchange=None, local=None):
        self.ex = exchange or Exchange()
        self.local = local or GpuLocal()

    def _agree(self, error):
        """Collective on every rank: None if every rank succeeded, else the first failing rank's error (as a
        MetricCalculationRuntimeException carrying its message) on every rank."""
        flags = self.ex.all_reduce_i64([0 if error is None else 1])
        if flags[0] == 0:
            return None
        msgs = self.ex.all_gather_blobs(b"" if error is None else ("%s: %s" % (type(error).__name__, error)).encode())
        for r, m in enumerate(msgs):
            if m:
                return MetricCalculationRuntimeException("rank %d failed: %s" % (r, m.decode(errors="replace")))
        return MetricCalculationRuntimeException("a rank failed")

    def run(self, shard, analyzers):
        uniq = []
        for a in analyzers:
            if a not in uniq:
                uniq.append(a)
        results = {}
        passed = []
        for a in uniq:
            e = Preconditions.findFirstFailing(shard.schema, a.preconditions())
            if e is not None:
                results[a] = a.toFailureMetric(e)
            else:
                passed.append(a)
        from .analyzers import KLLSketch
        kll = [a for a in passed if isinstance(a, KLLSketch)]
        shareable = [a for a in passed if isinstance(a, ScanShareableAnalyzer) and not isinstance(a, KLLSketch)]
        if kll:
            self._kll_metrics(shard, kll, results)
        if shareable:
            local_err = None
            try:
                batch = ScanBatch(shard)
                offsets = [a.addOps(batch) for a in shareable]
                local_states, local_q = self.local.scan_states(batch)
            except Exception as e:
                local_err = e
            agreed = self._agree(local_err)
            if agreed is not None:
                for a in shareable:
                    results[a] = a.toFailureMetric(agreed)
                shareable = []
        if shareable:
            try:
                gathered = self.ex.all_gather_bytes(local_states)
                states = ScanResult(fold_states(gathered.cpu().numpy(), self.ex.world, len(batch.ops)))
                if batch.quantile_reqs:
                    # ApproxQuantile digests: every rank's PercentileDigest (serialized), merged in rank
                    # order with QuantileSummaries.merge — as Spark merges per-partition digests
                    from .quantiles import PercentileDigest
                    merged = []
                    for dg in local_q:
                        acc = None
                        for blob in self.ex.all_gather_blobs(dg.serialize()):
                            d = PercentileDigest.deserialize(blob)
                            acc = d if acc is None else acc.merge(d)
                        merged.append(acc)
                    states.quantiles = merged
                for a, ops in zip(shareable, offsets):
                    try:
                        results[a] = a.metricFromAggregationResult(states, ops)
                    except Exception as e:
                        results[a] = a.toFailureMetric(e)
            except Exception as e:
                for a in shareable:
                    results[a] = a.toFailureMetric(e)
        by_cols = {}
        for a in passed:
            if isinstance(a, Histogram) and a.binningUdf is not None:
                # the binning UDF is a host function of this process; the sharded path groups raw keys
                results[a] = a.toFailureMetric(UnsupportedOnDevice(
                    "Histogram with a binningUdf is not supported by the multi-GPU runner"))
                continue
            if isinstance(a, (GroupingAnalyzer, Histogram)):
                cols = tuple(a.groupingColumns()) if isinstance(a, GroupingAnalyzer) else (a.column,)
                by_cols.setdefault(cols, []).append(a)
        for cols, group in by_cols.items():
            try:
                freq = self._frequencies(shard, list(cols))
            except Exception as e:
                for a in group:
                    results[a] = a.toFailureMetric(wrap_if_necessary(e))
                continue
            for a in group:
                results[a] = self._grouping_metric(a, freq)
        return AnalyzerContext(results)

    def _kll_metrics(self, shard, analyzers, results):
        """KLLRunner.computeKLLSketchesInExtraPass (R/KLLRunner.scala:91-116) over row shards: each rank
        sketches its shard as one partition (dq_kll_sketch), the KLLState bytes are all-gathered and merged
        in rank order with KLLState.sum — the reference's treeReduce over partition sketches."""
        from .kll import KLLState, DEFAULT_SKETCH_SIZE, DEFAULT_SHRINKING_FACTOR
        params = {}
        for a in analyzers:
            params[a.column] = a.kllParameters
        merged = {}
        for column, p in params.items():
            size, f = (p.sketchSize, p.shrinkingFactor) if p is not None else \
                (DEFAULT_SKETCH_SIZE, DEFAULT_SHRINKING_FACTOR)
            blob, local_err = None, None
            try:
                blob = self.local.kll_state(shard, column, size, f)
            except Exception as e:
                local_err = e
            agreed = self._agree(local_err)
            if agreed is not None:
                merged[column] = agreed
                continue
            try:
                acc = None
                for b in self.ex.all_gather_blobs(blob):
                    st = KLLState.fromBytes(b)
                    acc = st if acc is None else acc.sum(st)
                merged[column] = acc
            except Exception as e:
                merged[column] = e
        for a in analyzers:
            st = merged[a.column]
            results[a] = a.toFailureMetric(st) if isinstance(st, Exception) else a.calculateMetric(st)

    def _frequencies(self, shard, cols):
        if len(cols) != 1 or shard[cols[0]].spark_type == N.TYPE_STRING:
            raise UnsupportedOnDevice(
                "multi-GPU grouping supports one fixed-width key column (strings / multi-column: single GPU)")
        column = shard[cols[0]]
        local_err = None
        try:
            keys, send, nulls = self.local.partition(column, self.ex.world)
        except Exception as e:
            local_err = e
        agreed = self._agree(local_err)
        if agreed is not None:
            raise agreed
        owned = self.ex.all_to_all_keys(keys, send)
        local_err, local_table = None, None
        try:
            local_table = self.local.frequencies_of_keys(owned)
        except Exception as e:
            local_err = e
        agreed = self._agree(local_err)
        if agreed is not None:
            raise agreed
        taking, nulls_g = self.ex.all_reduce_i64([int(local_table.num_rows), nulls])
        return DistributedFrequencies(self.ex, local_table, column, taking, nulls_g)

    def _grouping_metric(self, a, freq):
        if isinstance(a, Histogram):
            try:
                total = freq.num_rows + freq.null_rows
                details = {}
                from .analyzers import _hist_key
                for key, c in freq.top(a.maxDetailBins):
                    details[_hist_key(key[0], freq.column)] = DistributionValue(int(c), int(c) / total)
                return HistogramMetric(a.column, Success(Distribution(details, freq.num_groups)))
            except Exception as e:
                return HistogramMetric(a.column, Failure(wrap_if_necessary(e)))
        if isinstance(a, ScanShareableFrequencyBasedAnalyzer):
            state = FrequenciesAndNumRows(freq, freq.num_rows, a.groupingColumns())
            state.summary = lambda entropy_rows=None: freq.summary(entropy_rows)
            return a.computeMetricFrom(state)
        return a.toFailureMetric(MetricCalculationRuntimeException(
            "%s is not supported by the multi-GPU runner" % type(a).__name__))
