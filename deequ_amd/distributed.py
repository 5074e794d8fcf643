"""Row-sharded multi-GPU AnalysisRunner: one process per GPU, torch.distributed
(backend "nccl" = RCCL over xGMI; "gloo" for CPU tests).

Scan-shareable analyzers: every rank runs the fused scan over its row shard, the fixed-size dq_state
records of all ranks are all-gathered in ONE collective, and every rank folds them in rank order
with the reference semigroup merges (dq_state_merge = State.sum, e.g. A/StandardDeviation.scala:37-44)
— deterministic and identical on every rank; a plain all-reduce cannot express the Chan merge.

Grouping analyzers (any key columns: fixed-width, strings, several columns): every rank builds the frequency
table of its shard (the partition-local pre-aggregation of Spark's groupBy), exports its groups as a GroupBlock
(key columns at the groups' representative rows + counts, deequ_amd/groups.py) and sends each group to the owner
rank picked by a hash of its key, in one all-to-all. Each owner rebuilds one table over what it received, weighted
by the counts, so duplicates across ranks merge and group sets are disjoint across ranks. The global numRows is an
all-reduce; #groups / #unique are sums; entropy terms use the global numRows and their per-rank sums are folded in
rank order (A/GroupingAnalyzers.scala:53-79, R/AnalysisRunner.scala:480-548). MutualInformation runs the joint
groups through two owners: by hash(x), where every x's marginal px is complete, then by hash(y), where py is, and
sums the terms (A/MutualInformation.scala:35-97).

The per-rank compute is behind `GpuLocal` (libdq.so); the collective choreography is shared with the
CPU test double in tests/test_distributed_gloo.py.
"""
import ctypes
import math

import numpy as np

from . import native as N
from . import engine
from . import groups as G
from .analyzers import (ScanShareableAnalyzer, GroupingAnalyzer, ScanShareableFrequencyBasedAnalyzer, Histogram,
                        MutualInformation, FrequenciesAndNumRows, Preconditions, metricFromFailure, metricFromValue,
                        metricFromEmpty)
from .metrics import Entity
from .table import Column
from .metrics import (HistogramMetric, Distribution, DistributionValue, Success, Failure, wrap_if_necessary,
                      MetricCalculationRuntimeException, UnsupportedOnDevice)
from .runners import AnalyzerContext, ScanBatch, ScanResult


def fold_states(raw, world, nops):
    """Rank-ordered semigroup fold of all-gathered dq_state records (rank-major bytes), in one
    dq_state_fold call."""
    raw = np.ascontiguousarray(np.asarray(raw, dtype=np.uint8))
    return N.fold_states(raw, world, nops)


def _signed64(c):
    return c - (1 << 64) if c >= 1 << 63 else c


_MIX_C1, _MIX_C2 = _signed64(0xBF58476D1CE4E5B9), _signed64(0x94D049BB133111EB)


def owner_ranks(torch, keys, world):
    """Owner rank of each canonical 64-bit key (int64 tensor): (mix64(key) >> 32) % world, the splitmix64 finalizer
    of freq.hip / groups.py on wrapping int64 arithmetic (logical shifts masked out of torch's arithmetic ones).
    Raw canonical bits would not do: integer-valued DOUBLE keys have all-zero low bits and FLOAT keys zero high
    bits, which would send every such group to one rank."""
    z = keys ^ ((keys >> 30) & 0x3FFFFFFFF)
    z = z * _MIX_C1
    z = z ^ ((z >> 27) & 0x1FFFFFFFFF)
    z = z * _MIX_C2
    z = z ^ ((z >> 31) & 0x1FFFFFFFF)
    return torch.remainder((z >> 32) & 0xFFFFFFFF, world)


_M64 = (1 << 64) - 1


def _i64(v):
    """A 64-bit pattern as a signed int64 (for an int64 tensor)."""
    v &= _M64
    return v - (1 << 64) if v >> 63 else v


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

    def all_gather_i64(self, values):
        """A fixed-length int64 vector of every rank, in rank order."""
        t = self.torch.tensor(values, dtype=self.torch.int64, device=self.device)
        out = self.torch.empty(self.world * len(values), dtype=self.torch.int64, device=self.device)
        self.dist.all_gather_into_tensor(out, t, group=self.group)
        flat = [int(v) for v in out.cpu().tolist()]
        return [flat[r * len(values):(r + 1) * len(values)] for r in range(self.world)]

    def all_gather_f64(self, value):
        t = self.torch.tensor([value], dtype=self.torch.float64, device=self.device)
        out = self.torch.empty(self.world, dtype=self.torch.float64, device=self.device)
        self.dist.all_gather_into_tensor(out, t, group=self.group)
        return out.cpu().tolist()

    def all_to_all_tensors(self, tensors, send_counts):
        """Rows of each tensor (same leading length, grouped by destination rank, send_counts[r] rows to rank r) to
        their destination ranks, on the exchange device (RCCL over xGMI for nccl): the received tensors, in source
        rank order, and the received counts."""
        torch = self.torch
        sc = send_counts.to(device=self.device, dtype=torch.int64)
        rc = torch.empty_like(sc)
        self.dist.all_to_all_single(rc, sc, group=self.group)
        send = [int(v) for v in sc.cpu().tolist()]
        recv = [int(v) for v in rc.cpu().tolist()]
        out = []
        for t in tensors:
            src = t.to(self.device).contiguous()
            dst = torch.empty(sum(recv), dtype=t.dtype, device=self.device)
            self.dist.all_to_all_single(dst, src, output_split_sizes=recv, input_split_sizes=send, group=self.group)
            out.append(dst)
        return out, recv

    def all_to_all_blobs(self, blobs):
        """blobs[r] goes to rank r; returns the blobs every rank sent to this one, in rank order."""
        torch = self.torch
        sizes = [len(b) for b in blobs]
        sc = torch.tensor(sizes, dtype=torch.int64, device=self.device)
        rc = torch.empty_like(sc)
        self.dist.all_to_all_single(rc, sc, group=self.group)
        recv = [int(v) for v in rc.cpu().tolist()]
        send = torch.frombuffer(bytearray(b"".join(blobs) or b"\0"), dtype=torch.uint8)[:sum(sizes)].to(self.device)
        out = torch.empty(sum(recv), dtype=torch.uint8, device=self.device)
        self.dist.all_to_all_single(out, send, output_split_sizes=recv, input_split_sizes=sizes, group=self.group)
        raw = out.cpu().numpy().tobytes()
        res, at = [], 0
        for n in recv:
            res.append(raw[at:at + n])
            at += n
        return res


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

    def group_block(self, shard, cols, include_nulls):
        """This shard's groups over `cols` (dq_frequencies on the GPU), as a host GroupBlock."""
        ft = engine.frequencies(shard, cols, include_nulls)
        keys, counts = ft.export_raw()
        s = ft.summary(None)
        if ft.key_kind() == N.FREQ_KEYS_VALUES:
            c = shard[cols[0]]
            columns = [G.column_from_canonical(c.name, c.spark_type, keys, c.decimal_precision, c.decimal_scale)]
        else:
            columns = [G.take(_host_column(shard[c]), keys) for c in cols]
        return G.GroupBlock(columns, counts, s["num_rows"], s["null_count"])

    def pair_export(self, shard, col, include_nulls):
        """This shard's table over one fixed-width key column as device (canonical key, count) int64 tensors, plus
        its rows taking part and its NULL-key rows; None when the table is not keyed by values."""
        import torch
        ft = engine.frequencies(shard, [col], include_nulls)
        if ft.key_kind() != N.FREQ_KEYS_VALUES:
            return None
        n = ft.num_groups
        keys = torch.empty(max(n, 1), dtype=torch.int64, device="cuda")
        counts = torch.empty(max(n, 1), dtype=torch.int64, device="cuda")
        torch.cuda.current_stream().synchronize()  # allocated on torch's stream; written on the context's
        ctx = engine.ctx()
        got = ctx.lib.dq_freq_export_device(ctx.handle, ft.handle, n, keys.data_ptr(), counts.data_ptr())
        if got < 0:
            raise N.NativeError(int(got), "dq_freq_export_device: %s" % ctx.last_error())
        ctx.synchronize()
        s = ft.summary(None)
        keys, counts = keys[:got], counts[:got]
        return keys, counts, int(counts.sum().item()) if got else 0, int(s["null_count"])

    def pairs_table(self, key_type, keys, counts, decimal_scale=0):
        """The owner's table of the (canonical key, count) pairs it received (device tensors; duplicates add)."""
        import torch
        keys = keys.to("cuda").contiguous()
        counts = counts.to("cuda").contiguous()
        torch.cuda.current_stream().synchronize()
        n = int(keys.numel())
        return engine.FrequencyTable.from_pairs(key_type, (keys.data_ptr(), n), (counts.data_ptr(), n),
                                                int(counts.sum().item()) if n else 0, 0, decimal_scale,
                                                device_ptrs=True)

    def owned_table(self, block, include_nulls):
        """The owner's table over the groups it received, weighted by their counts (dq_frequencies_ex)."""
        return engine.frequencies(block.table(), block.names, include_nulls, weights=block.counts)

    def table_summary(self, table, n):
        return table.summary(n)

    def top_block(self, table, block, k):
        keys, counts = table.top_raw(k)
        return self._block_of(table, block, keys, counts)

    def merged_block(self, table, block):
        keys, counts = table.export_raw()
        return self._block_of(table, block, keys, counts)

    def row_counts(self, block, cols):
        """Per group of `block`: the total count of the groups sharing its `cols` key (0 when that key is NULL)."""
        return engine.frequencies(block.table(), cols, False, weights=block.counts).row_counts()

    def cast_column(self, shard, name, to_type):
        from .profiles import _cast_column
        return _cast_column(shard, name, to_type)

    @staticmethod
    def _block_of(table, block, keys, counts):
        if table.key_kind() == N.FREQ_KEYS_VALUES:
            c = block.columns[0]
            return G.GroupBlock([G.column_from_canonical(c.name, c.spark_type, keys, c.decimal_precision,
                                                         c.decimal_scale)], counts)
        sub = block.subset(keys)
        return G.GroupBlock(sub.columns, counts)


def _host_column(col):
    """A column's host buffers (device-only columns are copied back)."""
    if col.values is not None or col.device is None:
        return col
    from .table import Column
    d = col.device
    vals = d["values"].cpu().numpy()
    if col.spark_type != N.TYPE_STRING:
        from .table import NUMPY_OF
        vals = vals.view(NUMPY_OF[col.spark_type])[:col.length]
    validity = d["validity"].cpu().numpy() if d.get("validity") is not None else None
    offsets = d["offsets"].cpu().numpy() if d.get("offsets") is not None else None
    return Column(col.name, col.spark_type, vals, validity, offsets, col.decimal_precision, col.decimal_scale,
                  length=col.length)


class DistributedFrequencies:
    """Global view of a grouping whose groups are spread over the ranks by owner (disjoint key sets)."""

    def __init__(self, runner, table, owned, column, num_rows, null_rows):
        self.runner, self.ex, self.local = runner, runner.ex, runner.local
        self.table, self.owned, self.schema, self.column = table, owned, owned.schema(), column
        self.num_rows = num_rows  # global rows taking part (excluding Histogram's all-NULL rows)
        self.null_rows = null_rows  # global all-NULL rows (Histogram's NULL group)
        self._summary = {}

    def summary(self, n=None):
        n = self.num_rows if n is None else n
        if n not in self._summary:
            s = self.runner._local_step(lambda: self.local.table_summary(self.table, n))
            groups, unique = self.ex.all_reduce_i64([s["num_groups"], s["num_unique"]])
            # the ranks' exact fixed-point entropy sums add exactly: the same bits for any world size
            fx = s["entropy_fx"]
            rows = self.ex.all_gather_i64([_i64(fx & _M64), _i64(fx >> 64), 0 if math.isfinite(s["entropy"]) else 1])
            total = sum(((hi << 64) | (lo & _M64)) for lo, hi, _ in rows)
            ent = N.fx_to_float(total) if not any(bad for _, _, bad in rows) else float("nan")
            self._summary[n] = {"num_rows": self.num_rows, "num_groups": groups, "num_unique": unique,
                                "entropy": ent}
        return self._summary[n]

    @property
    def num_groups(self):
        return self.summary()["num_groups"] + (1 if self.null_rows else 0)

    def top(self, k):
        """The k largest groups over all ranks: each owner's top k, all-gathered and merged."""
        blob = self.runner._local_step(lambda: G.pack(self.local.top_block(self.table, self.owned, k)))
        cands = []
        for b in self.ex.all_gather_blobs(blob):
            blk = G.unpack(b, self.schema)
            cands += list(zip(blk.keys(), blk.counts.tolist()))
        if self.null_rows:
            cands.append(((None,) * len(self.schema), self.null_rows))
        cands.sort(key=lambda kv: -kv[1])
        return cands[:k]


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
                try:
                    results[a] = self._binned_histogram(shard, a)
                except Exception as e:
                    results[a] = a.toFailureMetric(wrap_if_necessary(e))
                continue
            if isinstance(a, MutualInformation):
                try:
                    results[a] = self._mutual_information(shard, a)
                except Exception as e:
                    results[a] = a.toFailureMetric(wrap_if_necessary(e))
                continue
            if isinstance(a, Histogram):
                by_cols.setdefault(((a.column,), True), []).append(a)
            elif isinstance(a, GroupingAnalyzer):
                by_cols.setdefault((tuple(a.groupingColumns()), False), []).append(a)
        for (cols, include_nulls), group in by_cols.items():
            try:
                freq = self._frequencies(shard, list(cols), include_nulls)
            except Exception as e:
                for a in group:
                    results[a] = a.toFailureMetric(wrap_if_necessary(e))
                continue
            for a in group:
                results[a] = self._grouping_metric(a, freq)
        return AnalyzerContext(results)

    def _binned_histogram(self, shard, a):
        """Histogram with a binningUdf: every rank bins its shard's distinct values (the UDF is a deterministic host
        function of the value, so a value lands in the same bin on every rank) and the per-rank bin counts add up —
        the same (bin, count) table as binning the whole column (A/Histogram.scala:59-65)."""
        import json
        def binned():
            block = self.local.group_block(shard, [a.column], False)
            groups = ((k[0], c) for k, c in zip(block.keys(), block.counts.tolist()))
            col = shard[a.column] if getattr(a, "udfInputAsString", False) else None
            return a.bin_groups(groups, shard.count() - block.num_rows, col)
        local = self._local_step(binned)
        blob = json.dumps([[k[0], int(c)] for k, c in local.items()]).encode()
        bins = {}
        for b in self.ex.all_gather_blobs(blob):
            for label, c in json.loads(b.decode()):
                bins[(label,)] = bins.get((label,), 0) + c
        rows = self.ex.all_reduce_i64([shard.count()])[0]
        return a.computeMetricFrom(FrequenciesAndNumRows(bins, rows, [a.column]))

    def _local_step(self, fn):
        """Run one piece of per-rank compute, then agree on it: every rank returns its result, or every rank
        raises the first failing rank's error."""
        out, err = None, None
        try:
            out = fn()
        except Exception as e:
            err = e
        agreed = self._agree(err)
        if agreed is not None:
            raise agreed
        return out

    def _shuffle(self, block, key_columns=None, null_is_value=False):
        """Every group of this rank's `block` to its owner rank (hash of its key, or of `key_columns`): the groups
        this rank owns, from every rank, as one block."""
        world = self.ex.world

        def split():
            dest = G.owners(block, world, null_is_value, key_columns)
            return [G.pack(block, np.nonzero(dest == r)[0]) for r in range(world)]
        blobs = self._local_step(split)
        received = self.ex.all_to_all_blobs(blobs)
        schema = block.schema()
        return self._local_step(lambda: G.concat([G.unpack(b, schema) for b in received], schema))

    def _frequencies(self, shard, cols, include_nulls=False):
        if len(cols) == 1 and shard[cols[0]].spark_type != N.TYPE_STRING and hasattr(self.local, "pair_export"):
            freq = self._frequencies_pairs(shard, cols[0], include_nulls)
            if freq is not None:
                return freq
        block = self._local_step(lambda: self.local.group_block(shard, cols, include_nulls))
        owned = self._shuffle(block, null_is_value=include_nulls)
        table = self._local_step(lambda: self.local.owned_table(owned, include_nulls))
        num_rows, null_rows = self.ex.all_reduce_i64([int(owned.counts.sum()), block.null_rows])
        return DistributedFrequencies(self, table, owned, shard[cols[0]], num_rows, null_rows)

    def _frequencies_pairs(self, shard, col, include_nulls):
        """One fixed-width key column: the shard's groups stay on the device as (canonical key, count) pairs, go to
        their owner rank (a hash of the key) in one all-to-all on the exchange device (RCCL for nccl), and each owner
        builds the weighted table of the pairs it received (dq_freq_from_pairs) — groups, not rows, cross ranks and
        nothing passes through host memory. None (on every rank) when the table is not keyed by values."""
        torch = self.ex.torch
        world = self.ex.world
        local = self._local_step(lambda: self.local.pair_export(shard, col, include_nulls))
        if self.ex.all_reduce_i64([0 if local is None else 1])[0] != world:
            return None
        keys, counts, rows, nulls = local

        def route():
            owner = owner_ranks(torch, keys, world)
            order = torch.sort(owner, stable=True).indices
            return keys[order], counts[order], torch.bincount(owner, minlength=world)
        k_sorted, c_sorted, send = self._local_step(route)
        (rk, rc), _ = self.ex.all_to_all_tensors([k_sorted, c_sorted], send)
        c = shard[col]
        table = self._local_step(lambda: self.local.pairs_table(c.spark_type, rk, rc, c.decimal_scale))
        num_rows, null_rows = self.ex.all_reduce_i64([rows, nulls])
        stub = G.GroupBlock([G.column_from_canonical(c.name, c.spark_type, np.zeros(0, dtype=np.int64),
                                                     c.decimal_precision, c.decimal_scale)], np.zeros(0, dtype=np.int64))
        return DistributedFrequencies(self, table, stub, c, num_rows, null_rows)

    def _mutual_information(self, shard, a):
        """MutualInformation over row shards (A/MutualInformation.scala:35-97): the joint (x, y) groups go to their
        owner by hash(x), which merges them (pxy) and sees every group of each of its x values (px); then to their
        owner by hash(y) (py); every rank sums its terms and the per-rank sums are folded in rank order."""
        x, y = a.columns
        joint = self._local_step(lambda: self.local.group_block(shard, [x, y], False))
        by_x = self._shuffle(joint, key_columns=[x])

        def merge_x():
            table = self.local.owned_table(by_x, False)
            merged = self.local.merged_block(table, by_x)
            px = self.local.row_counts(merged, [x])
            return merged.with_column(Column("__deequ_px", N.TYPE_LONG, np.ascontiguousarray(px, dtype=np.int64)))
        merged = self._local_step(merge_x)
        by_y = self._shuffle(merged, key_columns=[y])

        def terms():
            py = self.local.row_counts(by_y, [y]).astype(np.float64)
            both = ~by_y.column(x).null_mask() & ~by_y.column(y).null_mask()
            pxy = by_y.counts[both].astype(np.float64)
            px = np.asarray(by_y.column("__deequ_px").values)[both].astype(np.float64)
            return pxy, px, py[both]
        pxy, px, py = self._local_step(terms)
        total, nterms = self.ex.all_reduce_i64([int(merged.counts.sum()), len(pxy)])
        inst = ",".join(a.columns)
        if nterms == 0:
            return metricFromEmpty(a, "MutualInformation", inst, Entity.Mutlicolumn)
        n = float(total)
        # the reference's miUdf, term by term: (pxy / total) * log((pxy / total) / ((px / total) * (py / total)))
        t = (pxy / n) * np.log((pxy / n) / ((px / n) * (py / n)))
        value = math.fsum(self.ex.all_gather_f64(math.fsum(t.tolist())))
        return metricFromValue(value, "MutualInformation", inst, Entity.Mutlicolumn)

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

    def profile(self, shard, restrictToColumns=None, lowCardinalityHistogramThreshold=None, kllParameters=None,
                predefinedTypes=None):
        """ColumnProfiler.profile (M/profiles/ColumnProfiler.scala:91-208) over row shards: the same three passes,
        each through this runner — the generic and numeric statistics as sharded scans (+ KLL), the low-cardinality
        histograms as owner-sharded groupings (computeHistograms, :564-606). Every rank returns the same profiles."""
        from .profiles import ColumnProfiler
        thr = ColumnProfiler.DEFAULT_CARDINALITY_THRESHOLD if lowCardinalityHistogramThreshold is None \
            else lowCardinalityHistogramThreshold
        return ColumnProfiler.profile(shard, restrictToColumns, False, thr, kllParameters, predefinedTypes,
                                      passes=ShardedProfilerPasses(self))

    def _profile_histograms(self, shard, targets):
        from .analyzers import _hist_key
        out = {}
        for name in targets:
            freq = self._frequencies(shard, [name], include_nulls=True)
            total = freq.num_rows + freq.null_rows
            values = {}
            for key, c in freq.top(freq.num_groups):
                k = Histogram.NullFieldReplacement if key[0] is None else _hist_key(key[0], shard[name])
                values[k] = DistributionValue(int(c), c / total)
            out[name] = Distribution(values, len(values))
        return out

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


class ShardedProfilerPasses:
    """The ColumnProfiler's passes over this rank's row shard (see DistributedAnalysisRunner.profile)."""

    def __init__(self, runner):
        self.runner = runner

    def run(self, data, analyzers):
        return self.runner.run(data, analyzers)

    def cast(self, data, name, to_type):
        # per-row casts need no exchange; a failure still has to be agreed on before the next collective
        return self.runner._local_step(lambda: self.runner.local.cast_column(data, name, to_type))

    def histograms(self, data, targets):
        return self.runner._profile_histograms(data, targets)
