"""AnalysisRunner / AnalysisRunBuilder / AnalyzerContext / state providers — the deequ runner API
(R/AnalysisRunner.scala, R/AnalysisRunBuilder.scala, R/AnalyzerContext.scala, A/StateProvider.scala)
driving the MI355X engine. The scan-shareable analyzers of a run become ONE dq_scan call (one fused
pass over HBM), exactly where the reference issues one `data.agg(...)` Spark job."""
import json
import os
import sys
import threading

from . import native as N
from . import engine
from .analyzers import (Analyzer, ScanShareableAnalyzer, GroupingAnalyzer, ScanShareableFrequencyBasedAnalyzer,
                        FrequencyBasedAnalyzer, KLLSketch, Preconditions, Size, computeFrequencies, STATE_ONLY,
                        ApproxQuantile, ApproxQuantiles, Histogram)
from .analyzers import merge as merge_states
from .expr import compile_predicate
from .metrics import DoubleMetric, Success, UnsupportedOnDevice
from .table import ChunkedTable


def stream_chunk_rows():
    """DQ_STREAM_CHUNK_ROWS: host-resident tables larger than this many rows are scanned in streamed chunks
    (copy of the next chunk overlapped with the scan of the current one) instead of being staged whole."""
    v = os.environ.get("DQ_STREAM_CHUNK_ROWS")
    return int(float(v)) if v else 0


class _Pending:
    """A helper thread's result (its exception re-raised by result())."""

    def __init__(self, fn, name="dq-helper"):
        self.value, self.error = None, None
        self.thread = threading.Thread(target=self._run, args=(fn,), daemon=True, name=name)
        self.thread.start()

    def _run(self, fn):
        try:
            self.value = fn()
        except BaseException as e:  # handed to the caller
            self.error = e

    def join(self):
        self.thread.join()

    def result(self):
        self.thread.join()
        if self.error is not None:
            raise self.error
        return self.value


class _Done:
    """A result computed on the calling thread, behind _Pending's interface."""

    def __init__(self, value):
        self.value, self.error = value, None

    def join(self):
        pass

    def result(self):
        return self.value


def _beside(fn, slot, priority=None):
    """Run fn in a helper thread on a second context of this thread's device (own stream and scratch, leased to this
    helper alone), or None when the work must stay on this thread (DQ_RUN_SERIAL, a multi-device context, or already
    on a helper context). The helper selects the device before any engine call (a new thread starts on device 0)."""
    if os.environ.get("DQ_RUN_SERIAL") or os.environ.get("DQ_DEVICES"):
        return None
    if getattr(engine._local, "ctx", None) is not None and not getattr(engine._local, "helpers_ok", False):
        return None  # on a helper context: nothing nests (a runAsync thread is the one exception, one level deep)
    if priority is None:  # a runAsync thread's helpers run at its priority; others at DQ_HELPER_PRIORITY (default 0)
        priority = getattr(engine._local, "helper_priority", None)
        if priority is None:
            priority = int(os.environ.get("DQ_HELPER_PRIORITY", 0))
    dev = engine.device()
    aux = N.lease_aux_context(dev, slot, priority)

    def run():
        try:
            torch = sys.modules.get("torch")
            if torch is not None and torch.cuda.is_initialized():
                torch.cuda.set_device(dev)
            with engine.using_context(aux):
                return fn()
        finally:
            N.release_aux_context(aux)
    try:
        return _Pending(run, "dq-helper-" + slot)
    except BaseException:
        N.release_aux_context(aux)
        raise


class _Helpers:
    """The helper threads of one run: every one is joined before the run returns or raises (an exception on this
    thread or in one helper never leaves another helper driving its context over buffers the caller may free); the
    first error re-raised is the first one result() meets."""

    def __init__(self):
        self.pending = []

    def beside(self, fn, slot):
        h = _beside(fn, slot)
        if h is not None:
            self.pending.append(h)
        return h

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        for h in self.pending:
            h.join()
        return False


class ScanResult(list):
    """dq_state per op, plus the PercentileDigest of each quantile request."""
    quantiles = ()


class ScanBatch:
    """The dq_op list of one fused scan: deduplicated ops, predicates compiled once per string.
    ApproxQuantile(s) register quantile requests, one dq_quantile_summary per (column, relativeError)
    after the fused pass (they share one digest, as Spark computes identical digests)."""

    def __init__(self, data):
        self.data = data
        self.names = list(data.columns)
        self.col_index = {n: i for i, n in enumerate(self.names)}
        self.preds = []
        self.pred_index = {}
        self.ops = []
        self.op_index = {}
        self.quantile_reqs = []
        self.quantile_index = {}

    def predicate(self, text):
        if text not in self.pred_index:
            self.preds.append(compile_predicate(text, self.col_index, self._column_types()))
            self.pred_index[text] = len(self.preds) - 1
        return self.pred_index[text]

    def _column_types(self):
        types = {}
        for n in self.names:
            try:
                types[n] = self.data[n].spark_type
            except (KeyError, TypeError, AttributeError):
                pass
        return types

    def regex_predicate(self, column, pattern):
        """PatternMatch's `regexp_extract(col, pattern, 0) != ""` as the [COL, REGEX] program."""
        from .expr import CompiledPredicate
        from .regex import compile_regex
        key = ("\x00regex", column, pattern)
        if key not in self.pred_index:
            if column not in self.col_index:
                from .metrics import NoSuchColumnException
                raise NoSuchColumnException("Input data does not include column %s!" % column)
            image = compile_regex(pattern).to_bytes()
            k = N.DqConst()
            k.tag, k.str_len, k.str_offset = N.V_STRING, len(image), 0
            self.preds.append(CompiledPredicate("regexp_extract(%s, %r, 0) != ''" % (column, pattern),
                                                [N.P_COL, self.col_index[column], N.P_REGEX, 0], [k], image,
                                                [column]))
            self.pred_index[key] = len(self.preds) - 1
        return self.pred_index[key]

    def add_op(self, kind, columns=(), where=None, predicate=None, predicate_index=None):
        cols = [self.col_index[c] if c in self.col_index else -1 for c in columns]
        for c, name in zip(cols, columns):
            if c < 0:
                from .metrics import NoSuchColumnException
                raise NoSuchColumnException("Input data does not include column %s!" % name)
        w = self.predicate(where) if where is not None else -1
        p = self.predicate(predicate) if predicate is not None else -1
        if predicate_index is not None:
            p = predicate_index
        key = (kind, tuple(cols), w, p)
        if key not in self.op_index:
            op = N.DqOp()
            op.kind = kind
            op.column[0] = cols[0] if len(cols) > 0 else -1
            op.column[1] = cols[1] if len(cols) > 1 else -1
            op.where = w
            op.predicate = p
            self.ops.append(op)
            self.op_index[key] = len(self.ops) - 1
        return self.op_index[key]

    def add_quantile(self, column, relativeError):
        if column not in self.col_index:
            from .metrics import NoSuchColumnException
            raise NoSuchColumnException("Input data does not include column %s!" % column)
        key = (column, float(relativeError))
        if key not in self.quantile_index:
            self.quantile_reqs.append(key)
            self.quantile_index[key] = len(self.quantile_reqs) - 1
        return self.quantile_index[key]

    def native_columns(self):
        return [self.data[n].native() for n in self.names]

    def run(self, out_device_ptr=None):
        res = ScanResult()
        if self.ops:
            chunk = stream_chunk_rows()
            host = all(self.data[n].device is None for n in self.names)
            if chunk and host and out_device_ptr is None and self.data.nrows > chunk:
                # host-resident table streamed through HBM in row chunks (dq_scan_streamed)
                got = engine.ctx().scan_streamed(self.native_columns(), self.data.nrows, self.ops,
                                                 [p.to_native() for p in self.preds], chunk)
            else:
                got = engine.ctx().scan(self.native_columns(), self.data.nrows, self.ops,
                                        [p.to_native() for p in self.preds], out_device_ptr=out_device_ptr)
            if got is not None:
                res.extend(got)
        if self.quantile_reqs:
            from .quantiles import PercentileDigest, DEFAULT_HEAD_SIZE
            # below the head-buffer size Spark's digest is a function of the sorted values: get all of them (rank
            # spacing 1) and rebuild Spark's own summary; above it, a bounded summary. Every request in one call.
            small = self.data.nrows < DEFAULT_HEAD_SIZE
            got = engine.ctx().quantile_summaries(
                [(self.data[column].native_parts(), 0.0 if small else rel) for column, rel in self.quantile_reqs])
            res.quantiles = []
            for (column, rel), (vals, ranks, n) in zip(self.quantile_reqs, got):
                if small:
                    res.quantiles.append(PercentileDigest.spark_single_partition(rel, vals))
                else:
                    res.quantiles.append(PercentileDigest.from_order_statistics(rel, vals, ranks, n))
        return res


class AnalyzerContext:
    """R/AnalyzerContext.scala:29-105."""

    def __init__(self, metricMap=None):
        self.metricMap = dict(metricMap or {})

    @staticmethod
    def empty():
        return AnalyzerContext()

    @property
    def allMetrics(self):
        return list(self.metricMap.values())

    def metric(self, analyzer):
        return self.metricMap.get(analyzer)

    def __add__(self, other):  # `++`: right-hand side wins
        m = dict(self.metricMap)
        m.update(other.metricMap)
        return AnalyzerContext(m)

    @staticmethod
    def successMetricsAsJson(analyzerContext, forAnalyzers=()):
        rows = []
        for a, m in analyzerContext.metricMap.items():
            if forAnalyzers and a not in forAnalyzers:
                continue
            if not m.value.isSuccess:
                continue
            for dm in m.flatten():
                rows.append({"entity": str(dm.entity), "instance": dm.instance, "name": dm.name,
                             "value": dm.value.get()})
        return json.dumps(rows)


class InMemoryStateProvider:
    """A/StateProvider.scala:47-69."""

    def __init__(self):
        self.states = {}

    def load(self, analyzer):
        return self.states.get(analyzer)

    def persist(self, analyzer, state):
        self.states[analyzer] = state


class Analysis:
    """A/Analysis.scala: a list of analyzers (deprecated entry point kept for the reference tests)."""

    def __init__(self, analyzers=None):
        self.analyzers = list(analyzers or [])

    def addAnalyzer(self, analyzer):
        return Analysis(self.analyzers + [analyzer])

    def addAnalyzers(self, analyzers):
        return Analysis(self.analyzers + list(analyzers))

    def run(self, data, aggregateWith=None, saveStatesWith=None):
        return AnalysisRunner.doAnalysisRun(data, self.analyzers, aggregateWith, saveStatesWith)


class AnalysisRunBuilder:
    """R/AnalysisRunBuilder.scala:27-116."""

    def __init__(self, data):
        self.data = data
        self.analyzers = []
        self._aggregateWith = None
        self._saveStatesWith = None

    def addAnalyzer(self, analyzer):
        self.analyzers.append(analyzer)
        return self

    def addAnalyzers(self, analyzers):
        self.analyzers.extend(analyzers)
        return self

    def aggregateWith(self, stateLoader):
        self._aggregateWith = stateLoader
        return self

    def saveStatesWith(self, statePersister):
        self._saveStatesWith = statePersister
        return self

    def run(self):
        return AnalysisRunner.doAnalysisRun(self.data, self.analyzers, self._aggregateWith, self._saveStatesWith)

    def runAsync(self, priority=0):
        """run() on a helper context of this thread's device (own stream and scratch) in a helper thread, beside the
        caller's next GPU work: a Spark application submitting two jobs from two threads (e.g. the ColumnProfiler's
        passes and a VerificationSuite over the same table). Returns a handle: result() is the AnalyzerContext (a
        failure re-raised), join() waits. The caller joins it before it frees the table. Where run() cannot go to a
        helper (DQ_RUN_SERIAL, a multi-device context, already on a helper) it runs here and the handle is done.
        `priority` (1 high, 0 normal, -1 low) is the helper stream's HIP priority (dq_set_priority): 1 lets this run's
        kernels dispatch ahead of the caller's when it is the longer chain."""
        def run():
            # DQ_ASYNC_NESTED=1: the run's own helpers (its grouping sets beside its quantile / scan passes) may start
            # from this thread, one level deep, at the run's priority. Off by default: beside the ColumnProfiler the
            # extra contexts only add contention (C5 step 156-171 ms nested against 140-143 ms with the whole run on
            # one helper context, profiles/r06/c5_async_nested_ab_r06aa.txt)
            engine._local.helpers_ok = os.environ.get("DQ_ASYNC_NESTED", "0") == "1"
            engine._local.helper_priority = priority
            try:
                return self.run()
            finally:
                engine._local.helpers_ok = False
                engine._local.helper_priority = None
        h = _beside(run, "async", priority)
        return h if h is not None else _Done(self.run())


class KLLRunner:
    """R/KLLRunner.scala:91-179: KLL sketches in an extra pass. Each column's sketch is built by
    dq_kll_sketch on the GPU as ONE partition holding the rows in order (KLLRunner.sketchPartitions over a
    single-partition DataFrame); partition sketches of a sharded table merge with KLLState.sum, as the
    reference's treeReduce does."""

    _SUPPORTED = ("DoubleType", "FloatType", "ByteType", "ShortType", "IntegerType", "LongType")

    @staticmethod
    def sketch_column(data, column, sketchSize, shrinkingFactor):
        from .kll import KLLState
        t = data.schema[column]
        if t not in KLLRunner._SUPPORTED:  # KLLRunner.emptySketches (:118-145)
            raise ValueError("Cannot handle %s" % t)
        raw = engine.ctx().kll_sketch(data[column].native(), data.nrows, sketchSize, shrinkingFactor)
        return KLLState.fromBytes(raw)

    @staticmethod
    def computeKLLSketchesInExtraPass(data, analyzers, aggregateWith=None, saveStatesTo=None):
        from .kll import DEFAULT_SKETCH_SIZE, DEFAULT_SHRINKING_FACTOR
        params = {}
        for a in analyzers:  # columnsAndParameters: `.toMap`, the last analyzer of a column wins
            params[a.column] = a.kllParameters
        from .kll import KLLState
        by_params = {}
        for column, p in params.items():
            size, f = (p.sketchSize, p.shrinkingFactor) if p is not None else \
                (DEFAULT_SKETCH_SIZE, DEFAULT_SHRINKING_FACTOR)
            if data.schema[column] not in KLLRunner._SUPPORTED:  # KLLRunner.emptySketches (:118-145)
                raise ValueError("Cannot handle %s" % data.schema[column])
            by_params.setdefault((size, f), []).append(column)
        sketches = {}
        for (size, f), cols in by_params.items():  # one pass over the columns sharing sketch parameters
            raws = engine.ctx().kll_sketch_columns([data[c].native() for c in cols], data.nrows, size, f)
            for c, raw in zip(cols, raws):
                sketches[c] = KLLState.fromBytes(raw)
        results = {}
        for a in analyzers:
            results[a] = a.calculateMetric(sketches[a.column], aggregateWith, saveStatesTo)
        return AnalyzerContext(results)


class AnalysisRunner:
    """R/AnalysisRunner.scala:46-548."""

    @staticmethod
    def onData(data):
        return AnalysisRunBuilder(data)

    @staticmethod
    def run(data, analysis, aggregateWith=None, saveStatesWith=None):
        return AnalysisRunner.doAnalysisRun(data, analysis.analyzers, aggregateWith, saveStatesWith)

    @staticmethod
    def doAnalysisRun(data, analyzers, aggregateWith=None, saveStatesWith=None):
        """R/AnalysisRunner.scala:97-203 (repository reuse and file output are out of scope)."""
        if not analyzers:
            return AnalyzerContext.empty()
        if isinstance(data, ChunkedTable):
            return AnalysisRunner._run_chunked(data, analyzers, aggregateWith, saveStatesWith)
        allAnalyzers = list(dict.fromkeys(analyzers))  # VerificationSuite does not dedupe; the result map does
        passed = [a for a in allAnalyzers if Preconditions.findFirstFailing(data.schema, a.preconditions()) is None]
        passed_set = set(passed)
        failed = [a for a in allAnalyzers if a not in passed_set]
        preconditionFailures = AnalyzerContext(
            {a: a.toFailureMetric(Preconditions.findFirstFailing(data.schema, a.preconditions())) for a in failed})
        grouping = [a for a in passed if isinstance(a, GroupingAnalyzer)]
        allScanning = [a for a in passed if not isinstance(a, GroupingAnalyzer)]
        kllAnalyzers = [a for a in allScanning if isinstance(a, KLLSketch)]
        scanning = [a for a in allScanning if not isinstance(a, KLLSketch)]
        by_cols = {}
        for a in grouping:
            by_cols.setdefault(tuple(sorted(a.groupingColumns())), []).append(a)
        sets = list(by_cols.items())

        def run_set(cols, group):
            _, metrics = AnalysisRunner._runGroupingAnalyzers(data, list(cols), group, aggregateWith, saveStatesWith)
            return metrics
        # the grouping builds (one per grouping-column set) and the scanning / KLL passes read the table independently:
        # each set's build runs on its own helper context meanwhile (Spark runs them as separate jobs; at most three
        # helpers, the rest -- or the last set when nothing else runs -- on this thread)
        others = bool(scanning or kllAnalyzers)
        with _Helpers() as helpers:
            here = []
            for k, (cols, group) in enumerate(sets):
                h = None
                if k < 3 and (others or k < len(sets) - 1):
                    h = helpers.beside(lambda cols=cols, group=group: run_set(cols, group), "group%d" % k)
                if h is None:
                    here.append((cols, group))
            kllMetrics = AnalyzerContext.empty()
            if kllAnalyzers:
                kllMetrics = KLLRunner.computeKLLSketchesInExtraPass(data, kllAnalyzers, aggregateWith, saveStatesWith)
            nonGrouped = AnalysisRunner._runScanningAnalyzers(data, scanning, aggregateWith, saveStatesWith)
            grouped = AnalyzerContext.empty()
            for cols, group in here:
                grouped = grouped + run_set(cols, group)
            for h in helpers.pending:
                grouped = grouped + h.result()
        return preconditionFailures + nonGrouped + grouped + kllMetrics

    @staticmethod
    def _run_chunked(data, analyzers, aggregateWith=None, saveStatesWith=None):
        """A ChunkedTable: every chunk runs the analysis (its scan, grouping and KLL passes on the GPU) and persists
        its states in memory; the chunk states (and the states of `aggregateWith`) then merge in chunk order through
        runOnAggregatedStates — Spark's partial aggregates of one `agg` over the partitions, merged by the same
        State.sum. An analyzer whose state computation failed on any chunk (an exception, not an empty state) keeps
        that chunk's failure metric. A grouping-column set with no state on any chunk (its frequencies failed on every
        chunk) does not reach the merge (the reference's findStateForParticularGrouping would require one): it keeps
        the chunk failure metrics."""
        analyzers = list(dict.fromkeys(analyzers))  # one state per analyzer: the merge adds each loader's state once
        with _Helpers() as helpers:
            return AnalysisRunner._run_chunked_body(data, analyzers, aggregateWith, saveStatesWith, helpers)

    @staticmethod
    def _run_chunked_body(data, analyzers, aggregateWith, saveStatesWith, helpers):
        # grouping analyzers: one frequency table over the whole shard (the chunks' key columns concatenated where
        # they live, int64 string offsets) instead of per-chunk tables merged through host memory -- the same
        # groups as Spark's shuffle of the partitions' partial counts (R/AnalysisRunner.scala:259-287). A
        # multi-device context (DQ_DEVICES) shards every call itself and takes neither int64 offsets nor parted
        # columns: its chunks run one by one and merge like any other state.
        whole_table = len(data.chunks) > 1 and not getattr(engine.ctx(), "multi", False)
        # Histogram (a plain Analyzer whose state is a frequency table with the NULL group) likewise: one table over
        # the shard's column, not per-chunk tables joined on the host (A/Histogram.scala:54-70)
        grouping = [a for a in analyzers if isinstance(a, GroupingAnalyzer) or
                    (isinstance(a, Histogram) and a.binningUdf is None)]
        whole = AnalyzerContext.empty()
        if grouping and whole_table:
            analyzers = [a for a in analyzers if a not in set(grouping)]
            by_set = {}
            for a in grouping:
                key = ("\x00histogram", a.column) if isinstance(a, Histogram) else tuple(sorted(a.groupingColumns()))
                by_set.setdefault(key, []).append(a)
            sets = [((k[1],) if k[0] == "\x00histogram" else k, g) for k, g in by_set.items()]
            # each grouping-column set on its own helper context (at most three; the rest, or the last set when
            # nothing else runs, on this thread), beside the other analyzers' passes (see doAnalysisRun)
            for k, (cset, group) in enumerate(sets):
                def run_set(cset=cset, group=group):
                    cols = [c for c in cset if c in data]
                    return AnalysisRunner.doAnalysisRun(data.grouping_view(cols), group, aggregateWith, saveStatesWith)
                last_here = not analyzers and k == len(sets) - 1
                h = None if last_here or k >= 3 else helpers.beside(run_set, "group%d" % k)
                if h is None:
                    whole = whole + run_set()
            if not analyzers:
                for h in helpers.pending:
                    whole = whole + h.result()
                return whole
        # ApproxQuantile(s): one summary per column over every chunk (dq_quantile_summaries reads the chunks as
        # parts), the exact order statistics of the shard -- a GK summary inside the same rank bound as the merge of
        # per-partition digests (QuantileSummaries.merge)
        quant = [a for a in analyzers if isinstance(a, (ApproxQuantile, ApproxQuantiles))]
        if quant and whole_table:
            cols = sorted({a.column for a in quant if a.column in data})
            whole = whole + AnalysisRunner.doAnalysisRun(data.parted(cols), quant, aggregateWith, saveStatesWith)
            analyzers = [a for a in analyzers if not isinstance(a, (ApproxQuantile, ApproxQuantiles))]
            if not analyzers:
                for h in helpers.pending:
                    whole = whole + h.result()
                return whole
        grouping_pending = list(helpers.pending)

        def run_chunks(indices):
            out = {}
            for i in indices:
                p = InMemoryStateProvider()
                p.states_only = True  # states only: no per-chunk metric (an empty chunk state is no failure)
                out[i] = (p, AnalysisRunner.doAnalysisRun(data.chunks[i], analyzers, saveStatesWith=p))
            return out
        # the chunks' runs are independent until the merge: the odd chunks run on a second context in a helper thread
        # while this thread runs the even ones, so one chunk's host work (KLL schedules, state extraction) overlaps
        # the other's kernels
        nchunks = len(data.chunks)
        odd = helpers.beside(lambda: run_chunks(range(1, nchunks, 2)), "chunk") if nchunks > 1 else None
        done = run_chunks(range(0, nchunks, 2) if odd is not None else range(nchunks))
        if odd is not None:
            done.update(odd.result())
        providers, failures = [], {}
        for i in range(nchunks):  # chunk order: the merge and the first failure seen are those of a serial run
            p, res = done[i]
            for a, m in res.metricMap.items():
                if not m.value.isSuccess and a not in failures:
                    failures[a] = m
            providers.append(p)
        if aggregateWith is not None:
            providers.append(aggregateWith)
        by_cols = {}
        for a in analyzers:
            if isinstance(a, GroupingAnalyzer):
                by_cols.setdefault(tuple(sorted(a.groupingColumns())), []).append(a)
        stateless = set()
        for group in by_cols.values():
            if not any(p.load(a) is not None for p in providers for a in group):
                stateless.update(group)
        merged = AnalysisRunner.runOnAggregatedStates(
            data.schema, Analysis([a for a in analyzers if a not in stateless]), providers, saveStatesWith)
        # no chunk had a state (every chunk empty for it): the metric of an empty state, as one run over all rows
        empty = {}
        for a in dict.fromkeys(analyzers):
            if a not in merged.metricMap and a not in failures:
                try:
                    empty[a] = a.computeMetricFrom(None)
                except Exception as e:
                    empty[a] = a.toFailureMetric(e)
        for h in grouping_pending:
            whole = whole + h.result()
        return merged + AnalyzerContext(empty) + AnalyzerContext(failures) + whole

    @staticmethod
    def _runScanningAnalyzers(data, analyzers, aggregateWith=None, saveStatesTo=None):
        """R/AnalysisRunner.scala:289-336: one fused dq_scan for all shareable analyzers."""
        shareable = [a for a in analyzers if isinstance(a, ScanShareableAnalyzer)]
        others = [a for a in analyzers if not isinstance(a, ScanShareableAnalyzer)]
        results = {}
        if shareable:
            try:
                batch = ScanBatch(data)
                offsets = []
                for a in shareable:
                    try:
                        offsets.append(a.addOps(batch))
                    except UnsupportedOnDevice as e:  # this engine's limitation: only this analyzer fails
                        offsets.append(None)
                        results[a] = a.toFailureMetric(e)
                states = batch.run()
                for a, ops in zip(shareable, offsets):
                    if ops is None:
                        continue
                    try:
                        results[a] = a.metricFromAggregationResult(states, ops, aggregateWith, saveStatesTo)
                    except Exception as e:  # successOrFailureMetricFrom (:340-353)
                        results[a] = a.toFailureMetric(e)
            except Exception as e:  # any failure of the shared aggregation fails every analyzer (:320-323)
                for a in shareable:
                    results[a] = a.toFailureMetric(e)
        for a in others:
            results[a] = a.calculate(data, aggregateWith, saveStatesTo)
        return AnalyzerContext(results)

    @staticmethod
    def _runGroupingAnalyzers(data, groupingColumns, analyzers, aggregateWith=None, saveStatesTo=None):
        """R/AnalysisRunner.scala:259-287 (+ runAnalyzersForParticularGrouping :480-548)."""
        try:
            freq = computeFrequencies(data, groupingColumns)
        except Exception as e:
            return 0, AnalyzerContext({a: a.toFailureMetric(e) for a in analyzers})
        if aggregateWith is not None:
            prev = aggregateWith.load(analyzers[0])
            if prev is not None:
                freq = freq.sum(prev)
        ctx = AnalysisRunner._runAnalyzersForParticularGrouping(freq, analyzers, saveStatesTo)
        return freq.numRows, ctx

    @staticmethod
    def _runAnalyzersForParticularGrouping(freq, analyzers, saveStatesTo=None):
        if getattr(saveStatesTo, "states_only", False):  # a row chunk: the merged state computes the metrics
            saveStatesTo.persist(analyzers[0], freq)
            return AnalyzerContext({a: STATE_ONLY for a in analyzers})
        results = {}
        for a in analyzers:
            try:
                results[a] = a.computeMetricFrom(freq)
            except Exception as e:
                results[a] = a.toFailureMetric(e)
        if saveStatesTo is not None:
            saveStatesTo.persist(analyzers[0], freq)
        return AnalyzerContext(results)

    @staticmethod
    def runOnAggregatedStates(schema, analysis, stateLoaders, saveStatesWith=None):
        """R/AnalysisRunner.scala:385-460: metrics from merged persisted states, no data scan."""
        if not analysis.analyzers or not stateLoaders:
            return AnalyzerContext.empty()
        analyzers = analysis.analyzers
        passed = [a for a in analyzers if Preconditions.findFirstFailing(schema, a.preconditions()) is None]
        passed_set = set(passed)
        failed = [a for a in analyzers if a not in passed_set]
        pre = AnalyzerContext({a: a.toFailureMetric(Preconditions.findFirstFailing(schema, a.preconditions()))
                               for a in failed})
        agg = InMemoryStateProvider()
        # KLL states fold through the library's merge (a ctypes call that releases the GIL): the columns' folds run on
        # a thread pool, each in loader order as below; every other state folds in place
        kll = [a for a in passed if isinstance(a, KLLSketch)] if len(stateLoaders) > 1 else []
        if len(kll) < 2:
            kll = []
        if kll:
            from concurrent.futures import ThreadPoolExecutor

            def fold(a):
                st = None
                for loader in stateLoaders:
                    st = merge_states(st, loader.load(a))
                return st
            with ThreadPoolExecutor(max_workers=min(8, len(kll))) as ex:
                for a, st in zip(kll, ex.map(fold, kll)):
                    if st is not None:
                        agg.persist(a, st)
        kll_set = set(kll)
        for a in passed:
            if a in kll_set:
                continue
            for loader in stateLoaders:
                a.aggregateStateTo(agg, loader, agg)
        grouping = [a for a in passed if isinstance(a, GroupingAnalyzer)]
        scanning = [a for a in passed if not isinstance(a, GroupingAnalyzer)]
        res = {}
        for a in scanning:
            m = a.loadStateAndComputeMetric(agg)
            if saveStatesWith is not None:
                a.copyStateTo(agg, saveStatesWith)
            if m is not None:
                res[a] = m
        by_cols = {}
        for a in grouping:
            by_cols.setdefault(tuple(sorted(a.groupingColumns())), []).append(a)
        out = pre + AnalyzerContext(res)
        for cols, group in by_cols.items():
            states = [agg.load(a) for a in group if agg.load(a) is not None]
            if not states:
                raise ValueError("requirement failed")
            out = out + AnalysisRunner._runAnalyzersForParticularGrouping(states[0], group, saveStatesWith)
        return out
