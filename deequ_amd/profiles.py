"""ColumnProfiler on the MI355X engine (M/profiles/ColumnProfiler.scala, ColumnProfile.scala,
ColumnProfilerRunner.scala, ColumnProfilerRunBuilder.scala).

The same three passes as the reference, each one AnalysisRunner run over the device engine:
  1. Size + per column Completeness, ApproxCountDistinct (+ DataType for STRING columns without a
     predefined type) — one fused dq_scan;
  2. columns of inferred / known type Integral or Fractional cast to LONG / DOUBLE (dq_cast_column on the
     GPU; castNumericStringColumns, :427-445), then Minimum, Maximum, Mean, StandardDeviation, Sum (one fused
     dq_scan) and KLLSketch (KLLRunner's extra pass, dq_kll_sketch);
  3. exact histograms of the low-cardinality columns (computeHistograms, :564-606) from dq_frequencies tables.
The metrics repository / result reuse and the JSON file output of the runner are not part of this engine.
"""
import json
import math
import os

import numpy as np

from . import native as N
from .analyzers import (Size, Completeness, ApproxCountDistinct, DataType, Minimum, Maximum, Mean,
                        StandardDeviation, Sum, KLLSketch, Histogram, _hist_key)
from .metrics import Distribution, DistributionValue
from .runners import AnalysisRunner
from .table import ChunkedTable, Table, Column


class DataTypeInstances:
    """A/DataType.scala:25-29 (Scala Enumeration values, compared and printed by name)."""
    Unknown = "Unknown"
    Fractional = "Fractional"
    Integral = "Integral"
    Boolean = "Boolean"
    String = "String"


class ColumnProfile:
    _fields = ("column", "completeness", "approximateNumDistinctValues", "dataType", "isDataTypeInferred",
               "typeCounts", "histogram")

    def _key(self):
        return tuple(getattr(self, f) for f in self._fields)

    def __eq__(self, other):
        return type(self) is type(other) and self._key() == other._key()

    def __repr__(self):
        return "%s(%s)" % (type(self).__name__, ",".join(repr(v) for v in self._key()))


class StandardColumnProfile(ColumnProfile):
    """M/profiles/ColumnProfile.scala:34-42."""

    def __init__(self, column, completeness, approximateNumDistinctValues, dataType, isDataTypeInferred, typeCounts,
                 histogram):
        self.column, self.completeness = column, completeness
        self.approximateNumDistinctValues, self.dataType = approximateNumDistinctValues, dataType
        self.isDataTypeInferred, self.typeCounts, self.histogram = isDataTypeInferred, dict(typeCounts), histogram


class NumericColumnProfile(ColumnProfile):
    """M/profiles/ColumnProfile.scala:44-59."""
    _fields = ColumnProfile._fields + ("kll", "mean", "maximum", "minimum", "sum", "stdDev", "approxPercentiles")

    def __init__(self, column, completeness, approximateNumDistinctValues, dataType, isDataTypeInferred, typeCounts,
                 histogram, kll, mean, maximum, minimum, sum, stdDev, approxPercentiles):
        self.column, self.completeness = column, completeness
        self.approximateNumDistinctValues, self.dataType = approximateNumDistinctValues, dataType
        self.isDataTypeInferred, self.typeCounts, self.histogram = isDataTypeInferred, dict(typeCounts), histogram
        self.kll, self.mean, self.maximum, self.minimum = kll, mean, maximum, minimum
        self.sum, self.stdDev, self.approxPercentiles = sum, stdDev, approxPercentiles


class ColumnProfiles:
    """M/profiles/ColumnProfile.scala:61-178."""

    def __init__(self, profiles, numRecords):
        self.profiles, self.numRecords = dict(profiles), int(numRecords)

    def __eq__(self, other):
        return isinstance(other, ColumnProfiles) and self.profiles == other.profiles and \
            self.numRecords == other.numRecords

    @staticmethod
    def toJson(columnProfiles):
        """ColumnProfiles.toJson (:68-177); Gson's pretty printing is not reproduced byte for byte."""
        cols = []
        for p in columnProfiles:
            j = {"column": p.column, "dataType": p.dataType, "isDataTypeInferred": str(p.isDataTypeInferred).lower()}
            j["completeness"] = p.completeness
            j["approximateNumDistinctValues"] = p.approximateNumDistinctValues
            if p.histogram is not None:
                j["histogram"] = [{"value": k, "count": v.absolute, "ratio": v.ratio}
                                  for k, v in p.histogram.values.items()]
            if isinstance(p, NumericColumnProfile):
                for name in ("mean", "maximum", "minimum", "sum", "stdDev"):
                    if getattr(p, name) is not None:
                        j[name] = getattr(p, name)
                if p.kll is not None:
                    j["kll"] = {"buckets": [{"low_value": b.lowValue, "high_value": b.highValue, "count": b.count}
                                            for b in p.kll.buckets],
                                "sketch": {"parameters": {"c": p.kll.parameters[0], "k": p.kll.parameters[1]},
                                           "data": json.dumps(p.kll.data)}}
                j["approxPercentiles"] = list(p.approxPercentiles or [])
            cols.append(j)
        return json.dumps({"columns": cols}, indent=2)


# Spark type names -> DataTypeInstances for schema-typed columns (ColumnProfiler.extractGenericStatistics :401-420)
def _known_type(type_name):
    if type_name in ("ShortType", "LongType", "IntegerType"):
        return DataTypeInstances.Integral
    if type_name.startswith("DecimalType") or type_name in ("FloatType", "DoubleType"):
        return DataTypeInstances.Fractional
    if type_name == "BooleanType":
        return DataTypeInstances.Boolean
    if type_name == "TimestampType":
        return DataTypeInstances.String
    return DataTypeInstances.Unknown


_HISTOGRAM_TYPES = ("StringType", "BooleanType", "DoubleType", "FloatType", "IntegerType", "LongType", "ShortType")


class GenericColumnStatistics:
    """M/profiles/ColumnProfiler.scala:30-43."""

    def __init__(self, numRecords, inferredTypes, knownTypes, typeDetectionHistograms, approximateNumDistincts,
                 completenesses, predefinedTypes):
        self.numRecords, self.inferredTypes, self.knownTypes = numRecords, inferredTypes, knownTypes
        self.typeDetectionHistograms, self.approximateNumDistincts = typeDetectionHistograms, approximateNumDistincts
        self.completenesses, self.predefinedTypes = completenesses, predefinedTypes

    def typeOf(self, column):
        merged = dict(self.inferredTypes)
        merged.update(self.knownTypes)
        merged.update(self.predefinedTypes)
        return merged[column]


# schema types whose pass-2 cast is the identity (integers -> LONG, FLOAT / DOUBLE -> DOUBLE: _cast_column)
_IDENTITY_CAST_TYPES = ("ByteType", "ShortType", "IntegerType", "LongType", "FloatType", "DoubleType")


def _cast_column(data, name, to_type):
    """ColumnProfiler.castColumn (:346-355) on the GPU. Casts that cannot change a value are skipped:
    integer -> LONG, FLOAT / DOUBLE -> DOUBLE (every pass-2 analyzer casts its input to double or sums
    integers in a long either way)."""
    import torch
    from . import engine
    col = data[name]
    t = col.spark_type
    if (to_type == N.TYPE_LONG and t in (N.TYPE_BYTE, N.TYPE_SHORT, N.TYPE_INT, N.TYPE_LONG)) or \
            (to_type == N.TYPE_DOUBLE and t in (N.TYPE_FLOAT, N.TYPE_DOUBLE)):
        return col
    n = data.nrows
    ctx = engine.ctx()
    if ctx.multi:  # a multi-device context casts each device's row shard into host buffers (include/dq.h)
        import numpy as np
        vals = np.empty(max(n, 1), dtype=np.float64 if to_type == N.TYPE_DOUBLE else np.int64)
        mask = np.zeros(max((n + 63) // 64, 1) * 8, dtype=np.uint8)
        ctx.cast_column(col.native(), n, to_type, vals.ctypes.data, mask.ctypes.data)
        return Column(name, to_type, vals[:n], mask[:(n + 7) // 8], length=n)
    dev = torch.device("cuda", engine.device())
    vals = torch.empty(max(n, 1), dtype=torch.float64 if to_type == N.TYPE_DOUBLE else torch.int64, device=dev)
    mask = torch.zeros(max((n + 63) // 64, 1) * 8, dtype=torch.uint8, device=dev)
    ctx.cast_column(col.native(), n, to_type, vals.data_ptr(), mask.data_ptr())
    out = Column(name, to_type, None, None, length=n)
    out.device = {"values": vals, "validity": mask}
    return out


class ColumnProfiler:
    """M/profiles/ColumnProfiler.scala:69-712."""
    DEFAULT_CARDINALITY_THRESHOLD = 120

    @staticmethod
    def profile(data, restrictToColumns=None, printStatusUpdates=False,
                lowCardinalityHistogramThreshold=DEFAULT_CARDINALITY_THRESHOLD, kllParameters=None,
                predefinedTypes=None, passes=None):
        """`passes` runs the three passes' work: None = AnalysisRunner on this process's GPU (LocalPasses); the
        sharded runner passes its own (distributed.ShardedProfilerPasses), so the same code profiles row shards."""
        passes = passes or LocalPasses()
        predefinedTypes = dict(predefinedTypes or {})
        if restrictToColumns is not None:
            for c in restrictToColumns:
                if c not in data.fieldNames:
                    raise ValueError("requirement failed: Unable to find column %s" % c)
        schema = data.schema
        relevant = [f for f in data.fieldNames if restrictToColumns is None or f in restrictToColumns]

        # ---- pass 1 ------------------------------------------------------------------------------
        if printStatusUpdates:
            print("### PROFILING: Computing generic column statistics in pass (1/3)...")
        first = []
        for name in relevant:
            if schema[name] == "StringType" and name not in predefinedTypes:
                first += [Completeness(name), ApproxCountDistinct(name), DataType(name)]
            else:
                first += [Completeness(name), ApproxCountDistinct(name)]
        # A column whose schema type is an integer or floating type is numeric whatever pass 1 finds, and its pass-2
        # cast is the identity (_cast_column), so its pass-2 statistics are the same analyzers over the same values:
        # they join pass 1's scan (one read of the column instead of two); its KLL sketch stays in pass 2.
        early = [name for name in relevant
                 if name not in predefinedTypes and schema[name] in _IDENTITY_CAST_TYPES and
                 not os.environ.get("DQ_PROFILE_NO_EARLY_STATS")]
        for name in early:
            first += [Minimum(name), Maximum(name), Mean(name), StandardDeviation(name), Sum(name)]
        # Their KLL sketches (the extra pass of pass 2) do not depend on pass 1 either: on this process's GPU they are
        # sketched on a second context in a helper thread while this thread runs pass 1 (the KLL compactions are
        # VALU-bound, pass 1's string scan latency-bound); DQ_PROFILE_NO_EARLY_KLL=1 keeps them in pass 2
        kll_early = []
        kll_pending = None
        if early and type(passes) is LocalPasses and not os.environ.get("DQ_PROFILE_SERIAL") and \
                not os.environ.get("DQ_PROFILE_NO_EARLY_KLL"):
            from .runners import _beside
            kll_an = [KLLSketch(name, kllParameters) for name in early]
            kll_pending = _beside(lambda: passes.run(data, kll_an), "kll")
            if kll_pending is not None:
                kll_early = list(early)
        try:
            res1 = passes.run(data, first + [Size()])
        except BaseException:
            if kll_pending is not None:
                kll_pending.join()
            raise
        generic = ColumnProfiler._extract_generic(relevant, schema, res1, predefinedTypes)

        # pass 3's columns depend on pass 1 only: on this process's GPU its histogram builds run on a second context
        # (own stream) in a helper thread while this thread casts, scans and aggregates pass 2 (the host aggregation
        # of pass 2 otherwise leaves the GPU idle); DQ_PROFILE_SERIAL=1 runs the passes one after the other
        targets = [c for c, cnt in generic.approximateNumDistincts.items()
                   if schema[c] in _HISTOGRAM_TYPES and
                   generic.typeOf(c) in (DataTypeInstances.String, DataTypeInstances.Boolean,
                                         DataTypeInstances.Integral, DataTypeInstances.Fractional) and
                   cnt <= lowCardinalityHistogramThreshold]
        pending = None
        try:
            if targets and type(passes) is LocalPasses and not os.environ.get("DQ_PROFILE_SERIAL"):
                pending = _histograms_beside(passes, data, targets)  # None: the passes stay on this thread
        except BaseException:
            if kll_pending is not None:
                kll_pending.join()
            raise

        try:
            # ---- pass 2 ------------------------------------------------------------------------------
            if printStatusUpdates:
                print("### PROFILING: Computing numeric column statistics in pass (2/3)...")
            numeric = [n for n in relevant
                       if generic.typeOf(n) in (DataTypeInstances.Integral, DataTypeInstances.Fractional)]
            casts = {name: N.TYPE_LONG if generic.typeOf(name) == DataTypeInstances.Integral else N.TYPE_DOUBLE
                     for name in numeric}
            casted = _cast_table(passes, data, casts)
            second = []
            early_set, kll_early_set = set(early), set(kll_early)
            for name in numeric:
                if name not in early_set:
                    second += [Minimum(name), Maximum(name), Mean(name), StandardDeviation(name), Sum(name)]
                if name not in kll_early_set:
                    second += [KLLSketch(name, kllParameters)]
            res2 = passes.run(casted, second) if second else None
            if early:
                res2 = res1 if res2 is None else res1 + res2
            if kll_pending is not None:
                kres = kll_pending.result()
                res2 = kres if res2 is None else res2 + kres
            stats = ColumnProfiler._extract_numeric(res2, numeric, kllParameters)

            # ---- pass 3 ------------------------------------------------------------------------------
            if printStatusUpdates:
                print("### PROFILING: Computing histograms of low-cardinality columns in pass (3/3)...")
            if pending is not None:
                histograms = pending.result()
            else:
                histograms = passes.histograms(data, targets) if targets else {}
        finally:  # a failing pass 2 does not leave the histogram or KLL helper driving its context
            if pending is not None:
                pending.join()
            if kll_pending is not None:
                kll_pending.join()

        profiles = {}
        for name in relevant:
            t = generic.typeOf(name)
            common = (name, generic.completenesses[name], generic.approximateNumDistincts[name], t,
                      name in generic.inferredTypes, generic.typeDetectionHistograms.get(name, {}),
                      histograms.get(name))
            if t in (DataTypeInstances.Integral, DataTypeInstances.Fractional):
                profiles[name] = NumericColumnProfile(
                    *common, stats["kll"].get(name), stats["mean"].get(name), stats["maximum"].get(name),
                    stats["minimum"].get(name), stats["sum"].get(name), stats["stdDev"].get(name),
                    stats["approxPercentiles"].get(name))
            else:
                profiles[name] = StandardColumnProfile(*common)
        return ColumnProfiles(profiles, generic.numRecords)

    @staticmethod
    def _extract_generic(columns, schema, results, predefinedTypes):
        """ColumnProfiler.extractGenericStatistics (:357-424)."""
        numRecords = int(results.metric(Size()).value.get())
        inferred, type_hist = {}, {}
        for name in columns:
            a = DataType(name)
            m = results.metricMap.get(a)
            if m is None or name in predefinedTypes:
                continue
            dist = m.value.get()
            from .states import DataTypeHistogram
            inferred[name] = DataTypeHistogram.determineType(dist)
            type_hist[name] = {k: v.absolute for k, v in dist.values.items()}
        approx = {n: int(results.metric(ApproxCountDistinct(n)).value.get()) for n in columns}
        completeness = {n: results.metric(Completeness(n)).value.get() for n in columns}
        known = {n: _known_type(schema[n]) for n in columns
                 if n not in predefinedTypes and schema[n] != "StringType"}
        return GenericColumnStatistics(numRecords, inferred, known, type_hist, approx, completeness, predefinedTypes)

    @staticmethod
    def _extract_numeric(results, columns, kllParameters):
        """ColumnProfiler.extractNumericStatistics (:448-528): Success values only."""
        out = {k: {} for k in ("mean", "stdDev", "maximum", "minimum", "sum", "kll", "approxPercentiles")}
        if results is None:
            return out
        for name in columns:
            for key, a in (("mean", Mean(name)), ("stdDev", StandardDeviation(name)), ("maximum", Maximum(name)),
                           ("minimum", Minimum(name)), ("sum", Sum(name))):
                m = results.metricMap.get(a)
                if m is not None and m.value.isSuccess:
                    out[key][name] = m.value.get()
            m = results.metricMap.get(KLLSketch(name, kllParameters))
            if m is not None and m.value.isSuccess:
                bd = m.value.get()
                out["kll"][name] = bd
                out["approxPercentiles"][name] = sorted(bd.computePercentiles())
        return out

    @staticmethod
    def _compute_histograms(data, targets):
        """ColumnProfiler.computeHistograms (:564-606): exact per-value counts (NULL as "NullValue"), the
        value formatted as `row.get(index).toString`, ratio = count / rows."""
        from . import engine
        out = {}
        for name in targets:
            table = engine.frequencies(data, [name], include_nulls=True)
            counts = table.to_dict()
            total = sum(counts.values())
            values = {}
            for key, c in counts.items():
                k = Histogram.NullFieldReplacement if key[0] is None else _hist_key(key[0], data[name])
                values[k] = DistributionValue(int(c), c / total)
            out[name] = Distribution(values, len(values))
        return out


def _histograms_beside(passes, data, targets):
    from .runners import _beside
    return _beside(lambda: passes.histograms(data, targets), "hist")


def _cast_table(passes, data, casts):
    """castNumericStringColumns (:326-344): every column in `casts` cast to its type, the others as they are; a
    ChunkedTable casts chunk by chunk."""
    if isinstance(data, ChunkedTable):
        return ChunkedTable([_cast_table(passes, chunk, casts) for chunk in data.chunks])
    return Table([passes.cast(data, name, casts[name]) if name in casts else data[name] for name in data.fieldNames])


def _chunked_histograms(data, targets):
    """computeHistograms over a ChunkedTable: each chunk's exact per-value counts (dq_frequencies), summed per value
    (the histogram columns are the low-cardinality ones: at most lowCardinalityHistogramThreshold groups each)."""
    from . import engine
    out = {}
    for name in targets:
        counts = {}
        for chunk in data.chunks:
            for key, c in engine.frequencies(chunk, [name], include_nulls=True).to_dict().items():
                counts[key] = counts.get(key, 0) + int(c)
        total = sum(counts.values())
        values = {}
        for key, c in counts.items():
            k = Histogram.NullFieldReplacement if key[0] is None else _hist_key(key[0], data[name])
            values[k] = DistributionValue(int(c), c / total)
        out[name] = Distribution(values, len(values))
    return out


class LocalPasses:
    """The profiler's passes on this process's GPU: AnalysisRunner runs, GPU casts, dq_frequencies histograms."""

    def run(self, data, analyzers):
        return AnalysisRunner.onData(data).addAnalyzers(analyzers).run()

    def cast(self, data, name, to_type):
        return _cast_column(data, name, to_type)

    def histograms(self, data, targets):
        if isinstance(data, ChunkedTable):
            return _chunked_histograms(data, targets)
        return ColumnProfiler._compute_histograms(data, targets)


class ColumnProfilerRunBuilder:
    """M/profiles/ColumnProfilerRunBuilder.scala:24-177 (repository and file-output options excluded)."""

    def __init__(self, data):
        self.data = data
        self._print = False
        self._threshold = ColumnProfiler.DEFAULT_CARDINALITY_THRESHOLD
        self._restrict = None
        self._kll = None
        self._predefined = {}

    def printStatusUpdates(self, flag):
        self._print = bool(flag)
        return self

    def cacheInputs(self, flag):  # Spark caching has no analogue: inputs stay resident in HBM
        return self

    def withLowCardinalityHistogramThreshold(self, threshold):
        self._threshold = int(threshold)
        return self

    def restrictToColumns(self, columns):
        self._restrict = list(columns)
        return self

    def setKLLParameters(self, kllParameters):
        self._kll = kllParameters
        return self

    def setPredefinedTypes(self, dataTypes):
        self._predefined = dict(dataTypes)
        return self

    def run(self):
        return ColumnProfiler.profile(self.data, self._restrict, self._print, self._threshold, self._kll,
                                      self._predefined)


class ColumnProfilerRunner:
    """M/profiles/ColumnProfilerRunner.scala:37-113."""

    def onData(self, data):
        return ColumnProfilerRunBuilder(data)
