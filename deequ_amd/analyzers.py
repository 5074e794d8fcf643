"""deequ analyzers on the MI355X engine — the same case classes, preconditions, states and metrics as
the reference (A/*.scala), with the per-row work done by libdq.so.

Scan-shareable analyzers describe their Spark aggregations as dq_op records instead of Spark
Columns (`aggregationFunctions`, A/Analyzer.scala:172) and rebuild their state from the returned
dq_state (`fromAggregationResult`, A/Analyzer.scala:175). Grouping analyzers read the device
frequency table built by `computeFrequencies` (A/GroupingAnalyzers.scala:53-79).
"""
import math

import numpy as np

from . import native as N
from .expr import compile_predicate
from .metrics import (DoubleMetric, Entity, Failure, Success, EmptyStateException, NoSuchColumnException,
                      WrongColumnTypeException, NoColumnsSpecifiedException, NumberOfSpecifiedColumnsException,
                      IllegalAnalyzerParameterException, HistogramMetric, Distribution, DistributionValue,
                      MetricCalculationRuntimeException, KeyedDoubleMetric, UnsupportedOnDevice, wrap_if_necessary)
from .states import (NumMatches, NumMatchesAndCount, MeanState, SumState, MinState, MaxState, ApproxQuantileState,
                     DataTypeHistogram, state_from_native)
from . import engine

COL_PREFIX = "com_amazon_deequ_dq_metrics_"
COUNT_COL = COL_PREFIX + "count"


# ---- Preconditions (A/Analyzer.scala:285-359) ----------------------------------------------------
class Preconditions:
    NUMERIC = ("ByteType", "ShortType", "IntegerType", "LongType", "FloatType", "DoubleType")

    @staticmethod
    def findFirstFailing(schema, conditions):
        for c in conditions:
            try:
                c(schema)
            except Exception as e:  # only exceptions, as in the reference
                return e
        return None

    @staticmethod
    def atLeastOne(columns):
        def check(_):
            if not columns:
                raise NoColumnsSpecifiedException("At least one column needs to be specified!")
        return check

    @staticmethod
    def exactlyNColumns(columns, n):
        def check(_):
            if len(columns) != n:
                raise NumberOfSpecifiedColumnsException(
                    "%d columns have to be specified! Currently, columns contains only %d column(s): %s!"
                    % (n, len(columns), ",".join(columns)))
        return check

    @staticmethod
    def hasColumn(column):
        def check(schema):
            if column not in schema:
                raise NoSuchColumnException("Input data does not include column %s!" % column)
        return check

    @staticmethod
    def isNumeric(column):
        def check(schema):
            t = schema[column]
            if not (t in Preconditions.NUMERIC or t.startswith("DecimalType")):
                raise WrongColumnTypeException(
                    "Expected type of column %s to be one of (%s), but found %s instead!"
                    % (column, ",".join(Preconditions.NUMERIC + ("DecimalType",)), t))
        return check

    @staticmethod
    def isString(column):
        def check(schema):
            t = schema[column]
            if t != "StringType":
                raise WrongColumnTypeException(
                    "Expected type of column %s to be StringType, but found %s instead!" % (column, t))
        return check


def entityFrom(columns):
    return Entity.Column if len(columns) == 1 else Entity.Mutlicolumn


def metricFromValue(value, name, instance, entity=Entity.Column):
    return DoubleMetric(entity, name, instance, Success(value))


def emptyStateException(analyzer):
    return EmptyStateException("Empty state for analyzer %r, all input values were NULL." % (analyzer,))


def metricFromFailure(exception, name, instance, entity=Entity.Column):
    return DoubleMetric(entity, name, instance, Failure(wrap_if_necessary(exception)))


def metricFromEmpty(analyzer, name, instance, entity=Entity.Column):
    return metricFromFailure(emptyStateException(analyzer), name, instance, entity)


def merge(*states):
    """Analyzers.merge (A/Analyzer.scala:367-386): None is the identity."""
    out = None
    for s in states:
        if s is None:
            continue
        out = s if out is None else out.sum(s)
    return out


# Placeholder result of an analyzer whose state went to a states-only provider (see Analyzer.calculateMetric).
STATE_ONLY = DoubleMetric(Entity.Dataset, "StateOnly", "*", Success(0.0))


# ---- Analyzer base classes (A/Analyzer.scala:56-197) ---------------------------------------------
class Analyzer:
    _fields = ()

    def _key(self):
        k = self.__dict__.get("_cached_key")  # analyzers are values: fields are not changed after construction
        if k is None:
            k = (type(self).__name__,) + tuple(
                tuple(v) if isinstance(v, list) else v for v in (getattr(self, f) for f in self._fields))
            self.__dict__["_cached_key"] = k
        return k

    def __eq__(self, other):
        return type(self) is type(other) and self._key() == other._key()

    def __hash__(self):
        return hash(self._key())

    def __repr__(self):
        args = []
        for f in self._fields:
            v = getattr(self, f)
            if isinstance(v, list):
                v = "List(%s)" % ", ".join(_java_double_to_string(x) if isinstance(x, float) else str(x) for x in v)
            elif v is None:
                v = "None"
            elif f in ("where", "binningUdf"):
                v = "Some(%s)" % v
            elif isinstance(v, float):
                v = _java_double_to_string(v)  # Scala's Double.toString inside the case-class toString
            args.append(str(v))
        return "%s(%s)" % (type(self).__name__, ",".join(args))

    def preconditions(self):
        return []

    def computeStateFrom(self, data):
        raise NotImplementedError

    def computeMetricFrom(self, state):
        raise NotImplementedError

    def toFailureMetric(self, exception):
        raise NotImplementedError

    def calculate(self, data, aggregateWith=None, saveStatesWith=None):
        """Analyzer.calculate (A/Analyzer.scala:88-103)."""
        try:
            for c in self.preconditions():
                c(data.schema)
            state = self.computeStateFrom(data)
            return self.calculateMetric(state, aggregateWith, saveStatesWith)
        except Exception as e:
            return self.toFailureMetric(e)

    def calculateMetric(self, state, aggregateWith=None, saveStatesWith=None):
        """A/Analyzer.scala:107-128. A states-only provider (the row chunks of a ChunkedTable, whose states are merged
        before any metric) takes the state and no metric is computed (STATE_ONLY: not even the empty-state failure,
        which only the merged state decides)."""
        loaded = aggregateWith.load(self) if aggregateWith is not None else None
        to_use = merge(state, loaded)
        if to_use is not None and saveStatesWith is not None:
            saveStatesWith.persist(self, to_use)
        if getattr(saveStatesWith, "states_only", False):
            return STATE_ONLY
        return self.computeMetricFrom(to_use)

    def aggregateStateTo(self, sourceA, sourceB, target):
        a, b = sourceA.load(self), sourceB.load(self)
        agg = merge(a, b)
        if agg is not None:
            target.persist(self, agg)

    def loadStateAndComputeMetric(self, source):
        s = source.load(self)
        return None if s is None else self.computeMetricFrom(s)

    def copyStateTo(self, source, target):
        s = source.load(self)
        if s is not None:
            target.persist(self, s)


class ScanShareableAnalyzer(Analyzer):
    """Contributes dq_ops to the fused scan instead of Spark aggregation Columns."""

    def addOps(self, batch):
        """Register this analyzer's ops; return the op indices (the `offset` into the result)."""
        raise NotImplementedError

    def fromAggregationResult(self, states, ops):
        raise NotImplementedError

    def computeStateFrom(self, data):
        from .runners import ScanBatch
        batch = ScanBatch(data)
        ops = self.addOps(batch)
        states = batch.run()
        return self.fromAggregationResult(states, ops)

    def metricFromAggregationResult(self, states, ops, aggregateWith=None, saveStatesWith=None):
        return self.calculateMetric(self.fromAggregationResult(states, ops), aggregateWith, saveStatesWith)


class StandardScanShareableAnalyzer(ScanShareableAnalyzer):
    name = None
    entity = Entity.Column

    @property
    def instance(self):
        raise NotImplementedError

    def computeMetricFrom(self, state):
        if state is not None:
            return metricFromValue(state.metricValue(), self.name, self.instance, self.entity)
        return metricFromEmpty(self, self.name, self.instance, self.entity)

    def toFailureMetric(self, exception):
        return metricFromFailure(exception, self.name, self.instance, self.entity)

    def additionalPreconditions(self):
        return []

    def preconditions(self):
        return self.additionalPreconditions()

    def _one_state(self, states, ops):
        return state_from_native(states[ops[0]])

    def fromAggregationResult(self, states, ops):
        return self._one_state(states, ops)


# ---- scan-shareable analyzers --------------------------------------------------------------------
class Size(StandardScanShareableAnalyzer):
    """A/Size.scala:33-47."""
    _fields = ("where",)
    name = "Size"
    entity = Entity.Dataset

    def __init__(self, where=None):
        self.where = where

    instance = property(lambda self: "*")

    def addOps(self, batch):
        return [batch.add_op(N.OP_SIZE, where=self.where)]


class Completeness(StandardScanShareableAnalyzer):
    """A/Completeness.scala:26-46."""
    _fields = ("column", "where")
    name = "Completeness"

    def __init__(self, column, where=None):
        self.column, self.where = column, where

    instance = property(lambda self: self.column)

    def additionalPreconditions(self):
        return [Preconditions.hasColumn(self.column)]

    def addOps(self, batch):
        return [batch.add_op(N.OP_COMPLETENESS, (self.column,), where=self.where)]


class Compliance(StandardScanShareableAnalyzer):
    """A/Compliance.scala:37-53."""
    _fields = ("instance_", "predicate", "where")
    name = "Compliance"

    def __init__(self, instance, predicate, where=None):
        self.instance_, self.predicate, self.where = instance, predicate, where

    instance = property(lambda self: self.instance_)

    def addOps(self, batch):
        return [batch.add_op(N.OP_COMPLIANCE, where=self.where, predicate=self.predicate)]


class _NumericColumnAnalyzer(StandardScanShareableAnalyzer):
    _fields = ("column", "where")
    op_kind = None

    def __init__(self, column, where=None):
        self.column, self.where = column, where

    instance = property(lambda self: self.column)

    def additionalPreconditions(self):
        return [Preconditions.hasColumn(self.column), Preconditions.isNumeric(self.column)]

    def addOps(self, batch):
        return [batch.add_op(self.op_kind, (self.column,), where=self.where)]


class Mean(_NumericColumnAnalyzer):
    """A/Mean.scala:36-54."""
    name, op_kind = "Mean", N.OP_MEAN


class Sum(_NumericColumnAnalyzer):
    """A/Sum.scala:34-52."""
    name, op_kind = "Sum", N.OP_SUM


class Minimum(_NumericColumnAnalyzer):
    """A/Minimum.scala:34-53."""
    name, op_kind = "Minimum", N.OP_MINIMUM


class Maximum(_NumericColumnAnalyzer):
    """A/Maximum.scala:34-53."""
    name, op_kind = "Maximum", N.OP_MAXIMUM


class StandardDeviation(_NumericColumnAnalyzer):
    """A/StandardDeviation.scala:47-73."""
    name, op_kind = "StandardDeviation", N.OP_STANDARD_DEVIATION


class Correlation(StandardScanShareableAnalyzer):
    """A/Correlation.scala:66-105."""
    _fields = ("firstColumn", "secondColumn", "where")
    name = "Correlation"
    entity = Entity.Mutlicolumn

    def __init__(self, firstColumn, secondColumn, where=None):
        self.firstColumn, self.secondColumn, self.where = firstColumn, secondColumn, where

    instance = property(lambda self: "%s,%s" % (self.firstColumn, self.secondColumn))

    def additionalPreconditions(self):
        return [Preconditions.hasColumn(self.firstColumn), Preconditions.isNumeric(self.firstColumn),
                Preconditions.hasColumn(self.secondColumn), Preconditions.isNumeric(self.secondColumn)]

    def addOps(self, batch):
        return [batch.add_op(N.OP_CORRELATION, (self.firstColumn, self.secondColumn), where=self.where)]


class ApproxCountDistinct(StandardScanShareableAnalyzer):
    """A/ApproxCountDistinct.scala:43-64 (HLL++ registers, XXH64 seed 42)."""
    _fields = ("column", "where")
    name = "ApproxCountDistinct"

    def __init__(self, column, where=None):
        self.column, self.where = column, where

    instance = property(lambda self: self.column)

    def additionalPreconditions(self):
        return [Preconditions.hasColumn(self.column)]

    def addOps(self, batch):
        return [batch.add_op(N.OP_APPROX_COUNT_DISTINCT, (self.column,), where=self.where)]


class _StringLengthAnalyzer(StandardScanShareableAnalyzer):
    _fields = ("column", "where")
    op_kind = None

    def __init__(self, column, where=None):
        self.column, self.where = column, where

    instance = property(lambda self: self.column)

    def additionalPreconditions(self):
        return [Preconditions.hasColumn(self.column), Preconditions.isString(self.column)]

    def addOps(self, batch):
        return [batch.add_op(self.op_kind, (self.column,), where=self.where)]


class MinLength(_StringLengthAnalyzer):
    """A/MinLength.scala:25-41: min(length(when(where, col))) as Double."""
    name, op_kind = "MinLength", N.OP_MIN_LENGTH


class MaxLength(_StringLengthAnalyzer):
    """A/MaxLength.scala:25-41: max(length(when(where, col))) as Double."""
    name, op_kind = "MaxLength", N.OP_MAX_LENGTH


class DataType(ScanShareableAnalyzer):
    """A/DataType.scala:138-183: StatefulDataType histogram of the value cast to string."""
    _fields = ("column", "where")

    def __init__(self, column, where=None):
        self.column, self.where = column, where

    def preconditions(self):
        return [Preconditions.hasColumn(self.column)]

    def addOps(self, batch):
        return [batch.add_op(N.OP_DATATYPE, (self.column,), where=self.where)]

    def fromAggregationResult(self, states, ops):
        return state_from_native(states[ops[0]])

    def computeMetricFrom(self, state):
        if state is None:
            return self.toFailureMetric(emptyStateException(self))
        return HistogramMetric(self.column, Success(state.toDistribution()))

    def toFailureMetric(self, exception):
        return HistogramMetric(self.column, Failure(wrap_if_necessary(exception)))


class PatternMatch(StandardScanShareableAnalyzer):
    """A/PatternMatch.scala:37-55: sum(when(regexp_extract(col, pattern, 0) != "", 1).otherwise(0))
    under `where`, plus conditionalCount. The pattern runs on the GPU's backtracking regex engine
    (deequ_amd/regex.py, csrc/regex.hip); a NULL value counts 0.

    FLOAT / DOUBLE values are matched against the shortest round-trip digits laid out as Java's toString
    (csrc/java_dtoa.h). JDK 8's FloatingDecimal is not always shortest (JDK-4511638: some values print with
    more digits than needed): for such values the match count is parity unpinned against a Java 8 Spark."""
    _fields = ("column", "pattern_", "where")
    name = "PatternMatch"

    def __init__(self, column, pattern, where=None):
        self.column, self.where = column, where
        self.pattern_ = pattern.pattern if hasattr(pattern, "pattern") else str(pattern)

    instance = property(lambda self: self.column)

    @property
    def pattern(self):
        return self.pattern_

    def addOps(self, batch):
        # regexp_extract casts a non-string column to STRING (Spark's implicit cast): the device formats every cell
        # as Cast(x AS STRING) does — Java toString of numerics, BigDecimal.toString of decimals, "yyyy-MM-dd" of
        # dates and "yyyy-MM-dd HH:mm:ss[.ffffff]" of timestamps in a UTC session time zone (regex.hip)
        col = batch.data[self.column] if self.column in batch.col_index else None
        tz = getattr(col, "tz", None)
        if col is not None and col.spark_type == N.TYPE_TIMESTAMP and tz not in UTC_ZONES:
            # Spark formats timestamps in the session time zone; the device formats in UTC only
            raise UnsupportedOnDevice("PatternMatch over TIMESTAMP column %s in time zone %s: the device formats "
                                      "timestamps in a UTC session time zone only" % (self.column, tz))
        p = batch.regex_predicate(self.column, self.pattern_)
        return [batch.add_op(N.OP_COMPLIANCE, where=self.where, predicate_index=p)]


UTC_ZONES = (None, "UTC", "Etc/UTC", "GMT", "Etc/GMT", "Z", "+00:00", "-00:00", "Zulu", "Universal")


class Patterns:
    """A/PatternMatch.scala:57-72 (the reference's pattern constants)."""
    EMAIL = (r"""(?:[a-z0-9!#$%&'*+/=?^_`{|}~-]+(?:\.[a-z0-9!#$%&'*+/=?^_`{|}~-]+)*|"(?:[\x01-\x08\x0b\x0c\x0e-\x1f"""
             r"""\x21\x23-\x5b\x5d-\x7f]|\\[\x01-\x09\x0b\x0c\x0e-\x7f])*")@(?:(?:[a-z0-9](?:[a-z0-9-]*[a-z0-9])?\.)+"""
             r"""[a-z0-9](?:[a-z0-9-]*[a-z0-9])?|\[(?:(?:25[0-5]|2[0-4][0-9]|[01]?[0-9][0-9]?)\.){3}(?:25[0-5]|"""
             r"""2[0-4][0-9]|[01]?[0-9][0-9]?|[a-z0-9-]*[a-z0-9]:(?:[\x01-\x08\x0b\x0c\x0e-\x1f\x21-\x5a\x53-\x7f]|"""
             r"""\\[\x01-\x09\x0b\x0c\x0e-\x7f])+)\])""")
    URL = r"""(https?|ftp)://[^\s/$.?#].[^\s]*"""
    SOCIAL_SECURITY_NUMBER_US = (
        r"""((?!219-09-9999|078-05-1120)(?!666|000|9\d{2})\d{3}-(?!00)\d{2}-(?!0{4})\d{4})|((?!219 09 9999|078 05 1120)"""
        r"""(?!666|000|9\d{2})\d{3} (?!00)\d{2} (?!0{4})\d{4})|((?!219099999|078051120)(?!666|000|9\d{2})\d{3}"""
        r"""(?!00)\d{2}(?!0{4})\d{4})""")
    CREDITCARD = (r"""\b(?:3[47]\d{2}([\ \-]?)\d{6}\1\d|(?:(?:4\d|5[1-5]|65)\d{2}|6011)([\ \-]?)\d{4}\2\d{4}\2)"""
                  r"""\d{4}\b""")


def _quantile_param_checks(quantiles, relativeError):
    """PARAM_CHECKS of A/ApproxQuantile.scala:44-55 / A/ApproxQuantiles.scala:41-54."""
    def check(_):
        for q in quantiles:
            if q < 0.0 or q > 1.0:
                raise IllegalAnalyzerParameterException(
                    "Quantile parameter must be in the closed interval [0, 1]. Currently, the value is: %s!"
                    % _java_double_to_string(float(q)))
        if relativeError < 0.0 or relativeError > 1.0:
            raise IllegalAnalyzerParameterException(
                "Relative error parameter must be in the closed interval [0, 1]. Currently, the value is: %s!"
                % _java_double_to_string(float(relativeError)))
    return check


class ApproxQuantile(ScanShareableAnalyzer):
    """A/ApproxQuantile.scala:44-103. The digest comes from dq_quantile_summary (exact order
    statistics on the GPU, deequ_amd/quantiles.py); `where` is not supported, as in the reference."""
    _fields = ("column", "quantile", "relativeError")

    def __init__(self, column, quantile, relativeError=0.01):
        self.column, self.quantile, self.relativeError = column, float(quantile), float(relativeError)

    @property
    def _metric_name(self):
        return "ApproxQuantile-%s" % _java_double_to_string(self.quantile)

    def preconditions(self):
        return [_quantile_param_checks([self.quantile], self.relativeError), Preconditions.hasColumn(self.column),
                Preconditions.isNumeric(self.column)]

    def addOps(self, batch):
        return [batch.add_quantile(self.column, self.relativeError)]

    def fromAggregationResult(self, states, ops):
        digest = states.quantiles[ops[0]]
        # all values NULL: getPercentiles is empty (A/ApproxQuantile.scala:76-80)
        if not digest.getPercentiles([self.quantile]):
            return None
        return ApproxQuantileState(digest)

    def computeMetricFrom(self, state):
        if state is None:
            return metricFromEmpty(self, self._metric_name, self.column)
        v = state.percentileDigest.getPercentiles([self.quantile])[0]
        return metricFromValue(v, self._metric_name, self.column)

    def toFailureMetric(self, exception):
        return metricFromFailure(exception, self._metric_name, self.column)


class ApproxQuantiles(ScanShareableAnalyzer):
    """A/ApproxQuantiles.scala:39-101: several quantiles from one digest -> KeyedDoubleMetric."""
    _fields = ("column", "quantiles", "relativeError")

    def __init__(self, column, quantiles, relativeError=0.01):
        self.column, self.quantiles, self.relativeError = column, [float(q) for q in quantiles], float(relativeError)

    def preconditions(self):
        return [_quantile_param_checks(self.quantiles, self.relativeError), Preconditions.hasColumn(self.column),
                Preconditions.isNumeric(self.column)]

    def addOps(self, batch):
        return [batch.add_quantile(self.column, self.relativeError)]

    def fromAggregationResult(self, states, ops):
        # no empty check here: an all-NULL column yields Success(Map()) (A/ApproxQuantiles.scala:69-83)
        return ApproxQuantileState(states.quantiles[ops[0]])

    def computeMetricFrom(self, state):
        if state is None:
            return self.toFailureMetric(emptyStateException(self))
        got = state.percentileDigest.getPercentiles(self.quantiles)
        return KeyedDoubleMetric(Entity.Column, "ApproxQuantiles", self.column,
                                 Success({_java_double_to_string(q): v for q, v in zip(self.quantiles, got)}))

    def toFailureMetric(self, exception):
        return KeyedDoubleMetric(Entity.Column, "ApproxQuantiles", self.column, Failure(wrap_if_necessary(exception)))


class KLLSketch(ScanShareableAnalyzer):
    """A/KLLSketch.scala:82-176. AnalysisRunner routes it to KLLRunner (one extra pass per column,
    deequ_amd/runners.py); the sketching itself is dq_kll_sketch on the GPU. No `where` (commented out in
    the reference)."""
    _fields = ("column", "kllParameters")

    def __init__(self, column, kllParameters=None):
        from .kll import DEFAULT_SKETCH_SIZE, DEFAULT_SHRINKING_FACTOR, MAXIMUM_ALLOWED_DETAIL_BINS
        self.column, self.kllParameters = column, kllParameters
        self.sketchSize = DEFAULT_SKETCH_SIZE
        self.shrinkingFactor = DEFAULT_SHRINKING_FACTOR
        self.numberOfBuckets = MAXIMUM_ALLOWED_DETAIL_BINS
        if kllParameters is not None:
            self.sketchSize = kllParameters.sketchSize
            self.shrinkingFactor = kllParameters.shrinkingFactor
            self.numberOfBuckets = kllParameters.numberOfBuckets

    def __repr__(self):
        p = "None" if self.kllParameters is None else "Some(%r)" % (self.kllParameters,)
        return "KLLSketch(%s,%s)" % (self.column, p)

    def preconditions(self):
        from .kll import MAXIMUM_ALLOWED_DETAIL_BINS

        def param_check(_):
            if self.numberOfBuckets > MAXIMUM_ALLOWED_DETAIL_BINS:
                raise IllegalAnalyzerParameterException(
                    "Cannot return KLL Sketch related values for more than %d values" % MAXIMUM_ALLOWED_DETAIL_BINS)
        return [param_check, Preconditions.hasColumn(self.column), Preconditions.isNumeric(self.column)]

    def computeStateFrom(self, data):
        from .runners import KLLRunner
        return KLLRunner.sketch_column(data, self.column, self.sketchSize, self.shrinkingFactor)

    def computeMetricFrom(self, state):
        from .kll import KLLMetric, bucket_distribution
        if state is None:
            return KLLMetric(self.column, Failure(emptyStateException(self)))
        try:
            return KLLMetric(self.column, Success(bucket_distribution(state, self.numberOfBuckets)))
        except Exception as e:
            return KLLMetric(self.column, Failure(e))

    def toFailureMetric(self, exception):
        from .kll import KLLMetric
        return KLLMetric(self.column, Failure(wrap_if_necessary(exception)))


# ---- grouping analyzers (A/GroupingAnalyzers.scala) ----------------------------------------------
def _host_key_column(col):
    """A key column with host buffers (device-resident columns are copied back once; a parted column's chunks are
    concatenated on the host)."""
    from .table import PartedColumn, _concat_host
    if isinstance(col, PartedColumn):
        return _concat_host([_host_key_column(p) for p in col.parts])
    if getattr(col, "values", None) is not None or not getattr(col, "device", None):
        return col
    from .distributed import _host_column
    return _host_column(col)


def _canonical_group_key(key):
    """A group key tuple with every float wrapped as engine.GroupFloat (bitwise equality, NaN canonical,
    -0.0 != 0.0), so keys from device tables, persisted states and host dicts join exactly."""
    if not isinstance(key, tuple):
        key = (key,)
    if any(isinstance(v, float) and not isinstance(v, engine.GroupFloat) for v in key):
        return tuple(engine.GroupFloat(v) if isinstance(v, float) and not isinstance(v, engine.GroupFloat) else v
                     for v in key)
    return key


def _single_device_side(t):
    """A DQ_FREQ_KEYS_VALUES table of a multi-device context as host (canonical key, count) pairs; anything else as
    is."""
    if isinstance(t, engine.FrequencyTable) and getattr(t.ctx, "multi", False):
        keys, counts = t.export_pairs()
        return engine.PairFrequencies(t.key_type, keys, counts, t.num_rows, t.summary(None)["null_count"],
                                      t.decimal_scale, t.names)
    return t


class FrequenciesAndNumRows:
    """A/GroupingAnalyzers.scala:123-156. `frequencies` is one of
      * engine.FrequencyTable — the device (key -> count) table built by dq_frequencies;
      * engine.PairFrequencies — (canonical key, count) arrays of one fixed-width key (a persisted state);
      * groups.GroupBlock — the groups of any key shape as host key columns + counts (persisted / merged states;
        a merge concatenates blocks, so a key may repeat: the weighted GPU build that evaluates it adds them);
      * dict[tuple -> int] — a host state built in Python (small)."""

    def __init__(self, frequencies, numRows, columns=None, summary=None):
        self.frequencies = frequencies
        self.numRows = int(numRows)
        self.columns = columns
        self._device = None

    def as_dict(self):
        from . import groups as G
        f = self.frequencies
        if isinstance(f, dict):
            return f
        if isinstance(f, G.GroupBlock):
            out = {}
            for k, c in zip(f.keys(), f.counts.tolist()):
                k = _canonical_group_key(k)
                out[k] = out.get(k, 0) + int(c)
            return out
        return f.to_dict()

    def _values_side(self):
        """This state as a single fixed-width-key table (device FrequencyTable or host PairFrequencies), or None."""
        f = self.frequencies
        if isinstance(f, engine.PairFrequencies):
            return f
        if isinstance(f, engine.FrequencyTable) and f.key_kind() == N.FREQ_KEYS_VALUES:
            return f
        return None

    def sum(self, other):
        """Null-safe full outer join on the keys, counts added (A/GroupingAnalyzers.scala:127-147). Keys are
        compared with Spark's grouping equality (floating values bitwise, NaN canonical). Single fixed-width
        keys merge on the GPU (dq_freq_merge) when either side is a device table, as canonical 64-bit
        pairs otherwise; any other key shape concatenates the two sides' groups (GroupBlock), which the weighted
        GPU build behind every metric of the state aggregates."""
        a, b = self._values_side(), other._values_side()
        if a is not None and b is not None and a.key_type == b.key_type:
            rows = self.numRows + other.numRows
            # a multi-device context's table (the union of per-device parts, DQ_DEVICES) merges as host pairs:
            # dq_freq_merge joins single-device tables only
            a, b = _single_device_side(a), _single_device_side(b)
            if isinstance(a, engine.PairFrequencies) and isinstance(b, engine.PairFrequencies):
                keys, inv = np.unique(np.concatenate([a.keys, b.keys]), return_inverse=True)
                counts = np.zeros(len(keys), dtype=np.int64)  # Long counts: exact beyond 2^53
                np.add.at(counts, inv, np.concatenate([a.counts, b.counts]))
                return FrequenciesAndNumRows(engine.PairFrequencies(a.key_type, keys, counts, rows,
                                                                    a.null_count + b.null_count, a.decimal_scale,
                                                                    a.names), rows, self.columns)
            ta = a.to_device() if isinstance(a, engine.PairFrequencies) else a
            tb = b.to_device() if isinstance(b, engine.PairFrequencies) else b
            return FrequenciesAndNumRows(ta.merge(tb), rows, self.columns)
        ba, bb = self.group_block(), other.group_block()
        if ba is None and bb is not None and isinstance(self.frequencies, dict):
            ba = _block_from_dict(self.frequencies, bb)
        if bb is None and ba is not None and isinstance(other.frequencies, dict):
            bb = _block_from_dict(other.frequencies, ba)
        if ba is not None and bb is not None and ba.schema() == bb.schema():
            from . import groups as G
            merged = G.BlockParts([ba, bb], ba.schema())  # joined in HBM by the metric's build, not on the host
            return FrequenciesAndNumRows(merged, self.numRows + other.numRows, self.columns)
        merged = {}
        for src in (self.as_dict(), other.as_dict()):
            for k, v in src.items():
                k = _canonical_group_key(k)
                merged[k] = merged.get(k, 0) + v
        return FrequenciesAndNumRows(merged, self.numRows + other.numRows, self.columns)

    def group_block(self):
        """The groups as a host GroupBlock (key cells + counts, vectorised: no per-group Python), or None for a
        host dict, a Histogram table (NULL group) or a pair table without key columns."""
        from . import groups as G
        f = self.frequencies
        if isinstance(f, G.GroupBlock):
            return f
        if isinstance(f, engine.PairFrequencies):
            if f.null_count:
                return None
            name = (f.names or self.columns or ["c0"])[0]
            return G.GroupBlock([G.column_from_canonical(name, f.key_type, f.keys, 18 if f.decimal_scale else 0,
                                                         f.decimal_scale)], f.counts)
        if not isinstance(f, engine.FrequencyTable) or f.include_nulls or f.source is None:
            return None
        keys, counts = f.export_raw()
        if f.key_kind() == N.FREQ_KEYS_VALUES:
            c = f.key_columns[0]
            cols = [G.column_from_canonical(c.name, c.spark_type, keys, c.decimal_precision, c.decimal_scale)]
        else:
            cols = [G.take(_host_key_column(c), keys) for c in f.key_columns]
        return G.GroupBlock(cols, counts, f.num_rows, 0)

    def device_table(self):
        """The state as a device FrequencyTable: a GroupBlock is built once on the GPU, weighted by its counts
        (dq_frequencies_ex), so repeated keys of a merged block add up. A multi-device context (DQ_DEVICES) takes no
        weighted input: the weighted build then runs on a one-device context of this process's GPU."""
        f = self.frequencies
        if isinstance(f, engine.FrequencyTable):
            return f
        ctx = engine.ctx()
        if self._device is None and getattr(ctx, "multi", False):
            with engine.using_context(N.aux_context(ctx.device, "weighted")):
                return self._weighted_table()
        return self._weighted_table()

    def _weighted_table(self):
        from . import groups as G
        f = self.frequencies
        if self._device is None and isinstance(f, G.BlockParts):
            splits = f.split_by_key()
            tables = []
            for s in splits:
                table, counts = s.device_table()
                tables.append(engine.frequencies(table, s.names, False, weights=counts))
            self._device = tables[0] if len(tables) == 1 else SplitFrequencies(tables, f.names, splits)
        elif self._device is None and isinstance(f, G.GroupBlock):
            self._device = engine.frequencies(f.table(), f.names, False, weights=f.counts)
        if self._device is None and isinstance(f, engine.PairFrequencies):
            self._device = f.to_device()
        return self._device

    def summary(self, entropy_rows=None):
        n = self.numRows if entropy_rows is None else entropy_rows
        if isinstance(self.frequencies, dict):
            # a small host-built state (the reference's KAT-sized inputs): the device summary's exact fixed-point sum
            counts = list(self.frequencies.values())
            fx = sum(N.fx_of(-(c / n) * math.log(c / n)) for c in counts) if n else 0
            return {"num_groups": len(counts), "num_unique": sum(1 for c in counts if c == 1),
                    "entropy": N.fx_to_float(fx), "entropy_fx": fx}
        return self.device_table().summary(n)


class SplitFrequencies:
    """A merged string / multi-column state too large for one device build (its key bytes reach the int32 Arrow
    offsets): weighted tables over key-disjoint splits of its groups (groups.BlockParts.split_by_key). A key lives in
    exactly one split, so the fused aggregation over the whole table (A/GroupingAnalyzers.scala:83-120) is the sum
    of the splits' (groups, unique groups, entropy terms), as in the multi-device union of dq_open_devices."""

    def __init__(self, tables, names, splits=None):
        self.tables = list(tables)
        self.names = list(names)
        self.splits = list(splits) if splits is not None else None  # the BlockParts each table was built over
        self.source = None  # no single source table: MutualInformation's marginals need the joint groups in one

    def key_kind(self):
        return self.tables[0].key_kind()

    def summary(self, entropy_rows=None):
        parts = [t.summary(entropy_rows) for t in self.tables]
        fx = sum(p["entropy_fx"] for p in parts)  # exact: the same bits as one table over all the groups
        finite = all(math.isfinite(p["entropy"]) for p in parts)
        return {"num_rows": sum(p["num_rows"] for p in parts), "num_groups": sum(p["num_groups"] for p in parts),
                "num_unique": sum(p["num_unique"] for p in parts),
                "entropy": N.fx_to_float(fx) if finite else float("nan"), "entropy_fx": fx,
                "entropy_rows": parts[0]["entropy_rows"],
                "max_count": max(p["max_count"] for p in parts), "null_count": sum(p["null_count"] for p in parts)}

    def export_raw(self):
        raise ValueError("a split frequency state has no single source table to export representative rows from")

    def distinct_block(self):
        """The aggregated groups as one GroupBlock: each split's (representative row, count) pairs taken from that
        split's own key columns and concatenated -- the splits are key-disjoint, so the groups stay distinct (the
        persisted form of a merged state, state_provider._block_table)."""
        from . import groups as G
        if self.splits is None:
            raise ValueError("a split frequency state without its splits' key columns")
        blocks = []
        for blk, table in zip(self.splits, self.tables):
            keys, counts = table.export_raw()
            blocks.append(G.GroupBlock([G.take(c, keys) for c in blk.columns], counts))
        out = G.concat(blocks, self.splits[0].schema())
        out.distinct = True
        return out


def _block_from_dict(freq, like):
    """A host dict state as a GroupBlock of `like`'s key schema (small Python-built states)."""
    from . import groups as G
    from .table import _column_from_pylist
    if any(c.spark_type == N.TYPE_DECIMAL for c in like.columns):
        return None  # the Python decimal decoding picks its own scale
    keys = list(freq.keys())
    cols = []
    for i, c in enumerate(like.columns):
        items = [k[i] for k in keys]
        items = [float(v) if isinstance(v, engine.GroupFloat) else v for v in items]
        col = _column_from_pylist(c.name, c.spark_type, items)
        col.decimal_precision, col.decimal_scale = c.decimal_precision, c.decimal_scale
        cols.append(col)
    return G.GroupBlock(cols, np.array([freq[k] for k in keys], dtype=np.int64))


def computeFrequencies(data, groupingColumns, include_nulls=False):
    """FrequencyBasedAnalyzer.computeFrequencies (A/GroupingAnalyzers.scala:53-79) on the GPU."""
    table = engine.frequencies(data, list(groupingColumns), include_nulls=include_nulls)
    return FrequenciesAndNumRows(table, table.num_rows, list(groupingColumns))


class GroupingAnalyzer(Analyzer):
    def groupingColumns(self):
        raise NotImplementedError

    def preconditions(self):
        return [Preconditions.hasColumn(c) for c in self.groupingColumns()]


class FrequencyBasedAnalyzer(GroupingAnalyzer):
    _fields = ("columns",)

    def __init__(self, columns):
        self.columns = [columns] if isinstance(columns, str) else list(columns)

    def groupingColumns(self):
        return self.columns

    def computeStateFrom(self, data):
        return computeFrequencies(data, self.groupingColumns())

    def preconditions(self):
        return [Preconditions.atLeastOne(self.columns)] + [Preconditions.hasColumn(c) for c in self.columns]


class ScanShareableFrequencyBasedAnalyzer(FrequencyBasedAnalyzer):
    """A/GroupingAnalyzers.scala:83-120: one fused aggregation over the frequency table."""
    name = None

    @property
    def instance(self):
        return ",".join(self.columns)

    @property
    def entity(self):
        return entityFrom(self.columns)

    def valueFromSummary(self, summary, numRows):
        """The analyzer's aggregation over the table; None when Spark's aggregate is NULL."""
        raise NotImplementedError

    def computeMetricFrom(self, state):
        if state is None:
            return metricFromEmpty(self, self.name, self.instance, self.entity)
        try:
            summ = state.summary()
            v = self.valueFromSummary(summ, state.numRows)
        except Exception as e:
            return self.toFailureMetric(e)
        if v is None:
            return metricFromEmpty(self, self.name, self.instance, self.entity)
        return metricFromValue(v, self.name, self.instance, self.entity)

    def toFailureMetric(self, exception):
        return metricFromFailure(exception, self.name, self.instance, self.entity)


class Uniqueness(ScanShareableFrequencyBasedAnalyzer):
    """A/Uniqueness.scala:26-32: sum(count == 1) / numRows."""
    name = "Uniqueness"

    def valueFromSummary(self, s, numRows):
        return None if s["num_groups"] == 0 else s["num_unique"] / numRows


class Distinctness(ScanShareableFrequencyBasedAnalyzer):
    """A/Distinctness.scala:29-35: sum(count >= 1) / numRows."""
    name = "Distinctness"

    def valueFromSummary(self, s, numRows):
        return None if s["num_groups"] == 0 else s["num_groups"] / numRows


class UniqueValueRatio(ScanShareableFrequencyBasedAnalyzer):
    """A/UniqueValueRatio.scala:25-38: #unique / #groups (getDouble of a NULL sum throws on empty)."""
    name = "UniqueValueRatio"

    def valueFromSummary(self, s, numRows):
        if s["num_groups"] == 0:
            raise MetricCalculationRuntimeException(cause=TypeError("Value at index 0 is null"))
        return s["num_unique"] / s["num_groups"]


class CountDistinct(ScanShareableFrequencyBasedAnalyzer):
    """A/CountDistinct.scala:24-34: count(*) over the table."""
    name = "CountDistinct"

    def valueFromSummary(self, s, numRows):
        return float(s["num_groups"])


class Entropy(ScanShareableFrequencyBasedAnalyzer):
    """A/Entropy.scala:28-42: sum over groups of -(c/N) ln(c/N)."""
    name = "Entropy"
    _fields = ("column",)

    def __init__(self, column):
        super().__init__([column])
        self.column = column

    def valueFromSummary(self, s, numRows):
        return None if s["num_groups"] == 0 else s["entropy"]


class MutualInformation(FrequencyBasedAnalyzer):
    """A/MutualInformation.scala:35-97 (joint table + marginals)."""
    name = "MutualInformation"

    def preconditions(self):
        return [Preconditions.exactlyNColumns(self.columns, 2)] + super().preconditions()

    def computeMetricFrom(self, state):
        inst = ",".join(self.columns)
        if state is None:
            return metricFromEmpty(self, self.name, inst, Entity.Mutlicolumn)
        f = state.frequencies
        if not isinstance(f, (dict, engine.FrequencyTable)):
            f = state.device_table()  # a persisted / merged GroupBlock: its weighted build
        if isinstance(f, engine.FrequencyTable) and f.source is not None and len(f.names) == 2 and \
                state.numRows == f.num_rows:
            # on the GPU: the joint table plus the two marginal tables of the same rows (dq_freq_mutual_information);
            # a merged / loaded state is a weighted build over its groups, and so are its marginals
            x = engine.frequencies(f.source, [f.names[0]], weights=f.weights)
            y = engine.frequencies(f.source, [f.names[1]], weights=f.weights)
            value, present = f.mutual_information(x, y)
            if not present:
                return metricFromEmpty(self, self.name, inst, Entity.Mutlicolumn)
            return metricFromValue(value, self.name, inst, Entity.Mutlicolumn)
        joint = state.as_dict()
        if not joint:
            return metricFromEmpty(self, self.name, inst, Entity.Mutlicolumn)
        total = state.numRows
        px, py = {}, {}
        for (a, b), c in joint.items():
            px[a] = px.get(a, 0) + c
            py[b] = py.get(b, 0) + c
        terms = []
        for (a, b), c in joint.items():
            if a is None or b is None:
                continue  # Spark's equi-join on the marginals drops NULL keys
            pxy = c / total
            terms.append(pxy * math.log(pxy / ((px[a] / total) * (py[b] / total))))
        if not terms:  # sum over zero joined rows is NULL (A/MutualInformation.scala:82-86)
            return metricFromEmpty(self, self.name, inst, Entity.Mutlicolumn)
        return metricFromValue(math.fsum(terms), self.name, inst, Entity.Mutlicolumn)

    def toFailureMetric(self, exception):
        return metricFromFailure(exception, self.name, ",".join(self.columns), Entity.Mutlicolumn)


class Histogram(Analyzer):
    """A/Histogram.scala:41-117: counts per value (nulls as "NullValue"), top-N details."""
    NullFieldReplacement = "NullValue"
    MaximumAllowedDetailBins = 1000
    # case class Histogram(column, binningUdf: Option[UserDefinedFunction], maxDetailBins): the UDF takes
    # part in equality (by identity, as Scala compares the wrapped function object) and in toString
    _fields = ("column", "binningUdf", "maxDetailBins")

    def _key(self):
        udf = None if self.binningUdf is None else ("udf", id(self.binningUdf), self.udfInputAsString)
        return (type(self).__name__, self.column, udf, self.maxDetailBins)

    def __init__(self, column, binningUdf=None, maxDetailBins=MaximumAllowedDetailBins, udfInputAsString=False):
        """`binningUdf` receives each value as the column's type (int, float, Decimal, date, str), as a typed Scala
        UDF does. `udfInputAsString=True` hands it the value's Spark string form instead, as Spark's implicit cast
        does for a UDF declared over String on a non-string column (NULL stays None either way)."""
        self.column, self.binningUdf, self.maxDetailBins = column, binningUdf, maxDetailBins
        self.udfInputAsString = bool(udfInputAsString)

    def preconditions(self):
        def param_check(_):
            if self.maxDetailBins > Histogram.MaximumAllowedDetailBins:
                raise IllegalAnalyzerParameterException(
                    "Cannot return histogram values for more than %d values" % Histogram.MaximumAllowedDetailBins)
        return [param_check, Preconditions.hasColumn(self.column)]

    def computeStateFrom(self, data):
        if self.binningUdf is not None:
            return FrequenciesAndNumRows(self.binned_counts(data), data.count(), [self.column])
        table = engine.frequencies(data, [self.column], include_nulls=True)
        return FrequenciesAndNumRows(table, data.count(), [self.column])

    def binned_counts(self, data):
        """`data.withColumn(column, bin(col(column))).select(col(column).cast(StringType)).na.fill("NullValue")
        .groupBy(column).count()` (A/Histogram.scala:59-65) without a per-row Python call: the column's groups are
        counted on the GPU, the UDF runs once per DISTINCT value (and once for NULL, as a Scala UDF over an object
        type sees the nulls), and the bins add the groups' counts — exact for any deterministic UDF. The UDF receives
        the column's value (str, int, float, ...), as a Spark UDF receives the Scala value. {(bin label,): count}."""
        ft = engine.frequencies(data, [self.column], include_nulls=False)
        col = data[self.column] if self.udfInputAsString else None
        return self.bin_groups(((k[0], c) for k, c in ft.to_dict().items()), data.count() - ft.num_rows, col)

    def bin_groups(self, groups, null_rows, string_column=None):
        """(value, count) groups of the raw column + its NULL rows -> {(bin label,): count}: the UDF's result cast to
        STRING, NULL filled with "NullValue", counts added per bin."""
        bins = {}

        def add(value, count):
            label = self.binningUdf(value)
            label = Histogram.NullFieldReplacement if label is None else (
                label if isinstance(label, str) else _spark_string(label))
            bins[(label,)] = bins.get((label,), 0) + int(count)
        for v, c in groups:
            v = float(v) if isinstance(v, float) else v
            if self.udfInputAsString and v is not None and not isinstance(v, str):
                v = _spark_string(v, string_column)
            add(v, c)
        if null_rows:
            add(None, null_rows)
        return bins

    def computeMetricFrom(self, state):
        if state is None:
            return HistogramMetric(self.column, Failure(emptyStateException(self)))
        try:
            f = state.frequencies
            if isinstance(f, engine.PairFrequencies):  # a persisted state read back: top-N on the device
                f = f.to_device()
            if isinstance(f, dict):
                items = sorted(f.items(), key=lambda kv: -kv[1])[:self.maxDetailBins]
                nbins = len(f)
                details = {(_hist_key(k[0])): DistributionValue(c, c / state.numRows) for k, c in items}
            else:
                nbins = f.num_groups
                col = f.key_columns[0] if f.key_columns else _KeyTypeOnly(f.key_type)
                details = {}
                for key, c in f.top(self.maxDetailBins):
                    details[_hist_key(key[0], col)] = DistributionValue(int(c), int(c) / state.numRows)
            return HistogramMetric(self.column, Success(Distribution(details, nbins)))
        except Exception as e:
            return HistogramMetric(self.column, Failure(wrap_if_necessary(e)))

    def toFailureMetric(self, exception):
        return HistogramMetric(self.column, Failure(wrap_if_necessary(exception)))


class _KeyTypeOnly:
    """The Spark type of a table's key column when the table has no source column (merged / loaded states)."""

    def __init__(self, spark_type, decimal_scale=0):
        self.spark_type, self.decimal_scale = spark_type, decimal_scale


def _spark_string(v, column=None):
    """Spark `Cast(x AS STRING)` for a host value (only top-N keys are ever formatted)."""
    if v is None:
        return None
    t = column.spark_type if column is not None else None
    if isinstance(v, bool):
        return "true" if v else "false"
    if isinstance(v, float) or t in (N.TYPE_FLOAT, N.TYPE_DOUBLE):
        return _java_double_to_string(float(v), t == N.TYPE_FLOAT)
    return str(v)


def _hist_key(v, column=None):
    return Histogram.NullFieldReplacement if v is None else _spark_string(v, column)


def _java_double_to_string(d, is_float=False):
    """java.lang.Double.toString / Float.toString: shortest repr, sci notation outside [1e-3, 1e7)."""
    if math.isnan(d):
        return "NaN"
    if math.isinf(d):
        return "Infinity" if d > 0 else "-Infinity"
    if d == 0.0:
        return "-0.0" if math.copysign(1.0, d) < 0 else "0.0"
    r = repr(float(np.float32(d))) if is_float else repr(d)
    a = abs(d)
    if 1e-3 <= a < 1e7:
        if "e" in r or "E" in r:
            r = ("%f" % d).rstrip("0")
        if "." not in r:
            r += ".0"
        return r
    mant, _, exp = ("%.17e" % d).partition("e")
    digits = repr(d if not is_float else float(np.float32(d)))
    # shortest digits via repr, reformatted as Java's d.dddE<exp>
    m, e = _sci_parts(digits)
    return "%sE%d" % (m, e)


def _sci_parts(r):
    sign = "-" if r.startswith("-") else ""
    r = r.lstrip("-")
    if "e" in r:
        m, e = r.split("e")
        e = int(e)
    else:
        m, e = r, 0
    digits = m.replace(".", "")
    point = m.index(".") if "." in m else len(m)
    stripped = digits.lstrip("0")
    lead = len(digits) - len(stripped)
    e += point - lead - 1
    stripped = stripped.rstrip("0") or "0"
    mant = stripped[0] + "." + (stripped[1:] or "0")
    return sign + mant, e
