"""Metric result types (M/metrics/Metric.scala:21-68, M/metrics/HistogramMetric.scala:21-61) and the
exception taxonomy failures are wrapped in (R/MetricCalculationException.scala:19-78)."""
import enum
import math


class Entity(enum.Enum):
    Dataset = "Dataset"
    Column = "Column"
    Mutlicolumn = "Mutlicolumn"  # (sic) the reference's spelling, kept for JSON parity

    def __str__(self):
        return self.value


# ---- scala.util.Try ------------------------------------------------------------------------------
class Success:
    def __init__(self, value):
        self.value = value

    isSuccess = property(lambda self: True)
    isFailure = property(lambda self: False)

    def get(self):
        return self.value

    def __eq__(self, other):
        if not isinstance(other, Success):
            return False
        a, b = self.value, other.value
        if isinstance(a, float) and isinstance(b, float) and math.isnan(a) and math.isnan(b):
            return True
        return a == b

    def __hash__(self):
        return hash(("Success", self.value))

    def __repr__(self):
        return "Success(%r)" % (self.value,)


class Failure:
    def __init__(self, exception):
        self.exception = exception

    isSuccess = property(lambda self: False)
    isFailure = property(lambda self: True)

    def get(self):
        raise self.exception

    @property
    def failed(self):
        return self.exception

    def __eq__(self, other):
        return isinstance(other, Failure) and type(self.exception) is type(other.exception) and \
            str(self.exception) == str(other.exception)

    def __hash__(self):
        return hash(("Failure", type(self.exception).__name__))

    def __repr__(self):
        return "Failure(%s: %s)" % (type(self.exception).__name__, self.exception)


# ---- exceptions (R/MetricCalculationException.scala) --------------------------------------------
class MetricCalculationException(Exception):
    pass


class MetricCalculationRuntimeException(MetricCalculationException):
    def __init__(self, message=None, cause=None):
        if message is None and cause is not None:
            message = "%s: %s" % (type(cause).__name__, cause)
        super().__init__(message)
        self.cause = cause


class MetricCalculationPreconditionException(MetricCalculationException):
    pass


class NoSuchColumnException(MetricCalculationPreconditionException):
    pass


class WrongColumnTypeException(MetricCalculationPreconditionException):
    pass


class NoColumnsSpecifiedException(MetricCalculationPreconditionException):
    pass


class NumberOfSpecifiedColumnsException(MetricCalculationPreconditionException):
    pass


class IllegalAnalyzerParameterException(MetricCalculationPreconditionException):
    pass


class EmptyStateException(MetricCalculationRuntimeException):
    pass


class UnsupportedOnDevice(MetricCalculationRuntimeException):
    """An analyzer configuration this engine does not evaluate on the GPU (e.g. a regex construct
    outside the supported java.util.regex subset). It fails that analyzer only — never a CPU path."""


def wrap_if_necessary(exception):
    """MetricCalculationException.wrapIfNecessary (R/MetricCalculationException.scala:69-76)."""
    if isinstance(exception, MetricCalculationException):
        return exception
    return MetricCalculationRuntimeException(cause=exception)


# ---- metrics -------------------------------------------------------------------------------------
class Metric:
    entity = None
    instance = None
    name = None
    value = None

    def flatten(self):
        raise NotImplementedError


class DoubleMetric(Metric):
    def __init__(self, entity, name, instance, value):
        self.entity, self.name, self.instance, self.value = entity, name, instance, value

    def flatten(self):
        return [self]

    def __eq__(self, other):
        return isinstance(other, DoubleMetric) and (self.entity, self.name, self.instance) == \
            (other.entity, other.name, other.instance) and self.value == other.value

    def __hash__(self):
        return hash((self.entity, self.name, self.instance))

    def __repr__(self):
        return "DoubleMetric(%s,%s,%s,%r)" % (self.entity, self.name, self.instance, self.value)


class KeyedDoubleMetric(Metric):
    """M/metrics/Metric.scala:51-68 (ApproxQuantiles): a map of quantile string -> value."""

    def __init__(self, entity, name, instance, value):
        self.entity, self.name, self.instance, self.value = entity, name, instance, value

    def flatten(self):
        if self.value.isSuccess:
            return [DoubleMetric(self.entity, "%s-%s" % (self.name, k), self.instance, Success(v))
                    for k, v in self.value.get().items()]
        return [DoubleMetric(self.entity, self.name, self.instance, Failure(self.value.failed))]

    def __eq__(self, other):
        return isinstance(other, KeyedDoubleMetric) and (self.entity, self.name, self.instance) == \
            (other.entity, other.name, other.instance) and self.value == other.value

    def __hash__(self):
        return hash((self.entity, self.name, self.instance))

    def __repr__(self):
        return "KeyedDoubleMetric(%s,%s,%s,%r)" % (self.entity, self.name, self.instance, self.value)


class DistributionValue:
    def __init__(self, absolute, ratio):
        self.absolute, self.ratio = absolute, ratio

    def __eq__(self, other):
        return isinstance(other, DistributionValue) and self.absolute == other.absolute and self.ratio == other.ratio

    def __repr__(self):
        return "DistributionValue(%d,%r)" % (self.absolute, self.ratio)


class Distribution:
    def __init__(self, values, numberOfBins):
        self.values, self.numberOfBins = values, numberOfBins

    def __getitem__(self, key):
        return self.values[key]

    def __eq__(self, other):
        return isinstance(other, Distribution) and self.values == other.values and \
            self.numberOfBins == other.numberOfBins

    def __repr__(self):
        return "Distribution(%r,%d)" % (self.values, self.numberOfBins)


class HistogramMetric(Metric):
    """M/metrics/HistogramMetric.scala:21-61."""

    def __init__(self, column, value):
        self.column = column
        self.value = value
        self.entity = Entity.Column
        self.instance = column
        self.name = "Histogram"

    def flatten(self):
        if self.value.isFailure:
            return [DoubleMetric(self.entity, "%s.bins" % self.name, self.instance, Failure(self.value.failed))]
        dist = self.value.get()
        out = [DoubleMetric(self.entity, "%s.bins" % self.name, self.instance, Success(float(dist.numberOfBins)))]
        for key, v in dist.values.items():
            out.append(DoubleMetric(self.entity, "%s.abs.%s" % (self.name, key), self.instance,
                                    Success(float(v.absolute))))
            out.append(DoubleMetric(self.entity, "%s.ratio.%s" % (self.name, key), self.instance,
                                    Success(v.ratio)))
        return out

    def __eq__(self, other):
        return isinstance(other, HistogramMetric) and self.column == other.column and self.value == other.value

    def __repr__(self):
        return "HistogramMetric(%s,%r)" % (self.column, self.value)
