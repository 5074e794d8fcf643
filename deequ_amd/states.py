"""deequ's states: commutative semigroups of sufficient statistics (A/Analyzer.scala:29-48), with
conversion from the C-ABI dq_state records. Each `sum` follows the reference state's own file."""
import math

import numpy as np

from . import native as N


class State:
    def sum(self, other):
        raise NotImplementedError

    def __add__(self, other):
        return self.sum(other)


class DoubleValuedState(State):
    def metricValue(self):
        raise NotImplementedError


class NumMatches(DoubleValuedState):
    """A/Size.scala:23-31."""

    def __init__(self, numMatches):
        self.numMatches = int(numMatches)

    def sum(self, other):
        return NumMatches(self.numMatches + other.numMatches)

    def metricValue(self):
        return float(self.numMatches)

    def __eq__(self, o):
        if not isinstance(o, NumMatches):
            return NotImplemented  # let a foreign state (e.g. a test oracle's) compare
        return o.numMatches == self.numMatches

    def __repr__(self):
        return "NumMatches(%d)" % self.numMatches


class NumMatchesAndCount(DoubleValuedState):
    """A/Analyzer.scala:230-244."""

    def __init__(self, numMatches, count):
        self.numMatches, self.count = int(numMatches), int(count)

    def sum(self, other):
        return NumMatchesAndCount(self.numMatches + other.numMatches, self.count + other.count)

    def metricValue(self):
        return float("nan") if self.count == 0 else self.numMatches / self.count

    def __eq__(self, o):
        if not isinstance(o, NumMatchesAndCount):
            return NotImplemented  # let a foreign state (e.g. a test oracle's) compare
        return (o.numMatches, o.count) == (self.numMatches, self.count)

    def __repr__(self):
        return "NumMatchesAndCount(%d,%d)" % (self.numMatches, self.count)


def _long_add(a, b):
    """Spark sums an integral column in a Long (wrapping on overflow) and casts the final total to Double
    (A/Sum.scala:34-37, A/Mean.scala:37-42): partial states of one table split into chunks or shards carry that
    exact Long, so their merge is the Long sum re-cast, not a sum of rounded doubles. States without it (other
    column types, loaded from a state provider) merge as the reference's doubles."""
    ea, eb = getattr(a, "exact", None), getattr(b, "exact", None)
    if ea is None or eb is None:
        return None
    return (ea + eb + (1 << 63)) % (1 << 64) - (1 << 63)


class MeanState(DoubleValuedState):
    """A/Mean.scala:25-34."""

    def __init__(self, sum_, count, exact=None):
        self.sum_, self.count = float(sum_), int(count)
        self.exact = exact  # the exact Long partial of an integral column (see _long_add), else None

    def sum(self, other):
        e = _long_add(self, other)
        if e is not None:
            return MeanState(float(e), self.count + other.count, e)
        return MeanState(self.sum_ + other.sum_, self.count + other.count)

    def metricValue(self):
        return float("nan") if self.count == 0 else self.sum_ / self.count

    def __eq__(self, o):
        if not isinstance(o, MeanState):
            return NotImplemented  # let a foreign state (e.g. a test oracle's) compare
        return (o.sum_, o.count) == (self.sum_, self.count)

    def __repr__(self):
        return "MeanState(%r,%d)" % (self.sum_, self.count)


class SumState(DoubleValuedState):
    """A/Sum.scala:25-33."""

    def __init__(self, sum_, exact=None):
        self.sum_ = float(sum_)
        self.exact = exact

    def sum(self, other):
        e = _long_add(self, other)
        if e is not None:
            return SumState(float(e), e)
        return SumState(self.sum_ + other.sum_)

    def metricValue(self):
        return self.sum_

    def __eq__(self, o):
        if not isinstance(o, SumState):
            return NotImplemented  # let a foreign state (e.g. a test oracle's) compare
        return o.sum_ == self.sum_

    def __repr__(self):
        return "SumState(%r)" % self.sum_


def _java_min(a, b):
    if math.isnan(a) or math.isnan(b):
        return float("nan")
    if a == 0.0 and b == 0.0:
        return a if math.copysign(1, a) < 0 else b
    return a if a <= b else b


def _java_max(a, b):
    if math.isnan(a) or math.isnan(b):
        return float("nan")
    if a == 0.0 and b == 0.0:
        return b if math.copysign(1, a) < 0 else a
    return a if a >= b else b


class MinState(DoubleValuedState):
    """A/Minimum.scala:25-33 (merge = math.min)."""

    def __init__(self, minValue):
        self.minValue = float(minValue)

    def sum(self, other):
        return MinState(_java_min(self.minValue, other.minValue))

    def metricValue(self):
        return self.minValue

    def __eq__(self, o):
        if not isinstance(o, MinState):
            return NotImplemented  # let a foreign state (e.g. a test oracle's) compare
        return o.minValue == self.minValue

    def __repr__(self):
        return "MinState(%r)" % self.minValue


class MaxState(DoubleValuedState):
    """A/Maximum.scala:25-33 (merge = math.max)."""

    def __init__(self, maxValue):
        self.maxValue = float(maxValue)

    def sum(self, other):
        return MaxState(_java_max(self.maxValue, other.maxValue))

    def metricValue(self):
        return self.maxValue

    def __eq__(self, o):
        if not isinstance(o, MaxState):
            return NotImplemented  # let a foreign state (e.g. a test oracle's) compare
        return o.maxValue == self.maxValue

    def __repr__(self):
        return "MaxState(%r)" % self.maxValue


class StandardDeviationState(DoubleValuedState):
    """A/StandardDeviation.scala:25-45 (Chan merge)."""

    def __init__(self, n, avg, m2):
        if not n > 0.0:
            raise ValueError("requirement failed: Standard deviation is undefined for n = 0.")
        self.n, self.avg, self.m2 = float(n), float(avg), float(m2)

    def metricValue(self):
        return math.sqrt(self.m2 / self.n)

    def sum(self, other):
        newN = self.n + other.n
        delta = other.avg - self.avg
        deltaN = 0.0 if newN == 0.0 else delta / newN
        return StandardDeviationState(newN, self.avg + deltaN * other.n,
                                      self.m2 + other.m2 + delta * deltaN * self.n * other.n)

    def __eq__(self, o):
        if not isinstance(o, StandardDeviationState):
            return NotImplemented  # let a foreign state (e.g. a test oracle's) compare
        return (o.n, o.avg, o.m2) == (self.n, self.avg, self.m2)

    def __repr__(self):
        return "StandardDeviationState(%r,%r,%r)" % (self.n, self.avg, self.m2)


class CorrelationState(DoubleValuedState):
    """A/Correlation.scala:26-57."""

    def __init__(self, n, xAvg, yAvg, ck, xMk, yMk):
        if not n > 0.0:
            raise ValueError("requirement failed: Correlation undefined for n = 0.")
        self.n, self.xAvg, self.yAvg, self.ck, self.xMk, self.yMk = map(float, (n, xAvg, yAvg, ck, xMk, yMk))

    def sum(self, other):
        n1, n2 = self.n, other.n
        newN = n1 + n2
        dx = other.xAvg - self.xAvg
        dxN = 0.0 if newN == 0.0 else dx / newN
        dy = other.yAvg - self.yAvg
        dyN = 0.0 if newN == 0.0 else dy / newN
        return CorrelationState(newN, self.xAvg + dxN * n2, self.yAvg + dyN * n2,
                                self.ck + other.ck + dx * dyN * n1 * n2,
                                self.xMk + other.xMk + dx * dxN * n1 * n2,
                                self.yMk + other.yMk + dy * dyN * n1 * n2)

    def metricValue(self):
        d = math.sqrt(self.xMk * self.yMk)
        if d == 0.0:
            return float("nan") if self.ck == 0.0 else math.copysign(float("inf"), self.ck)
        return self.ck / d

    def __eq__(self, o):
        if not isinstance(o, CorrelationState):
            return NotImplemented  # let a foreign state (e.g. a test oracle's) compare
        return \
            (o.n, o.xAvg, o.yAvg, o.ck, o.xMk, o.yMk) == (self.n, self.xAvg, self.yAvg, self.ck, self.xMk, self.yMk)

    def __repr__(self):
        return "CorrelationState(%r,%r,%r,%r,%r,%r)" % (self.n, self.xAvg, self.yAvg, self.ck, self.xMk, self.yMk)


def hll_merge(w1, w2):
    """DeequHyperLogLogPlusPlusUtils.merge (C/StatefulHyperloglogPlus.scala:188-208)."""
    out = []
    idx = 0
    for a, b in zip(w1, w2):
        a &= 0xFFFFFFFFFFFFFFFF
        b &= 0xFFFFFFFFFFFFFFFF
        word, mask = 0, 63
        i = 0
        while idx < 512 and i < 10:
            word |= max(a & mask, b & mask)
            mask <<= 6
            i += 1
            idx += 1
        out.append(word)
    return out


class ApproxCountDistinctState(DoubleValuedState):
    """A/ApproxCountDistinct.scala:26-41: 52 words of 6-bit HLL++ registers (P = 9)."""

    def __init__(self, words):
        self.words = [int(w) & 0xFFFFFFFFFFFFFFFF for w in words]

    def sum(self, other):
        return ApproxCountDistinctState(hll_merge(self.words, other.words))

    def metricValue(self):
        return N.hll_count(self.words)

    def registers(self):
        regs = []
        for w in self.words:
            for k in range(10):
                if len(regs) < 512:
                    regs.append((w >> (6 * k)) & 63)
        return regs

    def __eq__(self, o):
        if not isinstance(o, ApproxCountDistinctState):
            return NotImplemented  # let a foreign state (e.g. a test oracle's) compare
        return o.words == self.words

    def __repr__(self):
        return "ApproxCountDistinctState(%s)" % ",".join(str(np.int64(np.uint64(w))) for w in self.words)


class DataTypeHistogram(State):
    """A/DataType.scala:81-92 (+ toBytes / toDistribution / determineType :94-183)."""
    NULL_POS, FRACTIONAL_POS, INTEGRAL_POS, BOOLEAN_POS, STRING_POS = range(5)
    SIZE_IN_BYTES = 40

    def __init__(self, numNull, numFractional, numIntegral, numBoolean, numString):
        self.numNull, self.numFractional, self.numIntegral = int(numNull), int(numFractional), int(numIntegral)
        self.numBoolean, self.numString = int(numBoolean), int(numString)

    def _t(self):
        return (self.numNull, self.numFractional, self.numIntegral, self.numBoolean, self.numString)

    def sum(self, other):
        return DataTypeHistogram(*[a + b for a, b in zip(self._t(), other._t())])

    def __eq__(self, o):
        if not isinstance(o, DataTypeHistogram):
            return NotImplemented  # let a foreign state (e.g. a test oracle's) compare
        return o._t() == self._t()

    def __repr__(self):
        return "DataTypeHistogram(%d,%d,%d,%d,%d)" % self._t()

    def toBytes(self):
        import struct
        return struct.pack(">5q", *self._t())

    @staticmethod
    def fromBytes(data):
        import struct
        if len(data) != DataTypeHistogram.SIZE_IN_BYTES:
            raise ValueError("requirement failed")
        return DataTypeHistogram(*struct.unpack(">5q", data))

    def toDistribution(self):
        from .metrics import Distribution, DistributionValue
        total = sum(self._t())

        def ratio(x):
            return x / total if total else float("nan")
        return Distribution({
            "Unknown": DistributionValue(self.numNull, ratio(self.numNull)),
            "Fractional": DistributionValue(self.numFractional, ratio(self.numFractional)),
            "Integral": DistributionValue(self.numIntegral, ratio(self.numIntegral)),
            "Boolean": DistributionValue(self.numBoolean, ratio(self.numBoolean)),
            "String": DistributionValue(self.numString, ratio(self.numString))}, 5)

    @staticmethod
    def determineType(dist):
        """DataTypeHistogram.determineType (A/DataType.scala:143-171)."""
        def r(k):
            v = dist.values.get(k)
            return 0.0 if v is None else v.ratio
        if r("Unknown") == 1.0:
            return "Unknown"
        if r("String") > 0.0 or (r("Boolean") > 0.0 and (r("Integral") > 0.0 or r("Fractional") > 0.0)):
            return "String"
        if r("Boolean") > 0.0:
            return "Boolean"
        if r("Fractional") > 0.0:
            return "Fractional"
        return "Integral"


class ApproxQuantileState(State):
    """A/ApproxQuantile.scala:28-36: wraps a PercentileDigest; sum = PercentileDigest.merge."""

    def __init__(self, percentileDigest):
        self.percentileDigest = percentileDigest

    def sum(self, other):
        return ApproxQuantileState(self.percentileDigest.merge(other.percentileDigest))

    def __repr__(self):
        s = self.percentileDigest.quantileSummaries
        return "ApproxQuantileState(count=%d, samples=%d)" % (s.count, len(s.sampled))


def state_to_native(kind, state):
    """Reference State (or None) -> dq_state record of op `kind` (persisted / exchanged states)."""
    st = N.DqState()
    st.kind = kind
    st.present = 0 if state is None else 1
    if state is None:
        return st
    u = st.u
    if isinstance(state, NumMatches):
        u.num_matches.num_matches = state.numMatches
    elif isinstance(state, NumMatchesAndCount):
        u.num_matches_and_count.num_matches = state.numMatches
        u.num_matches_and_count.count = state.count
    elif isinstance(state, MeanState):
        u.mean.sum, u.mean.count = state.sum_, state.count
        if getattr(state, "exact", None) is not None:
            u.mean.isum, u.mean.exact = state.exact, 1
    elif isinstance(state, SumState):
        u.dbl.value = state.sum_
        if getattr(state, "exact", None) is not None:
            u.dbl.isum, u.dbl.exact = state.exact, 1
    elif isinstance(state, MinState):
        u.dbl.value = state.minValue
    elif isinstance(state, MaxState):
        u.dbl.value = state.maxValue
    elif isinstance(state, StandardDeviationState):
        u.stddev.n, u.stddev.avg, u.stddev.m2 = state.n, state.avg, state.m2
    elif isinstance(state, CorrelationState):
        c = u.corr
        c.n, c.x_avg, c.y_avg, c.ck, c.x_mk, c.y_mk = state.n, state.xAvg, state.yAvg, state.ck, state.xMk, state.yMk
    elif isinstance(state, ApproxCountDistinctState):
        for i, w in enumerate(state.words):
            u.hll.words[i] = int(np.int64(np.uint64(w)))
    elif isinstance(state, DataTypeHistogram):
        d = u.datatype
        d.num_null, d.num_fractional, d.num_integral, d.num_boolean, d.num_string = state._t()
    else:
        raise ValueError("cannot encode %r" % (state,))
    return st


def state_from_native(st):
    """dq_state -> reference State (None for an absent state, i.e. ifNoNullsIn failed)."""
    if not st.present:
        return None
    k = st.kind
    u = st.u
    if k == N.OP_SIZE:
        return NumMatches(u.num_matches.num_matches)
    if k in (N.OP_COMPLETENESS, N.OP_COMPLIANCE):
        return NumMatchesAndCount(u.num_matches_and_count.num_matches, u.num_matches_and_count.count)
    if k == N.OP_MEAN:
        return MeanState(u.mean.sum, u.mean.count, u.mean.isum if u.mean.exact else None)
    if k == N.OP_SUM:
        return SumState(u.dbl.value, u.dbl.isum if u.dbl.exact else None)
    if k in (N.OP_MINIMUM, N.OP_MIN_LENGTH):
        return MinState(u.dbl.value)
    if k in (N.OP_MAXIMUM, N.OP_MAX_LENGTH):
        return MaxState(u.dbl.value)
    if k == N.OP_STANDARD_DEVIATION:
        if u.stddev.n == 0.0:
            return None
        return StandardDeviationState(u.stddev.n, u.stddev.avg, u.stddev.m2)
    if k == N.OP_CORRELATION:
        if not u.corr.n > 0.0:
            return None
        return CorrelationState(u.corr.n, u.corr.x_avg, u.corr.y_avg, u.corr.ck, u.corr.x_mk, u.corr.y_mk)
    if k == N.OP_APPROX_COUNT_DISTINCT:
        return ApproxCountDistinctState(list(u.hll.words))
    if k == N.OP_DATATYPE:
        d = u.datatype
        return DataTypeHistogram(d.num_null, d.num_fractional, d.num_integral, d.num_boolean, d.num_string)
    raise ValueError("unknown state kind %d" % k)
