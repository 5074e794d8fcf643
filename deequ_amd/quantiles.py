"""Spark's Greenwald-Khanna summary as deequ uses it for ApproxQuantile(s).

deequ's ApproxQuantileState wraps Spark's `ApproximatePercentile.PercentileDigest`
(A/ApproxQuantile.scala:28-36; StatefulApproxQuantile, C/StatefulApproxQuantile.scala:28-111,
adjusted from Spark v2.2.0). The digest is Spark's `QuantileSummaries` (spark-catalyst 2.2.2 —
third-party, absent from /root/reference); its published merge / compress / query / serialization
rules are restated here so states built on the GPU behave like the reference's: they merge
(`ApproxQuantileState.sum`), answer `getPercentiles`, and serialize in the PercentileDigest byte
layout the reference persists (A/StateProvider.scala, ApproxQuantile case).

The GPU (dq_quantile_summary, deequ_amd/csrc/quantile.hip) returns EXACT order statistics:
  * n < defaultHeadSize (50000): all n sorted values, from which the digest Spark builds for one
    partition is reproduced exactly (`spark_single_partition`) — Spark's own answer;
  * otherwise ranks 1, n and every max(1, floor(relativeError * n))-th rank: a summary whose samples
    have delta = 0 and g = the rank gap. That is a valid GK summary (g + delta <= 2 relativeError n),
    so every query is within the declared relativeError rank bound — the parity criterion
    BASELINE.json states for ApproxQuantile (Spark's own sketch, which depends on partitioning and
    row order at this size, returns different, equally bounded values).
"""
import math
import struct

DEFAULT_COMPRESS_THRESHOLD = 10000  # QuantileSummaries.defaultCompressThreshold
DEFAULT_HEAD_SIZE = 50000  # QuantileSummaries.defaultHeadSize: insert() flushes the head buffer at this size


class Stats:
    """QuantileSummaries.Stats(value, g, delta)."""
    __slots__ = ("value", "g", "delta")

    def __init__(self, value, g, delta):
        self.value, self.g, self.delta = float(value), int(g), int(delta)

    def __repr__(self):
        return "Stats(%r,%d,%d)" % (self.value, self.g, self.delta)

    def __eq__(self, other):
        return isinstance(other, Stats) and (self.value, self.g, self.delta) == (other.value, other.g, other.delta)


def _java_double_key(v):
    """Ordering.Double (java.lang.Double.compare): -0.0 < 0.0, NaN largest."""
    if v != v:
        return (2, 0.0, 0)
    return (0, v, 0 if math.copysign(1.0, v) < 0 else 1)  # -0.0 just below 0.0, above every negative


def _compress_immut(current, merge_threshold):
    """QuantileSummaries.compressImmut (Spark 2.2)."""
    if not current:
        return []
    res = []
    head = current[-1]
    i = len(current) - 2
    while i >= 1:  # the last element is never compressed
        sample1 = current[i]
        if sample1.g + head.g + head.delta < merge_threshold:
            head = Stats(head.value, head.g + sample1.g, head.delta)
        else:
            res.append(head)
            head = sample1
        i -= 1
    res.append(head)
    curr_head = current[0]
    # add the minimum unless `current` has a single element (IEEE `<=`, as in the Scala source)
    if curr_head.value <= head.value and len(current) > 1:
        res.append(curr_head)
    res.reverse()
    return res


class QuantileSummaries:
    """org.apache.spark.sql.catalyst.util.QuantileSummaries (Spark 2.2), compressed form only: the GPU
    delivers compressed summaries, so `headSampled` is always empty."""

    def __init__(self, compressThreshold, relativeError, sampled=None, count=0):
        self.compressThreshold = int(compressThreshold)
        self.relativeError = float(relativeError)
        self.sampled = list(sampled or [])
        self.count = int(count)

    def merge(self, other):
        """QuantileSummaries.merge: concatenate, sort by value, compress with threshold
        2 * relativeError * count (Spark uses the LEFT summary's count here)."""
        if other.count == 0:
            return QuantileSummaries(self.compressThreshold, self.relativeError, self.sampled, self.count)
        if self.count == 0:
            return QuantileSummaries(other.compressThreshold, other.relativeError, other.sampled, other.count)
        res = sorted(self.sampled + other.sampled, key=lambda s: _java_double_key(s.value))  # stable, like sortBy
        comp = _compress_immut(res, 2 * self.relativeError * self.count)
        return QuantileSummaries(other.compressThreshold, other.relativeError, comp, other.count + self.count)

    def query(self, quantile):
        """QuantileSummaries.query (Spark 2.2): the first sample whose rank interval, widened by
        ceil(relativeError * count), contains ceil(quantile * count)."""
        if not (0.0 <= quantile <= 1.0):
            raise ValueError("requirement failed: quantile should be in the range [0.0, 1.0]")
        if quantile <= self.relativeError:
            return self.sampled[0].value
        if quantile >= 1 - self.relativeError:
            return self.sampled[-1].value
        rank = int(math.ceil(quantile * self.count))
        target_error = math.ceil(self.relativeError * self.count)
        min_rank = 0
        i = 1
        while i < len(self.sampled) - 1:
            cur = self.sampled[i]
            min_rank += cur.g
            max_rank = min_rank + cur.delta
            if max_rank - target_error <= rank <= min_rank + target_error:
                return cur.value
            i += 1
        return self.sampled[-1].value


class PercentileDigest:
    """ApproximatePercentile.PercentileDigest (Spark 2.2) over an already-compressed summary."""

    def __init__(self, summaries):
        self.quantileSummaries = summaries

    @staticmethod
    def from_order_statistics(relativeError, values, ranks, count):
        """The zero-uncertainty summary built from the GPU's exact (value, rank) samples."""
        sampled = []
        prev = 0
        for v, r in zip(values, ranks):
            sampled.append(Stats(v, int(r) - prev, 0))
            prev = int(r)
        return PercentileDigest(QuantileSummaries(DEFAULT_COMPRESS_THRESHOLD, relativeError, sampled, count))

    @staticmethod
    def spark_single_partition(relativeError, sorted_values):
        """The digest Spark itself builds when all n < defaultHeadSize values of a column arrive in one
        partition (the reference's test harness runs `local`, one partition): no head-buffer flush
        happens during insert(), so the result depends only on the sorted values —
        withHeadBufferInserted (each value Stats(v, 1, floor(2 * relativeError * i)), delta 0 for
        the first and the last) followed by compress() = compressImmut(.., 2 * relativeError * n)."""
        n = len(sorted_values)
        samples = []
        for i, v in enumerate(sorted_values):
            cur = i + 1
            delta = 0 if (i == 0 or i == n - 1) else int(math.floor(2 * relativeError * cur))
            samples.append(Stats(v, 1, delta))
        comp = _compress_immut(samples, 2 * relativeError * n)
        return PercentileDigest(QuantileSummaries(DEFAULT_COMPRESS_THRESHOLD, relativeError, comp, n))

    def merge(self, other):
        return PercentileDigest(self.quantileSummaries.merge(other.quantileSummaries))

    def getPercentiles(self, percentages):
        s = self.quantileSummaries
        if s.count == 0 or len(percentages) == 0:
            return []
        return [s.query(p) for p in percentages]

    # PercentileDigestSerializer (big-endian ByteBuffer): relativeError, count, #samples, then
    # (value: double, g: int, delta: int) per sample.
    def serialize(self):
        s = self.quantileSummaries
        out = [struct.pack(">dqi", s.relativeError, s.count, len(s.sampled))]
        for st in s.sampled:
            out.append(struct.pack(">dii", st.value, st.g, st.delta))
        return b"".join(out)

    @staticmethod
    def deserialize(data):
        rel, count, n = struct.unpack_from(">dqi", data, 0)
        off = 20
        sampled = []
        for _ in range(n):
            v, g, d = struct.unpack_from(">dii", data, off)
            off += 16
            sampled.append(Stats(v, g, d))
        return PercentileDigest(QuantileSummaries(DEFAULT_COMPRESS_THRESHOLD, rel, sampled, count))
