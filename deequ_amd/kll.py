"""KLLSketch: deequ's deterministic KLL quantile sketch (A/KLLSketch.scala, A/QuantileNonSample.scala,
A/NonSampleCompactor.scala, R/KLLRunner.scala, M/metrics/KLLMetric.scala).

The per-row sketching (KLLRunner.sketchPartitions' `updateUntyped` loop) runs on the GPU
(dq_kll_sketch, deequ_amd/csrc/kll.hip), which returns the KLLState bytes of one partition holding
the column in row order. This module is the host side the reference runs on the driver: the state
(de)serialization (KLLState.fromBytes, KLLSketchSerializer), the sketch merge (QuantileNonSample.merge,
used by KLLState.sum and KLLRunner's treeReduce over partitions), rank and quantile queries, and the
metric (KLLSketch.computeMetricFrom -> BucketDistribution / KLLMetric). All of it works on a few
thousand sketch items, never on rows.
"""
import math
import struct

from .metrics import DoubleMetric, Entity, Failure, Success

DEFAULT_SKETCH_SIZE = 2048  # KLLSketch.DEFAULT_SKETCH_SIZE
DEFAULT_SHRINKING_FACTOR = 0.64  # KLLSketch.DEFAULT_SHRINKING_FACTOR
MAXIMUM_ALLOWED_DETAIL_BINS = 100  # KLLSketch.MAXIMUM_ALLOWED_DETAIL_BINS


def _order_key(v):
    """Ordering.Double.compare (java.lang.Double.compare): -0.0 < 0.0, NaN largest — what `.sorted`
    and `sortBy` use."""
    if v != v:
        return (2, 0.0, 0)
    return (0, v, 0 if math.copysign(1.0, v) < 0 else 1)  # -0.0 just below 0.0, above every negative


def _sorted_java(items):
    """sorted(items, key=_order_key) (a stable sort by Double.compare): on int64 keys that order like
    Double.compare (the bits of a canonical NaN, sign-flipped for negatives) for more than a few items."""
    if len(items) < 64:
        return sorted(items, key=_order_key)
    import numpy as np
    a = np.asarray(items, dtype=np.float64)
    b = a.view(np.int64).copy()
    b[np.isnan(a)] = 0x7FF8000000000000
    k = b ^ ((b >> 63) & 0x7FFFFFFFFFFFFFFF)
    return a[np.argsort(k, kind="stable")].tolist()


def _capacity(sketch_size, shrinking_factor, height):
    """QuantileNonSample.capacity (A/QuantileNonSample.scala:87-89)."""
    return 2 * (int(math.ceil(sketch_size * math.pow(shrinking_factor, height) / 2)) + 1)


class NonSampleCompactor:
    """A/NonSampleCompactor.scala:29-69 (the Random offset is commented out in the reference)."""

    __slots__ = ("numOfCompress", "offset", "buffer")

    def __init__(self, numOfCompress=0, offset=0, buffer=None):
        self.numOfCompress, self.offset = int(numOfCompress), int(offset)
        self.buffer = list(buffer or [])

    def copy(self):
        return NonSampleCompactor(self.numOfCompress, self.offset, self.buffer)

    def compact(self):
        items = len(self.buffer)
        ln = items - items % 2
        if self.numOfCompress % 2 == 1:
            self.offset = 1 - self.offset
        srt = _sorted_java(self.buffer[:ln])
        output = srt[self.offset:ln:2]
        self.buffer = [self.buffer[items - 1]] if items % 2 == 1 else []
        self.numOfCompress += 1
        return output


class QuantileNonSample:
    """A/QuantileNonSample.scala:24-306 over doubles (the only instantiation deequ uses)."""

    def __init__(self, sketchSize=DEFAULT_SKETCH_SIZE, shrinkingFactor=DEFAULT_SHRINKING_FACTOR, compactors=None,
                 curNumOfCompactors=None, compactorActualSize=None, compactorTotalSize=None):
        self.sketchSize = int(sketchSize)
        self.shrinkingFactor = float(shrinkingFactor)
        if compactors is None:  # the constructor calls expand() once
            self.compactors = []
            self.curNumOfCompactors = 0
            self.compactorActualSize = 0
            self.compactorTotalSize = 0
            self.expand()
        else:
            self.compactors = compactors
            self.curNumOfCompactors = int(curNumOfCompactors)
            self.compactorActualSize = int(compactorActualSize)
            self.compactorTotalSize = int(compactorTotalSize)
        self._np_levels = None  # the buffers as float64 arrays (read paths); dropped by every mutation

    def copy(self):
        return QuantileNonSample(self.sketchSize, self.shrinkingFactor, [c.copy() for c in self.compactors],
                                 self.curNumOfCompactors, self.compactorActualSize, self.compactorTotalSize)

    def capacity(self, height):
        return _capacity(self.sketchSize, self.shrinkingFactor, height)

    def expand(self):
        self._np_levels = None
        self.compactors.append(NonSampleCompactor())
        self.curNumOfCompactors = len(self.compactors)
        self.compactorTotalSize = self.getCompactorCapacityCount()

    def reconstruct(self, sketchSize, shrinkingFactor, data):
        self._np_levels = None
        self.sketchSize, self.shrinkingFactor = int(sketchSize), float(shrinkingFactor)
        self.compactors = [NonSampleCompactor(buffer=list(d)) for d in data]
        self.curNumOfCompactors = len(data)
        self.compactorActualSize = self.getCompactorItemsCount()
        self.compactorTotalSize = self.getCompactorCapacityCount()

    def getCompactorItems(self):
        return [list(c.buffer) for c in self.compactors]

    def update(self, item):
        """QuantileNonSample.update (host-side restatement; the GPU runs this loop for real data)."""
        self._np_levels = None
        self.compactors[0].buffer.append(float(item))
        self.compactorActualSize += 1
        if self.compactorActualSize > self.compactorTotalSize:
            self.condense()

    def condense(self):
        self._np_levels = None
        for height in range(len(self.compactors)):
            if len(self.compactors[height].buffer) >= self.capacity(height):
                if height + 1 >= self.curNumOfCompactors:
                    self.expand()
                output = self.compactors[height].compact()
                self.compactors[height + 1].buffer.extend(output)
                self.compactorActualSize = self.getCompactorItemsCount()
                break

    def merge(self, that):
        """QuantileNonSample.merge (A/QuantileNonSample.scala:218-234); returns a new sketch (the
        Scala version mutates and returns `this`)."""
        out = self.copy()
        while out.curNumOfCompactors < that.curNumOfCompactors:
            out.expand()
        for i in range(that.curNumOfCompactors):
            out.compactors[i].buffer = out.compactors[i].buffer + list(that.compactors[i].buffer)
        out.compactorActualSize = out.getCompactorItemsCount()
        while out.compactorActualSize >= out.compactorTotalSize:
            out.condense()
        return out

    def _output(self):
        out = []
        for i, c in enumerate(self.compactors[:self.curNumOfCompactors]):
            w = 1 << i
            out.extend((v, w) for v in c.buffer)
        return out

    def _levels(self):
        import numpy as np
        if self._np_levels is None:
            self._np_levels = [np.asarray(c.buffer, dtype=np.float64) for c in self.compactors]
        return self._np_levels

    def _output_arrays(self):
        import numpy as np
        lv = self._levels()
        items = np.concatenate(lv[:self.curNumOfCompactors] or [np.zeros(0)])
        weights = np.concatenate([np.full(len(c.buffer), 1 << i, dtype=np.int64)
                                  for i, c in enumerate(self.compactors[:self.curNumOfCompactors])] or
                                 [np.zeros(0, dtype=np.int64)])
        return items, weights

    def getRank(self, item):
        """Inclusive rank: Ordering.Double.gt is IEEE `>` in Scala 2.11, so NaN targets count."""
        return int(self.getRanks([item], exclusive=False)[0])

    def getRankExclusive(self, item):
        return int(self.getRanks([item], exclusive=True)[0])

    def _rank_index(self):
        """(IEEE-sorted non-NaN items, cumulative weights with a leading 0, total weight of NaN items)."""
        import numpy as np
        t, w = self._output_arrays()
        nan = np.isnan(t)
        keep = ~nan
        # any order of equal items gives the same cumulative weight at a tie group's ends, which is all the binary
        # searches below read: no stable sort needed (5x faster than kind="stable" on a sketch's ~6k items)
        order = np.argsort(t[keep])
        ts = t[keep][order]
        cw = np.concatenate([np.zeros(1, dtype=np.int64), np.cumsum(w[keep][order])])
        return ts, cw, int(w[nan].sum())

    def getRanks(self, items, exclusive, index=None):
        """getRank / getRankExclusive for many query items at once, with the reference's IEEE comparisons:
        exclusive = weight of items `< q` (none for a NaN query); inclusive = weight of items with `!(item > q)`,
        i.e. items <= q plus every NaN item (all items for a NaN query). Binary searches over the sorted items."""
        import numpy as np
        ts, cw, nanw = index if index is not None else self._rank_index()
        q = np.asarray(items, dtype=np.float64)
        qnan = np.isnan(q)
        qq = np.where(qnan, 0.0, q)
        if exclusive:
            r = cw[np.searchsorted(ts, qq, side="left")]
            return np.where(qnan, 0, r)
        r = cw[np.searchsorted(ts, qq, side="right")] + nanw
        return np.where(qnan, cw[-1] + nanw, r)

    def quantiles(self, q):
        """QuantileNonSample.quantiles (A/QuantileNonSample.scala:249-281): items sorted in Double.compare order,
        the walk over cumulative weights done with binary searches (same picks as the reference's loop, including
        the entries left at the first item once the walk has consumed the last one)."""
        import numpy as np
        t, w = self._output_arrays()
        n = len(t)
        if n == 0:
            return []
        u = t.view(np.uint64).copy()
        u[np.isnan(t)] = np.uint64(0x7ff8000000000000)
        key = np.where((u >> np.uint64(63)) != 0, ~u, u | np.uint64(1 << 63))
        order = np.argsort(key)  # the walk needs the stable order only inside runs of equal keys
        sk = key[order]
        if n > 1 and bool((sk[1:] == sk[:-1]).any()):
            order = np.argsort(key, kind="stable")
        ts, c = t[order], np.cumsum(w[order])
        total = int(c[-1])
        if q < 2:
            return []
        # the walk, vectorised: i_k = max(i_{k-1}, searchsorted(c, thresh_k) + 1) for thresh_k > 0 (the thresholds
        # rise, so a running maximum); entries whose walk has already passed the last item keep ts[0]
        curq = np.arange(1, q, dtype=np.int64)
        thresh = (curq * total) // q if total < (1 << 62) // max(q, 1) else \
            np.array([k * total // q for k in range(1, q)], dtype=object).astype(np.int64)
        step = np.where(thresh > 0, np.searchsorted(c, thresh, side="left") + 1, 0)
        i = np.maximum.accumulate(step)
        prev = np.concatenate([[0], i[:-1]])
        res = np.where(prev < n, ts[np.minimum(i, n - 1)], ts[0])
        return [float(x) for x in res]

    def getCompactorItemsCount(self):
        return sum(len(c.buffer) for c in self.compactors[:self.curNumOfCompactors])

    def getCompactorCapacityCount(self):
        return sum(self.capacity(h) for h in range(self.curNumOfCompactors))

    # KLLSketchSerializer (A/catalyst/KLLSketchSerializer.scala:60-118), big-endian ByteBuffer
    def serialize(self):
        out = [struct.pack(">idiiii", self.sketchSize, self.shrinkingFactor, self.curNumOfCompactors,
                           self.compactorActualSize, self.compactorTotalSize, len(self.compactors))]
        for c in self.compactors:
            out.append(struct.pack(">iii", c.numOfCompress, c.offset, len(c.buffer)))
            out.append(struct.pack(">%dd" % len(c.buffer), *c.buffer))
        return b"".join(out)

    @staticmethod
    def deserialize(data, off=0):
        size, f, cur, actual, total, ncomp = struct.unpack_from(">idiiii", data, off)
        off += 28
        import numpy as np
        comps, levels = [], []
        for _ in range(ncomp):
            nc, o, ln = struct.unpack_from(">iii", data, off)
            off += 12
            arr = np.frombuffer(data, dtype=">f8", count=ln, offset=off).astype(np.float64)
            off += 8 * ln
            comps.append(NonSampleCompactor(nc, o, arr.tolist()))
            levels.append(arr)
        q = QuantileNonSample(size, f, comps, cur, actual, total)
        q._np_levels = levels
        return q


def _java_min(a, b):
    """java.lang.Math.min on doubles (NaN-propagating, -0.0 < 0.0)."""
    if a != a or b != b:
        return float("nan")
    return a if _order_key(a) <= _order_key(b) else b


def _java_max(a, b):
    if a != a or b != b:
        return float("nan")
    return a if _order_key(a) >= _order_key(b) else b


class KLLState:
    """A/KLLSketch.scala:32-67."""

    def __init__(self, qSketch, globalMax, globalMin, raw=None):
        self._q, self.globalMax, self.globalMin = qSketch, float(globalMax), float(globalMin)
        self._raw = raw  # the serialized state this one was read from (the sketch is parsed on first use)

    @property
    def qSketch(self):
        if self._q is None:
            self._q = QuantileNonSample.deserialize(self._raw, 16)
        return self._q

    @qSketch.setter
    def qSketch(self, q):
        self._q, self._raw = q, None

    def sum(self, other):
        """KLLState.sum (A/KLLSketch.scala:49-54) through the library's merge (dq_kll_merge_states): the same
        QuantileNonSample.merge + condense as `self.qSketch.merge(other.qSketch)` below, without the Python list work
        (13 columns x chunk merges sat between the C5 profiler's passes)."""
        from .native import kll_merge_states, NativeError
        try:
            return KLLState.fromBytes(kll_merge_states(self.toBytes(), other.toBytes()))
        except (OSError, NativeError) as e:
            if isinstance(e, NativeError) and "malformed" in str(e):
                raise
            # the merge is host-only state algebra: without a loadable libdq.so (a host with no ROCm runtime merging
            # persisted states, runOnAggregatedStates) the restated merge gives the same bytes
            return self.sum_restated(other)

    def sum_restated(self, other):
        """KLLState.sum over the Python QuantileNonSample (the library's merge is checked against it)."""
        return KLLState(self.qSketch.merge(other.qSketch), _java_max(self.globalMax, other.globalMax),
                        _java_min(self.globalMin, other.globalMin))

    @staticmethod
    def fromBytes(data):
        mn, mx = struct.unpack_from(">dd", data, 0)
        off = 16 + 28  # the layout is checked now (headers only), as an eager parse would
        ncomp = struct.unpack_from(">i", data, 40)[0]
        for _ in range(ncomp):
            off += 12 + 8 * struct.unpack_from(">i", data, off + 8)[0]
        if off > len(data):
            raise struct.error("KLLState bytes truncated")
        return KLLState(None, mx, mn, raw=bytes(data))

    def toBytes(self):
        """StatefulKLLSketch.toBytes layout (C/StatefulKLLSketch.scala:86-92): min, max, sketch."""
        if self._q is None:
            return self._raw
        return struct.pack(">dd", self.globalMin, self.globalMax) + self.qSketch.serialize()

    def __eq__(self, other):
        return isinstance(other, KLLState) and self.toBytes() == other.toBytes()


class KLLParameters:
    """A/KLLSketch.scala:75-80."""

    def __init__(self, sketchSize, shrinkingFactor, numberOfBuckets):
        self.sketchSize, self.shrinkingFactor, self.numberOfBuckets = int(sketchSize), float(shrinkingFactor), \
            int(numberOfBuckets)

    def _key(self):
        return (self.sketchSize, self.shrinkingFactor, self.numberOfBuckets)

    def __eq__(self, other):
        return isinstance(other, KLLParameters) and self._key() == other._key()

    def __hash__(self):
        return hash(self._key())

    def __repr__(self):
        return "KLLParameters(%d,%r,%d)" % self._key()


class BucketValue:
    """M/metrics/KLLMetric.scala:24."""

    def __init__(self, lowValue, highValue, count):
        self.lowValue, self.highValue, self.count = float(lowValue), float(highValue), int(count)

    def __eq__(self, other):
        return isinstance(other, BucketValue) and (self.lowValue, self.highValue, self.count) == \
            (other.lowValue, other.highValue, other.count)

    def __repr__(self):
        return "BucketValue(%r,%r,%d)" % (self.lowValue, self.highValue, self.count)


class BucketDistribution:
    """M/metrics/KLLMetric.scala:26-96."""

    def __init__(self, buckets, parameters, data, _levels=None):
        self.buckets, self.parameters, self.data = list(buckets), [float(p) for p in parameters], \
            [list(d) for d in data]
        self._levels = _levels  # `data` as float64 arrays when the sketch had them

    def computePercentiles(self):
        # parameters = (shrinkingFactor, sketchSize) but are read back as (sketchSize, shrinkingFactor); the
        # quantiles depend only on `data`, so the swap (kept from the reference) is harmless.
        q = QuantileNonSample(int(self.parameters[0]), self.parameters[1])
        q.reconstruct(int(self.parameters[0]), self.parameters[1], self.data)
        if self._levels is not None and len(self._levels) == len(self.data):
            q._np_levels = self._levels
        return q.quantiles(100)

    def __getitem__(self, key):
        return self.buckets[key]

    def argmax(self):
        current, best = 0, 0
        for i, b in enumerate(self.buckets):
            if b.count > current:
                current, best = b.count, i
        return best

    def __eq__(self, other):
        if not isinstance(other, BucketDistribution):
            return False
        if self.buckets != other.buckets or self.parameters != other.parameters or \
                len(self.data) != len(other.data):
            return False
        return all(list(a) == list(b) for a, b in zip(self.data, other.data))

    def __repr__(self):
        return "BucketDistribution(%r,%r,%r)" % (self.buckets, self.parameters, self.data)


class KLLMetric:
    """M/metrics/KLLMetric.scala:98-126."""
    name = "KLL"

    def __init__(self, column, value):
        self.column, self.value = column, value
        self.entity = Entity.Column
        self.instance = column

    def flatten(self):
        if self.value.isFailure:
            return [DoubleMetric(self.entity, "%s.buckets" % self.name, self.instance, Failure(self.value.failed))]
        dist = self.value.get()
        out = [DoubleMetric(self.entity, "%s.buckets" % self.name, self.instance,
                            Success(float(len(dist.buckets))))]
        for b in dist.buckets:
            out.append(DoubleMetric(self.entity, "%s.low" % self.name, self.instance, Success(b.lowValue)))
            out.append(DoubleMetric(self.entity, "%s.high" % self.name, self.instance, Success(b.highValue)))
            out.append(DoubleMetric(self.entity, "%s.count" % self.name, self.instance, Success(float(b.count))))
        return out

    def __eq__(self, other):
        return isinstance(other, KLLMetric) and self.column == other.column and self.value == other.value

    def __hash__(self):
        return hash(("KLL", self.column))

    def __repr__(self):
        return "KLLMetric(%s,%r)" % (self.column, self.value)


def bucket_distribution(state, numberOfBuckets):
    """KLLSketch.computeMetricFrom's body (A/KLLSketch.scala:121-146)."""
    sk = state.qSketch
    start, end = state.globalMin, state.globalMax
    lows = [start + (end - start) * i / float(numberOfBuckets) for i in range(numberOfBuckets)]
    highs = [start + (end - start) * (i + 1) / float(numberOfBuckets) for i in range(numberOfBuckets)]
    index = sk._rank_index()
    ex_low = sk.getRanks(lows, exclusive=True, index=index) if numberOfBuckets else []
    ex_high = sk.getRanks(highs, exclusive=True, index=index) if numberOfBuckets else []
    buckets = []
    for i in range(numberOfBuckets):
        if i == numberOfBuckets - 1:
            cnt = int(sk.getRanks([highs[i]], exclusive=False, index=index)[0]) - int(ex_low[i])
        else:
            cnt = int(ex_high[i]) - int(ex_low[i])
        buckets.append(BucketValue(lows[i], highs[i], cnt))
    return BucketDistribution(buckets, [sk.shrinkingFactor, float(sk.sketchSize)], sk.getCompactorItems(),
                              _levels=list(sk._levels()))
