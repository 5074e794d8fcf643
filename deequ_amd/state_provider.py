"""File-system state persistence: HdfsStateProvider (A/StateProvider.scala:72-312).

States leave the engine as the reference's host State objects, so a state written here can be read
back by any run (GPU or restated) and merged with `aggregateWith` / `runOnAggregatedStates`
(R/AnalysisRunner.scala:385-460). File layouts follow the reference byte for byte:

- one `<prefix>-<id>.bin` file per analyzer, written as java.io.DataOutputStream does
  (big-endian longs/doubles, `writeInt(len)` + raw bytes for byte-array states);
- frequency states as a parquet directory `<prefix>-<id>-frequencies.pqt` (grouping columns +
  `com_amazon_deequ_dq_metrics_count` long, up to `numPartitionsForHistogram` part files) plus `<prefix>-<id>-num_rows.bin`;
- `<id>` = `MurmurHash3.stringHash(analyzer.toString, 42)` (scala.util.hashing, Scala 2.11/2.12),
  printed as a signed decimal Int.

Only local paths are supported (no Hadoop client in this build); `session` is accepted and ignored
so call sites read like the reference's `HdfsStateProvider(session, locationPrefix, ...)`.
"""
import os
import struct

from . import analyzers as A
from . import engine
from . import native as N
from .states import (NumMatches, NumMatchesAndCount, SumState, MeanState, MinState, MaxState,
                     StandardDeviationState, CorrelationState, ApproxCountDistinctState, DataTypeHistogram,
                     ApproxQuantileState)

_M32 = 0xFFFFFFFF
# Analyzers.COUNT_COL (A/Analyzer.scala:363-364): the count column of a frequency table
COUNT_COL = "com_amazon_deequ_dq_metrics_count"


def _rotl32(x, r):
    return ((x << r) | (x >> (32 - r))) & _M32


def _mix_last(h, k):
    k = (k * 0xCC9E2D51) & _M32
    k = _rotl32(k, 15)
    k = (k * 0x1B873593) & _M32
    return h ^ k


def _mix(h, k):
    h = _rotl32(_mix_last(h, k), 13)
    return (h * 5 + 0xE6546B64) & _M32


def _avalanche(h):
    h ^= h >> 16
    h = (h * 0x85EBCA6B) & _M32
    h ^= h >> 13
    h = (h * 0xC2B2AE35) & _M32
    h ^= h >> 16
    return h


def murmur3_string_hash(s, seed=42):
    """scala.util.hashing.MurmurHash3.stringHash: UTF-16 code units taken in pairs
    (`(c(i) << 16) + c(i+1)`), a trailing odd unit through mixLast, finalised with the unit count.
    Returns the signed 32-bit result (A/StateProvider.scala:82-84)."""
    units = struct.unpack(">%dH" % (len(s.encode("utf-16-be")) // 2), s.encode("utf-16-be"))
    h = seed & _M32
    i = 0
    n = len(units)
    while i + 1 < n:
        h = _mix(h, ((units[i] << 16) + units[i + 1]) & _M32)
        i += 2
    if i < n:
        h = _mix_last(h, units[i])
    h = _avalanche(h ^ n)
    return h - (1 << 32) if h & 0x80000000 else h


class StateAlreadyExistsError(FileExistsError):
    """Hadoop FileAlreadyExistsException / Spark AnalysisException("path ... already exists.")."""


class HdfsStateProvider:
    """A/StateProvider.scala:73-312 on a local file system."""

    def __init__(self, session=None, locationPrefix=None, numPartitionsForHistogram=10, allowOverwrite=False):
        if locationPrefix is None and isinstance(session, (str, os.PathLike)):
            session, locationPrefix = None, session
        if locationPrefix is None:
            raise ValueError("locationPrefix is required")
        self.locationPrefix = os.fspath(locationPrefix)
        self.numPartitionsForHistogram = int(numPartitionsForHistogram)
        self.allowOverwrite = bool(allowOverwrite)

    # ---- identifiers and raw files -------------------------------------------------------------
    @staticmethod
    def toIdentifier(analyzer):
        return str(murmur3_string_hash(str(analyzer), 42))

    def _bin(self, ident, suffix=""):
        return "%s-%s%s.bin" % (self.locationPrefix, ident, suffix)

    def _write(self, path, payload):
        """io/DfsUtils.scala:43-56: fs.create(path, overwrite) then the DataOutputStream writes."""
        if os.path.exists(path) and not self.allowOverwrite:
            raise StateAlreadyExistsError("%s already exists" % path)
        d = os.path.dirname(path)
        if d:
            os.makedirs(d, exist_ok=True)
        with open(path, "wb") as f:
            f.write(payload)

    @staticmethod
    def _read(path):
        with open(path, "rb") as f:
            return f.read()

    def _persist_bytes(self, data, ident):
        self._write(self._bin(ident), struct.pack(">i", len(data)) + bytes(data))

    def _load_bytes(self, ident):
        raw = self._read(self._bin(ident))
        (n,) = struct.unpack_from(">i", raw, 0)
        if len(raw) < 4 + n:
            raise EOFError("truncated state file %s" % self._bin(ident))
        return raw[4:4 + n]

    # ---- StatePersister ------------------------------------------------------------------------
    def persist(self, analyzer, state):
        ident = self.toIdentifier(analyzer)
        if isinstance(analyzer, A.Size):
            self._write(self._bin(ident), struct.pack(">q", state.numMatches))
        elif isinstance(analyzer, (A.Completeness, A.Compliance, A.PatternMatch)):
            self._write(self._bin(ident), struct.pack(">qq", state.numMatches, state.count))
        elif isinstance(analyzer, A.Sum):
            self._write(self._bin(ident), struct.pack(">d", state.sum_))
        elif isinstance(analyzer, A.Mean):
            self._write(self._bin(ident), struct.pack(">dq", state.sum_, state.count))
        elif isinstance(analyzer, (A.Minimum, A.MinLength)):
            self._write(self._bin(ident), struct.pack(">d", state.minValue))
        elif isinstance(analyzer, (A.Maximum, A.MaxLength)):
            self._write(self._bin(ident), struct.pack(">d", state.maxValue))
        elif isinstance(analyzer, (A.FrequencyBasedAnalyzer, A.Histogram)):
            self._persist_frequencies(state, ident)
        elif isinstance(analyzer, A.DataType):
            self._persist_bytes(state.toBytes(), ident)
        elif isinstance(analyzer, A.ApproxCountDistinct):
            self._persist_bytes(struct.pack(">%dq" % len(state.words),
                                            *[w - (1 << 64) if w >> 63 else w for w in state.words]), ident)
        elif isinstance(analyzer, A.Correlation):
            self._write(self._bin(ident), struct.pack(">6d", state.n, state.xAvg, state.yAvg, state.ck,
                                                      state.xMk, state.yMk))
        elif isinstance(analyzer, A.StandardDeviation):
            self._write(self._bin(ident), struct.pack(">3d", state.n, state.avg, state.m2))
        elif isinstance(analyzer, A.ApproxQuantile):
            self._persist_bytes(state.percentileDigest.serialize(), ident)
        else:
            raise ValueError("Unable to persist state for analyzer %s." % analyzer)

    # ---- StateLoader ---------------------------------------------------------------------------
    def load(self, analyzer):
        ident = self.toIdentifier(analyzer)
        if isinstance(analyzer, A.Size):
            return NumMatches(*struct.unpack(">q", self._read(self._bin(ident))[:8]))
        if isinstance(analyzer, (A.Completeness, A.Compliance, A.PatternMatch)):
            return NumMatchesAndCount(*struct.unpack(">qq", self._read(self._bin(ident))[:16]))
        if isinstance(analyzer, A.Sum):
            return SumState(*struct.unpack(">d", self._read(self._bin(ident))[:8]))
        if isinstance(analyzer, A.Mean):
            return MeanState(*struct.unpack(">dq", self._read(self._bin(ident))[:16]))
        if isinstance(analyzer, (A.Minimum, A.MinLength)):
            return MinState(*struct.unpack(">d", self._read(self._bin(ident))[:8]))
        if isinstance(analyzer, (A.Maximum, A.MaxLength)):
            return MaxState(*struct.unpack(">d", self._read(self._bin(ident))[:8]))
        if isinstance(analyzer, (A.FrequencyBasedAnalyzer, A.Histogram)):
            return self._load_frequencies(ident)
        if isinstance(analyzer, A.DataType):
            return DataTypeHistogram.fromBytes(self._load_bytes(ident))
        if isinstance(analyzer, A.ApproxCountDistinct):
            data = self._load_bytes(ident)
            if len(data) != 52 * 8:
                raise ValueError("requirement failed")
            return ApproxCountDistinctState(list(struct.unpack(">52q", data)))
        if isinstance(analyzer, A.Correlation):
            return CorrelationState(*struct.unpack(">6d", self._read(self._bin(ident))[:48]))
        if isinstance(analyzer, A.StandardDeviation):
            return StandardDeviationState(*struct.unpack(">3d", self._read(self._bin(ident))[:24]))
        if isinstance(analyzer, A.ApproxQuantile):
            from .quantiles import PercentileDigest
            return ApproxQuantileState(PercentileDigest.deserialize(self._load_bytes(ident)))
        raise ValueError("Unable to load state for analyzer %s." % analyzer)

    # ---- frequency tables (A/StateProvider.scala:222-240, 291-298) ----------------------------
    def _freq_dir(self, ident):
        return "%s-%s-frequencies.pqt" % (self.locationPrefix, ident)

    def _persist_frequencies(self, state, ident):
        import shutil
        import pyarrow as pa
        import pyarrow.parquet as pq
        path = self._freq_dir(ident)
        if os.path.exists(path):
            if not self.allowOverwrite:
                raise StateAlreadyExistsError("path %s already exists." % path)
            shutil.rmtree(path) if os.path.isdir(path) else os.remove(path)
        tbl = _pairs_table(state)
        if tbl is None:
            tbl = _block_table(state)
        if tbl is None:
            freq = state.as_dict()
            columns = list(state.columns) if state.columns else \
                ["c%d" % i for i in range(len(next(iter(freq))) if freq else 1)]
            keys = list(freq.keys())
            counts = [freq[k] for k in keys]
            arrays = [pa.array([k[i] for k in keys]) for i in range(len(columns))]
            tbl = pa.Table.from_arrays(arrays + [pa.array(counts, type=pa.int64())], names=columns + [COUNT_COL])
        keys = range(tbl.num_rows)
        os.makedirs(path)
        parts = max(1, min(self.numPartitionsForHistogram, len(keys)))
        step = -(-len(keys) // parts) if keys else 0
        for p in range(parts):
            pq.write_table(tbl.slice(p * step, step) if keys else tbl,
                           os.path.join(path, "part-%05d.snappy.parquet" % p), compression="snappy")
        open(os.path.join(path, "_SUCCESS"), "wb").close()
        self._write(self._bin(ident, "-num_rows"), struct.pack(">q", state.numRows))

    def _load_frequencies(self, ident):
        import pyarrow.parquet as pq
        path = self._freq_dir(ident)
        files = sorted(f for f in os.listdir(path) if f.endswith(".parquet"))
        (num_rows,) = struct.unpack(">q", self._read(self._bin(ident, "-num_rows"))[:8])
        table = _read_parts(path, files)
        pairs = _load_pairs(table, num_rows)
        if pairs is not None:
            return pairs
        block = _load_block(table, num_rows)
        if block is not None:
            return block
        freq = {}
        columns = None
        for f in files:
            t = pq.read_table(os.path.join(path, f))
            names = t.column_names
            columns = [n for n in names if n != COUNT_COL]
            cols = [t.column(n).to_pylist() for n in columns]
            for key, c in zip(zip(*cols), t.column(COUNT_COL).to_pylist()):
                key = A._canonical_group_key(key)  # floating keys join bitwise (GroupFloat), as in device tables
                freq[key] = freq.get(key, 0) + int(c)
        return A.FrequenciesAndNumRows(freq, num_rows, columns)


FileSystemStateProvider = HdfsStateProvider


# ---- columnar (key, count) persistence of single fixed-width-key frequency states --------------------
def _arrow_of(spark_type):
    import pyarrow as pa
    return {N.TYPE_BYTE: pa.int8(), N.TYPE_SHORT: pa.int16(), N.TYPE_INT: pa.int32(), N.TYPE_LONG: pa.int64(),
            N.TYPE_FLOAT: pa.float32(), N.TYPE_DOUBLE: pa.float64(), N.TYPE_BOOLEAN: pa.bool_(),
            N.TYPE_DATE: pa.date32()}.get(spark_type)


def _pairs_table(state):
    """The parquet table of a single fixed-width-key state straight from its canonical (key, count) arrays
    (no per-group Python objects), or None for other key shapes."""
    import numpy as np
    import pyarrow as pa
    side = state._values_side()
    if side is None or _arrow_of(side.key_type) is None:
        return None
    if isinstance(side, engine.PairFrequencies):
        keys, counts, nulls = side.keys, side.counts, side.null_count
    else:
        keys, counts = side.export_pairs()
        nulls = side.summary(None)["null_count"]
    t = side.key_type
    if t == N.TYPE_DOUBLE:
        vals = pa.array(keys.view(np.float64))
    elif t == N.TYPE_FLOAT:
        vals = pa.array((keys.view(np.uint64) & np.uint64(0xFFFFFFFF)).astype(np.uint32).view(np.float32))
    elif t == N.TYPE_BOOLEAN:
        vals = pa.array(keys != 0)
    elif t == N.TYPE_DATE:
        # Arrow casts int32 -> date32, not int64 -> date32 (canonical keys are sign-extended int32 days)
        vals = pa.array(keys.astype(np.int32), type=pa.int32()).cast(pa.date32())
    else:
        vals = pa.array(keys).cast(_arrow_of(t))
    counts = np.asarray(counts, dtype=np.int64)
    if nulls:
        vals = pa.concat_arrays([vals, pa.nulls(1, type=vals.type)])
        counts = np.append(counts, np.int64(nulls))
    name = (list(state.columns) or ["c0"])[0]
    return pa.Table.from_arrays([vals, pa.array(counts, type=pa.int64())], names=[name, COUNT_COL])


def _block_table(state):
    """The parquet table of a state whose groups are a GroupBlock (string / multi-column keys: key columns + the
    count column, built from the column buffers, no per-group Python); a merged block (keys may repeat) is first
    aggregated by its weighted GPU build. None for other states."""
    import pyarrow as pa
    from . import groups as G
    from .table import column_to_arrow
    f = state.frequencies
    if isinstance(f, G.GroupBlock) and not getattr(f, "distinct", False):
        ft = state.device_table()
        if hasattr(ft, "distinct_block"):  # a merged state past the int32 offsets: key-disjoint split builds
            f = ft.distinct_block()
        else:
            keys, counts = ft.export_raw()
            f = G.GroupBlock([G.take(c, keys) for c in f.columns], counts)
    elif not isinstance(f, G.GroupBlock):
        if not isinstance(f, engine.FrequencyTable) or f.key_kind() == N.FREQ_KEYS_VALUES:
            return None
        f = state.group_block()
        if f is None:
            return None
    arrays = [column_to_arrow(c, pa) for c in f.columns]
    return pa.Table.from_arrays(arrays + [pa.array(f.counts, type=pa.int64())], names=f.names + [COUNT_COL])


def _read_parts(path, files):
    """The part files of a frequency state as one Arrow table (read once, Arrow's own threads), or None."""
    import pyarrow as pa
    import pyarrow.parquet as pq
    if not files:
        return None
    return pa.concat_tables([pq.read_table(os.path.join(path, f)) for f in files]) if len(files) == 1 else \
        pq.ParquetDataset([os.path.join(path, f) for f in files]).read(use_threads=True)


def _load_block(t, num_rows):
    """A persisted state of any key shape as a GroupBlock (Arrow buffers -> columns, vectorised); its groups are
    distinct, and the weighted GPU build behind its metrics reads them with their counts."""
    import numpy as np
    from . import groups as G
    from .table import Table
    if t is None:
        return None
    keys = [n for n in t.column_names if n != COUNT_COL]
    if COUNT_COL not in t.column_names or not keys:
        return None
    try:
        kt = Table.from_arrow(t.select(keys))
    except ValueError:
        return None
    counts = np.asarray(t.column(COUNT_COL).combine_chunks().to_numpy(zero_copy_only=False), dtype=np.int64)
    block = G.GroupBlock([kt[k] for k in keys], counts, int(counts.sum()), 0)
    block.distinct = True
    return A.FrequenciesAndNumRows(block, num_rows, keys)


def _load_pairs(t, num_rows):
    """A persisted single fixed-width-key frequency state as canonical (key, count) arrays
    (engine.PairFrequencies), or None when the key columns are of another shape."""
    import numpy as np
    import pyarrow as pa
    if t is None:
        return None
    keys = [n for n in t.column_names if n != COUNT_COL]
    if len(keys) != 1:
        return None
    arr = t.column(keys[0]).combine_chunks()
    spark = {pa.int8(): N.TYPE_BYTE, pa.int16(): N.TYPE_SHORT, pa.int32(): N.TYPE_INT, pa.int64(): N.TYPE_LONG,
             pa.float32(): N.TYPE_FLOAT, pa.float64(): N.TYPE_DOUBLE, pa.bool_(): N.TYPE_BOOLEAN,
             pa.date32(): N.TYPE_DATE}.get(arr.type)
    if spark is None:
        return None
    counts = np.asarray(t.column(COUNT_COL).combine_chunks().to_numpy(zero_copy_only=False), dtype=np.int64)
    valid = ~np.asarray(arr.is_null().to_numpy(zero_copy_only=False), dtype=bool)
    if spark == N.TYPE_BOOLEAN:
        vals = np.asarray(arr.fill_null(False).to_numpy(zero_copy_only=False), dtype=np.int64)
    elif spark == N.TYPE_DATE:
        vals = np.asarray(arr.cast(pa.int32()).fill_null(0).to_numpy(zero_copy_only=False), dtype=np.int64)
    else:
        vals = np.asarray(arr.fill_null(0).to_numpy(zero_copy_only=False))
    canon = engine.canonical_keys(spark, vals)[valid]
    nulls = int(counts[~valid].sum())
    return A.FrequenciesAndNumRows(engine.PairFrequencies(spark, canon, counts[valid], num_rows, nulls, 0, keys),
                                   num_rows, keys)
