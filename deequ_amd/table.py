"""Columnar batches in the layout the C-ABI takes (Arrow-style buffers + the Spark physical type).

This stands where deequ takes a Spark DataFrame (`AnalysisRunner.onData(df)`,
R/AnalysisRunner.scala:51-53). A Table holds named columns; each column is a values buffer,
an LSB-first validity bitmap (None = no nulls) and, for strings, int32 offsets into UTF-8 data.
`Table.to_device()` moves the buffers into HBM (torch is used only as the device allocator) so
repeated runs read device-resident data, as the benchmark does.
"""
import csv
import math
import re
from collections import OrderedDict

import numpy as np

from . import native as N

SPARK_TYPE_NAMES = {
    N.TYPE_BOOLEAN: "BooleanType", N.TYPE_BYTE: "ByteType", N.TYPE_SHORT: "ShortType",
    N.TYPE_INT: "IntegerType", N.TYPE_LONG: "LongType", N.TYPE_FLOAT: "FloatType",
    N.TYPE_DOUBLE: "DoubleType", N.TYPE_STRING: "StringType", N.TYPE_DATE: "DateType",
    N.TYPE_TIMESTAMP: "TimestampType", N.TYPE_DECIMAL: "DecimalType",
}
_NAME_TO_TYPE = {v.lower().replace("type", ""): k for k, v in SPARK_TYPE_NAMES.items()}
_NAME_TO_TYPE.update({"int": N.TYPE_INT, "bigint": N.TYPE_LONG, "bool": N.TYPE_BOOLEAN, "str": N.TYPE_STRING,
                      "float64": N.TYPE_DOUBLE, "float32": N.TYPE_FLOAT, "int64": N.TYPE_LONG,
                      "int32": N.TYPE_INT, "int16": N.TYPE_SHORT, "int8": N.TYPE_BYTE})

NUMPY_OF = {N.TYPE_BOOLEAN: np.uint8, N.TYPE_BYTE: np.int8, N.TYPE_SHORT: np.int16, N.TYPE_INT: np.int32,
            N.TYPE_LONG: np.int64, N.TYPE_FLOAT: np.float32, N.TYPE_DOUBLE: np.float64, N.TYPE_DATE: np.int32,
            N.TYPE_TIMESTAMP: np.int64, N.TYPE_DECIMAL: np.int64}

NUMERIC_TYPES = (N.TYPE_BYTE, N.TYPE_SHORT, N.TYPE_INT, N.TYPE_LONG, N.TYPE_FLOAT, N.TYPE_DOUBLE, N.TYPE_DECIMAL)


def spark_type_of(name_or_code):
    if isinstance(name_or_code, int):
        return name_or_code
    key = str(name_or_code).lower().replace("type", "")
    key = re.sub(r"\(.*\)", "", key)
    if key not in _NAME_TO_TYPE:
        raise ValueError("unknown Spark type %r" % name_or_code)
    return _NAME_TO_TYPE[key]


def pack_validity(mask):
    """bool mask (True = non-null) -> Arrow LSB-first bitmap (uint8), padded to 8-byte multiples."""
    mask = np.asarray(mask, dtype=bool)
    bits = np.packbits(mask, bitorder="little")
    pad = (-len(bits)) % 8
    if pad:
        bits = np.concatenate([bits, np.zeros(pad, dtype=np.uint8)])
    return bits


def unpack_validity(bitmap, n):
    if bitmap is None:
        return np.ones(n, dtype=bool)
    return np.unpackbits(np.asarray(bitmap, dtype=np.uint8), bitorder="little", count=n).astype(bool)


class Column:
    """One column: Spark type, values, optional validity bitmap, optional string offsets."""

    def __init__(self, name, spark_type, values, validity=None, offsets=None, decimal_precision=0,
                 decimal_scale=0, length=None):
        self.name = name
        self.spark_type = spark_type_of(spark_type)
        self.values = values
        self.validity = validity
        self.offsets = offsets
        self.decimal_precision = decimal_precision
        self.decimal_scale = decimal_scale
        if length is None:
            length = len(offsets) - 1 if self.spark_type == N.TYPE_STRING else len(values)
        self.length = int(length)
        self.device = None  # dict of torch tensors once resident in HBM
        self.tz = None  # TIMESTAMP: the Arrow column's time zone (None = naive, read as the UTC session zone)

    @property
    def type_name(self):
        n = SPARK_TYPE_NAMES[self.spark_type]
        if self.spark_type == N.TYPE_DECIMAL:
            return "DecimalType(%d,%d)" % (self.decimal_precision, self.decimal_scale)
        return n

    def is_numeric(self):
        return self.spark_type in NUMERIC_TYPES

    def null_mask(self):
        return ~unpack_validity(self.validity, self.length)

    def to_pylist(self):
        """Python values with None for nulls (host-side formatting only, e.g. Histogram keys)."""
        valid = unpack_validity(self.validity, self.length)
        out = []
        for i in range(self.length):
            out.append(self.value_at(i) if valid[i] else None)
        return out

    def valid_at(self, i):
        """Row i is non-NULL (reads one validity byte from HBM for a device-only column)."""
        if self.validity is not None:
            return bool((self.validity[i >> 3] >> (i & 7)) & 1)
        if self.values is None and self.device is not None and self.device.get("validity") is not None:
            return bool((int(self.device["validity"][i >> 3].item()) >> (i & 7)) & 1)
        return True

    def value_at(self, i):
        if self.values is None and self.device is not None:
            return self._device_value_at(i)
        if self.spark_type == N.TYPE_STRING:
            o = self.offsets
            return bytes(self.values[o[i]:o[i + 1]]).decode("utf-8")
        return self._decode_cell(self.values[i])

    def _device_value_at(self, i):
        """One cell of a device-only column (top-N keys, representatives of a few groups: tiny copies)."""
        d = self.device
        if self.spark_type == N.TYPE_STRING:
            o = d["offsets"][i:i + 2].cpu().numpy()
            return bytes(d["values"][int(o[0]):int(o[1])].cpu().numpy()).decode("utf-8")
        t = d["values"]
        dt = np.dtype(NUMPY_OF[self.spark_type])
        if str(t.dtype) == "torch.uint8" and dt.itemsize > 1:
            v = t[i * dt.itemsize:(i + 1) * dt.itemsize].cpu().numpy().view(dt)[0]
        else:
            v = t[i:i + 1].cpu().numpy().astype(dt)[0]
        return self._decode_cell(v)

    def cells_at(self, rows):
        """The cells of `rows` (None for NULL) in one go: for a device-only column, one gather per buffer and one copy
        back each (the representatives of a table's groups), instead of a device round trip per row."""
        rows = np.asarray(rows, dtype=np.int64)
        if len(rows) == 0:
            return []
        if not (self.values is None and self.device is not None):
            return [self.value_at(int(r)) if self.valid_at(int(r)) else None for r in rows]
        import torch
        d = self.device
        dev = d["values"].device
        idx = torch.from_numpy(rows).to(dev)
        if d.get("validity") is not None:
            vb = d["validity"][idx >> 3].cpu().numpy()
            valid = ((vb >> (rows & 7).astype(np.uint8)) & 1).astype(bool)
        else:
            valid = np.ones(len(rows), dtype=bool)
        if self.spark_type == N.TYPE_STRING:
            off = d["offsets"]
            lo = off[idx].to(torch.int64)
            hi = off[idx + 1].to(torch.int64)
            lens = (hi - lo).cpu().numpy()
            total = int(lens.sum())
            if total:
                starts = np.repeat(lo.cpu().numpy() - np.concatenate([[0], np.cumsum(lens)[:-1]]), lens)
                pos = torch.from_numpy(starts + np.arange(total, dtype=np.int64)).to(dev)
                data = d["values"][pos].cpu().numpy().tobytes()
            else:
                data = b""
            out, at = [], 0
            for ok, n in zip(valid, lens):
                out.append(data[at:at + int(n)].decode("utf-8") if ok else None)
                at += int(n)
            return out
        t = d["values"]
        dt = np.dtype(NUMPY_OF[self.spark_type])
        if str(t.dtype) == "torch.uint8" and dt.itemsize > 1:
            pos = (idx[:, None] * dt.itemsize + torch.arange(dt.itemsize, device=dev)[None, :]).reshape(-1)
            vals = t[pos].cpu().numpy().view(dt)
        else:
            vals = t[idx].cpu().numpy().astype(dt)
        return [self._decode_cell(v) if ok else None for v, ok in zip(vals, valid)]

    def _decode_cell(self, v):
        if self.spark_type == N.TYPE_BOOLEAN:
            return bool(v)
        if self.spark_type in (N.TYPE_FLOAT, N.TYPE_DOUBLE):
            return float(v)
        if self.spark_type == N.TYPE_DECIMAL:
            return int(v) / (10 ** self.decimal_scale)
        return int(v)

    def native(self):
        """DqColumn for the C-ABI (device pointers when resident in HBM)."""
        c = N.DqColumn()
        c.spark_type = self.spark_type
        c.length = self.length
        c.decimal_precision = self.decimal_precision
        c.decimal_scale = self.decimal_scale
        if self.device is not None:
            c.flags = N.COL_DEVICE | (N.COL_OFFSETS64 if getattr(self, "offsets64", False) else 0)
            c.values = self.device["values"].data_ptr() if self.device.get("values") is not None else None
            c.validity = self.device["validity"].data_ptr() if self.device.get("validity") is not None else None
            c.offsets = self.device["offsets"].data_ptr() if self.device.get("offsets") is not None else None
        else:
            c.flags = N.COL_OFFSETS64 if getattr(self, "offsets64", False) else 0
            c.values = self.values.ctypes.data if self.values is not None and len(self.values) else None
            c.validity = self.validity.ctypes.data if self.validity is not None else None
            c.offsets = self.offsets.ctypes.data if self.offsets is not None else None
        return c

    def native_parts(self):
        """The column as consecutive row ranges for the ABIs that take parts (dq_quantile_summaries)."""
        return [self.native()]


class PartedColumn(Column):
    """A column of a ChunkedTable seen as its chunks' columns in row order, read where they lie (no concatenation):
    only the ABIs that take parts accept it (dq_quantile_summaries)."""

    def __init__(self, parts):
        first = parts[0]
        super().__init__(first.name, first.spark_type, None, None, decimal_precision=first.decimal_precision,
                         decimal_scale=first.decimal_scale, length=sum(p.length for p in parts))
        self.parts = list(parts)
        self.tz = first.tz

    def native(self):
        raise TypeError("column %s is held as %d chunks: only a per-part ABI reads it" % (self.name, len(self.parts)))

    def native_parts(self):
        return [p.native() for p in self.parts]

    def _locate(self, i):
        """(part, row inside it) of row i of the concatenation."""
        for p in self.parts:
            if i < p.length:
                return p, i
            i -= p.length
        raise IndexError(i)

    def valid_at(self, i):
        p, j = self._locate(int(i))
        return p.valid_at(j)

    def value_at(self, i):
        p, j = self._locate(int(i))
        return p.value_at(j)

    def cells_at(self, rows):
        """The cells of `rows` (indices into the concatenation): one batched gather per part."""
        rows = np.asarray(rows, dtype=np.int64)
        out = [None] * len(rows)
        base = 0
        for p in self.parts:
            sel = np.flatnonzero((rows >= base) & (rows < base + p.length))
            if len(sel):
                for k, v in zip(sel.tolist(), p.cells_at(rows[sel] - base)):
                    out[k] = v
            base += p.length
        return out


def _column_from_pylist(name, spark_type, items):
    t = spark_type_of(spark_type)
    n = len(items)
    mask = np.array([x is not None and not (isinstance(x, float) and math.isnan(x) and t == N.TYPE_STRING)
                     for x in items], dtype=bool)
    validity = None if mask.all() else pack_validity(mask)
    if t == N.TYPE_STRING:
        enc = [("" if x is None else str(x)).encode("utf-8") for x in items]
        offsets = np.zeros(n + 1, dtype=np.int32)
        if n:
            offsets[1:] = np.cumsum([len(b) for b in enc])
        data = np.frombuffer(b"".join(enc), dtype=np.uint8).copy() if n else np.zeros(0, dtype=np.uint8)
        return Column(name, t, data, validity, offsets, length=n)
    if t == N.TYPE_DECIMAL:
        from decimal import Decimal
        vals = [Decimal(str(x)) if x is not None else Decimal(0) for x in items]
        scale = max([max(0, -v.as_tuple().exponent) for v in vals] + [0])
        unscaled = np.array([int(v.scaleb(scale)) for v in vals], dtype=np.int64)
        prec = max([len(str(abs(int(u)))) for u in unscaled] + [1])
        return Column(name, t, unscaled, validity, decimal_precision=max(prec, scale + 1), decimal_scale=scale)
    dtype = NUMPY_OF[t]
    fill = 0
    vals = np.array([fill if x is None else x for x in items], dtype=dtype)
    return Column(name, t, vals, validity)


def _arrow_validity(arr, n):
    if arr.null_count == 0:
        return None
    bits = np.frombuffer(arr.buffers()[0], dtype=np.uint8)
    mask = np.unpackbits(bits, bitorder="little", count=arr.offset + n)[arr.offset:].astype(bool)
    return pack_validity(mask)


def _column_from_arrow(name, arr, pa):
    t, n = arr.type, len(arr)
    validity = _arrow_validity(arr, n)
    if pa.types.is_dictionary(t):
        return _column_from_arrow(name, arr.dictionary_decode(), pa)
    if pa.types.is_large_string(t):
        arr, t = arr.cast(pa.string()), pa.string()
    if pa.types.is_string(t):
        bufs = arr.buffers()
        offs = np.frombuffer(bufs[1], dtype=np.int32)[arr.offset:arr.offset + n + 1]
        data = np.frombuffer(bufs[2], dtype=np.uint8) if bufs[2] is not None else np.zeros(0, np.uint8)
        base = int(offs[0]) if n else 0
        end = int(offs[-1]) if n else 0
        return Column(name, N.TYPE_STRING, data[base:end], validity, (offs - base).astype(np.int32), length=n)
    if pa.types.is_boolean(t):
        bits = np.frombuffer(arr.buffers()[1], dtype=np.uint8)
        vals = np.unpackbits(bits, bitorder="little", count=arr.offset + n)[arr.offset:].astype(np.uint8)
        return Column(name, N.TYPE_BOOLEAN, vals, validity)
    if pa.types.is_decimal(t):
        if t.precision > 18:
            raise ValueError("column %s: DecimalType(%d,%d) exceeds the 64-bit unscaled range"
                             % (name, t.precision, t.scale))
        # decimal128 cells are 16-byte little-endian two's complement; precision <= 18 fits the low 8 bytes
        cells = np.frombuffer(arr.buffers()[1], dtype=np.int64)[2 * arr.offset:2 * (arr.offset + n)]
        unscaled = np.ascontiguousarray(cells[0::2])
        if validity is not None:
            unscaled = np.where(unpack_validity(validity, n), unscaled, 0)
        return Column(name, N.TYPE_DECIMAL, unscaled, validity, decimal_precision=t.precision,
                      decimal_scale=t.scale)
    if pa.types.is_timestamp(t):
        us = arr.cast(pa.timestamp("us", tz=t.tz), safe=False) if t.unit != "us" else arr
        vals = np.frombuffer(us.buffers()[1], dtype=np.int64)[us.offset:us.offset + n]
        col = Column(name, N.TYPE_TIMESTAMP, vals, validity)
        col.tz = t.tz
        return col
    spark = {pa.int8(): N.TYPE_BYTE, pa.int16(): N.TYPE_SHORT, pa.int32(): N.TYPE_INT, pa.int64(): N.TYPE_LONG,
             pa.float32(): N.TYPE_FLOAT, pa.float64(): N.TYPE_DOUBLE, pa.date32(): N.TYPE_DATE}.get(t)
    if spark is None:
        raise ValueError("column %s: Arrow type %s has no Spark counterpart here" % (name, t))
    vals = np.frombuffer(arr.buffers()[1], dtype=NUMPY_OF[spark])[arr.offset:arr.offset + n]
    return Column(name, spark, vals, validity)


def column_to_arrow(col, pa):
    """A host column -> pyarrow array of its Spark type (inverse of _column_from_arrow), from the buffers."""
    n = col.length
    valid = unpack_validity(col.validity, n)
    mask = None if valid.all() else ~valid
    vbuf = None if mask is None else pa.py_buffer(np.packbits(valid, bitorder="little").tobytes())
    t = col.spark_type
    if t == N.TYPE_STRING:
        off = np.ascontiguousarray(np.asarray(col.offsets, dtype=np.int32)[:n + 1])
        data = np.ascontiguousarray(np.asarray(col.values, dtype=np.uint8)[:int(off[-1]) if n else 0])
        return pa.Array.from_buffers(pa.string(), n, [vbuf, pa.py_buffer(off.tobytes()), pa.py_buffer(data.tobytes())],
                                     null_count=-1)
    if t == N.TYPE_BOOLEAN:
        return pa.array(np.asarray(col.values)[:n] != 0, mask=mask)
    if t == N.TYPE_DATE:
        return pa.array(np.asarray(col.values, dtype=np.int32)[:n], type=pa.int32(), mask=mask).cast(pa.date32())
    if t == N.TYPE_TIMESTAMP:
        return pa.array(np.asarray(col.values, dtype=np.int64)[:n], type=pa.int64(), mask=mask).cast(pa.timestamp("us"))
    if t == N.TYPE_DECIMAL:
        u = np.asarray(col.values, dtype=np.int64)[:n]
        cells = np.empty(2 * n, dtype=np.int64)
        cells[0::2] = u
        cells[1::2] = np.where(u < 0, -1, 0)
        return pa.Array.from_buffers(pa.decimal128(max(col.decimal_precision, 1), col.decimal_scale), n,
                                     [vbuf, pa.py_buffer(cells.tobytes())], null_count=-1)
    return pa.array(np.asarray(col.values, dtype=NUMPY_OF[t])[:n], mask=mask)


class Table:
    """Named columns of equal length (the DataFrame stand-in of the drop-in API)."""

    def __init__(self, columns):
        self.columns = OrderedDict()
        n = None
        for c in columns:
            if n is not None and c.length != n:
                raise ValueError("column %s has %d rows, expected %d" % (c.name, c.length, n))
            n = c.length
            self.columns[c.name] = c
        self.nrows = n or 0

    # ---- constructors ---------------------------------------------------------------------------
    @classmethod
    def from_rows(cls, rows, names, types=None):
        """Like Spark's `Seq((..),(..)).toDF(names...)`: None is null; types default from values."""
        cols = []
        for j, name in enumerate(names):
            items = [r[j] for r in rows]
            t = types[j] if types else _infer_py_type(items)
            cols.append(_column_from_pylist(name, t, items))
        return cls(cols)

    @classmethod
    def from_pydict(cls, data, types=None):
        cols = []
        for name, items in data.items():
            t = (types or {}).get(name) or _infer_py_type(list(items))
            cols.append(_column_from_pylist(name, t, list(items)))
        return cls(cols)

    @classmethod
    def from_arrays(cls, arrays, types=None, validity=None):
        """numpy arrays (fixed width) -> columns; `validity`: name -> bool mask."""
        cols = []
        for name, arr in arrays.items():
            arr = np.ascontiguousarray(arr)
            t = (types or {}).get(name)
            if t is None:
                t = {np.dtype(np.float64): N.TYPE_DOUBLE, np.dtype(np.float32): N.TYPE_FLOAT,
                     np.dtype(np.int64): N.TYPE_LONG, np.dtype(np.int32): N.TYPE_INT,
                     np.dtype(np.int16): N.TYPE_SHORT, np.dtype(np.int8): N.TYPE_BYTE,
                     np.dtype(np.bool_): N.TYPE_BOOLEAN}[arr.dtype]
            t = spark_type_of(t)
            vals = arr.astype(NUMPY_OF[t]) if t != N.TYPE_BOOLEAN else arr.astype(np.uint8)
            vm = (validity or {}).get(name)
            cols.append(Column(name, t, vals, pack_validity(vm) if vm is not None else None))
        return cls(cols)

    @classmethod
    def from_csv(cls, path, header=True, infer_schema=True):
        """CSV -> Table with Spark 2.2 CSV `inferSchema` typing (empty field = null)."""
        with open(path, newline="") as f:
            rows = list(csv.reader(f))
        names = rows[0] if header else ["_c%d" % i for i in range(len(rows[0]))]
        body = rows[1:] if header else rows
        cols = []
        for j, name in enumerate(names):
            raw = [(r[j] if j < len(r) else "") for r in body]
            items = [None if x == "" else x for x in raw]
            t = _csv_infer(items) if infer_schema else N.TYPE_STRING
            if t == N.TYPE_STRING:
                cols.append(_column_from_pylist(name, t, items))
            elif t == N.TYPE_DOUBLE:
                cols.append(_column_from_pylist(name, t, [None if x is None else float(x) for x in items]))
            elif t == N.TYPE_BOOLEAN:
                cols.append(_column_from_pylist(name, t, [None if x is None else x.lower() == "true" for x in items]))
            else:
                cols.append(_column_from_pylist(name, t, [None if x is None else int(x) for x in items]))
        return cls(cols)

    @classmethod
    def from_arrow(cls, table):
        """pyarrow.Table (a Spark DataFrame collected through Arrow, or a parquet read) -> Table.
        Fixed-width values and UTF-8 offsets/data are taken from the Arrow buffers without a
        per-row pass; validity bitmaps are realigned to bit 0 and padded; booleans are widened to one
        byte per row, timestamps normalised to Spark's microseconds, decimals (precision <= 18) to
        unscaled longs."""
        import pyarrow as pa
        cols = []
        for name, chunked in zip(table.column_names, table.columns):
            arr = chunked.combine_chunks() if chunked.num_chunks != 1 else chunked.chunk(0)
            cols.append(_column_from_arrow(name, arr, pa))
        return cls(cols)

    @classmethod
    def from_parquet(cls, path, columns=None):
        """Parquet file or directory -> Table (through pyarrow, then `from_arrow`)."""
        import pyarrow.parquet as pq
        return cls.from_arrow(pq.read_table(path, columns=columns))

    # ---- schema / access ------------------------------------------------------------------------
    @property
    def schema(self):
        return OrderedDict((n, c.type_name) for n, c in self.columns.items())

    @property
    def fieldNames(self):
        return list(self.columns)

    def __getitem__(self, name):
        return self.columns[name]

    def __contains__(self, name):
        return name in self.columns

    def count(self):
        return self.nrows

    def select_rows(self, mask):
        """Host-side row subset (test helper: builds partitions like parallelize(rows, numSlices))."""
        mask = np.asarray(mask, dtype=bool)
        out = []
        for c in self.columns.values():
            valid = unpack_validity(c.validity, c.length)[mask]
            if c.spark_type == N.TYPE_STRING:
                items = [c.value_at(i) for i in np.nonzero(mask)[0]]
                items = [x if v else None for x, v in zip(items, valid)]
                out.append(_column_from_pylist(c.name, c.spark_type, items))
            else:
                vals = c.values[mask]
                nc = Column(c.name, c.spark_type, np.ascontiguousarray(vals),
                            None if valid.all() else pack_validity(valid), decimal_precision=c.decimal_precision,
                            decimal_scale=c.decimal_scale)
                out.append(nc)
        return Table(out)

    def to_device(self, device=0):
        """Copy every buffer into HBM (torch tensors as the allocator); runs then read device memory."""
        import torch
        dev = torch.device("cuda", device)
        for c in self.columns.values():
            d = {}
            if c.spark_type == N.TYPE_STRING:
                d["values"] = torch.from_numpy(np.concatenate([c.values, np.zeros(16, np.uint8)])).to(dev)
                d["offsets"] = torch.from_numpy(c.offsets.astype(np.int32)).to(dev)
            else:
                d["values"] = torch.from_numpy(np.ascontiguousarray(c.values).view(np.uint8).copy()).to(dev)
            if c.validity is not None:
                d["validity"] = torch.from_numpy(pack_validity(unpack_validity(c.validity, c.length))).to(dev)
            c.device = d
        return self


class ChunkedTable:
    """A table held as consecutive row chunks (Arrow record batches) of one schema: the shape of a DataFrame's
    partitions, and how a shard whose string bytes exceed one column's int32 offsets (2^31 bytes) is held.
    AnalysisRunner runs every chunk and merges the chunk states with the reference's semigroup merges
    (runOnAggregatedStates, R/AnalysisRunner.scala:385-460) — the per-partition aggregation Spark performs inside
    one `agg`; ColumnProfiler runs its three passes the same way."""

    def __init__(self, chunks):
        chunks = list(chunks)
        if not chunks:
            raise ValueError("a ChunkedTable needs at least one chunk")
        schema = chunks[0].schema
        for t in chunks[1:]:
            if t.schema != schema:
                raise ValueError("chunks of a ChunkedTable must share one schema")
        self.chunks = chunks
        self.nrows = sum(t.nrows for t in chunks)

    @property
    def schema(self):
        return self.chunks[0].schema

    @property
    def fieldNames(self):
        return self.chunks[0].fieldNames

    def __getitem__(self, name):
        """The first chunk's column: type and metadata only (values live in every chunk)."""
        return self.chunks[0][name]

    def __contains__(self, name):
        return name in self.chunks[0]

    def count(self):
        return self.nrows

    def concat(self, names):
        """The named columns of every chunk as one Table, concatenated where the chunks live (HBM when every chunk is
        device-resident, else host memory): a string column's offsets become int64 (Arrow large_string,
        DQ_COL_OFFSETS64) so its bytes may pass 2^31. The grouping builds take it whole, so a grouping over the shard
        is one frequency table (not per-chunk tables merged through host memory)."""
        on_device = all(all(c[n].device is not None for n in names) for c in self.chunks)
        cols = [(_concat_device if on_device else _concat_host)([c[n] for c in self.chunks]) for n in names]
        if on_device and cols:
            import torch
            # the copies run on this thread's torch stream of the columns' device, the builds that read them on the
            # context's own stream
            torch.cuda.current_stream(cols[0].device["values"].device).synchronize()
        return Table(cols)

    def parted(self, names):
        """The named columns as PartedColumns over the chunks (no copy): the ApproxQuantile summaries of the shard
        read every chunk in one dq_quantile_summaries call."""
        return Table([PartedColumn([c[n] for c in self.chunks]) for n in names])

    def grouping_view(self, names):
        """The key columns of a grouping over the whole shard: read in place as two parts (dq_frequencies_parts) when
        the shard is two device chunks and a key is a string (the general build, no HBM concatenation and no host
        synchronisation), else concatenated (a fixed-width single key keeps the fast build over one column).
        DQ_GROUP_CONCAT=1 always concatenates."""
        import os
        cols = [self.chunks[0][n] for n in names]
        if len(self.chunks) == 2 and not os.environ.get("DQ_GROUP_CONCAT") and \
                any(c.spark_type == N.TYPE_STRING for c in cols) and \
                all(ch[n].device is not None and not getattr(ch[n], "offsets64", False)
                    for ch in self.chunks for n in names):
            return self.parted(names)
        return self.concat(names)


def _infer_py_type(items):
    nn = [x for x in items if x is not None]
    if not nn:
        return N.TYPE_STRING
    if all(isinstance(x, bool) for x in nn):
        return N.TYPE_BOOLEAN
    if all(isinstance(x, (int, np.integer)) and not isinstance(x, bool) for x in nn):
        return N.TYPE_INT if all(-2 ** 31 <= int(x) < 2 ** 31 for x in nn) else N.TYPE_LONG
    if all(isinstance(x, (int, float, np.integer, np.floating)) for x in nn):
        return N.TYPE_DOUBLE
    return N.TYPE_STRING


_INT_RE = re.compile(r"^[+-]?\d+$")


def _csv_infer(items):
    """Spark 2.2 CSVInferSchema per column: Integer -> Long -> Decimal(p,0) -> Double -> Boolean -> String."""
    rank = {None: 0, N.TYPE_INT: 1, N.TYPE_LONG: 2, N.TYPE_DOUBLE: 4, N.TYPE_BOOLEAN: 5, N.TYPE_STRING: 6}
    cur = None
    for x in items:
        if x is None:
            continue
        t = _csv_field_type(x)
        if cur is None:
            cur = t
        elif t != cur:
            if {t, cur} <= {N.TYPE_INT, N.TYPE_LONG, N.TYPE_DOUBLE}:
                cur = max(t, cur, key=lambda k: rank[k])
            else:
                cur = N.TYPE_STRING
        if cur == N.TYPE_STRING:
            break
    return cur if cur is not None else N.TYPE_STRING


def _csv_field_type(x):
    if _INT_RE.match(x):
        v = int(x)
        if -2 ** 31 <= v < 2 ** 31:
            return N.TYPE_INT
        if -2 ** 63 <= v < 2 ** 63:
            return N.TYPE_LONG
        return N.TYPE_DOUBLE
    try:
        float(x)
        if re.match(r"^[+-]?(\d+\.?\d*|\.\d+)([eE][+-]?\d+)?[dDfF]?$", x) or x in ("NaN", "Infinity", "-Infinity"):
            return N.TYPE_DOUBLE
    except ValueError:
        pass
    if x.lower() in ("true", "false"):
        return N.TYPE_BOOLEAN
    return N.TYPE_STRING


def _concat_host(parts):
    """Host columns of consecutive chunks as one column (int64 string offsets)."""
    first = parts[0]
    n = sum(p.length for p in parts)
    valid = np.concatenate([unpack_validity(p.validity, p.length) for p in parts]) if parts else np.zeros(0, bool)
    validity = None if valid.all() else pack_validity(valid)
    if first.spark_type == N.TYPE_STRING:
        offs, datas, base = [np.zeros(1, dtype=np.int64)], [], 0
        for p in parts:
            o = np.asarray(p.offsets, dtype=np.int64)[:p.length + 1]
            datas.append(np.asarray(p.values, dtype=np.uint8)[int(o[0]):int(o[-1])])
            offs.append(o[1:] - o[0] + base)
            base += int(o[-1] - o[0])
        col = Column(first.name, N.TYPE_STRING, np.concatenate(datas) if datas else np.zeros(0, np.uint8), validity,
                     np.concatenate(offs), length=n)
        col.offsets64 = True
        return col
    vals = np.concatenate([np.asarray(p.values)[:p.length] for p in parts])
    return Column(first.name, first.spark_type, vals, validity, decimal_precision=first.decimal_precision,
                  decimal_scale=first.decimal_scale, length=n)


def _device_valid_bits(col, torch):
    """One bool per row of a device column's validity (all True without a bitmap)."""
    d = col.device
    dev = d["values"].device
    if d.get("validity") is None:
        return torch.ones(col.length, dtype=torch.bool, device=dev)
    v = d["validity"][:(col.length + 7) // 8]
    bits = (v.unsqueeze(1) >> torch.arange(8, device=dev, dtype=torch.uint8)) & 1
    return bits.reshape(-1)[:col.length].bool()


def _concat_device(parts):
    """Device columns of consecutive chunks as one device column: values / UTF-8 bytes copied in HBM, validity bits
    re-packed at the chunk boundaries (byte-wise when every chunk but the last holds a multiple of 8 rows), string
    offsets rebased into int64 in place in the output."""
    import torch
    first = parts[0]
    dev = first.device["values"].device
    n = sum(p.length for p in parts)
    col = Column(first.name, first.spark_type, None, None, decimal_precision=first.decimal_precision,
                 decimal_scale=first.decimal_scale, length=n)
    d = {}
    if any(p.device.get("validity") is not None for p in parts):
        nwords = max((n + 63) // 64, 1)
        if all(p.length % 8 == 0 for p in parts[:-1]):
            out = torch.zeros(nwords * 8, dtype=torch.uint8, device=dev)
            at = 0
            for p in parts:
                nb = (p.length + 7) // 8
                v = p.device.get("validity")
                if v is None:
                    out[at:at + nb] = 0xFF
                    if p.length % 8:
                        out[at + nb - 1] = (1 << (p.length % 8)) - 1
                else:
                    out[at:at + nb].copy_(v[:nb])
                    if p.length % 8:  # bits past the chunk's last row read as NULL
                        out[at + nb - 1] &= (1 << (p.length % 8)) - 1
                at += nb
            d["validity"] = out
        else:
            bits = torch.cat([_device_valid_bits(p, torch) for p in parts])
            padded = torch.zeros(nwords * 64, dtype=torch.uint8, device=dev)
            padded[:n] = bits.to(torch.uint8)
            w = (1 << torch.arange(8, device=dev, dtype=torch.int32))
            d["validity"] = (padded.reshape(-1, 8).to(torch.int32) * w).sum(dim=1).to(torch.uint8)
    if first.spark_type == N.TYPE_STRING:
        spans = []
        for p in parts:
            o = p.device["offsets"]
            spans.append((int(o[0].item()), int(o[p.length].item())))
        total = sum(b - a for a, b in spans)
        data = torch.empty(total + 16, dtype=torch.uint8, device=dev)  # + read-past padding of the dword loads
        data[total:] = 0
        offs = torch.empty(n + 1, dtype=torch.int64, device=dev)
        offs[0] = 0
        at, base = 0, 0
        for p, (o0, o1) in zip(parts, spans):
            data[base:base + o1 - o0].copy_(p.device["values"][o0:o1])
            seg = offs[at + 1:at + 1 + p.length]
            seg.copy_(p.device["offsets"][1:p.length + 1])
            seg.add_(base - o0)
            at += p.length
            base += o1 - o0
        d["values"], d["offsets"] = data, offs
        col.offsets64 = True
    else:
        width = np.dtype(NUMPY_OF[first.spark_type]).itemsize
        d["values"] = torch.cat([p.device["values"].reshape(-1).view(torch.uint8)[:p.length * width] for p in parts])
    col.device = d
    return col
