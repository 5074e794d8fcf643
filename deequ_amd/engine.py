"""Device selection and the frequency-table handle (the GPU side of computeFrequencies)."""
import contextlib
import ctypes
import os
import threading

import numpy as np

from . import native as N
from .table import PartedColumn

_device = None


def set_device(device):
    global _device
    _device = int(device)


def device():
    if _device is not None:
        return _device
    return int(os.environ.get("LOCAL_RANK", "0"))


_local = threading.local()


def ctx():
    """This thread's context: the process-wide one of the device, unless `using_context` set another."""
    c = getattr(_local, "ctx", None)
    return c if c is not None else N.context(device())


@contextlib.contextmanager
def using_context(context):
    """Run this thread's engine calls on `context` (a second context of the device has its own stream and scratch,
    so work on it may proceed while another thread drives the first)."""
    prev = getattr(_local, "ctx", None)
    _local.ctx = context
    try:
        yield context
    finally:
        _local.ctx = prev


class GroupFloat(float):
    """A float group key with Spark's grouping equality: bitwise, NaN canonical (so NaN == NaN and
    -0.0 != 0.0, unlike Python floats). Formats like a float."""

    def _bits(self):
        v = float(self)
        if v != v:
            return 0x7FF8000000000000
        return int(np.array([v], dtype=np.float64).view(np.uint64)[0])

    def __eq__(self, other):
        if isinstance(other, float):
            return self._bits() == GroupFloat(other)._bits()
        return NotImplemented

    def __ne__(self, other):
        r = self.__eq__(other)
        return r if r is NotImplemented else not r

    def __hash__(self):
        return hash(("GroupFloat", self._bits()))


def decode_canonical(spark_type, decimal_scale, k):
    """Canonical 64-bit key (DQ_FREQ_KEYS_VALUES) of a fixed-width column -> its Python group value."""
    u = np.uint64(int(k) & 0xFFFFFFFFFFFFFFFF)
    if spark_type == N.TYPE_DOUBLE:
        return GroupFloat(u.view(np.float64))
    if spark_type == N.TYPE_FLOAT:
        return GroupFloat(np.uint32(int(u) & 0xFFFFFFFF).view(np.float32))
    i = int(u.view(np.int64))
    if spark_type == N.TYPE_BOOLEAN:
        return bool(i)
    if spark_type == N.TYPE_DECIMAL:
        from decimal import Decimal
        return Decimal(i).scaleb(-decimal_scale)
    return i


def canonical_keys(spark_type, values):
    """numpy values of a fixed-width key column -> canonical 64-bit keys (int64 view): integers sign-extended,
    FLOAT / DOUBLE bit patterns with NaN canonical (Spark's binary grouping equality)."""
    v = np.asarray(values)
    if spark_type == N.TYPE_DOUBLE:
        b = v.astype(np.float64).view(np.uint64).copy()
        b[np.isnan(v)] = np.uint64(0x7FF8000000000000)
        return b.view(np.int64)
    if spark_type == N.TYPE_FLOAT:
        f = v.astype(np.float32)
        b = f.view(np.uint32).astype(np.uint64)
        b[np.isnan(f)] = np.uint64(0x7FC00000)
        return b.view(np.int64)
    return v.astype(np.int64)


class PairFrequencies:
    """A frequency state held as (canonical key, count) arrays on the host — a persisted state read back by
    HdfsStateProvider — for one fixed-width key column. Merges with a device table on the GPU
    (dq_freq_from_pairs + dq_freq_merge); as_dict() decodes it for host-side consumers."""

    def __init__(self, key_type, keys, counts, num_rows, null_count=0, decimal_scale=0, names=None):
        self.key_type, self.decimal_scale = key_type, decimal_scale
        self.keys = np.ascontiguousarray(keys, dtype=np.int64)
        self.counts = np.ascontiguousarray(counts, dtype=np.int64)
        self.num_rows, self.null_count = int(num_rows), int(null_count)
        self.names = names

    def to_dict(self):
        out = {}
        for k, c in zip(self.keys.tolist(), self.counts.tolist()):
            key = (decode_canonical(self.key_type, self.decimal_scale, k),)
            out[key] = out.get(key, 0) + int(c)
        if self.null_count:
            out[(None,)] = self.null_count
        return out

    def to_device(self):
        return FrequencyTable.from_pairs(self.key_type, self.keys, self.counts, self.num_rows, self.null_count,
                                         self.decimal_scale, self.names)


class FrequencyTable:
    """Device-resident (key -> count) table built by dq_frequencies over `key_columns` of `source` (or from
    (key, count) pairs: source None, `key_type` the canonical keys' Spark type)."""

    def __init__(self, context, handle, source, key_columns, include_nulls, key_type=None, decimal_scale=0):
        self.ctx = context
        self.handle = handle
        self.source = source
        self.key_columns = [source[c] for c in key_columns] if source is not None else []
        self.names = list(key_columns)
        self.include_nulls = include_nulls
        if key_type is None and self.key_columns:
            key_type, decimal_scale = self.key_columns[0].spark_type, self.key_columns[0].decimal_scale
        self.key_type, self.decimal_scale = key_type, decimal_scale
        self.weights = None  # per source row counts of a weighted build (dq_frequencies_ex)
        s = self.summary(None)
        self.num_rows = s["num_rows"]
        self.num_groups = s["num_groups"]

    @classmethod
    def from_pairs(cls, key_type, keys, counts, num_rows, null_count=0, decimal_scale=0, names=None,
                   device_ptrs=False):
        """dq_freq_from_pairs: the table of (canonical key, count) pairs (numpy arrays, or device pointers)."""
        context = ctx()
        handle = ctypes.c_void_p()
        if device_ptrs:
            kp, cp, n = keys[0], counts[0], keys[1]
        else:
            keys = np.ascontiguousarray(keys, dtype=np.int64)
            counts = np.ascontiguousarray(counts, dtype=np.int64)
            kp, cp, n = keys.ctypes.data, counts.ctypes.data, len(keys)
        rc = context.lib.dq_freq_from_pairs(context.handle, int(key_type), ctypes.c_void_p(kp), ctypes.c_void_p(cp),
                                            int(n), N.FREQ_PAIRS_DEVICE if device_ptrs else 0, int(num_rows),
                                            int(null_count), ctypes.byref(handle))
        context.check(rc, "dq_freq_from_pairs")
        return cls(context, handle, None, list(names or ["k"]), bool(null_count), key_type, decimal_scale)

    def merge(self, other):
        """FrequenciesAndNumRows.sum on the GPU (dq_freq_merge)."""
        handle = ctypes.c_void_p()
        rc = self.ctx.lib.dq_freq_merge(self.ctx.handle, self.handle, other.handle, ctypes.byref(handle))
        self.ctx.check(rc, "dq_freq_merge")
        return FrequencyTable(self.ctx, handle, None, self.names, self.include_nulls or other.include_nulls,
                              self.key_type, self.decimal_scale)

    def export_pairs(self):
        """(canonical keys, counts) numpy arrays of a DQ_FREQ_KEYS_VALUES table (NULL group excluded)."""
        n = self.num_groups
        keys = np.zeros(max(n, 1), dtype=np.int64)
        counts = np.zeros(max(n, 1), dtype=np.int64)
        got = self.ctx.lib.dq_freq_export(self.ctx.handle, self.handle, n, keys.ctypes.data, counts.ctypes.data)
        if got < 0:
            raise N.NativeError(int(got), "dq_freq_export: %s" % self.ctx.last_error())
        return keys[:got], counts[:got]

    def mutual_information(self, x_table, y_table):
        """dq_freq_mutual_information over this (x, y) table and the x / y tables: (value, present)."""
        mi = ctypes.c_double(0.0)
        present = ctypes.c_int32(0)
        rc = self.ctx.lib.dq_freq_mutual_information(self.ctx.handle, self.handle, x_table.handle, y_table.handle,
                                                     ctypes.byref(mi), ctypes.byref(present))
        self.ctx.check(rc, "dq_freq_mutual_information")
        return mi.value, bool(present.value)

    def export_raw(self):
        """Every group as (key, count) int64 arrays: the canonical value (DQ_FREQ_KEYS_VALUES) or the smallest row
        index of the group in the source (DQ_FREQ_KEYS_ROWS); the NULL group of an include_nulls table excluded."""
        n = self.num_groups
        keys = np.zeros(max(n, 1), dtype=np.int64)
        counts = np.zeros(max(n, 1), dtype=np.int64)
        got = self.ctx.lib.dq_freq_export(self.ctx.handle, self.handle, n, keys.ctypes.data, counts.ctypes.data)
        if got < 0:
            raise N.NativeError(int(got), "dq_freq_export: %s" % self.ctx.last_error())
        return keys[:got], counts[:got]

    def top_raw(self, k):
        """The k largest groups as (key, count) int64 arrays (keys as in export_raw)."""
        k = int(min(k, self.num_groups))
        keys = np.zeros(max(k, 1), dtype=np.int64)
        counts = np.zeros(max(k, 1), dtype=np.int64)
        n = self.ctx.lib.dq_freq_top(self.ctx.handle, self.handle, k, keys.ctypes.data, counts.ctypes.data)
        if n < 0:
            raise N.NativeError(int(n), "dq_freq_top: %s" % self.ctx.last_error())
        return keys[:n], counts[:n]

    def row_counts(self):
        """dq_freq_row_counts: per source row, the count of its group (0 for rows taking no part)."""
        n = self.source.nrows
        out = np.zeros(max(n, 1), dtype=np.int64)
        rc = self.ctx.lib.dq_freq_row_counts(self.ctx.handle, self.handle, out.ctypes.data, n, 0)
        self.ctx.check(rc, "dq_freq_row_counts")
        return out[:n]

    def __del__(self):
        try:
            if self.handle:
                self.ctx.lib.dq_freq_free(self.ctx.handle, self.handle)
                self.handle = None
        except Exception:
            pass

    def summary(self, entropy_rows=None):
        out = N.DqFreqSummary()
        rc = self.ctx.lib.dq_freq_summarize(self.ctx.handle, self.handle, int(entropy_rows or 0), ctypes.byref(out))
        self.ctx.check(rc, "dq_freq_summarize")
        return {"num_rows": out.num_rows, "num_groups": out.num_groups, "num_unique": out.num_unique,
                "entropy": out.entropy, "entropy_rows": out.entropy_rows, "max_count": out.max_count,
                "null_count": out.null_count, "entropy_fx": N.fx_value(out.entropy_fx_lo, out.entropy_fx_hi)}

    def key_kind(self):
        return self.ctx.lib.dq_freq_key_kind(self.handle)

    def _key_of_row(self, r):
        key = []
        for c in self.key_columns:
            v = c.value_at(int(r)) if c.valid_at(int(r)) else None
            key.append(GroupFloat(v) if isinstance(v, float) else v)
        return tuple(key)

    def _decode_value(self, k):
        """Canonical 64-bit key of the single fixed-width key column -> Python value."""
        return decode_canonical(self.key_type, self.decimal_scale, k)

    def _decode(self, k):
        if self.key_kind() == N.FREQ_KEYS_VALUES:
            return (self._decode_value(int(k)),)
        return self._key_of_row(int(k))

    def _decode_many(self, keys):
        """_decode over many keys; a representative-row table gathers every key column's cells in one batch."""
        if self.key_kind() == N.FREQ_KEYS_VALUES:
            return [(self._decode_value(int(k)),) for k in keys]
        cols = [c.cells_at(keys) for c in self.key_columns]
        out = []
        for i in range(len(keys)):
            out.append(tuple(GroupFloat(col[i]) if isinstance(col[i], float) else col[i] for col in cols))
        return out

    def top(self, k):
        """[(key tuple, count)] of the k largest groups (NULL group included for Histogram)."""
        k = int(min(k, self.num_groups))
        keys = np.zeros(max(k, 1), dtype=np.int64)
        counts = np.zeros(max(k, 1), dtype=np.int64)
        n = self.ctx.lib.dq_freq_top(self.ctx.handle, self.handle, k, keys.ctypes.data, counts.ctypes.data)
        if n < 0:
            raise N.NativeError(int(n), "dq_freq_top: %s" % self.ctx.last_error())
        dec = self._decode_many(keys[:n])
        out = [(dec[i], int(counts[i])) for i in range(n)]
        nulls = self.summary(None)["null_count"]
        if nulls:
            out.append(((None,) * max(len(self.names), 1), int(nulls)))
            out.sort(key=lambda kv: -kv[1])
            out = out[:k]
        return out

    def to_dict(self):
        n = self.num_groups
        keys = np.zeros(max(n, 1), dtype=np.int64)
        counts = np.zeros(max(n, 1), dtype=np.int64)
        got = self.ctx.lib.dq_freq_export(self.ctx.handle, self.handle, n, keys.ctypes.data, counts.ctypes.data)
        if got < 0:
            raise N.NativeError(int(got), "dq_freq_export: %s" % self.ctx.last_error())
        dec = self._decode_many(keys[:got])
        out = {dec[i]: int(counts[i]) for i in range(got)}
        nulls = self.summary(None)["null_count"]
        if nulls:
            out[(None,) * max(len(self.names), 1)] = int(nulls)
        return out


def frequencies(table, key_columns, include_nulls=False, weights=None):
    """dq_frequencies over `key_columns` of `table`; with `weights` (int64 numpy array, one count per row) each row
    stands for that many rows (dq_frequencies_ex: the pre-aggregated groups of other shards)."""
    context = ctx()
    names = list(table.columns)
    keys = np.array([names.index(c) for c in key_columns], dtype=np.int32)
    parted = [table[c] for c in names if isinstance(table[c], PartedColumn)]
    if parted:  # a ChunkedTable's columns read in place (dq_frequencies_parts): part-major column array
        if weights is not None or len(parted) != len(names):
            raise TypeError("a parted table takes an unweighted grouping over parted columns only")
        per = [table[c].native_parts() for c in names]
        nparts = len(per[0])
        arr = (N.DqColumn * (nparts * len(names)))(*[per[c][p] for p in range(nparts) for c in range(len(names))])
        opt = N.DqFreqOptions()
        opt.flags = N.FREQ_INCLUDE_NULLS if include_nulls else 0
        handle = ctypes.c_void_p()
        rc = context.lib.dq_frequencies_parts(context.handle, arr, nparts, len(names), keys.ctypes.data, len(keys),
                                              ctypes.byref(opt), ctypes.byref(handle))
        context.check(rc, "dq_frequencies_parts")
        return FrequencyTable(context, handle, table, key_columns, include_nulls)
    cols = [table[c].native() for c in names]
    arr = (N.DqColumn * max(len(cols), 1))(*cols)
    handle = ctypes.c_void_p()
    flags = N.FREQ_INCLUDE_NULLS if include_nulls else 0
    if weights is None:
        rc = context.lib.dq_frequencies(context.handle, arr, len(cols), table.nrows, keys.ctypes.data, len(keys),
                                        flags, ctypes.byref(handle))
    else:
        on_device = hasattr(weights, "data_ptr")  # a torch tensor in HBM (int64, one count per row)
        w = weights if on_device else np.ascontiguousarray(weights, dtype=np.int64)
        if len(w) != table.nrows:
            raise ValueError("weights: %d entries for %d rows" % (len(w), table.nrows))
        opt = N.DqFreqOptions()
        opt.flags = flags
        opt.weights_device = 1 if on_device else 0
        opt.weights = (w.data_ptr() if on_device else w.ctypes.data) if len(w) else None
        rc = context.lib.dq_frequencies_ex(context.handle, arr, len(cols), table.nrows, keys.ctypes.data, len(keys),
                                           ctypes.byref(opt), ctypes.byref(handle))
    context.check(rc, "dq_frequencies")
    ft = FrequencyTable(context, handle, table, key_columns, include_nulls)
    ft.weights = None if weights is None else w
    return ft
