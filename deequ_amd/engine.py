"""Device selection and the frequency-table handle (the GPU side of computeFrequencies)."""
import ctypes
import os

import numpy as np

from . import native as N

_device = None


def set_device(device):
    global _device
    _device = int(device)


def device():
    if _device is not None:
        return _device
    return int(os.environ.get("LOCAL_RANK", "0"))


def ctx():
    return N.context(device())


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


class FrequencyTable:
    """Device-resident (key -> count) table built by dq_frequencies over `key_columns` of `source`."""

    def __init__(self, context, handle, source, key_columns, include_nulls):
        self.ctx = context
        self.handle = handle
        self.source = source
        self.key_columns = [source[c] for c in key_columns]
        self.names = list(key_columns)
        self.include_nulls = include_nulls
        s = self.summary(None)
        self.num_rows = s["num_rows"]
        self.num_groups = s["num_groups"]

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
                "null_count": out.null_count}

    def key_kind(self):
        return self.ctx.lib.dq_freq_key_kind(self.handle)

    def _key_of_row(self, r):
        key = []
        for c in self.key_columns:
            valid = c.validity is None or bool((c.validity[r >> 3] >> (r & 7)) & 1)
            v = c.value_at(int(r)) if valid else None
            key.append(GroupFloat(v) if isinstance(v, float) else v)
        return tuple(key)

    def _decode_value(self, k):
        """Canonical 64-bit key of the single fixed-width key column -> Python value."""
        c = self.key_columns[0]
        u = np.uint64(k & 0xFFFFFFFFFFFFFFFF)
        if c.spark_type == N.TYPE_DOUBLE:
            return GroupFloat(u.view(np.float64))
        if c.spark_type == N.TYPE_FLOAT:
            return GroupFloat(np.uint32(int(u) & 0xFFFFFFFF).view(np.float32))
        i = int(u.view(np.int64))
        if c.spark_type == N.TYPE_BOOLEAN:
            return bool(i)
        if c.spark_type == N.TYPE_DECIMAL:
            from decimal import Decimal
            return Decimal(i).scaleb(-c.decimal_scale)
        return i

    def _decode(self, k):
        if self.key_kind() == N.FREQ_KEYS_VALUES:
            return (self._decode_value(int(k)),)
        return self._key_of_row(int(k))

    def top(self, k):
        """[(key tuple, count)] of the k largest groups (NULL group included for Histogram)."""
        k = int(min(k, self.num_groups))
        keys = np.zeros(max(k, 1), dtype=np.int64)
        counts = np.zeros(max(k, 1), dtype=np.int64)
        n = self.ctx.lib.dq_freq_top(self.ctx.handle, self.handle, k, keys.ctypes.data, counts.ctypes.data)
        if n < 0:
            raise N.NativeError(int(n), "dq_freq_top: %s" % self.ctx.last_error())
        out = [(self._decode(keys[i]), int(counts[i])) for i in range(n)]
        nulls = self.summary(None)["null_count"]
        if nulls:
            out.append(((None,) * len(self.key_columns), int(nulls)))
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
        out = {self._decode(keys[i]): int(counts[i]) for i in range(got)}
        nulls = self.summary(None)["null_count"]
        if nulls:
            out[(None,) * len(self.key_columns)] = int(nulls)
        return out


def frequencies(table, key_columns, include_nulls=False):
    context = ctx()
    names = list(table.columns)
    cols = [table[c].native() for c in names]
    keys = np.array([names.index(c) for c in key_columns], dtype=np.int32)
    arr = (N.DqColumn * max(len(cols), 1))(*cols)
    handle = ctypes.c_void_p()
    rc = context.lib.dq_frequencies(context.handle, arr, len(cols), table.nrows, keys.ctypes.data, len(keys),
                                    N.FREQ_INCLUDE_NULLS if include_nulls else 0, ctypes.byref(handle))
    context.check(rc, "dq_frequencies")
    return FrequencyTable(context, handle, table, key_columns, include_nulls)
