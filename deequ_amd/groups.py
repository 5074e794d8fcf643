"""Group blocks: the groups of a pre-aggregated frequency table as host columns, in the form the sharded runner
exchanges them between ranks.

The reference computes a grouping with one Spark shuffle: `groupBy(columns).count()` pre-aggregates each
partition and hash-partitions the partial groups by key (A/GroupingAnalyzers.scala:53-79). The sharded runner
does the same. Each rank builds its shard's frequency table on its GPU. Its groups become a GroupBlock (the key
columns at the groups' representative rows, plus the counts). A group goes to the rank picked by a hash of its key
(`owners`), as packed bytes (`pack` / `unpack`, one all-to-all). The owner rebuilds one table over everything it
received, weighted by the counts, so duplicates from different ranks merge into one group.

Everything here is vectorised numpy over whole blocks, with no per-group Python. Strings are hashed with a
polynomial hash over the concatenated bytes (prefix sums of b_j * P^j, rescaled by P^-start). It only has to be a
deterministic function of the key bytes, identical on every rank; equality inside a group is decided by the
owner's table build, never by this hash.
"""
import struct

import numpy as np

from . import native as N
from .table import Column, Table, NUMPY_OF, pack_validity, unpack_validity
from .engine import canonical_keys, decode_canonical, GroupFloat

_M64 = (1 << 64) - 1
_P = 0x9E3779B97F4A7C15  # odd: invertible mod 2^64
_NULL_COMPONENT = np.uint64(0x6A09E667F3BCC909)
_NULL_VALUE = b"NullValue"  # Histogram's NullFieldReplacement (A/Histogram.scala:45)


def _inverse(a):
    x = a
    for _ in range(6):  # Newton: each step doubles the correct low bits
        x = (x * (2 - a * x)) & _M64
    return x


_P_INV = _inverse(_P)


def mix64(z):
    """splitmix64 finalizer over a uint64 array (wrapping arithmetic)."""
    z = np.asarray(z, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def _powers(base, n):
    p = np.empty(n + 1, dtype=np.uint64)
    p[0] = 1
    if n:
        with np.errstate(over="ignore"):
            p[1:] = np.cumprod(np.full(n, base, dtype=np.uint64), dtype=np.uint64)
    return p


def _string_hashes_span(values, start, end):
    """string_hashes over strings [start_i, end_i) that all lie in `values` (one bounded slice)."""
    total = len(values)
    with np.errstate(over="ignore"):
        pw = _powers(_P, total)
        pref = np.zeros(total + 1, dtype=np.uint64)
        if total:
            pref[1:] = np.cumsum(values.astype(np.uint64) * pw[:total], dtype=np.uint64)
        inv = _powers(_P_INV, total)
        h = (pref[end] - pref[start]) * inv[start]
        h = h + (end - start).astype(np.uint64) * np.uint64(0xC2B2AE3D27D4EB4F)
    return mix64(h)


_HASH_SLICE_BYTES = 1 << 24
# A device string column carries int32 Arrow offsets: a merged block whose key bytes reach this is built in
# key-disjoint splits (BlockParts.split_by_key). Module-level so tests can inject a small limit.
STRING_KEY_LIMIT = 2 ** 31 - 1


def string_hashes(values, offsets, slice_bytes=None):
    """Per string of a (UTF-8 bytes, int32 offsets) column: a 64-bit hash of its bytes and length. The polynomial
    prefix sums run over row slices of about `slice_bytes` bytes (the hash of a string does not depend on where it
    sits), so host memory stays ~24 B per byte of one slice rather than of the whole column."""
    values = np.asarray(values, dtype=np.uint8)
    offsets = np.asarray(offsets, dtype=np.int64)
    n = max(len(offsets) - 1, 0)
    out = np.empty(n, dtype=np.uint64)
    budget = max(1, int(slice_bytes or _HASH_SLICE_BYTES))
    r = 0
    while r < n:
        base = int(offsets[r])
        # last row whose end stays within the budget (at least one row per slice)
        e = int(np.searchsorted(offsets, base + budget, side="right")) - 1
        e = min(max(e, r + 1), n)
        lo, hi = offsets[r:e] - base, offsets[r + 1:e + 1] - base
        out[r:e] = _string_hashes_span(values[base:int(offsets[e])], lo, hi)
        r = e
    return out


def column_hashes(col, null_is_value=False):
    """64-bit hash of each cell of a key column, NULL cells a fixed component (or "NullValue"'s hash for a
    Histogram string column, where NULL and the literal are one group)."""
    valid = unpack_validity(col.validity, col.length)
    if col.spark_type == N.TYPE_STRING:
        h = string_hashes(col.values, col.offsets)
        if not valid.all():
            if null_is_value:
                nv = string_hashes(np.frombuffer(_NULL_VALUE, np.uint8), np.array([0, len(_NULL_VALUE)]))[0]
                h[~valid] = nv
            else:
                h[~valid] = _NULL_COMPONENT
        return h
    h = mix64(canonical_keys(col.spark_type, col.values).view(np.uint64))
    h[~valid] = _NULL_COMPONENT
    return h


def key_hashes(columns, null_is_value=False):
    acc = np.full(columns[0].length if columns else 0, 0x243F6A8885A308D3, dtype=np.uint64)
    with np.errstate(over="ignore"):
        for i, c in enumerate(columns):
            acc = mix64(acc + np.uint64((0xC2B2AE3D27D4EB4F * (i + 1)) & _M64) + column_hashes(c, null_is_value))
    return acc


def owners(block, world, null_is_value=False, key_columns=None):
    """Owner rank of every group of `block`: a hash of its key (or of the named subset of its key columns)."""
    cols = block.columns if key_columns is None else [block.column(n) for n in key_columns]
    if block.size == 0:
        return np.zeros(0, dtype=np.int64)
    return ((key_hashes(cols, null_is_value) >> np.uint64(32)) % np.uint64(world)).astype(np.int64)


def take(col, rows):
    """Rows `rows` (int64 indices) of a host column, as a new column."""
    rows = np.asarray(rows, dtype=np.int64)
    valid = unpack_validity(col.validity, col.length)[rows]
    validity = None if valid.all() else pack_validity(valid)
    if col.spark_type == N.TYPE_STRING:
        off = np.asarray(col.offsets, dtype=np.int64)
        starts = off[rows]
        lens = off[rows + 1] - starts
        new_off = np.zeros(len(rows) + 1, dtype=np.int64)
        np.cumsum(lens, out=new_off[1:])
        total = int(new_off[-1])
        idx = np.repeat(starts - new_off[:-1], lens) + np.arange(total, dtype=np.int64)
        data = np.ascontiguousarray(np.asarray(col.values, dtype=np.uint8)[idx])
        return Column(col.name, col.spark_type, data, validity, new_off.astype(np.int32), length=len(rows))
    return Column(col.name, col.spark_type, np.ascontiguousarray(np.asarray(col.values)[rows]), validity,
                  decimal_precision=col.decimal_precision, decimal_scale=col.decimal_scale)


def column_from_canonical(name, spark_type, keys, decimal_precision=0, decimal_scale=0):
    """Canonical 64-bit keys (DQ_FREQ_KEYS_VALUES export) -> a host column of the key's own type."""
    u = np.asarray(keys, dtype=np.int64).view(np.uint64)
    if spark_type == N.TYPE_DOUBLE:
        vals = u.view(np.float64).copy()
    elif spark_type == N.TYPE_FLOAT:
        vals = (u & np.uint64(0xFFFFFFFF)).astype(np.uint32).view(np.float32)
    elif spark_type == N.TYPE_BOOLEAN:
        vals = (u & np.uint64(1)).astype(np.uint8)
    else:
        vals = u.view(np.int64).astype(NUMPY_OF[spark_type])
    return Column(name, spark_type, np.ascontiguousarray(vals), None, decimal_precision=decimal_precision,
                  decimal_scale=decimal_scale)


class GroupBlock:
    """Groups as host columns: columns[i][g] is the i-th key component of group g (NULL where the group's key has
    NULL there), counts[g] its row count. num_rows / null_rows describe the table the groups came from (rows taking
    part; Histogram's all-NULL rows, which are not exported as a group)."""

    def __init__(self, columns, counts, num_rows=0, null_rows=0):
        self.columns = list(columns)
        self.counts = np.ascontiguousarray(counts, dtype=np.int64)
        self.num_rows = int(num_rows)
        self.null_rows = int(null_rows)

    @property
    def size(self):
        return len(self.counts)

    @property
    def names(self):
        return [c.name for c in self.columns]

    def column(self, name):
        for c in self.columns:
            if c.name == name:
                return c
        raise KeyError(name)

    def table(self):
        return Table(self.columns)

    def schema(self):
        return [(c.name, c.spark_type, c.decimal_precision, c.decimal_scale) for c in self.columns]

    def subset(self, rows):
        return GroupBlock([take(c, rows) for c in self.columns], self.counts[np.asarray(rows, dtype=np.int64)])

    def with_column(self, col):
        return GroupBlock(self.columns + [col], self.counts, self.num_rows, self.null_rows)

    def keys(self):
        """Python key tuples (GroupFloat for floating values, None for NULL) — for small blocks (top-k)."""
        out = []
        valid = [unpack_validity(c.validity, c.length) for c in self.columns]
        for g in range(self.size):
            key = []
            for c, v in zip(self.columns, valid):
                if not v[g]:
                    key.append(None)
                elif c.spark_type == N.TYPE_STRING:
                    key.append(c.value_at(g))
                else:
                    key.append(decode_canonical(c.spark_type, c.decimal_scale,
                                                int(canonical_keys(c.spark_type, c.values[g:g + 1])[0])))
            out.append(tuple(key))
        return out


def pack(block, rows=None):
    """Groups `rows` of `block` (all when None) -> bytes: the count, then per key column a validity byte per group
    and the values (fixed width) or lengths + UTF-8 bytes (strings)."""
    if rows is not None:
        block = block.subset(rows)
    g = block.size
    parts = [struct.pack("<q", g), block.counts.tobytes()]
    for c in block.columns:
        parts.append(unpack_validity(c.validity, c.length).astype(np.uint8).tobytes())
        if c.spark_type == N.TYPE_STRING:
            off = np.asarray(c.offsets, dtype=np.int64)
            lens = (off[1:] - off[:-1]).astype(np.int32)
            parts.append(lens.tobytes())
            parts.append(np.asarray(c.values, dtype=np.uint8)[:int(off[-1]) if g else 0].tobytes())
        else:
            parts.append(np.ascontiguousarray(c.values, dtype=NUMPY_OF[c.spark_type]).tobytes())
    return b"".join(parts)


def unpack(blob, schema):
    """Inverse of `pack` for the key schema [(name, spark type, decimal precision, decimal scale)]."""
    mv = memoryview(blob)
    (g,) = struct.unpack_from("<q", mv, 0)
    at = 8
    counts = np.frombuffer(mv, dtype=np.int64, count=g, offset=at).copy()
    at += 8 * g
    cols = []
    for name, t, prec, scale in schema:
        valid = np.frombuffer(mv, dtype=np.uint8, count=g, offset=at).astype(bool)
        at += g
        validity = None if valid.all() else pack_validity(valid)
        if t == N.TYPE_STRING:
            lens = np.frombuffer(mv, dtype=np.int32, count=g, offset=at).astype(np.int64)
            at += 4 * g
            off = np.zeros(g + 1, dtype=np.int64)
            np.cumsum(lens, out=off[1:])
            total = int(off[-1])
            data = np.frombuffer(mv, dtype=np.uint8, count=total, offset=at).copy()
            at += total
            cols.append(Column(name, t, data, validity, off.astype(np.int32), length=g))
        else:
            dt = np.dtype(NUMPY_OF[t])
            vals = np.frombuffer(mv, dtype=dt, count=g, offset=at).copy()
            at += dt.itemsize * g
            cols.append(Column(name, t, vals, validity, decimal_precision=prec, decimal_scale=scale))
    return GroupBlock(cols, counts)


class BlockParts(GroupBlock):
    """The groups of several blocks of one schema, concatenated lazily: the host columns are joined only when read;
    device_table() copies each part straight into device buffers (no host-side concatenation of the key bytes)."""

    def __init__(self, parts, schema):
        self.parts = [p for b in parts for p in (b.parts if isinstance(b, BlockParts) else [b]) if p.size]
        self._schema = list(schema)
        self._joined = None
        self.num_rows = sum(p.num_rows for p in self.parts)
        self.null_rows = sum(p.null_rows for p in self.parts)

    def _join(self):
        if self._joined is None:
            self._joined = concat(self.parts, self._schema)
        return self._joined

    columns = property(lambda self: self._join().columns)
    counts = property(lambda self: self._join().counts)

    @property
    def size(self):
        return sum(p.size for p in self.parts)

    @property
    def names(self):
        return [n for n, _, _, _ in self._schema]

    def schema(self):
        return list(self._schema)

    def key_bytes(self):
        """The largest total of UTF-8 key bytes over this block's string key columns (0 without string keys)."""
        most = 0
        for i, (_, t, _, _) in enumerate(self._schema):
            if t == N.TYPE_STRING:
                most = max(most, sum(int(p.columns[i].offsets[p.columns[i].length]) - int(p.columns[i].offsets[0])
                                     for p in self.parts))
        return most

    def split_by_key(self, limit=None):
        """The groups split into key-disjoint BlockParts (by a hash of the whole key, so every copy of a key lands
        in the same split), each with fewer than `limit` string key bytes per column: one weighted build per split
        stays within the int32 Arrow offsets of a device string column. One split when the block already fits."""
        limit = int(limit or STRING_KEY_LIMIT)
        total = self.key_bytes()
        if total < limit:
            return [self]
        k = max(2, -(-total * 5 // (4 * limit)))
        while True:
            splits = [[] for _ in range(k)]
            for p in self.parts:
                own = (key_hashes(p.columns) >> np.uint64(32)) % np.uint64(k)
                for s in range(k):
                    rows = np.flatnonzero(own == s)
                    if len(rows):
                        splits[s].append(p.subset(rows))
            out = [BlockParts(s, self._schema) for s in splits]
            if all(b.key_bytes() < limit for b in out):
                return out
            k *= 2
            if k > 4096:
                raise ValueError("string group keys do not split under the int32 Arrow offsets")

    def device_table(self):
        """(deequ_amd.table.Table of device columns, device int64 counts): each part's buffers copied into its
        slice of the device buffers, string offsets rebased on the device."""
        import torch
        dev = torch.device("cuda", torch.cuda.current_device())
        n = self.size
        if self.key_bytes() >= STRING_KEY_LIMIT:
            raise ValueError("string group keys of %d bytes exceed the int32 Arrow offsets of one device column "
                             "(split_by_key first)" % self.key_bytes())
        cols = []
        for i, (name, t, prec, scale) in enumerate(self._schema):
            parts = [b.columns[i] for b in self.parts]
            c = Column(name, t, None, None, length=n, decimal_precision=prec, decimal_scale=scale)
            d = {}
            if t == N.TYPE_STRING:
                nbytes = sum(int(p.offsets[p.length]) - int(p.offsets[0]) for p in parts)
                data = torch.zeros(nbytes + 16, dtype=torch.uint8, device=dev)
                off = torch.empty(n + 1, dtype=torch.int32, device=dev)
                off[0] = 0
                at, base = 0, 0
                for p in parts:
                    o = np.asarray(p.offsets, dtype=np.int64)[:p.length + 1]
                    a, b = int(o[0]), int(o[-1])
                    data[base:base + b - a].copy_(_host_tensor(np.asarray(p.values, dtype=np.uint8)[a:b]))
                    po = _host_tensor(o[1:]).to(dev)  # int64 on the device: the rebase cannot wrap
                    off[at + 1:at + 1 + p.length] = (po - a + base).to(torch.int32)
                    at += p.length
                    base += b - a
                d["values"], d["offsets"] = data, off
            else:
                dt = NUMPY_OF[t]
                vals = torch.empty(max(n, 1), dtype=torch.from_numpy(np.zeros(1, dtype=dt)).dtype, device=dev)
                at = 0
                for p in parts:
                    vals[at:at + p.length].copy_(_host_tensor(np.asarray(p.values)[:p.length]))
                    at += p.length
                d["values"] = vals
            if any(p.validity is not None for p in parts):
                d["validity"] = _device_validity(parts, n, dev)
            c.device = d
            cols.append(c)
        counts = torch.empty(max(n, 1), dtype=torch.int64, device=dev)
        at = 0
        for p in self.parts:
            counts[at:at + p.size].copy_(_host_tensor(p.counts))
            at += p.size
        torch.cuda.synchronize()
        return Table(cols), counts[:n]


def _host_tensor(a):
    """A CPU tensor over a numpy array, copied only when the array is read-only or strided (np.frombuffer views of
    persisted / received bytes are read-only, and torch.from_numpy warns on those)."""
    import torch
    return torch.from_numpy(np.require(a, requirements=["C", "W"]))


def _device_validity(parts, n, dev):
    """The validity bitmaps of several columns joined on the device: each part's packed bits (LSB first) unpacked
    to one byte per row in its slice, then repacked into one bitmap padded to whole 64-bit words."""
    import torch
    valid = torch.ones(max(n, 1), dtype=torch.uint8, device=dev)
    shifts = torch.arange(8, dtype=torch.uint8, device=dev)
    at = 0
    for p in parts:
        if p.validity is not None and p.length:
            packed = _host_tensor(np.asarray(p.validity, dtype=np.uint8)[:(p.length + 7) // 8]).to(dev)
            bits = (packed.unsqueeze(1) >> shifts) & 1
            valid[at:at + p.length] = bits.reshape(-1)[:p.length]
        at += p.length
    words = (n + 63) // 64
    rows = torch.zeros(words * 64, dtype=torch.uint8, device=dev)
    rows[:n] = valid[:n]
    return (rows.reshape(-1, 8) << shifts).sum(dim=1, dtype=torch.uint8) if n else \
        torch.zeros(8, dtype=torch.uint8, device=dev)


def concat(blocks, schema):
    """One block of the groups of several (same schema): buffers concatenated once, offsets rebased in place."""
    blocks = [b for b in blocks if b.size]
    if not blocks:
        return unpack(struct.pack("<q", 0), schema)
    if len(blocks) == 1:
        return GroupBlock(blocks[0].columns, blocks[0].counts)
    cols = []
    for i, (name, t, prec, scale) in enumerate(schema):
        parts = [b.columns[i] for b in blocks]
        validity = None
        if any(c.validity is not None for c in parts):
            valid = np.concatenate([unpack_validity(c.validity, c.length) for c in parts])
            validity = None if valid.all() else pack_validity(valid)
        n = sum(c.length for c in parts)
        if t == N.TYPE_STRING:
            off = np.empty(n + 1, dtype=np.int64)
            off[0] = 0
            at, base = 1, 0
            for c in parts:
                o = np.asarray(c.offsets, dtype=np.int64)[:c.length + 1]
                off[at:at + c.length] = o[1:] - o[0] + base
                base += int(o[-1] - o[0])
                at += c.length
            if base >= 2 ** 31:
                raise ValueError("concatenated string keys exceed the int32 Arrow offsets")
            data = np.concatenate([np.asarray(c.values, dtype=np.uint8)[int(c.offsets[0]):int(c.offsets[c.length])]
                                   for c in parts])
            cols.append(Column(name, t, data, validity, off.astype(np.int32), length=n))
        else:
            cols.append(Column(name, t, np.concatenate([np.asarray(c.values)[:c.length] for c in parts]), validity,
                               decimal_precision=prec, decimal_scale=scale))
    return GroupBlock(cols, np.concatenate([b.counts for b in blocks]))