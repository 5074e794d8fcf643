"""Parity oracle (TEST INFRASTRUCTURE — never imported by deequ_amd/).

Expected deequ states for a Table, restated from the reference's semantics:
  - per-row aggregates through the C restatement in oracle/dq_oracle.c (liboracle.so),
  - `where` / Compliance predicates by a pure-Python three-valued-logic evaluator of the parsed
    expression tree (small inputs only),
  - frequency tables (computeFrequencies, A/GroupingAnalyzers.scala:53-79) with Python dicts / numpy,
    entropy with math.fsum (exact summation).
Citations per function; SURVEY.md §8a restates every rule used here.
"""
import ctypes
import math
import os
import subprocess
import sys

import weakref

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "liboracle.so")

T_BOOLEAN, T_BYTE, T_SHORT, T_INT, T_LONG, T_FLOAT, T_DOUBLE, T_STRING, T_DATE, T_TIMESTAMP, T_DECIMAL = range(1, 12)


class OracleCol(ctypes.Structure):
    _fields_ = [("n", ctypes.c_int64), ("isum", ctypes.c_int64), ("dsum", ctypes.c_double),
                ("imin", ctypes.c_int64), ("imax", ctypes.c_int64), ("dmin", ctypes.c_double),
                ("dmax", ctypes.c_double), ("w_n", ctypes.c_double), ("w_avg", ctypes.c_double),
                ("w_m2", ctypes.c_double), ("ex_mean", ctypes.c_double), ("ex_m2", ctypes.c_double)]


class OracleCorr(ctypes.Structure):
    _fields_ = [("n", ctypes.c_double), ("x_avg", ctypes.c_double), ("y_avg", ctypes.c_double),
                ("ck", ctypes.c_double), ("x_mk", ctypes.c_double), ("y_mk", ctypes.c_double),
                ("ex_ck", ctypes.c_double), ("ex_x_mk", ctypes.c_double), ("ex_y_mk", ctypes.c_double)]


class OracleGenSpec(ctypes.Structure):
    _fields_ = [("kind", ctypes.c_int32), ("spark_type", ctypes.c_int32), ("seed", ctypes.c_uint64),
                ("vseed", ctypes.c_uint64), ("permille", ctypes.c_int32), ("hll", ctypes.c_int32),
                ("pred_gt0", ctypes.c_int32), ("pad", ctypes.c_int32)]


class OracleGenCol(ctypes.Structure):
    _fields_ = [("n", ctypes.c_int64), ("nnan", ctypes.c_int64), ("isum", ctypes.c_int64), ("imin", ctypes.c_int64),
                ("imax", ctypes.c_int64), ("pred_true", ctypes.c_int64), ("dmin", ctypes.c_double),
                ("dmax", ctypes.c_double), ("ex_sum", ctypes.c_double), ("ex_mean", ctypes.c_double),
                ("ex_m2", ctypes.c_double), ("sp_sum", ctypes.c_double), ("sp_mean", ctypes.c_double),
                ("sp_m2", ctypes.c_double), ("regs", ctypes.c_uint8 * 512)]


class OracleGenCorr(ctypes.Structure):
    _fields_ = [("n", ctypes.c_double), ("x_avg", ctypes.c_double), ("y_avg", ctypes.c_double),
                ("ck", ctypes.c_double), ("x_mk", ctypes.c_double), ("y_mk", ctypes.c_double)]


class OracleGenLeaf(ctypes.Structure):
    _fields_ = [("col", ctypes.c_int32), ("op", ctypes.c_int32), ("is_dbl", ctypes.c_int32), ("pad", ctypes.c_int32),
                ("ci", ctypes.c_int64), ("cd", ctypes.c_double)]


class OracleGenPred(ctypes.Structure):
    _fields_ = [("nleaves", ctypes.c_int32), ("comb", ctypes.c_int32), ("leaf", OracleGenLeaf * 4)]


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            subprocess.run(["make", "-s", "-C", HERE], check=True)
        L = ctypes.CDLL(LIB)
        L.oracle_xxh64.restype = ctypes.c_uint64
        L.oracle_xxh64.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_uint64]
        L.oracle_spark_hash.restype = ctypes.c_uint64
        L.oracle_spark_hash.argtypes = [ctypes.c_int, ctypes.c_void_p]
        L.oracle_column.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64,
                                    ctypes.POINTER(OracleCol)]
        L.oracle_correlation.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                                         ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.POINTER(OracleCorr)]
        L.oracle_hll_fixed.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p]
        L.oracle_hll_strings.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64,
                                         ctypes.c_void_p]
        L.oracle_hll_pack.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
        L.oracle_hll_count.restype = ctypes.c_double
        L.oracle_hll_count.argtypes = [ctypes.c_void_p]
        L.oracle_splitmix64.restype = ctypes.c_uint64
        L.oracle_splitmix64.argtypes = [ctypes.c_uint64, ctypes.c_uint64]
        L.oracle_synth_column.argtypes = [ctypes.c_int, ctypes.c_uint64, ctypes.c_int64, ctypes.c_int64,
                                          ctypes.c_void_p]
        L.oracle_synth_validity.argtypes = [ctypes.c_uint64, ctypes.c_int64, ctypes.c_int64, ctypes.c_int,
                                            ctypes.c_void_p]
        L.oracle_synth_freq_keys.argtypes = [ctypes.c_int64, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64,
                                             ctypes.c_void_p]
        L.oracle_generated_suite.restype = ctypes.c_int
        L.oracle_generated_suite.argtypes = [ctypes.c_int, ctypes.POINTER(OracleGenSpec), ctypes.c_int64,
                                             ctypes.c_int64, ctypes.c_int, ctypes.c_void_p, ctypes.c_int,
                                             ctypes.POINTER(OracleGenCol), ctypes.POINTER(OracleGenCorr)]
        L.oracle_generated_suite_ex.restype = ctypes.c_int
        L.oracle_generated_suite_ex.argtypes = [ctypes.c_int, ctypes.POINTER(OracleGenSpec), ctypes.c_int64,
                                                ctypes.c_int64, ctypes.c_int, ctypes.c_void_p, ctypes.c_int,
                                                ctypes.POINTER(OracleGenPred), ctypes.c_int,
                                                ctypes.POINTER(OracleGenPred), ctypes.POINTER(OracleGenCol),
                                                ctypes.POINTER(OracleGenCorr), ctypes.c_void_p, ctypes.c_void_p]
        L.oracle_group_counts.restype = ctypes.c_int64
        L.oracle_group_counts.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64,
                                          ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                          ctypes.POINTER(ctypes.c_int64)]
        _lib = L
    return _lib


def group_counts_raw(spark_type, values, validity, nrows):
    """count(*) GROUP BY one fixed-width key column from its raw Arrow buffers (values, LSB-first validity bitmap
    or None) in C (oracle_group_counts, A/GroupingAnalyzers.scala:53-79): (canonical keys as uint64 ascending,
    int64 counts, NULL rows). Canonical: integers sign-extended, FLOAT / DOUBLE bits with NaN canonical."""
    vals = np.ascontiguousarray(values)
    n = int(nrows)
    keys = np.empty(max(n, 1), dtype=np.int64)
    counts = np.empty(max(n, 1), dtype=np.int64)
    scratch = np.empty(max(n, 1), dtype=np.uint64)
    nulls = ctypes.c_int64(0)
    vb = None if validity is None else np.ascontiguousarray(validity, dtype=np.uint8)
    g = lib().oracle_group_counts(int(spark_type), vals.ctypes.data, None if vb is None else vb.ctypes.data, n,
                                  keys.ctypes.data, counts.ctypes.data, scratch.ctypes.data, ctypes.byref(nulls))
    return keys[:g].view(np.uint64).copy(), counts[:g].copy(), int(nulls.value)


def group_strings_raw(parts, queries=()):
    """count(*) GROUP BY one UTF-8 string key column over row-range parts [(bytes uint8, int32 offsets, LSB-first
    validity or None, rows), ...] in C (oracle_group_strings: keys <= 23 bytes packed with their length into 24-byte
    records, bucketed, sorted and run-length counted -- equal groups are equal byte strings, no fingerprint;
    A/GroupingAnalyzers.scala:53-79). Returns {"valid_rows", "null_rows", "num_groups", "count_values",
    "count_groups" (the distinct group counts and how many groups have each), "query_counts" (the exact count of each
    query string, 0 when absent)}."""
    L = lib()
    fn = L.oracle_group_strings
    fn.restype = ctypes.c_int64
    P = ctypes.c_void_p
    fn.argtypes = [ctypes.c_int, P, P, P, P, P, P, P, P, P, P, P, ctypes.c_int64, P]
    keep = []
    np_parts = []
    for b, o, v, n in parts:
        b = np.ascontiguousarray(b, dtype=np.uint8)
        o = np.ascontiguousarray(o, dtype=np.int32)
        v = None if v is None else np.ascontiguousarray(v, dtype=np.uint8)
        np_parts.append((b, o, v, int(n)))
        keep += [b, o, v]
    k = len(np_parts)
    bp = (ctypes.c_void_p * k)(*[p[0].ctypes.data for p in np_parts])
    op = (ctypes.c_void_p * k)(*[p[1].ctypes.data for p in np_parts])
    vp = (ctypes.c_void_p * k)(*[None if p[2] is None else p[2].ctypes.data for p in np_parts])
    rows = np.array([p[3] for p in np_parts], dtype=np.int64)
    enc = [q.encode("utf-8") for q in queries]
    qb = np.frombuffer(b"".join(enc) or b"\0", dtype=np.uint8).copy()
    qo = np.zeros(len(enc) + 1, dtype=np.int64)
    qo[1:] = np.cumsum([len(e) for e in enc]) if enc else []
    qc = np.zeros(max(len(enc), 1), dtype=np.int64)
    cap = 1 << 20
    cv = np.zeros(cap, dtype=np.int64)
    cm = np.zeros(cap, dtype=np.int64)
    ncc = ctypes.c_int64(cap)
    vr, nr = ctypes.c_int64(0), ctypes.c_int64(0)
    g = fn(k, ctypes.cast(bp, P), ctypes.cast(op, P), ctypes.cast(vp, P), rows.ctypes.data, ctypes.addressof(vr),
           ctypes.addressof(nr), cv.ctypes.data, cm.ctypes.data, ctypes.addressof(ncc), qb.ctypes.data, qo.ctypes.data,
           len(enc), qc.ctypes.data)
    if g < 0:
        raise ValueError("oracle_group_strings failed (%d)" % g)
    m = ncc.value
    return {"valid_rows": vr.value, "null_rows": nr.value, "num_groups": int(g), "count_values": cv[:m].copy(),
            "count_groups": cm[:m].copy(), "query_counts": qc[:len(enc)].copy()}


def group_summary_from_count_groups(values, mult, num_rows):
    """group_summary_from_counts over (distinct count, number of groups with it) pairs."""
    terms = []
    for v, m in zip(np.asarray(values).tolist(), np.asarray(mult).tolist()):
        p = v / num_rows
        terms.append(-m * p * math.log(p))
    vals = np.asarray(values)
    mult = np.asarray(mult)
    return {"num_groups": int(mult.sum()), "num_unique": int(mult[vals == 1].sum()),
            "entropy": math.fsum(terms) if terms else 0.0}


def group_summary_from_counts(counts, num_rows):
    """The fused aggregation of A/GroupingAnalyzers.scala:83-120 over a table's counts: groups, groups seen once,
    and the entropy terms -(c/N) ln(c/N) summed exactly (math.fsum over the distinct counts' multiplicities)."""
    c = np.asarray(counts, dtype=np.int64)
    vals, mult = np.unique(c, return_counts=True)
    terms = []
    for v, m in zip(vals.tolist(), mult.tolist()):
        p = v / num_rows
        terms.append(-m * p * math.log(p))
    return {"num_groups": int(len(c)), "num_unique": int((c == 1).sum()), "entropy": math.fsum(terms) if terms else 0.0}


# ---- raw helpers ---------------------------------------------------------------------------------
def xxh64(data, seed=42):
    b = bytes(data)
    buf = ctypes.create_string_buffer(b, max(len(b), 1))
    return lib().oracle_xxh64(buf, len(b), seed)


def spark_hash(spark_type, value):
    dtype = {T_BOOLEAN: np.uint8, T_BYTE: np.int8, T_SHORT: np.int16, T_INT: np.int32, T_DATE: np.int32,
             T_LONG: np.int64, T_TIMESTAMP: np.int64, T_DECIMAL: np.int64, T_FLOAT: np.float32,
             T_DOUBLE: np.float64}[spark_type]
    a = np.array([value], dtype=dtype)
    return lib().oracle_spark_hash(spark_type, a.ctypes.data)


def hll_count(words):
    w = np.array([int(np.int64(np.uint64(x & 0xFFFFFFFFFFFFFFFF))) for x in words], dtype=np.int64)
    return lib().oracle_hll_count(w.ctypes.data)


def synth_column(kind, seed, row0, n):
    dt = np.int64 if kind in (4, 5) else np.float64
    out = np.zeros(n, dtype=dt)
    lib().oracle_synth_column(kind, seed, row0, n, out.ctypes.data)
    return out


def synth_freq_keys(total, distinct, row0, n):
    out = np.zeros(n, dtype=np.int64)
    lib().oracle_synth_freq_keys(total, distinct, row0, n, out.ctypes.data)
    return out


def synth_validity(seed, row0, n, permille):
    m = np.zeros(n, dtype=np.uint8)
    lib().oracle_synth_validity(seed, row0, n, permille, m.ctypes.data)
    return m.astype(bool)


_GEN_OPS = {"<": 0, "<=": 1, "=": 2, "!=": 3, ">": 4, ">=": 5}


def _gen_pred(specs, pred):
    """(comb, [(column index, op, constant)...]) -> OracleGenPred. comb is "and" / "or"; a Python float constant
    compares as double, an int as long (as double against a DOUBLE column)."""
    comb, leaves = pred
    if not 1 <= len(leaves) <= 4:
        raise ValueError("1..4 leaves")
    p = OracleGenPred()
    p.nleaves = len(leaves)
    p.comb = {"and": 0, "or": 1}[comb]
    for i, (c, op, k) in enumerate(leaves):
        is_dbl = isinstance(k, float) or specs[c]["spark_type"] == T_DOUBLE
        p.leaf[i] = OracleGenLeaf(c, _GEN_OPS[op], int(is_dbl), 0, 0 if isinstance(k, float) else int(k), float(k))
    return p


def generated_suite(specs, row0, nrows, pairs=(), threads=None, where=None, preds=()):
    """Streamed oracle over generated columns (dq_oracle.c oracle_generated_suite_ex): `specs` are dicts
    with kind, spark_type, seed, vseed, permille (< 0 = no nulls), hll, pred_gt0. Returns (per-column
    dicts, per-pair correlation dicts). Exact counts / Long sums / min / max / Compliance counts / HLL
    registers; exact (compensated long double) sums, moments and co-moments.

    `where` (comb, leaves) filters every aggregate (conditionalSelection, A/Analyzer.scala:409-432); `preds` are
    Compliance predicates counted over the where-TRUE rows. Given either, a third value is returned:
    {"where_true", "where_nn", "preds": [(true, not_null), ...]}."""
    if threads is None:
        threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or os.cpu_count() or 1
        threads = max(1, min(threads, 16))
    arr = (OracleGenSpec * len(specs))()
    for i, sp in enumerate(specs):
        arr[i] = OracleGenSpec(sp["kind"], sp["spark_type"], sp["seed"], sp.get("vseed", 0), sp.get("permille", -1),
                               int(sp.get("hll", 0)), int(sp.get("pred_gt0", 0)), 0)
    outc = (OracleGenCol * len(specs))()
    npairs = len(pairs)
    pa = np.array([c for p in pairs for c in p] or [0], dtype=np.int32)
    outp = (OracleGenCorr * max(npairs, 1))()
    wp = _gen_pred(specs, where) if where is not None else None
    parr = (OracleGenPred * max(len(preds), 1))(*[_gen_pred(specs, p) for p in preds])
    wc = np.zeros(2, dtype=np.int64)
    pc = np.zeros(2 * max(len(preds), 1), dtype=np.int64)
    rc = lib().oracle_generated_suite_ex(len(specs), arr, row0, nrows, npairs, pa.ctypes.data, threads,
                                         ctypes.byref(wp) if wp is not None else None, len(preds), parr, outc, outp,
                                         wc.ctypes.data, pc.ctypes.data)
    if rc != 0:
        raise RuntimeError("oracle_generated_suite_ex failed: %d" % rc)
    cols = []
    for o in outc:
        d = {f: getattr(o, f) for f, _ in OracleGenCol._fields_ if f != "regs"}
        d["regs"] = np.frombuffer(bytes(o.regs), dtype=np.uint8).copy()
        words = np.zeros(52, dtype=np.int64)
        lib().oracle_hll_pack(d["regs"].ctypes.data, words.ctypes.data)
        d["words"] = [int(w) for w in words]
        cols.append(d)
    corrs = [{f: getattr(outp[i], f) for f, _ in OracleGenCorr._fields_} for i in range(npairs)]
    if where is None and not preds:
        return cols, corrs
    counts = {"where_true": int(wc[0]), "where_nn": int(wc[1]),
              "preds": [(int(pc[2 * i]), int(pc[2 * i + 1])) for i in range(len(preds))]}
    return cols, corrs, counts


# ---- the oracle's own State algebra and metric formulas -----------------------------------------------
# Restated from the reference state files, independent of deequ_amd/states.py: field names match the
# reference case classes (so tests compare field by field, and `==` against a product state compares
# the fields), metricValue / sum follow each file.
class OState:
    fields = ()

    def key(self):
        return tuple(getattr(self, f) for f in self.fields)

    def __eq__(self, other):
        if type(other).__name__ != type(self).__name__:
            return NotImplemented
        return self.key() == tuple(getattr(other, f) for f in self.fields)

    def __ne__(self, other):
        r = self.__eq__(other)
        return r if r is NotImplemented else not r

    __hash__ = None

    def __repr__(self):
        return "oracle.%s%r" % (type(self).__name__, self.key())


def _java_div(a, b):
    """Java double division (x / 0.0 = +-Infinity, 0.0 / 0.0 = NaN)."""
    if b == 0.0:
        if a == 0.0 or a != a:
            return float("nan")
        return math.copysign(float("inf"), a) * math.copysign(1.0, b)
    return a / b


class NumMatches(OState):  # A/Size.scala:23-31
    fields = ("numMatches",)

    def __init__(self, numMatches):
        self.numMatches = int(numMatches)

    def sum(self, o):
        return NumMatches(self.numMatches + o.numMatches)

    def metricValue(self):
        return float(self.numMatches)


class NumMatchesAndCount(OState):  # A/Analyzer.scala:230-244
    fields = ("numMatches", "count")

    def __init__(self, numMatches, count):
        self.numMatches, self.count = int(numMatches), int(count)

    def sum(self, o):
        return NumMatchesAndCount(self.numMatches + o.numMatches, self.count + o.count)

    def metricValue(self):
        return float("nan") if self.count == 0 else self.numMatches / self.count


class MeanState(OState):  # A/Mean.scala:25-35
    fields = ("sum_", "count")

    def __init__(self, sum_, count):
        self.sum_, self.count = float(sum_), int(count)

    def sum(self, o):
        return MeanState(self.sum_ + o.sum_, self.count + o.count)

    def metricValue(self):
        return float("nan") if self.count == 0 else self.sum_ / self.count


class SumState(OState):  # A/Sum.scala:25-32
    fields = ("sum_",)

    def __init__(self, sum_):
        self.sum_ = float(sum_)

    def sum(self, o):
        return SumState(self.sum_ + o.sum_)

    def metricValue(self):
        return self.sum_


def _java_min(a, b):  # math.min: NaN wins, -0.0 < 0.0
    if a != a or b != b:
        return float("nan")
    if a == b == 0.0:
        return a if math.copysign(1.0, a) < 0 else b
    return a if a < b else b


def _java_max(a, b):
    if a != a or b != b:
        return float("nan")
    if a == b == 0.0:
        return b if math.copysign(1.0, a) < 0 else a
    return a if a > b else b


class MinState(OState):  # A/Minimum.scala:25-32
    fields = ("minValue",)

    def __init__(self, minValue):
        self.minValue = float(minValue)

    def sum(self, o):
        return MinState(_java_min(self.minValue, o.minValue))

    def metricValue(self):
        return self.minValue


class MaxState(OState):  # A/Maximum.scala:25-32
    fields = ("maxValue",)

    def __init__(self, maxValue):
        self.maxValue = float(maxValue)

    def sum(self, o):
        return MaxState(_java_max(self.maxValue, o.maxValue))

    def metricValue(self):
        return self.maxValue


class StandardDeviationState(OState):  # A/StandardDeviation.scala:25-50
    fields = ("n", "avg", "m2")

    def __init__(self, n, avg, m2):
        self.n, self.avg, self.m2 = float(n), float(avg), float(m2)

    def sum(self, o):
        newN = self.n + o.n
        delta = o.avg - self.avg
        deltaN = 0.0 if newN == 0.0 else delta / newN
        return StandardDeviationState(newN, self.avg + deltaN * o.n, self.m2 + o.m2 + delta * deltaN * self.n * o.n)

    def metricValue(self):
        return math.sqrt(_java_div(self.m2, self.n))


class CorrelationState(OState):  # A/Correlation.scala:26-60
    fields = ("n", "xAvg", "yAvg", "ck", "xMk", "yMk")

    def __init__(self, n, xAvg, yAvg, ck, xMk, yMk):
        self.n, self.xAvg, self.yAvg = float(n), float(xAvg), float(yAvg)
        self.ck, self.xMk, self.yMk = float(ck), float(xMk), float(yMk)

    def sum(self, o):
        n1, n2 = self.n, o.n
        newN = n1 + n2
        dx, dy = o.xAvg - self.xAvg, o.yAvg - self.yAvg
        dxN = 0.0 if newN == 0.0 else dx / newN
        dyN = 0.0 if newN == 0.0 else dy / newN
        return CorrelationState(newN, self.xAvg + dxN * n2, self.yAvg + dyN * n2,
                                self.ck + o.ck + dx * dyN * n1 * n2, self.xMk + o.xMk + dx * dxN * n1 * n2,
                                self.yMk + o.yMk + dy * dyN * n1 * n2)

    def metricValue(self):
        return _java_div(self.ck, math.sqrt(self.xMk * self.yMk))


class ApproxCountDistinctState(OState):  # A/ApproxCountDistinct.scala:26-40
    fields = ("words",)

    def __init__(self, words):
        self.words = [int(w) for w in words]

    def sum(self, o):
        ra, rb = _unpack_regs(self.words), _unpack_regs(o.words)
        return ApproxCountDistinctState(_pack_regs(np.maximum(ra, rb)))

    def metricValue(self):
        return hll_count(self.words)


def _unpack_regs(words):
    regs = np.zeros(512, dtype=np.uint8)
    for i in range(512):
        regs[i] = (int(words[i // 10]) >> (6 * (i % 10))) & 63
    return regs


def _pack_regs(regs):
    words = np.zeros(52, dtype=np.int64)
    lib().oracle_hll_pack(np.ascontiguousarray(regs, dtype=np.uint8).ctypes.data, words.ctypes.data)
    return [int(w) for w in words]


class OracleDistValue:
    def __init__(self, absolute, ratio):
        self.absolute, self.ratio = absolute, ratio


class OracleDistribution:
    def __init__(self, values, numberOfBins):
        self.values, self.numberOfBins = values, numberOfBins


class DataTypeHistogram(OState):  # A/DataType.scala:32-110
    fields = ("numNull", "numFractional", "numIntegral", "numBoolean", "numString")

    def __init__(self, numNull, numFractional, numIntegral, numBoolean, numString):
        self.numNull, self.numFractional, self.numIntegral = int(numNull), int(numFractional), int(numIntegral)
        self.numBoolean, self.numString = int(numBoolean), int(numString)

    def sum(self, o):
        return DataTypeHistogram(*[a + b for a, b in zip(self.key(), o.key())])

    def toDistribution(self):
        total = sum(self.key())
        names = ("Unknown", "Fractional", "Integral", "Boolean", "String")
        return OracleDistribution({n: OracleDistValue(c, c / total if total else 0.0)
                                   for n, c in zip(names, self.key())}, 5)


# ---- the oracle's own SQL predicate parser ------------------------------------------------------------
# Spark SQL expression strings as deequ passes them (where filters, Compliance predicates, the checks'
# generated constraints M/checks/Check.scala:594-943), parsed by precedence climbing — independent of
# deequ_amd/expr.py — into the nodes _eval below evaluates with three-valued logic.
class PNode:
    def __init__(self, kind, *children, value=None):
        self.kind, self.children, self.value = kind, list(children), value


def _lex(text):
    out, i, n = [], 0, len(text)
    ops3 = ("<=>",)
    ops2 = ("<=", ">=", "<>", "!=", "==")
    while i < n:
        ch = text[i]
        if ch.isspace():
            i += 1
            continue
        if ch.isdigit() or (ch == "." and i + 1 < n and text[i + 1].isdigit()):
            j = i
            while j < n and text[j].isdigit():
                j += 1
            is_float = False
            if j < n and text[j] == ".":
                is_float = True
                j += 1
                while j < n and text[j].isdigit():
                    j += 1
            if j < n and text[j] in "eE" and j + 1 < n and (text[j + 1].isdigit() or text[j + 1] in "+-"):
                is_float = True
                j += 2
                while j < n and text[j].isdigit():
                    j += 1
            lit = text[i:j]
            if j < n and text[j] in "dD":
                is_float, j = True, j + 1
            elif j < n and text[j] in "lL":
                j += 1
            out.append(("num", float(lit) if is_float else int(lit)))
            i = j
            continue
        if ch in "'\"":
            j, buf = i + 1, []
            while j < n:
                c = text[j]
                if c == "\\" and j + 1 < n:
                    buf.append({"n": "\n", "t": "\t"}.get(text[j + 1], text[j + 1]))
                    j += 2
                    continue
                if c == ch:
                    if ch == "'" and j + 1 < n and text[j + 1] == "'":
                        buf.append("'")
                        j += 2
                        continue
                    break
                buf.append(c)
                j += 1
            out.append(("str", "".join(buf)))
            i = j + 1
            continue
        if ch == "`":
            j = text.index("`", i + 1)
            out.append(("name", text[i + 1:j]))
            i = j + 1
            continue
        if ch.isalpha() or ch == "_":
            j = i
            while j < n and (text[j].isalnum() or text[j] in "_."):
                j += 1
            out.append(("word", text[i:j]))
            i = j
            continue
        if text[i:i + 3] in ops3:
            out.append(("op", text[i:i + 3]))
            i += 3
            continue
        if text[i:i + 2] in ops2:
            out.append(("op", text[i:i + 2]))
            i += 2
            continue
        if ch in "=<>+-*/%(),":
            out.append(("op", ch))
            i += 1
            continue
        raise ValueError("oracle parser: bad character %r in %r" % (ch, text))
    out.append(("end", None))
    return out


class OracleParser:
    _CMP = {"=": "=", "==": "=", "!=": "!=", "<>": "!=", "<": "<", "<=": "<=", ">": ">", ">=": ">=", "<=>": "<=>"}

    def __init__(self, text):
        self.t, self.i, self.text = _lex(text), 0, text

    def _peek(self, k=0):
        return self.t[self.i + k]

    def _word(self, k=0):
        tok = self._peek(k)
        return tok[1].upper() if tok[0] == "word" else None

    def _next(self):
        tok = self.t[self.i]
        self.i += 1
        return tok

    def _expect_op(self, op):
        tok = self._next()
        if tok != ("op", op):
            raise ValueError("oracle parser: expected %r in %r" % (op, self.text))

    def parse(self):
        node = self._expr(0)
        if self._peek()[0] != "end":
            raise ValueError("oracle parser: trailing input in %r" % self.text)
        return node

    # binding powers: OR 1, AND 2, NOT 3 (prefix), predicates 4, + - 5, * / % 6, unary 7
    def _expr(self, min_bp):
        if self._word() == "NOT":
            self._next()
            left = PNode("not", self._expr(3))
        else:
            left = self._arith(0)
        while True:
            w = self._word()
            if w == "OR" and min_bp < 1:
                self._next()
                left = PNode("or", left, self._expr(1))
            elif w == "AND" and min_bp < 2:
                self._next()
                left = PNode("and", left, self._expr(2))
            elif min_bp < 4 and self._postfix_predicate_ahead():
                left = self._predicate(left)
            else:
                return left

    def _postfix_predicate_ahead(self):
        tok = self._peek()
        if tok[0] == "op" and tok[1] in self._CMP:
            return True
        w = self._word()
        return w in ("IS", "IN", "LIKE", "BETWEEN", "RLIKE", "REGEXP") or \
            (w == "NOT" and self._word(1) in ("IN", "LIKE", "BETWEEN", "RLIKE", "REGEXP"))

    def _predicate(self, left):
        tok = self._peek()
        if tok[0] == "op":
            self._next()
            return PNode("cmp", left, self._arith(0), value=self._CMP[tok[1]])
        negate = False
        if self._word() == "NOT":
            self._next()
            negate = True
        w = self._word()
        self._next()
        if w == "IS":
            neg = self._word() == "NOT"
            if neg:
                self._next()
            if self._word() != "NULL":
                raise ValueError("oracle parser: IS [NOT] NULL expected in %r" % self.text)
            self._next()
            return PNode("isnotnull" if neg else "isnull", left)
        if w == "IN":
            self._expect_op("(")
            items = [self._arith(0)]
            while self._peek() == ("op", ","):
                self._next()
                items.append(self._arith(0))
            self._expect_op(")")
            node = PNode("in", left, *items)
        elif w == "LIKE":
            pat = self._next()
            if pat[0] != "str":
                raise ValueError("oracle parser: LIKE pattern must be a string literal")
            node = PNode("like", left, value=pat[1])
        elif w in ("RLIKE", "REGEXP"):
            pat = self._next()
            if pat[0] != "str":
                raise ValueError("oracle parser: RLIKE pattern must be a string literal")
            node = PNode("rlike", left, value=pat[1])
        else:  # BETWEEN lo AND hi
            lo = self._arith(0)
            if self._word() != "AND":
                raise ValueError("oracle parser: BETWEEN without AND in %r" % self.text)
            self._next()
            hi = self._arith(0)
            node = PNode("and", PNode("cmp", left, lo, value=">="), PNode("cmp", left, hi, value="<="))
        return PNode("not", node) if negate else node

    def _arith(self, min_bp):
        tok = self._peek()
        if tok == ("op", "-"):
            self._next()
            left = PNode("neg", self._arith(7))
        elif tok == ("op", "+"):
            self._next()
            left = self._arith(7)
        else:
            left = self._primary()
        while True:
            tok = self._peek()
            if tok[0] != "op" or tok[1] not in "+-*/%" or len(tok[1]) != 1:
                return left
            bp = 5 if tok[1] in "+-" else 6
            if bp <= min_bp:
                return left
            self._next()
            left = PNode("arith", left, self._arith(bp), value=tok[1])

    def _primary(self):
        kind, val = self._next()
        if kind == "op" and val == "(":
            node = self._expr(0)
            self._expect_op(")")
            return node
        if kind == "num":
            return PNode("const", value=("double" if isinstance(val, float) else "long", val))
        if kind == "str":
            return PNode("const", value=("string", val))
        if kind == "name":
            return PNode("col", value=val)
        if kind != "word":
            raise ValueError("oracle parser: unexpected %r in %r" % (val, self.text))
        up = val.upper()
        if up in ("TRUE", "FALSE"):
            return PNode("const", value=("bool", up == "TRUE"))
        if up == "NULL":
            return PNode("null")
        if up == "DATE" and self._peek()[0] == "str":
            import datetime
            y, m, d = (int(x) for x in self._next()[1].strip().split("-"))
            return PNode("const", value=("long", (datetime.date(y, m, d) - datetime.date(1970, 1, 1)).days))
        if up == "CASE":
            subject = None if self._word() == "WHEN" else self._expr(0)
            parts = []
            while self._word() == "WHEN":
                self._next()
                cond = self._expr(0)
                if subject is not None:
                    cond = PNode("cmp", subject, cond, value="=")
                if self._word() != "THEN":
                    raise ValueError("oracle parser: CASE WHEN without THEN")
                self._next()
                parts.append((cond, self._expr(0)))
            other = None
            if self._word() == "ELSE":
                self._next()
                other = self._expr(0)
            if self._word() != "END":
                raise ValueError("oracle parser: CASE without END")
            self._next()
            return PNode("case", value=(parts, other))
        if up == "CAST":
            self._expect_op("(")
            inner = self._expr(0)
            if self._word() != "AS":
                raise ValueError("oracle parser: CAST without AS")
            self._next()
            target = self._next()[1].lower()
            if self._peek() == ("op", "("):
                while self._next() != ("op", ")"):
                    pass
            self._expect_op(")")
            if target in ("double", "float", "decimal"):
                return PNode("cast_double", inner)
            if target in ("int", "integer", "long", "bigint", "short", "smallint", "tinyint", "byte"):
                return PNode("cast_long", inner)
            if target == "string":
                return inner
            raise ValueError("oracle parser: CAST target %s" % target)
        if self._peek() == ("op", "("):
            self._next()
            args = []
            if self._peek() != ("op", ")"):
                args.append(self._expr(0))
                while self._peek() == ("op", ","):
                    self._next()
                    args.append(self._expr(0))
            self._expect_op(")")
            f = val.lower()
            if f == "coalesce":
                return PNode("coalesce", *args)
            if f in ("length", "char_length", "character_length"):
                return PNode("length", args[0])
            if f == "isnull":
                return PNode("isnull", args[0])
            if f == "isnotnull":
                return PNode("isnotnull", args[0])
            if f in ("nvl", "ifnull"):
                return PNode("coalesce", *args)
            if f == "if":
                return PNode("case", value=([(args[0], args[1])], args[2]))
            if f in ("substring", "substr"):
                return PNode("substr", *args)
            unary = {"isnan": "isnan", "abs": "abs", "lower": "lower", "lcase": "lower", "upper": "upper",
                     "ucase": "upper", "trim": "trim", "ltrim": "ltrim", "rtrim": "rtrim", "year": "year",
                     "month": "month", "dayofmonth": "day", "day": "day", "nanvl": "nanvl"}
            if f in unary:
                return PNode(unary[f], *args)
            raise ValueError("oracle parser: function %s" % f)
        return PNode("col", value=val)

# ---- predicate evaluation (3VL) ------------------------------------------------------------------
def _cmp_vals(a, b):
    """Spark comparison after PromoteStrings (string vs number -> double). None = NULL result."""
    if isinstance(a, str) and isinstance(b, str):
        ab, bb = a.encode(), b.encode()
        return (ab > bb) - (ab < bb)
    if isinstance(a, str) or isinstance(b, str):
        try:
            a = float(a) if isinstance(a, str) else float(a)
            b = float(b) if isinstance(b, str) else float(b)
        except ValueError:
            return None
    if isinstance(a, bool):
        a = int(a)
    if isinstance(b, bool):
        b = int(b)
    an = isinstance(a, float) and math.isnan(a)
    bn = isinstance(b, float) and math.isnan(b)
    if an or bn:
        return 0 if an and bn else (1 if an else -1)
    return (a > b) - (a < b)


def _like(s, pat):
    import re
    rx, i = "", 0
    while i < len(pat):
        c = pat[i]
        if c == "\\" and i + 1 < len(pat):
            rx += re.escape(pat[i + 1])
            i += 2
            continue
        rx += ".*" if c == "%" else ("." if c == "_" else re.escape(c))
        i += 1
    return re.fullmatch(rx, s, flags=re.S) is not None


def _eval(node, row):
    k = node.kind
    if k == "col":
        return row[node.value]
    if k == "const":
        kind, v = node.value
        return v
    if k == "null":
        return None
    if k == "cmp":
        a, b = _eval(node.children[0], row), _eval(node.children[1], row)
        if node.value == "<=>":
            if a is None or b is None:
                return a is None and b is None
            return _cmp_vals(a, b) == 0
        if a is None or b is None:
            return None
        c = _cmp_vals(a, b)
        if c is None:
            return None
        return {"=": c == 0, "!=": c != 0, "<": c < 0, "<=": c <= 0, ">": c > 0, ">=": c >= 0}[node.value]
    if k == "and":
        a, b = _eval(node.children[0], row), _eval(node.children[1], row)
        if a is False or b is False:
            return False
        if a is None or b is None:
            return None
        return True
    if k == "or":
        a, b = _eval(node.children[0], row), _eval(node.children[1], row)
        if a is True or b is True:
            return True
        if a is None or b is None:
            return None
        return False
    if k == "not":
        a = _eval(node.children[0], row)
        return None if a is None else (not a)
    if k == "isnull":
        return _eval(node.children[0], row) is None
    if k == "isnotnull":
        return _eval(node.children[0], row) is not None
    if k == "in":
        x = _eval(node.children[0], row)
        if x is None:
            return None
        any_null = False
        for ch in node.children[1:]:
            e = _eval(ch, row)
            if e is None:
                any_null = True
            elif _cmp_vals(x, e) == 0:
                return True
        return None if any_null else False
    if k == "like":
        x = _eval(node.children[0], row)
        return None if x is None else _like(x, node.value)
    if k == "arith":
        a, b = _eval(node.children[0], row), _eval(node.children[1], row)
        if a is None or b is None:
            return None
        a = float(a) if isinstance(a, str) else a
        b = float(b) if isinstance(b, str) else b
        op = node.value
        if op == "/":
            return None if b == 0 else float(a) / float(b)
        if op == "%":
            if b == 0:
                return None
            return math.fmod(a, b) if isinstance(a, float) or isinstance(b, float) else int(math.fmod(a, b))
        return {"+": a + b, "-": a - b, "*": a * b}[op]
    if k == "neg":
        a = _eval(node.children[0], row)
        return None if a is None else -a
    if k == "coalesce":
        for ch in node.children:
            v = _eval(ch, row)
            if v is not None:
                return v
        return None
    if k == "length":
        a = _eval(node.children[0], row)
        return None if a is None else len(a)
    if k == "cast_double":
        a = _eval(node.children[0], row)
        if a is None:
            return None
        try:
            return float(a)
        except ValueError:
            return None
    if k == "cast_long":
        a = _eval(node.children[0], row)
        if a is None:
            return None
        try:
            return int(float(a)) if isinstance(a, str) else int(a)
        except ValueError:
            return None
    if k == "case":
        parts, other = node.value
        for cond, val in parts:
            c = _eval(cond, row)
            if c is True or (c is not None and not isinstance(c, bool) and c != 0):
                return _eval(val, row)
        return None if other is None else _eval(other, row)
    if k == "rlike":
        # Spark RLike: Pattern.compile(p).matcher(str).find() -- any match, even an empty one
        a = _eval(node.children[0], row)
        if a is None:
            return None
        text = a if isinstance(a, str) else ("true" if a is True else "false" if a is False else str(a))
        return compile_java_regex(node.value).search(text) is not None
    if k in ("lower", "upper"):
        a = _eval(node.children[0], row)
        return a if not isinstance(a, str) else (a.lower() if k == "lower" else a.upper())
    if k in ("trim", "ltrim", "rtrim"):  # Spark 2.2 UTF8String.trim*: ASCII spaces only
        a = _eval(node.children[0], row)
        if not isinstance(a, str):
            return a
        return a.strip(" ") if k == "trim" else (a.lstrip(" ") if k == "ltrim" else a.rstrip(" "))
    if k == "substr":
        # UTF8String.substringSQL(pos, len): one-based, 0 = the first character, negative from the end
        vals = [_eval(c, row) for c in node.children]
        if any(v is None for v in vals):
            return None
        s, pos = vals[0], int(vals[1])
        length = int(vals[2]) if len(vals) > 2 else 2 ** 31 - 1
        n = len(s)
        start = pos - 1 if pos > 0 else (n + pos if pos < 0 else 0)
        until = n if length == 2 ** 31 - 1 else start + length
        if until <= start or start >= len(s.encode()):
            return ""
        return s[max(start, 0):max(until, 0)]
    if k == "isnan":
        a = _eval(node.children[0], row)
        if a is None:
            return False
        try:
            return math.isnan(float(a))
        except ValueError:
            return False
    if k == "abs":
        a = _eval(node.children[0], row)
        if isinstance(a, str):
            try:
                return abs(float(a))
            except ValueError:
                return None
        return None if a is None else abs(a)
    if k == "nanvl":
        a, b = _eval(node.children[0], row), _eval(node.children[1], row)
        if a is None or b is None:
            return None
        return b if isinstance(a, float) and math.isnan(a) else a
    if k in ("year", "month", "day"):
        # Spark 2.2 DateTimeUtils.getYear / getMonth / getDayOfMonth: the proleptic Gregorian date of the day number,
        # 10 days earlier on or before 1582-10-04; a TIMESTAMP's day in the UTC session zone
        import datetime
        a = _eval(node.children[0], row)
        if a is None:
            return None
        days = a // 86400000000 if node.value == T_TIMESTAMP else a
        if days <= -141428:
            days -= 10
        d = datetime.date(1970, 1, 1) + datetime.timedelta(days=days)
        return {"year": d.year, "month": d.month, "day": d.day}[k]
    raise ValueError(k)


def _annotate_types(node, table):
    """year / month / day of a column: the column's Spark type decides DATE (days) or TIMESTAMP (micros)."""
    if node.kind in ("year", "month", "day") and node.children and node.children[0].kind == "col":
        node.value = table[node.children[0].value].spark_type
    for c in node.children:
        _annotate_types(c, table)
    if node.kind == "case":
        for cond, val in node.value[0]:
            _annotate_types(cond, table)
            _annotate_types(val, table)
        if node.value[1] is not None:
            _annotate_types(node.value[1], table)


_MASKS = weakref.WeakKeyDictionary()  # table -> {predicate text: masks} (tables are not mutated by the tests)
_CELLS = weakref.WeakKeyDictionary()  # column -> its cells as Python objects


def predicate_masks(table, text):
    """(TRUE mask, NOT-NULL mask) of a SQL predicate over every row."""
    memo = _MASKS.setdefault(table, {})
    if text in memo:
        return memo[text]
    tree = OracleParser(text).parse()
    _annotate_types(tree, table)
    cols = {n: _pylist(table[n]) for n in table.columns}
    t = np.zeros(table.nrows, dtype=bool)
    nn = np.zeros(table.nrows, dtype=bool)
    for i in range(table.nrows):
        v = _eval(tree, {n: cols[n][i] for n in cols})
        nn[i] = v is not None
        t[i] = v is True or (v is not None and not isinstance(v, bool) and v != 0)
    memo[text] = (t, nn)
    return t, nn


# ---- the oracle's own reading of a column's Arrow-style buffers (never the product's decoders) ----------
def _host_buffer(col, key):
    """A column buffer as numpy: host arrays as they are; a device-resident column's buffer copied back."""
    v = getattr(col, {"values": "values", "validity": "validity", "offsets": "offsets"}[key])
    if v is None and getattr(col, "device", None):
        d = col.device.get(key)
        v = None if d is None else d.cpu().numpy()
    return v


def _valid(col):
    """Validity: bit (i mod 8) of byte (i div 8), LSB first; no bitmap = every row valid."""
    n = col.length
    vb = _host_buffer(col, "validity")
    if vb is None:
        return np.ones(n, dtype=bool)
    b = np.frombuffer(bytes(np.asarray(vb, dtype=np.uint8)[:(n + 7) // 8]), dtype=np.uint8)
    i = np.arange(n, dtype=np.int64)
    return ((b[i >> 3] >> (i & 7).astype(np.uint8)) & 1).astype(bool)


def _cell(col, i):
    """Row i's value as a Python object: UTF-8 text between offsets[i] and offsets[i + 1], or the fixed-width cell
    read as its Spark type (BOOLEAN a byte, DECIMAL the unscaled long / 10^scale)."""
    t = col.spark_type
    vals = _host_buffer(col, "values")
    if t == T_STRING:
        off = _host_buffer(col, "offsets")
        a, b = int(off[i]), int(off[i + 1])
        return bytes(np.asarray(vals, dtype=np.uint8)[a:b]).decode("utf-8")
    width = {T_BOOLEAN: 1, T_BYTE: 1, T_SHORT: 2, T_INT: 4, T_DATE: 4, T_FLOAT: 4}.get(t, 8)
    raw = np.asarray(vals).view(np.uint8)[i * width:(i + 1) * width].tobytes()
    if t == T_BOOLEAN:
        return raw != b"\x00"
    if t == T_FLOAT:
        return float(np.frombuffer(raw, dtype="<f4")[0])
    if t == T_DOUBLE:
        return float(np.frombuffer(raw, dtype="<f8")[0])
    x = int.from_bytes(raw, "little", signed=True)
    return x / (10 ** col.decimal_scale) if t == T_DECIMAL else x


_LE = {T_BYTE: "<i1", T_SHORT: "<i2", T_INT: "<i4", T_DATE: "<i4", T_FLOAT: "<f4", T_DOUBLE: "<f8"}


def _pylist(col):
    """Every row's cell (None for NULL), the column decoded once: the same reading as _cell, vectorised."""
    if col in _CELLS:
        return _CELLS[col]
    valid = _valid(col)
    n = col.length
    t = col.spark_type
    vals = _host_buffer(col, "values")
    if t == T_STRING:
        off = [int(x) for x in np.asarray(_host_buffer(col, "offsets"))[:n + 1]]
        data = bytes(np.asarray(vals, dtype=np.uint8)[:off[-1] if n else 0])
        cells = [data[off[i]:off[i + 1]].decode("utf-8") if valid[i] else None for i in range(n)]
    else:
        width = {T_BOOLEAN: 1, T_BYTE: 1, T_SHORT: 2, T_INT: 4, T_DATE: 4, T_FLOAT: 4}.get(t, 8)
        raw = np.asarray(vals).view(np.uint8)[:n * width].tobytes()
        if t == T_BOOLEAN:
            xs = [b != 0 for b in raw]
        else:
            xs = np.frombuffer(raw, dtype=_LE.get(t, "<i8")).tolist()
            if t == T_DECIMAL:
                xs = [x / (10 ** col.decimal_scale) for x in xs]
        cells = [x if valid[i] else None for i, x in enumerate(xs)]
    try:
        _CELLS[col] = cells
    except TypeError:  # a column type that cannot be weakly referenced: no memo
        pass
    return cells


# ---- expected states per analyzer ---------------------------------------------------------------


def _where(table, where):
    if where is None:
        return np.ones(table.nrows, dtype=bool), np.ones(table.nrows, dtype=bool)
    return predicate_masks(table, where)


def _cond_count(table, where):
    """conditionalCount (A/Analyzer.scala:426-432): (value, present)."""
    if where is None:
        return table.nrows, True
    t, nn = _where(table, where)
    return int(t.sum()), bool(nn.any())


def column_stats(table, column, where=None):
    c = table[column]
    wt, _ = _where(table, where)
    mask = (_valid(c) & wt).astype(np.uint8)
    out = OracleCol()
    vals = np.ascontiguousarray(c.values)
    lib().oracle_column(c.spark_type, c.decimal_scale, vals.ctypes.data, mask.ctypes.data, c.length,
                        ctypes.byref(out))
    return out


def expected_state(table, analyzer, exact=True):
    """The reference State for `analyzer` on `table` (None = empty state), oracle semantics."""
    S = sys.modules[__name__]  # this module's own State classes (not deequ_amd's)
    name = type(analyzer).__name__
    if name == "Size":
        v, present = _cond_count(table, analyzer.where)
        return S.NumMatches(v) if present else None
    if name == "Completeness":
        c = table[analyzer.column]
        wt, _ = _where(table, analyzer.where)
        cnt, present = _cond_count(table, analyzer.where)
        if table.nrows == 0 or not present:
            return None
        return S.NumMatchesAndCount(int((_valid(c) & wt).sum()), cnt)
    if name == "Compliance":
        wt, _ = _where(table, analyzer.where)
        pt, pnn = predicate_masks(table, analyzer.predicate)
        cnt, present = _cond_count(table, analyzer.where)
        if not (wt & pnn).any() or not present:
            return None
        return S.NumMatchesAndCount(int((wt & pt).sum()), cnt)
    if name in ("Mean", "Sum", "Minimum", "Maximum", "StandardDeviation"):
        c = table[analyzer.column]
        st = column_stats(table, analyzer.column, analyzer.where)
        if st.n == 0:
            return None
        frac = c.spark_type in (T_FLOAT, T_DOUBLE)
        scale = 10.0 ** c.decimal_scale if c.spark_type == T_DECIMAL else 1.0
        total = st.dsum if frac else st.isum / scale
        if name == "Mean":
            return S.MeanState(total, st.n)
        if name == "Sum":
            return S.SumState(total)
        if name == "Minimum":
            return S.MinState(st.dmin if frac else st.imin / scale)
        if name == "Maximum":
            return S.MaxState(st.dmax if frac else st.imax / scale)
        if exact:
            return S.StandardDeviationState(float(st.n), st.ex_mean, st.ex_m2)
        return S.StandardDeviationState(st.w_n, st.w_avg, st.w_m2)
    if name == "Correlation":
        x, y = table[analyzer.firstColumn], table[analyzer.secondColumn]
        wt, _ = _where(table, analyzer.where)
        mask = (_valid(x) & _valid(y) & wt).astype(np.uint8)
        out = OracleCorr()
        xv, yv = np.ascontiguousarray(x.values), np.ascontiguousarray(y.values)
        lib().oracle_correlation(x.spark_type, x.decimal_scale, xv.ctypes.data, y.spark_type, y.decimal_scale,
                                 yv.ctypes.data, mask.ctypes.data, x.length, ctypes.byref(out))
        if out.n == 0:
            return None
        if exact:
            return S.CorrelationState(out.n, out.x_avg, out.y_avg, out.ex_ck, out.ex_x_mk, out.ex_y_mk)
        return S.CorrelationState(out.n, out.x_avg, out.y_avg, out.ck, out.x_mk, out.y_mk)
    if name == "ApproxCountDistinct":
        c = table[analyzer.column]
        wt, _ = _where(table, analyzer.where)
        mask = (_valid(c) & wt).astype(np.uint8)
        regs = np.zeros(512, dtype=np.uint8)
        if c.spark_type == T_STRING:
            lib().oracle_hll_strings(c.values.ctypes.data if len(c.values) else None, c.offsets.ctypes.data,
                                     mask.ctypes.data, c.length, regs.ctypes.data)
        else:
            vals = np.ascontiguousarray(c.values)
            lib().oracle_hll_fixed(c.spark_type, vals.ctypes.data, mask.ctypes.data, c.length, regs.ctypes.data)
        words = np.zeros(52, dtype=np.int64)
        lib().oracle_hll_pack(regs.ctypes.data, words.ctypes.data)
        return S.ApproxCountDistinctState([int(w) for w in words])
    if name == "PatternMatch":
        # sum(when(regexp_extract(col, p, 0) != "", 1).otherwise(0)) under where (A/PatternMatch.scala:46-48):
        # the third-party `regex` module (2026.7.19, V1 syntax) is, like java.util.regex, a leftmost-first
        # backtracking engine with atomic groups, possessive quantifiers, lookbehind, named groups, nested sets
        # and `&&` intersections; regex.ASCII gives Java's default \d \s \w classes and ASCII-only
        # CASE_INSENSITIVE (Java's Unicode \b, `.` and `$` line terminators differ only on non-ASCII word
        # characters / \r, \u0085, \u2028, \u2029, absent from the tests).
        c = table[analyzer.column]
        rx = compile_java_regex(analyzer.pattern)
        wt, _ = _where(table, analyzer.where)
        valid = _valid(c)
        cnt, present = _cond_count(table, analyzer.where)
        hits = 0
        for i in range(c.length):
            if wt[i] and valid[i]:
                m = rx.search(spark_cast_to_string(c, i))
                hits += 1 if (m is not None and m.group(0) != "") else 0
        if not wt.any() or not present:
            return None
        return S.NumMatchesAndCount(hits, cnt)
    if name in ("MinLength", "MaxLength"):
        # min/max(length(when(where, col))): Spark's length = characters (A/MinLength.scala:28-30)
        c = table[analyzer.column]
        wt, _ = _where(table, analyzer.where)
        m = _valid(c) & wt
        lens = [len(_cell(c, i)) for i in range(c.length) if m[i]]
        if not lens:
            return None
        return S.MinState(float(min(lens))) if name == "MinLength" else S.MaxState(float(max(lens)))
    if name == "DataType":
        # StatefulDataType.update over the value cast to string (C/StatefulDataType.scala:58-69),
        # NULL for rows outside `where` (conditionalSelection, A/DataType.scala:146-148)
        c = table[analyzer.column]
        wt, _ = _where(table, analyzer.where)
        m = _valid(c) & wt
        counts = [0, 0, 0, 0, 0]
        for i in range(c.length):
            if not m[i]:
                counts[0] += 1
                continue
            counts[datatype_class(spark_cast_to_string(c, i))] += 1
        return S.DataTypeHistogram(*counts)
    raise ValueError("no oracle for %s" % name)


_POSIX_ORACLE = {  # java.util.regex.Pattern's US-ASCII POSIX classes, as set contents
    "Lower": "a-z", "Upper": "A-Z", "ASCII": "\\x00-\\x7f", "Alpha": "a-zA-Z", "Digit": "0-9", "Alnum": "a-zA-Z0-9",
    "Punct": "!-/:-@\\[-`{-~", "Graph": "!-~", "Print": " -~", "Blank": " \\t", "Cntrl": "\\x00-\\x1f\\x7f",
    "XDigit": "0-9a-fA-F", "Space": " \\t\\n\\x0b\\f\\r",
}
_JAVA_PROPS_ORACLE = {"javaLowerCase": "Ll", "javaUpperCase": "Lu", "javaLetter": "L", "javaDigit": "Nd",
                      "javaAlphabetic": "Alphabetic", "IsAlphabetic": "Alphabetic", "IsLetter": "L",
                      "IsDigit": "Nd", "IsLowercase": "Ll", "IsUppercase": "Lu", "IsPunctuation": "P",
                      "IsControl": "Cc", "IsWhite_Space": "White_Space"}


def java_regex_to_python(p):
    """A java.util.regex pattern in the `regex` module's V1 syntax: the spellings that differ are rewritten —
    \\z -> \\Z, \\Z -> (?=\\n?\\Z), POSIX \\p{Lower}..\\p{Space} -> their US-ASCII sets, java* / Is* properties ->
    Unicode property names, \\h \\v \\R \\e \\cX \\x{..} \\0oo -> explicit forms, \\Q..\\E -> escaped text, the
    Java-only flags d / u dropped (inputs hold no \\r and no non-ASCII letters), and a MULTILINE ^ never matching at
    the end of input (Java's Caret)."""
    import regex
    out, i, depth = [], 0, 0
    multiline = False
    while i < len(p):
        ch = p[i]
        if ch == "\\" and i + 1 < len(p):
            nxt = p[i + 1]
            if nxt == "z":
                out.append("\\Z")
            elif nxt == "Z":
                out.append("(?=\\n?\\Z)")
            elif nxt in "pP":
                if i + 2 < len(p) and p[i + 2] == "{":
                    j = p.index("}", i)
                    name = p[i + 3:j]
                else:
                    j, name = i + 2, p[i + 2]
                neg = nxt == "P"
                if name.startswith("^"):
                    neg, name = not neg, name[1:]
                if name in _POSIX_ORACLE:
                    body = _POSIX_ORACLE[name]
                    out.append(("[^%s]" if neg else "[%s]") % body if depth == 0 else
                               ("[^%s]" % body if neg else body))
                else:
                    name = _JAVA_PROPS_ORACLE.get(name, name)
                    for prefix in ("general_category=", "gc=", "Is"):
                        if name.startswith(prefix):
                            name = name[len(prefix):]
                    out.append("\\%s{%s}" % ("P" if neg else "p", name))
                i = j + 1
                continue
            elif nxt == "h":
                out.append("[ \\t\\xa0\\u1680\\u180e\\u2000-\\u200a\\u202f\\u205f\\u3000]" if depth == 0 else
                           " \\t\\xa0\\u1680\\u180e\\u2000-\\u200a\\u202f\\u205f\\u3000")
            elif nxt == "v":
                out.append("[\\n\\x0b\\f\\r\\x85\\u2028\\u2029]" if depth == 0 else "\\n\\x0b\\f\\r\\x85\\u2028\\u2029")
            elif nxt == "R":
                out.append("(?>\\r\\n|[\\n\\x0b\\f\\r\\x85\\u2028\\u2029])")
            elif nxt == "k":
                j = p.index(">", i)
                out.append("(?P=%s)" % p[i + 3:j])
                i = j + 1
                continue
            elif nxt == "e":
                out.append("\\x1b")
            elif nxt == "c":
                out.append("\\x%02x" % (ord(p[i + 2]) ^ 64))
                i += 3
                continue
            elif nxt == "x" and i + 2 < len(p) and p[i + 2] == "{":
                j = p.index("}", i)
                out.append("\\U%08x" % int(p[i + 3:j], 16))
                i = j + 1
                continue
            elif nxt == "0":
                j = i + 2
                while j < len(p) and j < i + 5 and p[j] in "01234567" and int(p[i + 2:j + 1], 8) <= 0o377:
                    j += 1
                out.append("\\x%02x" % int(p[i + 2:j], 8))
                i = j
                continue
            elif nxt == "Q":
                j = p.find("\\E", i + 2)
                lit = p[i + 2:] if j < 0 else p[i + 2:j]
                out.append(regex.escape(lit, special_only=False) if depth == 0 else
                           "".join("\\" + c if not c.isalnum() else c for c in lit))
                i = len(p) if j < 0 else j + 2
                continue
            else:
                out.append(p[i:i + 2])
            i += 2
            continue
        if ch == "[":
            depth += 1
        elif ch == "]" and depth > 0 and not (out and out[-1] in ("[", "[^")):
            depth -= 1
        elif ch == "(" and p[i + 1:i + 2] == "?" and depth == 0:
            j = i + 2
            flags = ""
            while j < len(p) and (p[j].isalpha() or p[j] == "-"):
                flags += p[j]
                j += 1
            if flags and j < len(p) and p[j] in ":)":
                if "m" in flags.split("-")[0]:
                    multiline = True
                kept = "".join(c for c in flags if c not in "du")
                if kept.strip("-") == "":
                    out.append("(?:" if p[j] == ":" else "")
                    if p[j] == ")":
                        i = j + 1
                        continue
                    i = j + 1
                    continue
                out.append("(?" + kept.rstrip("-") + p[j])
                i = j + 1
                continue
        elif ch == "^" and depth == 0 and multiline:
            out.append("(?:^(?!\\Z))")
            i += 1
            continue
        out.append("[" if ch == "[" and depth == 1 and (i + 1 >= len(p) or p[i + 1] != "^") else ch)
        i += 1
    return "".join(out)


def compile_java_regex(pattern):
    """The oracle's compiled form of a java.util.regex pattern (`regex` module, V1, ASCII classes)."""
    import regex
    return regex.compile(java_regex_to_python(pattern), regex.ASCII | regex.V1)


# StatefulDataType's regexes (C/StatefulDataType.scala:36-38), ASCII \d as in java.util.regex
_FRACTIONAL = __import__("re").compile(r"^(-|\+)? ?[0-9]*\.[0-9]*$")
_INTEGRAL = __import__("re").compile(r"^(-|\+)? ?[0-9]*$")
_BOOLEAN = __import__("re").compile(r"^(true|false)$")


def datatype_class(text):
    """1 Fractional, 2 Integral, 3 Boolean, 4 String; Regex.unapplySeq is a full match (`matches`)."""
    if _FRACTIONAL.fullmatch(text):
        return 1
    if _INTEGRAL.fullmatch(text):
        return 2
    if _BOOLEAN.fullmatch(text):
        return 3
    return 4


def java_double_to_string(d, is_float=False):
    """java.lang.Double/Float.toString: shortest round-trip digits (Python repr), plain notation for
    1e-3 <= |d| < 1e7, otherwise d.dddE<exp>; "NaN", "Infinity"."""
    if d != d:
        return "NaN"
    if d in (float("inf"), float("-inf")):
        return "Infinity" if d > 0 else "-Infinity"
    if d == 0.0:
        return "-0.0" if math.copysign(1.0, d) < 0 else "0.0"
    r = str(np.float32(d)) if is_float else repr(float(d))  # shortest round-trip digits of the float / double
    sign = "-" if r.startswith("-") else ""
    r = r.lstrip("-")
    mant, _, exp = r.partition("e")
    digits = mant.replace(".", "")
    point = mant.index(".") if "." in mant else len(mant)
    e10 = (int(exp) if exp else 0) + point  # value = 0.digits * 10^e10
    lead = len(digits) - len(digits.lstrip("0"))
    digits = digits.strip("0") or "0"
    e10 -= lead
    thr = np.float32(1e-3) if is_float else 1e-3
    if thr <= abs(d) < 1e7:
        if e10 <= 0:
            return sign + "0." + "0" * (-e10) + digits
        if e10 >= len(digits):
            return sign + digits + "0" * (e10 - len(digits)) + ".0"
        return sign + digits[:e10] + "." + digits[e10:]
    frac = digits[1:] or "0"
    return "%s%s.%sE%d" % (sign, digits[0], frac, e10 - 1)


def spark_cast_to_string(col, i):
    """Cast(value AS STRING) for row i (Spark 2.2: Java toString of the boxed value, BigDecimal.toString)."""
    from decimal import Decimal
    t = col.spark_type
    if t == T_STRING:
        return _cell(col, i)
    v = col.values[i]
    if t == T_BOOLEAN:
        return "true" if v else "false"
    if t in (T_BYTE, T_SHORT, T_INT, T_LONG):
        return str(int(v))
    if t == T_DOUBLE:
        return java_double_to_string(float(v))
    if t == T_FLOAT:
        return java_double_to_string(float(v), is_float=True)
    if t == T_DECIMAL:
        return java_bigdecimal_to_string(int(v), col.decimal_scale)
    if t == T_DATE:
        return java_date_to_string(int(v))
    return java_timestamp_to_string_utc(int(v))


def _java_civil(days):
    """(year of era, month, day) of a day number (days since 1970-01-01) in java.util.GregorianCalendar's hybrid
    calendar, the one java.text.SimpleDateFormat prints with: Gregorian from 1582-10-15, Julian before (Java's
    published cutover; restated with Python's proleptic-Gregorian date arithmetic and the Julian leap rule, not
    with the device's day-number formulas)."""
    import datetime
    if days >= -141427:  # 1582-10-15 and later: Gregorian
        shift = 0
        if days > 2932896:  # past 9999-12-31 (Python's date range): whole 400-year Gregorian cycles of 146097 days
            shift = (days - 2932896) // 146097 + 1
        d = datetime.date(1970, 1, 1) + datetime.timedelta(days=days - 146097 * shift)
        return d.year + 400 * shift, d.month, d.day
    # Julian calendar: whole 4-year cycles of 1461 days counted from Julian 0001-01-01 (day -719164), then the year
    # inside the cycle (the fourth year is the leap year) and the month from cumulative month lengths
    off = days + 719164
    cycles, rem = divmod(off, 1461)
    yin = min(rem // 365, 3)
    y = 1 + 4 * cycles + yin
    doy = rem - 365 * yin
    leap = y % 4 == 0
    m = 1
    for ml in (31, 29 if leap else 28, 31, 30, 31, 30, 31, 31, 30, 31, 30, 31):
        if doy < ml:
            break
        doy -= ml
        m += 1
    return (y if y >= 1 else 1 - y), m, doy + 1


def java_date_to_string(days):
    """Spark 2.2 Cast(date AS STRING) = DateTimeUtils.dateToString: SimpleDateFormat("yyyy-MM-dd")."""
    y, m, d = _java_civil(days)
    return "%04d-%02d-%02d" % (y, m, d)


def java_timestamp_to_string_utc(micros):
    """Spark 2.2 Cast(timestamp AS STRING) = DateTimeUtils.timestampToString in a UTC session time zone:
    SimpleDateFormat("yyyy-MM-dd HH:mm:ss") of the floored second, plus java.sql.Timestamp.toString's fraction
    (nanoseconds with trailing zeros dropped) unless it is ".0". Other session time zones: parity unpinned."""
    secs, frac = divmod(micros, 1_000_000)
    days, sod = divmod(secs, 86400)
    out = "%s %02d:%02d:%02d" % (java_date_to_string(days), sod // 3600, sod // 60 % 60, sod % 60)
    if frac:
        out += "." + ("%06d" % frac).rstrip("0")
    return out


def java_bigdecimal_to_string(unscaled, scale):
    """java.math.BigDecimal.toString (scientific when scale < 0 or adjusted exponent < -6)."""
    neg = unscaled < 0
    digits = str(abs(unscaled))
    adjusted = len(digits) - 1 - scale
    if scale >= 0 and adjusted >= -6:
        if scale == 0:
            body = digits
        elif len(digits) > scale:
            body = digits[:-scale] + "." + digits[-scale:]
        else:
            body = "0." + "0" * (scale - len(digits)) + digits
    else:
        body = digits[0] + ("." + digits[1:] if len(digits) > 1 else "") + "E" + ("+" if adjusted > 0 else "") + str(adjusted)
    return ("-" if neg else "") + body


def frequencies(table, columns, include_nulls=False):
    """computeFrequencies: {key tuple: count} over rows with >= 1 non-null key (all rows if
    include_nulls, Histogram semantics), plus numRows."""
    cols = [_pylist(table[c]) for c in columns]
    freq = {}
    nrows = 0
    for i in range(table.nrows):
        key = tuple(_group_key(c[i]) for c in cols)
        if not include_nulls and all(k is None for k in key):
            continue
        nrows += 1
        freq[key] = freq.get(key, 0) + 1
    return freq, nrows


def _group_key(v):
    """Spark groups on binary equality: NaN canonical, -0.0 != 0.0."""
    if isinstance(v, float):
        fv = float(v)
        if math.isnan(fv):
            return ("nan",)
        if fv == 0.0 and math.copysign(1.0, fv) < 0:
            return ("-0.0",)
        return fv
    return v


def grouping_summary(freq, num_rows):
    counts = list(freq.values())
    ent = math.fsum(-(c / num_rows) * math.log(c / num_rows) for c in counts) if counts else 0.0
    return {"num_groups": len(counts), "num_unique": sum(1 for c in counts if c == 1), "entropy": ent,
            "num_rows": num_rows}


# ---- ApproxQuantile(s): exact order statistics (A/ApproxQuantile.scala:28-103) ----------------------
def java_sorted_doubles(table, column):
    """The column's non-NULL values cast to double (Spark's implicit DoubleType cast of the child,
    C/StatefulApproxQuantile.scala:50-52; Decimal.toDouble = unscaled / 10^scale for compact
    decimals), sorted in java.lang.Double.compare order (-0.0 < 0.0, NaN largest), which is the order
    of QuantileSummaries' `sortBy(_.value)`."""
    col = table[column]
    valid = _valid(col)
    v = np.asarray(col.values)[: col.length][valid]
    if col.spark_type == T_DECIMAL:
        d = v.astype(np.float64) / (10.0 ** col.decimal_scale) if col.decimal_scale else v.astype(np.float64)
    else:
        d = v.astype(np.float64)
    bits = d.view(np.uint64).copy()
    bits[np.isnan(d)] = np.uint64(0x7FF8000000000000)
    neg = (bits >> np.uint64(63)) == 1
    keys = np.where(neg, ~bits, bits | np.uint64(1 << 63))
    keys.sort()
    neg = (keys >> np.uint64(63)) == 0
    out = np.where(neg, ~keys, keys & np.uint64(0x7FFFFFFFFFFFFFFF))
    return out.view(np.float64)


def summary_ranks(n, relative_error):
    """Ranks of the zero-uncertainty summary dq_quantile_summary returns: 1, n and every
    max(1, floor(relativeError * n))-th rank in between."""
    if n == 0:
        return np.zeros(0, dtype=np.int64)
    s = max(1, int(math.floor(relative_error * n)))
    r = list(range(1, n + 1, s))
    if r[-1] != n:
        r.append(n)
    return np.array(r, dtype=np.int64)


def rank_interval(sorted_values, value):
    """1-based [lowest, highest] rank `value` occupies in the sorted (Java-ordered) values."""
    keys = _java_keys(sorted_values)
    k = _java_keys(np.array([value], dtype=np.float64))[0]
    lo = int(np.searchsorted(keys, k, side="left")) + 1
    hi = int(np.searchsorted(keys, k, side="right"))
    return lo, hi


def _java_keys(d):
    bits = np.asarray(d, dtype=np.float64).view(np.uint64).copy()
    bits[np.isnan(np.asarray(d, dtype=np.float64))] = np.uint64(0x7FF8000000000000)
    neg = (bits >> np.uint64(63)) == 1
    return np.where(neg, ~bits, bits | np.uint64(1 << 63))


# ---- KLLSketch (A/KLLSketch.scala, A/QuantileNonSample.scala, A/NonSampleCompactor.scala,
#      R/KLLRunner.scala) ---------------------------------------------------------------------------

def _java_total_order(a):
    """uint64 keys ordering float64 like java.lang.Double.compare (-0.0 < 0.0, NaN largest)."""
    a = np.asarray(a, dtype=np.float64).copy()
    a[np.isnan(a)] = np.nan  # canonical NaN
    b = a.view(np.uint64)
    neg = (b >> np.uint64(63)).astype(bool)
    return np.where(neg, ~b, b | np.uint64(1 << 63))


def _kll_capacity(sketch_size, shrinking_factor, height):
    """QuantileNonSample.capacity (A/QuantileNonSample.scala:87-89)."""
    return 2 * (int(math.ceil(sketch_size * math.pow(shrinking_factor, height) / 2)) + 1)


def kll_sketch_sequential(values, sketch_size=2048, shrinking_factor=0.64):
    """The sketch of one partition whose items arrive in `values` order: QuantileNonSample.update /
    condense / expand (A/QuantileNonSample.scala:80-121) with NonSampleCompactor.compact
    (A/NonSampleCompactor.scala:40-66; the Random offset is commented out in the reference, so the
    offset flips deterministically after every odd-numbered compaction). Returns a dict with the
    serializer fields (A/catalyst/KLLSketchSerializer.scala:60-80)."""
    cap = lambda h: _kll_capacity(sketch_size, shrinking_factor, h)
    bufs, ncomp, offs = [[]], [0], [0]
    total = cap(0)
    actual = 0
    for v in values:
        bufs[0].append(float(v))
        actual += 1
        if actual > total:
            for h in range(len(bufs)):
                if len(bufs[h]) >= cap(h):
                    if h + 1 >= len(bufs):
                        bufs.append([]); ncomp.append(0); offs.append(0)
                        total = sum(cap(i) for i in range(len(bufs)))
                    items = len(bufs[h])
                    ln = items - items % 2
                    if ncomp[h] % 2 == 1:
                        offs[h] = 1 - offs[h]
                    part = np.asarray(bufs[h][:ln], dtype=np.float64)
                    srt = part[np.argsort(_java_total_order(part), kind="stable")]
                    bufs[h + 1].extend(srt[offs[h]:ln:2].tolist())
                    bufs[h] = [bufs[h][items - 1]] if items % 2 else []
                    ncomp[h] += 1
                    actual = sum(len(b) for b in bufs)
                    break
    return {"sketchSize": sketch_size, "shrinkingFactor": shrinking_factor, "curNumOfCompactors": len(bufs),
            "compactorActualSize": actual, "compactorTotalSize": total,
            "compactors": [(ncomp[h], offs[h], bufs[h]) for h in range(len(bufs))]}


def kll_runner_min_max(values):
    """UntypedQuantileNonSample min/max (R/KLLRunner.scala:27-36): math.min / math.max folds starting
    from Int.MaxValue.toDouble / Int.MinValue.toDouble (NaN-propagating, -0.0 < 0.0)."""
    lo, hi = 2147483647.0, -2147483648.0
    for v in values:
        v = float(v)
        if v != v or lo != lo:
            lo = float("nan")
        elif v < lo or (v == lo == 0.0 and math.copysign(1.0, v) < 0):
            lo = v
        if v != v or hi != hi:
            hi = float("nan")
        elif v > hi or (v == hi == 0.0 and math.copysign(1.0, v) > 0):
            hi = v
    return lo, hi


def kll_state_bytes(values, sketch_size=2048, shrinking_factor=0.64):
    """KLLState bytes for one partition (A/KLLSketch.scala:56-66 read order: min, max, sketch)."""
    import struct
    sk = kll_sketch_sequential(values, sketch_size, shrinking_factor)
    lo, hi = kll_runner_min_max(values)
    out = [struct.pack(">dd", lo, hi),
           struct.pack(">idiiii", sk["sketchSize"], sk["shrinkingFactor"], sk["curNumOfCompactors"],
                       sk["compactorActualSize"], sk["compactorTotalSize"], len(sk["compactors"]))]
    for nc, off, buf in sk["compactors"]:
        out.append(struct.pack(">iii", nc, off, len(buf)))
        out.append(struct.pack(">%dd" % len(buf), *buf))
    return b"".join(out)


# ---- Spark 2.2 string -> number casts (ColumnProfiler.castColumn, M/profiles/ColumnProfiler.scala:346-355) --

def spark_string_to_long(s):
    """UTF8String.toLong (spark-unsafe 2.2.2, third-party): no trimming, optional sign, digits, an optional
    '.' followed by digits only (truncated), overflow -> None."""
    b = s.encode("utf-8")
    if not b:
        return None
    neg = b[0:1] == b"-"
    i = 1 if b[0:1] in (b"-", b"+") else 0
    if i == 1 and len(b) == 1:
        return None
    digits = []
    while i < len(b):
        c = b[i]
        i += 1
        if c == ord("."):
            break
        if not 48 <= c <= 57:
            return None
        digits.append(c - 48)
    while i < len(b):
        if not 48 <= b[i] <= 57:
            return None
        i += 1
    v = 0
    for d in digits:
        v = v * 10 + d
    v = -v if neg else v
    if not -(1 << 63) <= v < (1 << 63):
        return None
    return v


_JAVA_DOUBLE = None


def java_parse_double(s):
    """java.lang.Double.parseDouble for decimal literals (String.trim of chars <= ' ', optional sign,
    NaN / Infinity, digits with an optional point, optional exponent, optional f/F/d/D suffix); the value
    is Python's correctly rounded float() of the same digits. Returns None where Java throws."""
    import re
    global _JAVA_DOUBLE
    if _JAVA_DOUBLE is None:
        _JAVA_DOUBLE = re.compile(r"([+-]?)(NaN|Infinity|(?:[0-9]+\.?[0-9]*|\.[0-9]+)(?:[eE][+-]?[0-9]+)?)[fFdD]?\Z")
    t = s
    i, j = 0, len(t)
    while i < j and ord(t[i]) <= 32:
        i += 1
    while j > i and ord(t[j - 1]) <= 32:
        j -= 1
    m = _JAVA_DOUBLE.match(t[i:j])
    if not m:
        return None
    body = m.group(2)
    if body == "NaN":
        return float("nan")
    v = float("inf") if body == "Infinity" else float(body)
    return -v if m.group(1) == "-" else v


# ---- ColumnProfiler passes 1-3 (M/profiles/ColumnProfiler.scala:91-208, 357-606) --------------------
def determine_type(counts):
    """DataTypeHistogram.determineType (A/DataType.scala:116-143) over class counts
    {Unknown, Fractional, Integral, Boolean, String}."""
    total = sum(counts.values())
    ratio = {k: (v / total if total else 0.0) for k, v in counts.items()}
    if ratio["Unknown"] == 1.0:
        return "Unknown"
    if ratio["String"] > 0.0 or (ratio["Boolean"] > 0.0 and (ratio["Integral"] > 0.0 or ratio["Fractional"] > 0.0)):
        return "String"
    if ratio["Boolean"] > 0.0:
        return "Boolean"
    if ratio["Fractional"] > 0.0:
        return "Fractional"
    return "Integral"


_KNOWN = {T_SHORT: "Integral", T_INT: "Integral", T_LONG: "Integral", T_FLOAT: "Fractional", T_DOUBLE: "Fractional",
          T_DECIMAL: "Fractional", T_BOOLEAN: "Boolean", T_TIMESTAMP: "String"}
_HIST_TYPES = (T_STRING, T_BOOLEAN, T_DOUBLE, T_FLOAT, T_INT, T_LONG, T_SHORT)


def _hll_words_of(table, name):
    c = table[name]
    mask = _valid(c).astype(np.uint8)
    regs = np.zeros(512, dtype=np.uint8)
    if c.spark_type == T_STRING:
        lib().oracle_hll_strings(c.values.ctypes.data if len(c.values) else None, c.offsets.ctypes.data,
                                 mask.ctypes.data, c.length, regs.ctypes.data)
    else:
        vals = np.ascontiguousarray(c.values)
        lib().oracle_hll_fixed(c.spark_type, vals.ctypes.data, mask.ctypes.data, c.length, regs.ctypes.data)
    words = np.zeros(52, dtype=np.int64)
    lib().oracle_hll_pack(regs.ctypes.data, words.ctypes.data)
    return words


def _exact_stats(values):
    """count, sum, min, max, mean, population stddev of a 1-D float array; sums in long double."""
    n = len(values)
    if n == 0:
        return None
    ld = values.astype(np.longdouble)
    s = ld.sum()
    mean = s / n
    m2 = ((ld - mean) ** 2).sum()
    return {"n": n, "sum": float(s), "min": float(values.min()), "max": float(values.max()), "mean": float(mean),
            "stdDev": float(np.sqrt(m2 / n))}


def expected_profile(table, threshold=120):
    """Per column: completeness, approximateNumDistinctValues (HLL++ of the C oracle), dataType,
    isDataTypeInferred, typeCounts (StatefulDataType classes of Cast(x AS STRING)), pass-2 numeric
    statistics over the column cast as ColumnProfiler.castColumn does (Spark string -> long / double
    casts, non-parsing strings NULL), and the exact pass-3 histogram (counts; NULL as "NullValue") of
    columns whose approximate distinct count is <= threshold."""
    n = table.nrows
    out = {}
    for name in table.columns:
        c = table[name]
        valid = _valid(c)
        p = {"completeness": int(valid.sum()) / n}
        p["approx_distinct"] = int(hll_count([int(w) for w in _hll_words_of(table, name)]))
        if c.spark_type == T_STRING:
            py = _pylist(c)
            cache, counts = {}, {"Unknown": 0, "Fractional": 0, "Integral": 0, "Boolean": 0, "String": 0}
            names = {1: "Fractional", 2: "Integral", 3: "Boolean", 4: "String"}
            for v in py:
                if v is None:
                    counts["Unknown"] += 1
                    continue
                k = cache.get(v)
                if k is None:
                    k = cache[v] = names[datatype_class(v)]
                counts[k] += 1
            p["typeCounts"] = counts
            p["dataType"] = determine_type(counts)
            p["inferred"] = True
        else:
            p["typeCounts"] = {}
            p["dataType"] = _KNOWN.get(c.spark_type, "Unknown")
            p["inferred"] = False
        if p["dataType"] in ("Integral", "Fractional"):
            if c.spark_type == T_STRING:
                conv = spark_string_to_long if p["dataType"] == "Integral" else java_parse_double
                cache, vals = {}, []
                for v in _pylist(c):
                    if v is None:
                        continue
                    if v not in cache:
                        cache[v] = conv(v)
                    if cache[v] is not None:
                        vals.append(cache[v])
                arr = np.array(vals, dtype=np.int64 if p["dataType"] == "Integral" else np.float64)
            else:
                arr = np.asarray(c.values)[: c.length][valid]
            st = _exact_stats(arr.astype(np.float64))
            if st is not None and p["dataType"] == "Integral":
                # Spark's Long sum wraps around, then is cast to Double (A/Sum.scala:34-37, A/Mean.scala:36-40)
                with np.errstate(over="ignore"):
                    st["sum"] = float(int(arr.astype(np.int64).sum(dtype=np.int64)))
                st["mean"] = st["sum"] / st["n"]
                st["min"], st["max"] = float(int(arr.min())), float(int(arr.max()))
            p["numeric"] = st
        if c.spark_type in _HIST_TYPES and p["dataType"] in ("String", "Boolean", "Integral", "Fractional") and \
                p["approx_distinct"] <= threshold:
            freq, _ = frequencies(table, [name], include_nulls=True)
            hist = {}
            for (k,), cnt in freq.items():
                if k is None:
                    key = "NullValue"
                elif c.spark_type == T_STRING:
                    key = k
                elif c.spark_type == T_BOOLEAN:
                    key = "true" if k else "false"
                elif c.spark_type in (T_DOUBLE, T_FLOAT):
                    key = java_double_to_string(float("nan") if isinstance(k, tuple) and k[0] == "nan" else
                                                (-0.0 if isinstance(k, tuple) else k), c.spark_type == T_FLOAT)
                else:
                    key = str(int(k))
                hist[key] = cnt
            p["histogram"] = hist
        else:
            p["histogram"] = None
        out[name] = p
    return out
