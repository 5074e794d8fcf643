"""ctypes binding of libdq.so (include/dq.h) — the same C-ABI a JVM host binds over JNI.

The library is loaded from the package directory (built in-tree by __graft_entry__.build()).
There is no CPU fallback: if the library or a GPU is missing, operations raise.
"""
import ctypes
import sys
import os
import threading

import numpy as np

# Hardware queues per process. A run drives up to ~7 streams at once (the main context, helper contexts for the
# second row chunk, the early KLL pass, the pass-3 histograms, the groupings and AnalysisRunBuilder.runAsync, plus
# torch's); with HIP's default of 4 queues, streams share a queue and one stream's kernels wait behind another's (the
# C5 step's histograms queued ~60 ms behind the text grouping). Read by the HIP runtime when it initialises (the first
# HIP call of the process): set here, before that, unless the user set it. C5 step: 4 queues 159-173 ms, 8 queues
# 143-145 ms (profiles/r06/c5_hw_queues_ab_r06v.txt).
os.environ.setdefault("GPU_MAX_HW_QUEUES", "8")

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("DQ_LIBRARY") or os.path.join(_HERE, "libdq.so")

# ---- constants mirrored from include/dq.h -------------------------------------------------------
DQ_OK = 0
STATUS_NAMES = {0: "DQ_OK", -1: "DQ_ERR_INVALID_ARGUMENT", -2: "DQ_ERR_UNSUPPORTED", -3: "DQ_ERR_DEVICE",
                -4: "DQ_ERR_OUT_OF_MEMORY", -5: "DQ_ERR_NO_DEVICE", -6: "DQ_ERR_PREDICATE",
                -7: "DQ_ERR_ALIGNMENT"}

TYPE_BOOLEAN, TYPE_BYTE, TYPE_SHORT, TYPE_INT, TYPE_LONG, TYPE_FLOAT, TYPE_DOUBLE, TYPE_STRING, \
    TYPE_DATE, TYPE_TIMESTAMP, TYPE_DECIMAL = range(1, 12)

COL_DEVICE = 0x1
COL_OFFSETS64 = 0x2  # STRING: int64 offsets (dq_frequencies only)
SCAN_OUT_DEVICE = 0x1
FREQ_INCLUDE_NULLS = 0x1
FREQ_KEYS_VALUES, FREQ_KEYS_ROWS = 0, 1
FREQ_PAIRS_DEVICE = 0x1

OP_SIZE, OP_COMPLETENESS, OP_COMPLIANCE, OP_MEAN, OP_SUM, OP_MINIMUM, OP_MAXIMUM, OP_STANDARD_DEVIATION, \
    OP_CORRELATION, OP_APPROX_COUNT_DISTINCT, OP_MIN_LENGTH, OP_MAX_LENGTH, OP_DATATYPE = range(1, 14)

# predicate opcodes
P_COL, P_CONST, P_NULL = 1, 2, 3
P_EQ, P_NE, P_LT, P_LE, P_GT, P_GE, P_EQ_NULLSAFE = 10, 11, 12, 13, 14, 15, 16
P_AND, P_OR, P_NOT, P_IS_NULL, P_IS_NOT_NULL, P_IN, P_COALESCE = 20, 21, 22, 23, 24, 25, 26
P_ADD, P_SUB, P_MUL, P_DIV, P_MOD, P_NEG = 30, 31, 32, 33, 34, 35
P_LIKE, P_LENGTH, P_CAST_DOUBLE, P_CAST_LONG, P_CAST_STRING_NUM, P_REGEX = 40, 41, 42, 43, 44, 45
P_RLIKE, P_LOWER, P_UPPER, P_TRIM, P_CASE, P_ISNAN, P_ABS, P_SUBSTR, P_YEAR, P_MONTH, P_DAY, P_NANVL = range(46, 58)
V_BOOL, V_LONG, V_DOUBLE, V_STRING = 1, 2, 3, 4

SYNTH_DYADIC, SYNTH_UNIFORM, SYNTH_NORMAL, SYNTH_INT32R, SYNTH_KEY30, SYNTH_GAUSS01, SYNTH_GAUSS_CORR = range(1, 8)
SYNTH_STR_CAT50, SYNTH_STR_BOOL, SYNTH_STR_CAT100, SYNTH_STR_INT, SYNTH_STR_DEC, SYNTH_STR_MIXNUM, SYNTH_STR_TEXT = \
    101, 102, 103, 104, 105, 106, 107

HLL_NUM_WORDS = 52

# dq_scan_kernel, in enum order
FREQ_PATHS = ("fast", "fast_narrow", "fast_done", "exact", "partitioned", "sorted", "small", "small_optimistic", "fast_spill",
              "split_buckets", "long_tuples")
SCAN_KERNELS = ("striped", "striped_heavy", "heavy8", "heavy8_full", "bits", "pred_simple", "pred_vm", "regex",
                "strings", "where_fused", "where_masks")

# Every symbol include/dq.h declares (checked by tests/test_native_abi.py).
EXPORTED_SYMBOLS = (
    "dq_abi_version", "dq_open", "dq_close", "dq_last_error", "dq_set_stream", "dq_synchronize", "dq_scan",
    "dq_scan_launch_count", "dq_state_merge", "dq_state_fold", "dq_hll_count", "dq_spark_hash64", "dq_frequencies",
    "dq_freq_summarize", "dq_freq_key_kind", "dq_freq_top", "dq_freq_export", "dq_freq_free", "dq_partition_keys",
    "dq_quantile_summary", "dq_quantile_summaries", "dq_kll_sketch", "dq_cast_column", "dq_synth_column", "dq_synth_freq_keys",
    "dq_synth_validity", "dq_frequencies_ex", "dq_freq_export_device", "dq_freq_from_pairs", "dq_freq_merge", "dq_freq_row_counts", "dq_synth_strings",
    "dq_freq_mutual_information", "dq_open_devices", "dq_ctx_num_devices", "dq_ctx_uses_rccl", "dq_scan_sharded",
    "dq_scan_streamed", "dq_scan_kernel_launches", "dq_freq_path_count", "dq_kll_sketch_columns",
    "dq_kll_merge_states", "dq_scratch_trim", "dq_frequencies_parts", "dq_set_priority",
)


class DqColumn(ctypes.Structure):
    _fields_ = [("spark_type", ctypes.c_int32), ("flags", ctypes.c_uint32), ("length", ctypes.c_int64),
                ("values", ctypes.c_void_p), ("validity", ctypes.c_void_p), ("offsets", ctypes.c_void_p),
                ("decimal_precision", ctypes.c_int32), ("decimal_scale", ctypes.c_int32)]


class DqConst(ctypes.Structure):
    _fields_ = [("tag", ctypes.c_int32), ("str_len", ctypes.c_int32), ("i64", ctypes.c_int64),
                ("f64", ctypes.c_double), ("str_offset", ctypes.c_int64)]


class DqPredicate(ctypes.Structure):
    _fields_ = [("code", ctypes.c_void_p), ("code_len", ctypes.c_int32), ("n_consts", ctypes.c_int32),
                ("consts", ctypes.c_void_p), ("strings", ctypes.c_void_p), ("strings_len", ctypes.c_int64)]


class DqOp(ctypes.Structure):
    _fields_ = [("kind", ctypes.c_int32), ("column", ctypes.c_int32 * 2), ("where", ctypes.c_int32),
                ("predicate", ctypes.c_int32)]


class _NumMatches(ctypes.Structure):
    _fields_ = [("num_matches", ctypes.c_int64)]


class _NumMatchesAndCount(ctypes.Structure):
    _fields_ = [("num_matches", ctypes.c_int64), ("count", ctypes.c_int64)]


class _Mean(ctypes.Structure):
    _fields_ = [("sum", ctypes.c_double), ("count", ctypes.c_int64), ("isum", ctypes.c_int64), ("exact", ctypes.c_int32),
                ("pad", ctypes.c_int32)]


class _Dbl(ctypes.Structure):
    _fields_ = [("value", ctypes.c_double), ("isum", ctypes.c_int64), ("exact", ctypes.c_int32), ("pad", ctypes.c_int32)]


class _StdDev(ctypes.Structure):
    _fields_ = [("n", ctypes.c_double), ("avg", ctypes.c_double), ("m2", ctypes.c_double)]


class _Corr(ctypes.Structure):
    _fields_ = [("n", ctypes.c_double), ("x_avg", ctypes.c_double), ("y_avg", ctypes.c_double),
                ("ck", ctypes.c_double), ("x_mk", ctypes.c_double), ("y_mk", ctypes.c_double)]


class _Hll(ctypes.Structure):
    _fields_ = [("words", ctypes.c_int64 * HLL_NUM_WORDS)]


class _DataType(ctypes.Structure):
    _fields_ = [("num_null", ctypes.c_int64), ("num_fractional", ctypes.c_int64), ("num_integral", ctypes.c_int64),
                ("num_boolean", ctypes.c_int64), ("num_string", ctypes.c_int64)]


class _StateUnion(ctypes.Union):
    _fields_ = [("num_matches", _NumMatches), ("num_matches_and_count", _NumMatchesAndCount), ("mean", _Mean),
                ("dbl", _Dbl), ("stddev", _StdDev), ("corr", _Corr), ("hll", _Hll), ("datatype", _DataType)]


class DqState(ctypes.Structure):
    _fields_ = [("kind", ctypes.c_int32), ("present", ctypes.c_int32), ("u", _StateUnion)]


class DqFreqSummary(ctypes.Structure):
    _fields_ = [("num_rows", ctypes.c_int64), ("num_groups", ctypes.c_int64), ("num_unique", ctypes.c_int64),
                ("entropy", ctypes.c_double), ("entropy_rows", ctypes.c_int64), ("max_count", ctypes.c_int64),
                ("null_count", ctypes.c_int64), ("entropy_fx_lo", ctypes.c_uint64), ("entropy_fx_hi", ctypes.c_int64)]


def fx_value(lo, hi):
    """The exact fixed-point entropy sum of a dq_freq_summary (2^-104 units) as a Python int."""
    return (int(hi) << 64) | int(lo)


def fx_of(t):
    """dq_common.h fx_of: a double rounded once to signed fixed point of 2^-104 units (round half up in magnitude)."""
    import struct
    u = struct.unpack("<Q", struct.pack("<d", float(t)))[0]
    e = (u >> 52) & 0x7FF
    m = (u & ((1 << 52) - 1)) | ((1 << 52) if e else 0)
    sh = (e if e else 1) - 1075 + 104
    if sh >= 0:
        v = m << min(sh, 74)
    elif sh > -64:
        v = (m + (1 << (-sh - 1))) >> -sh
    else:
        v = 0
    return -v if u >> 63 else v


def fx_to_float(v):
    """dq_common.h fx_to_double: one correctly rounded conversion (Python's int / float true division of an int by a
    power of two rounds correctly), then an exact scale."""
    return v / float(1 << 104) if abs(v) < (1 << 1000) else float("nan")


class DqFreqOptions(ctypes.Structure):
    _fields_ = [("flags", ctypes.c_uint32), ("weights_device", ctypes.c_uint32), ("weights", ctypes.c_void_p),
                ("key_type", ctypes.c_int32), ("pad", ctypes.c_int32)]


STATE_SIZE = ctypes.sizeof(DqState)


class NativeError(RuntimeError):
    """A failed libdq call (status code + dq_last_error message)."""

    def __init__(self, status, message):
        self.status = status
        super().__init__("%s: %s" % (STATUS_NAMES.get(status, status), message))


_lib = None
_lib_lock = threading.Lock()


def load_library(path=None):
    """Load libdq.so and declare its prototypes. Raises if the library was not built."""
    global _lib
    with _lib_lock:
        if _lib is not None and path is None:
            return _lib
        p = path or LIB_PATH
        if not os.path.exists(p):
            raise NativeError(-5, "libdq.so not found at %s: run __graft_entry__.build() (no CPU fallback exists)" % p)
        lib = ctypes.CDLL(p, mode=ctypes.RTLD_GLOBAL)
        c_void_p, c_int, c_int64, c_uint32 = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_uint32
        sig = {
            "dq_abi_version": (c_int, []),
            "dq_open": (c_void_p, [c_int, ctypes.POINTER(c_int)]),
            "dq_close": (None, [c_void_p]),
            "dq_last_error": (ctypes.c_char_p, [c_void_p]),
            "dq_set_stream": (c_int, [c_void_p, c_void_p]),
            "dq_synchronize": (c_int, [c_void_p]),
            "dq_scratch_trim": (None, [c_void_p, c_int64]),
            "dq_set_priority": (c_int, [c_void_p, c_int]),
            "dq_frequencies_parts": (c_int, [c_void_p, c_void_p, c_int, c_int, c_void_p, c_int, c_void_p, c_void_p]),
            "dq_scan": (c_int, [c_void_p, c_void_p, c_int, c_int64, c_void_p, c_int, c_void_p, c_int, c_void_p,
                                c_uint32]),
            "dq_scan_launch_count": (c_int64, [c_void_p]),
            "dq_scan_kernel_launches": (c_int64, [c_void_p, ctypes.c_int32]),
            "dq_freq_path_count": (c_int64, [c_void_p, ctypes.c_int32]),
            "dq_state_merge": (c_int, [c_void_p, c_void_p, c_void_p]),
            "dq_state_fold": (c_int, [c_void_p, c_int, c_int, c_void_p]),
            "dq_hll_count": (ctypes.c_double, [c_void_p]),
            "dq_spark_hash64": (c_int64, [ctypes.c_int32, c_void_p, c_int64]),
            "dq_frequencies": (c_int, [c_void_p, c_void_p, c_int, c_int64, c_void_p, c_int, c_uint32, c_void_p]),
            "dq_freq_summarize": (c_int, [c_void_p, c_void_p, c_int64, c_void_p]),
            "dq_freq_key_kind": (c_int, [c_void_p]),
            "dq_freq_top": (c_int64, [c_void_p, c_void_p, c_int64, c_void_p, c_void_p]),
            "dq_freq_export": (c_int64, [c_void_p, c_void_p, c_int64, c_void_p, c_void_p]),
            "dq_freq_free": (None, [c_void_p, c_void_p]),
            "dq_partition_keys": (c_int, [c_void_p, c_void_p, c_int64, c_int, c_void_p, c_void_p, c_void_p]),
            "dq_quantile_summary": (c_int64, [c_void_p, c_void_p, c_int64, ctypes.c_double, c_int64, c_void_p,
                                              c_void_p, c_void_p]),
            "dq_quantile_summaries": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_int64, c_void_p,
                                              c_void_p, c_void_p, c_void_p]),
            "dq_kll_sketch": (c_int64, [c_void_p, c_void_p, c_int64, ctypes.c_int32, ctypes.c_double, c_void_p,
                                        c_int64]),
            "dq_kll_sketch_columns": (c_int64, [c_void_p, c_void_p, ctypes.c_int32, c_int64, ctypes.c_int32,
                                                ctypes.c_double, c_void_p, c_int64, c_void_p]),
            "dq_kll_merge_states": (c_int64, [c_void_p, c_int64, c_void_p, c_int64, c_void_p, c_int64]),
            "dq_cast_column": (c_int, [c_void_p, c_void_p, c_int64, ctypes.c_int32, c_void_p, c_void_p]),
            "dq_synth_column": (c_int, [c_void_p, ctypes.c_int32, ctypes.c_uint64, c_int64, c_int64, c_void_p]),
            "dq_synth_freq_keys": (c_int, [c_void_p, c_int64, c_int64, c_int64, c_int64, c_void_p]),
            "dq_synth_validity": (c_int, [c_void_p, ctypes.c_uint64, c_int64, c_int64, ctypes.c_int32, c_void_p]),
            "dq_frequencies_ex": (c_int, [c_void_p, c_void_p, c_int, c_int64, c_void_p, c_int, c_void_p, c_void_p]),
            "dq_freq_row_counts": (c_int, [c_void_p, c_void_p, c_void_p, c_int64, c_uint32]),
            "dq_synth_strings": (c_int, [c_void_p, ctypes.c_int32, ctypes.c_uint64, c_int64, c_int64, c_void_p, c_void_p,
                                         c_void_p]),
            "dq_freq_export_device": (c_int64, [c_void_p, c_void_p, c_int64, c_void_p, c_void_p]),
            "dq_freq_from_pairs": (c_int, [c_void_p, ctypes.c_int32, c_void_p, c_void_p, c_int64, c_uint32, c_int64,
                                           c_int64, c_void_p]),
            "dq_freq_merge": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p]),
            "dq_freq_mutual_information": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
            "dq_open_devices": (c_void_p, [c_void_p, c_int, ctypes.POINTER(c_int)]),
            "dq_scan_streamed": (c_int, [c_void_p, c_void_p, c_int, c_int64, c_void_p, c_int, c_void_p, c_int, c_void_p,
                                         c_int64]),
            "dq_ctx_num_devices": (c_int, [c_void_p]),
            "dq_ctx_uses_rccl": (c_int, [c_void_p]),
            "dq_scan_sharded": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_int, c_void_p, c_int,
                                        c_void_p]),
        }
        for name, (res, args) in sig.items():
            f = getattr(lib, name)
            f.restype = res
            f.argtypes = args
        if path is None:
            _lib = lib
        return lib


def hll_count(words):
    """DeequHyperLogLogPlusPlusUtils.count over 52 packed register words (host-side, C-ABI)."""
    lib = load_library()
    arr = (ctypes.c_int64 * HLL_NUM_WORDS)(*[int(np.int64(np.uint64(w & 0xFFFFFFFFFFFFFFFF))) for w in words])
    return lib.dq_hll_count(arr)


def kll_merge_states(a, b):
    """dq_kll_merge_states: KLLState.sum of two serialized KLLStates (host-side, C-ABI)."""
    lib = load_library()
    cap = len(a) + len(b) + 64
    while True:
        out = ctypes.create_string_buffer(cap)
        n = lib.dq_kll_merge_states(a, len(a), b, len(b), out, cap)
        if n < 0:
            raise NativeError(int(n), "dq_kll_merge_states: malformed KLLState bytes")
        if n <= cap:
            return out.raw[:n]
        cap = int(n)


def spark_hash64(spark_type, value):
    """Spark XxHash64Function.hash(value, type, 42) as a signed 64-bit int (test hook)."""
    lib = load_library()
    if spark_type == TYPE_STRING:
        b = value.encode("utf-8") if isinstance(value, str) else bytes(value)
        buf = ctypes.create_string_buffer(b, len(b))
        return lib.dq_spark_hash64(spark_type, buf, len(b))
    dtype = {TYPE_BOOLEAN: np.uint8, TYPE_BYTE: np.int8, TYPE_SHORT: np.int16, TYPE_INT: np.int32,
             TYPE_DATE: np.int32, TYPE_LONG: np.int64, TYPE_TIMESTAMP: np.int64, TYPE_DECIMAL: np.int64,
             TYPE_FLOAT: np.float32, TYPE_DOUBLE: np.float64}[spark_type]
    a = np.array([value], dtype=dtype)
    return lib.dq_spark_hash64(spark_type, a.ctypes.data, a.nbytes)


def merge_states(a, b):
    """State.sum through the C-ABI (dq_state_merge)."""
    lib = load_library()
    out = DqState()
    rc = lib.dq_state_merge(ctypes.byref(a), ctypes.byref(b), ctypes.byref(out))
    if rc != DQ_OK:
        raise NativeError(rc, "dq_state_merge")
    return out


def fold_states(buf, nparts, nops):
    """dq_state_fold over a part-major buffer of nparts x nops dq_state records (any object exposing
    the buffer protocol, e.g. a pinned host tensor's numpy view); returns nops DqState."""
    lib = load_library()
    arr = np.frombuffer(buf, dtype=np.uint8, count=nparts * nops * STATE_SIZE)
    out = (DqState * max(nops, 1))()
    rc = lib.dq_state_fold(arr.ctypes.data, int(nparts), int(nops), out)
    if rc != DQ_OK:
        raise NativeError(rc, "dq_state_fold")
    return [out[i] for i in range(nops)]


class Context:
    """One dq_ctx bound to one GPU (one per process / rank), or — `devices` given — one context over several
    GPUs of this node (dq_open_devices: row-sharded scans, RCCL exchange of grouping keys)."""

    def __init__(self, device=0, devices=None):
        self.lib = load_library()
        status = ctypes.c_int(0)
        if devices is not None:
            arr = (ctypes.c_int * len(devices))(*[int(d) for d in devices])
            self.handle = self.lib.dq_open_devices(arr, len(devices), ctypes.byref(status))
            device = int(devices[0])
        else:
            self.handle = self.lib.dq_open(int(device), ctypes.byref(status))
        if not self.handle:
            raise NativeError(status.value, "dq_open(%r) failed: a MI355X GPU is required" % (devices or device))
        self.device = device
        self.devices = list(devices) if devices is not None else [device]
        self.multi = devices is not None  # dq_open_devices: host columns in, host results out

    def num_devices(self):
        return self.lib.dq_ctx_num_devices(self.handle)

    def uses_rccl(self):
        return bool(self.lib.dq_ctx_uses_rccl(self.handle))

    def close(self):
        if self.handle:
            self.lib.dq_close(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def last_error(self):
        msg = self.lib.dq_last_error(self.handle)
        return msg.decode() if msg else ""

    def check(self, rc, what):
        if rc != DQ_OK:
            raise NativeError(rc, "%s: %s" % (what, self.last_error()))

    def set_stream(self, stream_ptr):
        self.check(self.lib.dq_set_stream(self.handle, ctypes.c_void_p(stream_ptr or 0)), "dq_set_stream")

    def set_priority(self, priority):
        """dq_set_priority: 1 high, 0 normal, -1 low stream priority for this context's work."""
        if getattr(self, "_priority", 0) != priority:
            self.check(self.lib.dq_set_priority(self.handle, int(priority)), "dq_set_priority")
            self._priority = priority

    def synchronize(self):
        self.check(self.lib.dq_synchronize(self.handle), "dq_synchronize")

    def scan_launch_count(self):
        return self.lib.dq_scan_launch_count(self.handle)

    def kernel_launches(self):
        """{kernel name: launches so far} of the scan path (dq_scan_kernel_launches)."""
        return {name: int(self.lib.dq_scan_kernel_launches(self.handle, i)) for i, name in enumerate(SCAN_KERNELS)}

    def freq_paths(self):
        """{grouping build path: count so far} (dq_freq_path_count): which build produced the tables."""
        return {name: int(self.lib.dq_freq_path_count(self.handle, i)) for i, name in enumerate(FREQ_PATHS)}

    def scan(self, columns, nrows, ops, preds, out_device_ptr=None):
        """Run dq_scan. `columns`: list of DqColumn, `ops`: list of DqOp, `preds`: list of DqPredicate.
        Returns a list of DqState (host) or None when writing to a device buffer."""
        ncol = len(columns)
        col_arr = (DqColumn * max(ncol, 1))(*columns)
        op_arr = (DqOp * max(len(ops), 1))(*ops)
        pred_arr = (DqPredicate * max(len(preds), 1))(*preds)
        if out_device_ptr is not None:
            rc = self.lib.dq_scan(self.handle, col_arr, ncol, int(nrows), op_arr, len(ops), pred_arr, len(preds),
                                  ctypes.c_void_p(out_device_ptr), SCAN_OUT_DEVICE)
            self.check(rc, "dq_scan")
            return None
        out = (DqState * max(len(ops), 1))()
        rc = self.lib.dq_scan(self.handle, col_arr, ncol, int(nrows), op_arr, len(ops), pred_arr, len(preds), out, 0)
        self.check(rc, "dq_scan")
        return [out[i] for i in range(len(ops))]

    def scan_streamed(self, columns, nrows, ops, preds, chunk_rows):
        """dq_scan_streamed: host columns streamed through HBM in row chunks (copy / scan overlapped)."""
        col_arr = (DqColumn * max(len(columns), 1))(*columns)
        op_arr = (DqOp * max(len(ops), 1))(*ops)
        pred_arr = (DqPredicate * max(len(preds), 1))(*preds)
        out = (DqState * max(len(ops), 1))()
        rc = self.lib.dq_scan_streamed(self.handle, col_arr, len(columns), int(nrows), op_arr, len(ops), pred_arr,
                                       len(preds), out, int(chunk_rows))
        self.check(rc, "dq_scan_streamed")
        return [out[i] for i in range(len(ops))]

    def quantile_summary(self, column, nrows, relative_error):
        """dq_quantile_summary: exact (value, rank) samples of a zero-uncertainty GK summary of the
        column's non-NULL values, and their count n."""
        cap = int(nrows) if relative_error <= 0.0 else min(int(nrows), int(2.0 / relative_error) + 8)
        cap = max(cap, 2)
        vals = np.empty(cap, dtype=np.float64)
        ranks = np.empty(cap, dtype=np.int64)
        count = ctypes.c_int64(0)
        ns = self.lib.dq_quantile_summary(self.handle, ctypes.byref(column), int(nrows), float(relative_error), cap,
                                          vals.ctypes.data, ranks.ctypes.data, ctypes.byref(count))
        if ns < 0:
            self.check(int(ns), "dq_quantile_summary")
        return vals[:ns].copy(), ranks[:ns].copy(), int(count.value)

    def quantile_summaries(self, requests):
        """dq_quantile_summaries: requests = [(parts, relative_error)], parts = the DqColumns of one column's
        consecutive row ranges; returns [(values, ranks, n)] per request, as quantile_summary over the parts
        concatenated."""
        if not requests:
            return []
        parts, begin, rels, cap = [], [0], [], 2
        for cols, rel in requests:
            parts.extend(cols)
            begin.append(len(parts))
            rels.append(float(rel))
            rows = sum(int(c.length) for c in cols)
            cap = max(cap, rows if rel <= 0.0 else min(rows, int(2.0 / rel) + 8))
        nreq = len(requests)
        part_arr = (DqColumn * len(parts))(*parts)
        begin_arr = np.asarray(begin, dtype=np.int32)
        rel_arr = np.asarray(rels, dtype=np.float64)
        vals = np.empty(nreq * cap, dtype=np.float64)
        ranks = np.empty(nreq * cap, dtype=np.int64)
        counts = np.zeros(nreq, dtype=np.int64)
        nsamp = np.zeros(nreq, dtype=np.int64)
        rc = self.lib.dq_quantile_summaries(self.handle, part_arr, begin_arr.ctypes.data, nreq, rel_arr.ctypes.data,
                                            cap, vals.ctypes.data, ranks.ctypes.data, counts.ctypes.data,
                                            nsamp.ctypes.data)
        self.check(rc, "dq_quantile_summaries")
        return [(vals[r * cap:r * cap + nsamp[r]].copy(), ranks[r * cap:r * cap + nsamp[r]].copy(), int(counts[r]))
                for r in range(nreq)]

    def kll_sketch(self, column, nrows, sketch_size, shrinking_factor):
        """dq_kll_sketch: the KLLState bytes of one partition holding the column's rows in order."""
        cap = 1 << 16
        while True:
            buf = np.empty(cap, dtype=np.uint8)
            n = self.lib.dq_kll_sketch(self.handle, ctypes.byref(column), int(nrows), int(sketch_size),
                                       float(shrinking_factor), buf.ctypes.data, cap)
            if n < 0:
                self.check(int(n), "dq_kll_sketch")
            if n <= cap:
                return buf[:n].tobytes()
            cap = int(n)

    def kll_sketch_columns(self, columns, nrows, sketch_size, shrinking_factor):
        """dq_kll_sketch_columns: the KLLState bytes of each column (one partition each, rows in order), sketched in
        one call (parallel host schedules, one round trip)."""
        arr = (DqColumn * max(len(columns), 1))(*columns)
        sizes = np.zeros(max(len(columns), 1), dtype=np.int64)
        cap = (1 << 18) * max(len(columns), 1)  # a default sketch's state is ~40 KB: one call, not a size probe + a rerun
        while True:
            buf = np.empty(cap, dtype=np.uint8)
            n = self.lib.dq_kll_sketch_columns(self.handle, arr, len(columns), int(nrows), int(sketch_size),
                                               float(shrinking_factor), buf.ctypes.data, cap, sizes.ctypes.data)
            if n < 0:
                self.check(int(n), "dq_kll_sketch_columns")
            if n <= cap:
                out, at = [], 0
                for k in range(len(columns)):
                    out.append(buf[at:at + int(sizes[k])].tobytes())
                    at += int(sizes[k])
                return out
            cap = int(n)

    def cast_column(self, column, nrows, to_type, values_dev_ptr, validity_dev_ptr):
        """dq_cast_column: Spark Cast(column -> long | double) into caller-owned device buffers (torch's queued work
        on them, e.g. a zero fill, completes first: the cast runs on the context's stream)."""
        self._after_torch_stream()
        self.check(self.lib.dq_cast_column(self.handle, ctypes.byref(column), int(nrows), int(to_type),
                                            ctypes.c_void_p(values_dev_ptr), ctypes.c_void_p(validity_dev_ptr)),
                   "dq_cast_column")

    def _after_torch_stream(self):
        """The generators run on the context's stream; a buffer torch just allocated and filled (torch.zeros) on its
        own stream must be complete before they write into it. The stream is this thread's current stream of the
        context's device (explicitly: a helper thread starts on device 0)."""
        torch = sys.modules.get("torch")
        if torch is not None and torch.cuda.is_initialized():
            for d in self.devices:
                torch.cuda.current_stream(int(d)).synchronize()

    def synth_column(self, kind, seed, row0, nrows, dev_ptr):
        self._after_torch_stream()
        self.check(self.lib.dq_synth_column(self.handle, kind, seed & 0xFFFFFFFFFFFFFFFF, row0, nrows,
                                            ctypes.c_void_p(dev_ptr)), "dq_synth_column")

    def synth_freq_keys(self, total_rows, distinct, row0, nrows, dev_ptr):
        self._after_torch_stream()
        self.check(self.lib.dq_synth_freq_keys(self.handle, int(total_rows), int(distinct), int(row0), int(nrows),
                                               ctypes.c_void_p(dev_ptr)), "dq_synth_freq_keys")

    def synth_strings(self, kind, seed, row0, nrows, offsets_ptr, bytes_ptr=None):
        """dq_synth_strings: offsets first (returns the text bytes), then the bytes."""
        self._after_torch_stream()
        total = ctypes.c_int64(0)
        self.check(self.lib.dq_synth_strings(self.handle, int(kind), seed & 0xFFFFFFFFFFFFFFFF, int(row0), int(nrows),
                                             ctypes.c_void_p(offsets_ptr),
                                             ctypes.c_void_p(bytes_ptr) if bytes_ptr else None, ctypes.byref(total)),
                   "dq_synth_strings")
        return int(total.value)

    def synth_validity(self, seed, row0, nrows, null_permille, dev_ptr):
        self._after_torch_stream()
        self.check(self.lib.dq_synth_validity(self.handle, seed & 0xFFFFFFFFFFFFFFFF, row0, nrows, null_permille,
                                              ctypes.c_void_p(dev_ptr)), "dq_synth_validity")


_contexts = {}
_aux_lock = threading.Lock()
_aux_pool = {}     # (device, slot) -> [Context, ...]
_aux_leased = set()  # id() of the aux contexts a helper thread drives right now


def lease_aux_context(device=0, slot="aux", priority=0):
    """A single-device context of `device` (its own stream and scratch cache) for one helper thread: the cached
    context of `slot` unless another thread holds it (dq.h: calls on one ctx are not re-entrant), else another one of
    the slot's pool. Return it with release_aux_context. Helper work overlaps the main context's (the
    ColumnProfiler's histogram pass beside its numeric pass, a run's grouping builds beside its scans)."""
    key = (int(device), slot)
    ctx = None
    with _aux_lock:
        pool = _aux_pool.setdefault(key, [])
        for c in pool:
            if id(c) not in _aux_leased:
                _aux_leased.add(id(c))
                ctx = c
                break
    if ctx is None:
        ctx = Context(device)  # outside the lock: dq_open may take a while
        with _aux_lock:
            _aux_pool[key].append(ctx)
            _aux_leased.add(id(ctx))
    try:
        ctx.set_priority(priority)  # (the leased context is idle: its stream can be replaced)
    except BaseException:
        release_aux_context(ctx)
        raise
    return ctx


def release_aux_context(ctx):
    """The helper is done with `ctx`: its cached scratch beyond the idle cap is released and the context may be leased
    again."""
    try:
        ctx.lib.dq_scratch_trim(ctx.handle, AUX_IDLE_SCRATCH_BYTES)
    finally:
        with _aux_lock:
            _aux_leased.discard(id(ctx))


# idle device scratch an aux context keeps between runs (its builds re-use it instead of hipMalloc'ing again; an
# allocation that fails on any context of the device releases the others' idle scratch first, dq_api.cpp). r06: the
# same 48 GB as a context's own cap (dq_api.cpp kScratchCacheCap). At 16 GiB the C5 text grouping's ~27 GB working set
# was freed and re-allocated every run; on some boxes those hipFree / hipMalloc rounds made the overlapped C5 step
# 340-560 ms, with the scratch-heavy passes alone 5-16x slower afterwards (profiles/r06/c5_priority_risk_r06bg.txt)
AUX_IDLE_SCRATCH_BYTES = int(float(os.environ.get("DQ_AUX_IDLE_SCRATCH", 48e9)))


def aux_context(device=0, slot="aux"):
    """The cached context of `slot` (see lease_aux_context) without a lease: single-threaded callers only."""
    key = (int(device), slot)
    with _aux_lock:
        pool = _aux_pool.setdefault(key, [])
        if pool:
            return pool[0]
    ctx = Context(device)
    with _aux_lock:
        _aux_pool[key].append(ctx)
    return ctx


def context(device=0):
    """Process-wide cached context for a device. DQ_DEVICES="0,1,..." makes it one multi-device context over
    those GPUs (every host-column scan / grouping of the runner is then row-sharded across them)."""
    spec = os.environ.get("DQ_DEVICES")
    key = ("multi", spec) if spec else device
    ctx = _contexts.get(key)
    if ctx is None:
        ctx = Context(device, devices=[int(d) for d in spec.split(",")] if spec else None)
        _contexts[key] = ctx
    return ctx
