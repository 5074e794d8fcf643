"""libdq.so loads, exports every symbol include/dq.h declares, and its host-side functions (HLL
estimate, Spark hash, state merge) agree with the oracle. No GPU needed."""
import ctypes
import os
import random
import re

import numpy as np
import pytest
import xxhash

import deequ_amd.native as N
import oracle as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    text = open(os.path.join(ROOT, "include", "dq.h")).read()
    return sorted(set(re.findall(r"\b(dq_[a-z0-9_]+)\s*\(", text)))


def test_library_exports_every_declared_symbol():
    lib = N.load_library()
    decl = declared_symbols()
    assert set(decl) == set(N.EXPORTED_SYMBOLS), set(decl) ^ set(N.EXPORTED_SYMBOLS)
    for s in decl:
        assert hasattr(lib, s), s
    assert lib.dq_abi_version() == 2


def test_struct_sizes_match_header_layout():
    assert ctypes.sizeof(N.DqColumn) == 48
    assert ctypes.sizeof(N.DqOp) == 20
    assert ctypes.sizeof(N.DqState) == 8 + 52 * 8
    assert ctypes.sizeof(N.DqConst) == 32


def test_open_without_gpu_fails_loudly():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(N.NativeError):
        N.Context(0)


def test_hll_count_matches_oracle_random_registers():
    rng = random.Random(3)
    for trial in range(300):
        maxr = rng.choice([1, 3, 8, 20, 40, 56])
        density = rng.random()
        regs = [rng.randint(0, maxr) if rng.random() < density else 0 for _ in range(512)]
        words = []
        for w in range(52):
            word = 0
            for k in range(10):
                i = w * 10 + k
                if i < 512:
                    word |= regs[i] << (6 * k)
            words.append(word)
        assert N.hll_count(words) == O.hll_count(words), trial


def test_spark_hash_matches_oracle_and_xxhash():
    for t, v in [(N.TYPE_INT, 6), (N.TYPE_LONG, -7), (N.TYPE_DOUBLE, 2.5), (N.TYPE_FLOAT, 1.25),
                 (N.TYPE_SHORT, -3), (N.TYPE_BYTE, 100), (N.TYPE_BOOLEAN, 1), (N.TYPE_DATE, 17000)]:
        assert N.spark_hash64(t, v) & 0xFFFFFFFFFFFFFFFF == O.spark_hash(t, v), t
    for s in ["", "a", "hello world", "x" * 31, "y" * 32, "ünïcødé" * 9]:
        assert N.spark_hash64(N.TYPE_STRING, s) & 0xFFFFFFFFFFFFFFFF == \
            xxhash.xxh64_intdigest(s.encode("utf-8"), seed=42)


def _st(kind, **fields):
    s = N.DqState()
    s.kind = kind
    s.present = 1
    for k, v in fields.items():
        path = k.split("__")
        obj = s.u
        for p in path[:-1]:
            obj = getattr(obj, p)
        setattr(obj, path[-1], v)
    return s


def test_state_merge_follows_reference_semigroups():
    from deequ_amd.states import StandardDeviationState, CorrelationState, hll_merge
    a = _st(N.OP_STANDARD_DEVIATION, stddev__n=3.0, stddev__avg=2.0, stddev__m2=2.0)
    b = _st(N.OP_STANDARD_DEVIATION, stddev__n=3.0, stddev__avg=5.0, stddev__m2=2.0)
    m = N.merge_states(a, b)
    ref = StandardDeviationState(3, 2, 2).sum(StandardDeviationState(3, 5, 2))
    assert (m.u.stddev.n, m.u.stddev.avg, m.u.stddev.m2) == (ref.n, ref.avg, ref.m2)
    c1 = _st(N.OP_CORRELATION, corr__n=2, corr__x_avg=1.5, corr__y_avg=4.5, corr__ck=0.5, corr__x_mk=0.5,
             corr__y_mk=0.5)
    c2 = _st(N.OP_CORRELATION, corr__n=1, corr__x_avg=3, corr__y_avg=6, corr__ck=0, corr__x_mk=0, corr__y_mk=0)
    m = N.merge_states(c1, c2)
    ref = CorrelationState(2, 1.5, 4.5, .5, .5, .5).sum(CorrelationState(1, 3, 6, 0, 0, 0))
    assert abs(m.u.corr.ck / (m.u.corr.x_mk * m.u.corr.y_mk) ** 0.5 - ref.metricValue()) < 1e-15
    rng = random.Random(1)
    w1 = [rng.getrandbits(60) for _ in range(52)]
    w2 = [rng.getrandbits(60) for _ in range(52)]
    h1 = _st(N.OP_APPROX_COUNT_DISTINCT)
    h2 = _st(N.OP_APPROX_COUNT_DISTINCT)
    for i in range(52):
        h1.u.hll.words[i] = w1[i]
        h2.u.hll.words[i] = w2[i]
    m = N.merge_states(h1, h2)
    assert [x & 0xFFFFFFFFFFFFFFFF for x in m.u.hll.words] == hll_merge(w1, w2)
    # None is the identity (Analyzers.merge)
    empty = N.DqState()
    empty.kind = N.OP_MINIMUM
    mn = _st(N.OP_MINIMUM, dbl__value=3.0)
    assert N.merge_states(empty, mn).u.dbl.value == 3.0
    nan = _st(N.OP_MAXIMUM, dbl__value=float("nan"))
    assert np.isnan(N.merge_states(nan, _st(N.OP_MAXIMUM, dbl__value=1.0)).u.dbl.value)


def test_integral_sum_partials_merge_as_wrapped_long():
    """Chunks / shards of one integral column merge their exact Long partials (Spark: Long sum that wraps,
    cast once to Double, A/Sum.scala:34-37), natively and in the host states; a rounded-double merge differs."""
    from deequ_amd.states import MeanState, SumState, state_from_native, state_to_native
    big, small = (1 << 63) - 7, 1 << 60
    wrapped = (big + small + (1 << 63)) % (1 << 64) - (1 << 63)
    a = _st(N.OP_MEAN, mean__sum=float(big), mean__count=2, mean__isum=big, mean__exact=1)
    b = _st(N.OP_MEAN, mean__sum=float(small), mean__count=3, mean__isum=small, mean__exact=1)
    m = N.merge_states(a, b)
    assert (m.u.mean.isum, m.u.mean.exact, m.u.mean.sum, m.u.mean.count) == (wrapped, 1, float(wrapped), 5)
    s = N.merge_states(_st(N.OP_SUM, dbl__value=float(big), dbl__isum=big, dbl__exact=1),
                       _st(N.OP_SUM, dbl__value=float(small), dbl__isum=small, dbl__exact=1))
    assert s.u.dbl.value == float(wrapped)
    # one side without the exact partial (e.g. a persisted state): the reference's double merge
    s = N.merge_states(_st(N.OP_SUM, dbl__value=1.5), _st(N.OP_SUM, dbl__value=2.0, dbl__isum=2, dbl__exact=1))
    assert (s.u.dbl.value, s.u.dbl.exact) == (3.5, 0)
    hm = MeanState(float(big), 2, big).sum(MeanState(float(small), 3, small))
    assert (hm.sum_, hm.count, hm.exact) == (float(wrapped), 5, wrapped)
    assert SumState(1.0, 1).sum(SumState(2.5)) == SumState(3.5)
    back = state_from_native(state_to_native(N.OP_MEAN, hm))
    assert back.exact == wrapped and back == hm
