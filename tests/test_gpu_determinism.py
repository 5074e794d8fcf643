"""Entropy and MutualInformation do not depend on how a table was built.

A GPU frequency table's slot order is decided by atomics (LDS compare-and-swap inserts, global merges of the small
build), so a floating-point fold over slots changes with the build path, the launch geometry and the device split.
The product sums every group's term as a 128-bit fixed-point integer instead (dq_common.h fx_of, freq.hip
SummaryPartial): the same groups must give the same bits — and the same exact fixed-point sum — on the fast /
exact / unpartitioned / small / optimistic / regular builds, with the summary fused into the build or scanned with
any grid, and on one device or split over several, and stay within 1e-12 of the exact oracle
(A/Entropy.scala:28-42, A/MutualInformation.scala:35-97)."""
import math
import struct

import numpy as np
import pytest

import deequ_amd as D
import deequ_amd.native as N
from deequ_amd import engine
from deequ_amd.table import Table, Column, pack_validity
import oracle as O

pytestmark = pytest.mark.gpu

# build path x summary geometry: each entry is the environment one table is built and summarised under
VARIANTS = [{}, {"DQ_FREQ_NO_FUSED_SUMMARY": "1"}, {"DQ_FREQ_NO_FUSED_SUMMARY": "1", "DQ_FREQ_SUMMARY_GRID": "1"},
            {"DQ_FREQ_NO_FUSED_SUMMARY": "1", "DQ_FREQ_SUMMARY_GRID": "7"}]
FIXED_PATHS = [{}, {"DQ_FREQ_EXACT": "1"}, {"DQ_FREQ_NO_PARTITION": "1"}, {"DQ_FREQ_WIDE": "1"}]
GENERAL_PATHS = [{}, {"DQ_FREQ_NO_SMALL": "1"}, {"DQ_FREQ_NO_OPTIMISTIC": "1"}]


def _bits(x):
    return struct.unpack("<Q", struct.pack("<d", x))[0]


def _summaries(monkeypatch, table, cols, include_nulls, paths, devices=(None,)):
    """devices: DQ_DEVICES specs (None = the plain single-device context, "0,0,0" = one context over 3 shards)."""
    out = []
    for dev in devices:
        if dev is None:
            monkeypatch.delenv("DQ_DEVICES", raising=False)
        else:
            monkeypatch.setenv("DQ_DEVICES", dev)
        for path in paths:
            for var in VARIANTS:
                env = dict(path, **var)
                for k, v in env.items():
                    monkeypatch.setenv(k, v)
                ft = engine.frequencies(table, cols, include_nulls=include_nulls)
                s = ft.summary(None)
                out.append((dev, env, s, None))
                del ft
                for k in env:
                    monkeypatch.delenv(k)
    monkeypatch.delenv("DQ_DEVICES", raising=False)
    return out


def _assert_identical(results, exp_entropy):
    ref = results[0][2]
    for dev, env, s, _ in results:
        for key in ("num_rows", "num_groups", "num_unique", "max_count", "null_count", "entropy_fx"):
            assert s[key] == ref[key], (dev, env, key, s[key], ref[key])
        assert _bits(s["entropy"]) == _bits(ref["entropy"]), (dev, env, s["entropy"], ref["entropy"])
    assert N.fx_to_float(ref["entropy_fx"]) == ref["entropy"]
    assert abs(ref["entropy"] - exp_entropy) <= 1e-12 * max(1.0, exp_entropy)


def _freq_counts_oracle(table, cols, include_nulls):
    freq, n = O.frequencies(table, cols, include_nulls=include_nulls)
    return O.grouping_summary(freq, n)["entropy"]


def test_fixed_width_entropy_bits_do_not_depend_on_the_build(monkeypatch):
    """2^24 + 4097 int64 rows (the fast path's minimum), ~1.5e6 groups, one value whose mixed key is the EMPTY slot
    marker (kept as a side group on the fast path, inside the table on the exact path) and 2 % NULLs (Histogram's
    NULL group with include_nulls)."""
    from test_gpu_grouping import _value_mixing_to_all_ones
    rng = np.random.default_rng(23)
    n = (1 << 24) + 4097
    v = rng.integers(0, 1_500_000, n).astype(np.int64)
    v[::999_983] = _value_mixing_to_all_ones()
    valid = rng.random(n) > 0.02
    t = Table.from_arrays({"k": v}, validity={"k": valid})
    t.to_device(0)
    vs = np.where(valid, v, 0)
    for include_nulls in (False, True):
        # oracle entropy from numpy counts (exact fsum of the terms)
        _, counts = np.unique(vs[valid], return_counts=True)
        cl = counts.tolist() + ([int((~valid).sum())] if include_nulls else [])
        nn = n if include_nulls else int(valid.sum())
        exp = math.fsum(-(c / nn) * math.log(c / nn) for c in cl)
        res = _summaries(monkeypatch, t, ["k"], include_nulls, FIXED_PATHS)
        _assert_identical(res, exp)


def test_general_key_entropy_bits_do_not_depend_on_the_build(monkeypatch):
    """String and (string, int) keys over 3e5 rows on the small one-pass build, the regular extract / build / verify
    path and the sized path, on one device and split over 3 (copy transport) and 1 (RCCL) devices."""
    rng = np.random.default_rng(29)
    n = 300_001
    words = np.array(["w%d" % i for i in range(1500)] + ["", "ü" * 3, "x" * 60], dtype=object)
    s = [None if rng.random() < 0.05 else words[rng.integers(0, len(words))] for _ in range(n)]
    k = [None if rng.random() < 0.1 else int(rng.integers(0, 5)) for _ in range(n)]
    t = Table.from_pydict({"s": s, "k": k}, types={"s": "string", "k": "int"})
    for cols, nulls in ((["s"], True), (["s", "k"], False)):
        exp = _freq_counts_oracle(t, cols, nulls)
        res = _summaries(monkeypatch, t, cols, nulls, GENERAL_PATHS, devices=(None, "0", "0,0,0"))
        _assert_identical(res, exp)


def test_entropy_bits_equal_across_a_device_split(monkeypatch):
    """The same fixed-width groups summarised on one device and as the union of 4 disjoint device parts."""
    rng = np.random.default_rng(31)
    n = 400_003
    v = rng.integers(-50_000, 50_000, n).astype(np.int64)
    t = Table.from_arrays({"k": v}, validity={"k": rng.random(n) > 0.01})
    exp = _freq_counts_oracle(t, ["k"], False)
    res = _summaries(monkeypatch, t, ["k"], False, [{}, {"DQ_FREQ_EXACT": "1"}], devices=(None, "0,0,0,0"))
    _assert_identical(res, exp)


def test_mutual_information_bits_do_not_depend_on_the_build(monkeypatch):
    """MutualInformation of two correlated columns (A/MutualInformation.scala:35-97) with its joint table built by the
    small and the regular path and scanned with three grids: identical bits, within 1e-12 of the oracle."""
    rng = np.random.default_rng(37)
    n = 200_003
    x = rng.integers(0, 300, n)
    y = (x * 7 + rng.integers(0, 40, n)) % 500
    valid = rng.random(n) > 0.03
    t = Table.from_arrays({"x": x.astype(np.int64), "y": y.astype(np.int64)}, validity={"y": valid})
    a = D.MutualInformation(["x", "y"])
    got = []
    for path in GENERAL_PATHS:
        for var in VARIANTS[1:]:
            env = dict(path, **var)
            for kk, vv in env.items():
                monkeypatch.setenv(kk, vv)
            m = a.calculate(t)
            assert m.value.isSuccess, (env, m)
            got.append((env, m.value.get()))
            for kk in env:
                monkeypatch.delenv(kk)
    ref = got[0][1]
    for env, val in got:
        assert _bits(val) == _bits(ref), (env, val, ref)
    from test_distributed_gloo import _oracle_mi
    mi = _oracle_mi(t, ["x", "y"])
    assert abs(ref - mi) <= 1e-12 * abs(mi), (ref, mi)


def test_fixed_point_term_rounding_matches_the_host_restatement():
    """native.fx_of (the host mirror used for small host states and the CPU gloo tests) equals the device's rounding:
    a table of one group per count value c gives the exact sum of fx_of(-(c/N) ln(c/N))."""
    counts = np.array([1, 2, 3, 5, 8, 13, 21, 34, 55, 89, 144, 1000, 77777], dtype=np.int64)
    v = np.repeat(np.arange(len(counts), dtype=np.int64), counts)
    t = Table.from_arrays({"k": v})
    s = engine.frequencies(t, ["k"], include_nulls=False).summary(None)
    n = int(counts.sum())
    host = sum(N.fx_of(-(c / n) * math.log(c / n)) for c in counts.tolist())
    # host glibc log and the device log may differ in the last ulp of a term; the fixed-point sums then differ by
    # at most one term ulp (2^-53 relative) each
    assert abs(s["entropy_fx"] - host) <= len(counts) * (1 << (104 - 53)), (s["entropy_fx"], host)
