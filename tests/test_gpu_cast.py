"""GPU parity of dq_cast_column (cast.hip + dq_parse.h) against the oracle's restatements of Spark 2.2's
Cast(string -> long) (UTF8String.toLong) and Cast(string -> double) (java.lang.Double.parseDouble, whose
correctly rounded value is Python's float() of the same digits). Bar: bit-exact values and identical
NULLs. Strings with more than 19 significant digits either match or fail loudly (DQ_ERR_UNSUPPORTED)."""
import numpy as np
import pytest
import torch

from deequ_amd import engine
from deequ_amd import native as N
from deequ_amd.native import NativeError
from deequ_amd.table import Table, unpack_validity
import oracle as O

pytestmark = pytest.mark.gpu


def gpu_cast(strings, to_type, device=False):
    valid = [s is not None for s in strings]
    t = Table.from_rows([(s,) for s in strings], ["s"], ["string"])
    if device:
        t.to_device(0)
    n = len(strings)
    vals = torch.empty(max(n, 1), dtype=torch.float64 if to_type == N.TYPE_DOUBLE else torch.int64, device="cuda")
    mask = torch.zeros(max((n + 63) // 64, 1) * 8, dtype=torch.uint8, device="cuda")
    engine.ctx().cast_column(t["s"].native(), n, to_type, vals.data_ptr(), mask.data_ptr())
    ok = unpack_validity(mask.cpu().numpy(), n)
    return vals.cpu().numpy()[:n], ok, valid


def random_numeric_strings(rng, n, max_digits=19):
    out = []
    for _ in range(n):
        k = int(rng.integers(0, 6))
        nd = int(rng.integers(1, max_digits + 1))
        digits = "".join(str(d) for d in rng.integers(0, 10, nd))
        sign = ["", "-", "+", "- ", " "][int(rng.integers(0, 5))]
        if k == 0:
            s = sign + digits
        elif k == 1:
            p = int(rng.integers(0, nd + 1))
            s = sign + digits[:p] + "." + digits[p:]
        elif k == 2:
            s = sign + digits[:1] + "." + digits[1:] + "e" + str(int(rng.integers(-330, 320)))
        elif k == 3:
            s = sign + "0." + "0" * int(rng.integers(0, 30)) + digits
        elif k == 4:
            s = sign + digits + ["d", "f", "D", "x", "", "\n", "  "][int(rng.integers(0, 7))]
        else:
            s = ["", ".", "-", "+", "NaN", "-Infinity", "Infinity", "1e", "e5", "--1", "1.2.3", " 42 ", "\t7\n",
                 "9223372036854775807", "9223372036854775808", "-9223372036854775808", "-9223372036854775809",
                 "1.", ".5", "-.5", "+.", "0.1e-5", "1E+3", "4.9e-324", "2.4703282292062328e-324",
                 "1.7976931348623157e308", "1.7976931348623159e308", "0x1p3", "007"][int(rng.integers(0, 29))]
        out.append(s)
    return out


def test_cast_to_long_matches_spark():
    rng = np.random.default_rng(1)
    strings = random_numeric_strings(rng, 50_000) + [None, "123", None]
    strings = [s for s in strings if s != "0x1p3"]
    vals, ok, valid = gpu_cast(strings, N.TYPE_LONG)
    for i, s in enumerate(strings):
        exp = O.spark_string_to_long(s) if s is not None else None
        assert bool(ok[i]) == (exp is not None), (s, exp)
        if exp is not None:
            assert int(vals[i]) == exp, (s, exp, int(vals[i]))


@pytest.mark.parametrize("device", [False, True])
def test_cast_to_double_matches_java(device):
    rng = np.random.default_rng(2 + device)
    strings = random_numeric_strings(rng, 60_000) + [None, "2.5", None]
    strings = [s for s in strings if s != "0x1p3"]
    vals, ok, valid = gpu_cast(strings, N.TYPE_DOUBLE, device=device)
    bad = []
    for i, s in enumerate(strings):
        exp = O.java_parse_double(s) if s is not None else None
        if bool(ok[i]) != (exp is not None):
            bad.append((s, exp, ok[i]))
            continue
        if exp is not None:
            a, b = np.float64(vals[i]), np.float64(exp)
            if not (np.isnan(a) and np.isnan(b)) and a.view(np.uint64) != b.view(np.uint64):
                bad.append((s, exp, float(a)))
    assert not bad, bad[:10]


def test_cast_long_significands_match_or_fail_loudly():
    rng = np.random.default_rng(5)
    strings = random_numeric_strings(rng, 3000, max_digits=30)
    strings = [s for s in strings if s != "0x1p3"]
    try:
        vals, ok, _ = gpu_cast(strings, N.TYPE_DOUBLE)
    except NativeError:
        return
    for i, s in enumerate(strings):
        exp = O.java_parse_double(s)
        assert bool(ok[i]) == (exp is not None), s
        if exp is not None and not np.isnan(exp):
            assert np.float64(vals[i]).view(np.uint64) == np.float64(exp).view(np.uint64), s
    with pytest.raises(NativeError):
        gpu_cast(["0x1p3"], N.TYPE_DOUBLE)


def test_cast_empty_and_all_null():
    vals, ok, _ = gpu_cast([], N.TYPE_LONG)
    assert len(vals) == 0
    vals, ok, _ = gpu_cast([None] * 100, N.TYPE_DOUBLE)
    assert not ok.any()


@pytest.mark.parametrize("to_type", [N.TYPE_LONG, N.TYPE_DOUBLE])
@pytest.mark.parametrize("device", [False, True])
def test_short_numbers_fast_path_matches_the_parsers(to_type, device, monkeypatch):
    """Strings of <= 15 bytes are parsed by one branch-free DFA step per byte ([+|-] digits [. digits]; cast.hip
    cast_short_number): every form of that grammar at every length up to 15 (and the near misses around it: lone signs
    and points, second points, inner signs, spaces, exponents, letters, 16-byte numbers) equals the oracle's
    UTF8String.toLong / Double.parseDouble and the general device parsers (DQ_CAST_NO_SHORT=1), bit for bit."""
    rng = np.random.default_rng(40 + device + 2 * (to_type == N.TYPE_DOUBLE))
    strings = ["", ".", "+", "-", "+.", "-.", "-.5", ".5", "1.", "00", "-0", "-0.000", "+0", "0.", "1.2.3", "1-2", "+-1",
               " 1", "1 ", "1e5", "1d", "NaN", "a", "999999999999999", "-99999999999999", "9999999.9999999",
               "0.000000000001", "1234567890123456", "-123456789012345", "1.23456789012345", "..1", "1..", "-",
               None]
    for _ in range(30_000):
        nd = int(rng.integers(0, 15))
        digits = "".join(str(d) for d in rng.integers(0, 10, nd))
        p = int(rng.integers(0, nd + 1))
        form = int(rng.integers(0, 4))
        s = digits if form == 0 else digits[:p] + "." + digits[p:] if form == 1 else \
            ["-", "+"][int(rng.integers(0, 2))] + (digits[:p] + "." + digits[p:] if rng.random() < 0.5 else digits)
        if form == 3 and s:  # a near miss: one byte replaced
            i = int(rng.integers(0, len(s)))
            s = s[:i] + ["x", " ", "e", "-", "."][int(rng.integers(0, 5))] + s[i + 1:]
        strings.append(s[:16])
    strings += ["%d" % v for v in rng.integers(-1_000_000, 1_000_000, 2000)]  # the C5 generators' forms
    strings += ["%d.%02d" % (v // 100, v % 100) for v in rng.integers(0, 100_000, 2000)]
    strings += ["%s%d.%03d" % ("-" if v < 0 else "", abs(v) // 1000, abs(v) % 1000)
                for v in rng.integers(-999_999, 999_999, 2000)]
    fast, ok_f, _ = gpu_cast(strings, to_type, device=device)
    monkeypatch.setenv("DQ_CAST_NO_SHORT", "1")
    slow, ok_s, _ = gpu_cast(strings, to_type, device=device)
    assert np.array_equal(ok_f, ok_s)
    assert np.array_equal(fast[ok_f].view(np.uint64), slow[ok_s].view(np.uint64))
    for i, s in enumerate(strings):
        exp = None if s is None else (O.spark_string_to_long(s) if to_type == N.TYPE_LONG else O.java_parse_double(s))
        assert bool(ok_f[i]) == (exp is not None), (s, exp)
        if exp is not None and to_type == N.TYPE_LONG:
            assert int(fast[i]) == exp, (s, exp)
        elif exp is not None and not np.isnan(exp):
            assert np.float64(fast[i]).view(np.uint64) == np.float64(exp).view(np.uint64), (s, exp, fast[i])
