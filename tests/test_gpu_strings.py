"""GPU parity of the string-shaped scan ops (strings.hip) against the oracle: MinLength / MaxLength
(UTF-8 characters), DataType (StatefulDataType's regexes over the value cast to string, with the
oracle formatting numbers through a Java toString restatement), and ApproxCountDistinct over UTF-8
(HLL registers bit-exact against the oracle's XXH64, itself pinned to the `xxhash` package)."""
import numpy as np
import pytest

import deequ_amd as D
from deequ_amd import engine
from deequ_amd.table import Table, Column, pack_validity, _column_from_pylist
import oracle as O

pytestmark = pytest.mark.gpu

SPECIAL = ["", "-", "+", " ", "- ", "+ 1", "-1", " 7", "1.", ".", "-.5", "+ .5", "1.5.", "12a", "true", "false",
           "True", "FALSE", "1e5", "12\n", "NaN", "0", "007", "9" * 40, "é", "中文字符", "😀x", "a" * 33,
           "ab" * 40, "tr ue", "--1", "+-1", "1 ", "١٢"]


def random_strings(rng, n):
    alphabet = list("abcxyz0123456789 .-+") + ["é", "ß", "中", "😀"]
    out = []
    for i in range(n):
        r = rng.random()
        if r < 0.3:
            out.append(SPECIAL[rng.integers(len(SPECIAL))])
        elif r < 0.5:
            out.append(str(rng.integers(-10 ** 6, 10 ** 6)) + ("." + str(rng.integers(0, 999)) if rng.random() < 0.5
                                                              else ""))
        else:
            k = int(rng.integers(0, 70))
            out.append("".join(alphabet[j] for j in rng.integers(0, len(alphabet), k)))
    return out


def string_table(n=50_000, seed=0, null_frac=0.1):
    rng = np.random.default_rng(seed)
    vals = random_strings(rng, n)
    items = [None if rng.random() < null_frac else v for v in vals]
    col = _column_from_pylist("s", "string", items)
    key = _column_from_pylist("k", "int", [int(x) for x in rng.integers(0, 10, n)])
    return Table([col, key])


def run_states(t, analyzers):
    batch = D.ScanBatch(t)
    offs = [a.addOps(batch) for a in analyzers]
    res = batch.run()
    return [a.fromAggregationResult(res, o) for a, o in zip(analyzers, offs)]


@pytest.mark.parametrize("device", [False, True])
@pytest.mark.parametrize("where", [None, "k < 4"])
def test_string_ops_match_oracle(device, where):
    t = string_table(seed=1 if device else 2)
    if device:
        t.to_device(0)
    analyzers = [D.MinLength("s", where), D.MaxLength("s", where), D.DataType("s", where),
                 D.ApproxCountDistinct("s", where), D.Completeness("s", where), D.Size(where)]
    got = run_states(t, analyzers)
    for a, g in zip(analyzers, got):
        exp = O.expected_state(t, a)
        assert g == exp or (g is not None and exp is not None and repr(g) == repr(exp)), (a, g, exp)
    words = got[3].words
    assert [int(w) & 0xFFFFFFFFFFFFFFFF for w in words] == \
        [int(w) & 0xFFFFFFFFFFFFFFFF for w in O.expected_state(t, analyzers[3]).words]


def test_datatype_digit_runs_match_oracle():
    """DataType's digit runs are scanned four bytes at a time: strings of digits with the bytes next to '0'..'9'
    ('/', ':'), signs, spaces, points and multi-byte characters at every offset and length 0-40."""
    rng = np.random.default_rng(11)
    alphabet = list("0123456789") * 4 + list("/:.-+ ") + ["°", "é", "٣"]
    vals = []
    for i in range(60_000):
        k = int(rng.integers(0, 41))
        body = "".join(alphabet[j] for j in rng.integers(0, len(alphabet), k))
        r = rng.random()
        if r < 0.3:
            body = "".join(c for c in body if c.isdigit() and c.isascii())
        elif r < 0.5:
            d = "".join(c for c in body if c.isdigit() and c.isascii())
            body = ("-" if rng.random() < 0.3 else "") + d[: len(d) // 2] + "." + d[len(d) // 2:]
        vals.append(body)
    t = Table([_column_from_pylist("s", "string", vals)])
    t.to_device(0)
    a = D.DataType("s")
    got = run_states(t, [a])[0]
    exp = O.expected_state(t, a)
    fields = ("numNull", "numFractional", "numIntegral", "numBoolean", "numString")
    assert [getattr(got, f) for f in fields] == [getattr(exp, f) for f in fields], (got, exp)


def test_string_all_null_and_empty():
    t = Table([_column_from_pylist("s", "string", [None] * 100)])
    ctx = D.AnalysisRunner.onData(t).addAnalyzers(
        [D.MinLength("s"), D.MaxLength("s"), D.DataType("s"), D.ApproxCountDistinct("s")]).run()
    assert ctx.metric(D.MinLength("s")).value.isFailure
    assert ctx.metric(D.MaxLength("s")).value.isFailure
    assert ctx.metric(D.DataType("s")).value.get().values["Unknown"].ratio == 1.0
    assert ctx.metric(D.ApproxCountDistinct("s")).value.get() == 0.0
    t0 = Table([_column_from_pylist("s", "string", [])])
    m = D.DataType("s").calculate(t0)
    assert m.value.isSuccess and m.value.get().values["Unknown"].absolute == 0


def test_datatype_of_numeric_columns_matches_java_tostring_rules():
    rng = np.random.default_rng(3)
    n = 20_000
    edge = [0.0, -0.0, 1e-3, np.nextafter(1e-3, 0), 1e7, np.nextafter(1e7, 0), -1e7, 5e-324, np.nan, np.inf, -np.inf,
            123.456, 1e-300, 1e300]
    d = np.concatenate([np.array(edge), rng.normal(0, 10, n) * 10.0 ** rng.integers(-6, 9, n)])
    f = d.astype(np.float32)
    dec = rng.integers(-10 ** 12, 10 ** 12, len(d), dtype=np.int64)
    dec[:5] = [0, 1, -1, 10 ** 6, 5]
    ints = rng.integers(-2 ** 40, 2 ** 40, len(d), dtype=np.int64)
    bools = (rng.random(len(d)) < 0.5).astype(np.uint8)
    cols = [Column("d", "double", d), Column("f", "float", f), Column("i", "long", ints), Column("b", "boolean", bools),
            Column("dec0", "DecimalType", dec, decimal_precision=18, decimal_scale=0),
            Column("dec9", "DecimalType", dec, decimal_precision=18, decimal_scale=9),
            Column("dec14", "DecimalType", dec, decimal_precision=18, decimal_scale=14),
            Column("date", "date", rng.integers(0, 20000, len(d)).astype(np.int32))]
    t = Table(cols)
    analyzers = [D.DataType(c.name) for c in cols]
    got = run_states(t, analyzers)
    for a, g in zip(analyzers, got):
        assert g == O.expected_state(t, a), (a, g, O.expected_state(t, a))
