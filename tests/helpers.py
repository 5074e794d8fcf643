"""Test helpers: fixture tables and analyzers from tests/golden/kats.json specs."""
import math

import deequ_amd as D
from deequ_amd.table import Table


def table_from_fixture(fx):
    return Table.from_rows([tuple(r) for r in fx["rows"]], fx["names"], fx["types"])


def analyzer_from_spec(spec):
    name, args = spec[0], spec[1:]
    cls = getattr(D, name)
    if name == "Histogram" and len(args) == 2:
        return cls(args[0], None, args[1])
    if name in ("Completeness", "Mean", "Sum", "Minimum", "Maximum", "StandardDeviation", "ApproxCountDistinct",
                "MinLength", "MaxLength", "DataType"):
        return cls(args[0], args[1] if len(args) > 1 else None)
    if name == "Compliance":
        return cls(args[0], args[1], args[2] if len(args) > 2 else None)
    if name == "Correlation":
        return cls(args[0], args[1], args[2] if len(args) > 2 else None)
    if name == "PatternMatch":
        pat = args[1]
        if pat.startswith("@"):
            pat = getattr(D.Patterns, pat[1:])
        return cls(args[0], pat, args[2] if len(args) > 2 else None)
    if name == "Size":
        return cls(args[0] if args else None)
    return cls(*args)


def check_metric(metric, expected, rel=0.0):
    """Compare a metric against a KAT expectation (value, "NaN", failure or histogram spec)."""
    if isinstance(expected, dict) and "failure" in expected:
        assert metric.value.isFailure, metric
        if expected["failure"] != "*":
            assert type(metric.value.failed).__name__ == expected["failure"], metric
        return
    assert metric.value.isSuccess, metric
    v = metric.value.get()
    if isinstance(expected, dict) and "between" in expected:
        lo, hi = expected["between"]
        assert lo < v < hi, (metric, expected)
        return
    if isinstance(expected, dict) and "datatype" in expected:
        want = {k: (0, 0.0) for k in ("Unknown", "Fractional", "Integral", "Boolean", "String")}
        want.update({k: tuple(x) for k, x in expected["datatype"].items()})
        assert v.numberOfBins == 5, v
        got = {k: (dv.absolute, dv.ratio) for k, dv in v.values.items()}
        assert got == want, (got, want)
        return
    if isinstance(expected, dict):
        assert v.numberOfBins == expected["bins"], v
        if "keys" in expected:
            assert set(v.values) == set(expected["keys"]), v
        if "nkeys" in expected:
            assert len(v.values) == expected["nkeys"], v
        return
    if expected == "NaN":
        assert math.isnan(v), v
        return
    if rel == 0.0:
        assert v == expected, (metric, expected)
    else:
        assert abs(v - expected) <= rel * max(abs(expected), 1e-300), (metric, expected)
