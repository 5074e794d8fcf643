"""ColumnProfiler on the GPU engine against the reference's profiler known answers
(T/profiles/ColumnProfilerTest.scala, T/KLL/KLLProfileTest.scala; fixtures FixtureSupport.scala)."""
import json
import math
import os

import numpy as np
import pytest

import deequ_amd as D
from deequ_amd.kll import BucketValue
from deequ_amd.metrics import Distribution, DistributionValue
from deequ_amd.table import Table

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
DTI = D.DataTypeInstances


def df_complete_and_incomplete():
    # FixtureSupport.scala:74-84
    rows = [("1", "a", "f"), ("2", "b", "d"), ("3", "a", None), ("4", "a", "f"), ("5", "b", None), ("6", "a", "f")]
    return Table.from_rows(rows, ["item", "att1", "att2"], ["string", "string", "string"])


def df_numeric_fractional():
    # FixtureSupport.scala:137-147
    rows = [(str(i), float(i), a2) for i, a2 in zip(range(1, 7), [0.0, 0.0, 0.0, 5.0, 6.0, 7.0])]
    return Table.from_rows(rows, ["item", "att1", "att2"], ["string", "double", "double"])


TYPE_COUNTS_ATT2 = {"Boolean": 0, "Fractional": 0, "Integral": 0, "Unknown": 2, "String": 4}


def test_standard_column_profile():
    p = D.ColumnProfiler.profile(df_complete_and_incomplete(), ["att2"], False, 1).profiles["att2"]
    assert p == D.StandardColumnProfile("att2", 2.0 / 3.0, 2, DTI.String, True, TYPE_COUNTS_ATT2, None)


def test_predefined_types():
    t = df_complete_and_incomplete()
    p = D.ColumnProfiler.profile(t, ["item"], False, 1, predefinedTypes={"item": DTI.String}).profiles["item"]
    assert p == D.StandardColumnProfile("item", 1.0, 6, DTI.String, False, {}, None)
    p = D.ColumnProfiler.profile(t, ["att2"], False, 1, predefinedTypes={"item": DTI.String}).profiles["att2"]
    assert p == D.StandardColumnProfile("att2", 2.0 / 3.0, 2, DTI.String, True, TYPE_COUNTS_ATT2, None)


def assert_numeric(p, column, completeness, distinct, dtype, inferred, typeCounts, histogram, mean, maximum, minimum,
                   total, stdDev):
    # ColumnProfilerTest.assertProfilesEqual (:31-47)
    assert isinstance(p, D.NumericColumnProfile)
    assert p.column == column and p.completeness == completeness
    assert abs(p.approximateNumDistinctValues - distinct) <= 1
    assert p.dataType == dtype and p.isDataTypeInferred == inferred and p.typeCounts == typeCounts
    assert p.histogram == histogram
    assert (p.mean, p.maximum, p.minimum, p.sum, p.stdDev) == (mean, maximum, minimum, total, stdDev)


def test_numeric_profile_for_numeric_strings():
    p = D.ColumnProfiler.profile(df_complete_and_incomplete(), ["item"], False, 1).profiles["item"]
    assert_numeric(p, "item", 1.0, 6, DTI.Integral, True,
                   {"Boolean": 0, "Fractional": 0, "Integral": 6, "Unknown": 0, "String": 0}, None,
                   3.5, 6.0, 1.0, 21.0, 1.707825127659933)


def test_numeric_profile_for_numeric_columns():
    p = D.ColumnProfiler.profile(df_numeric_fractional(), ["att1"], False, 1).profiles["att1"]
    assert_numeric(p, "att1", 1.0, 6, DTI.Fractional, False, {}, None, 3.5, 6.0, 1.0, 21.0, 1.707825127659933)
    assert p.kll is not None and sum(b.count for b in p.kll.buckets) == 6


def test_kll_profiles():
    # T/KLL/KLLProfileTest.scala:49-116
    with open(os.path.join(HERE, "golden", "kll_kats.json")) as f:
        kats = {c["name"]: c for c in json.load(f)}
    params = D.KLLParameters(2, 0.64, 2)
    for name, table in (("NumericFractionalValues", df_numeric_fractional()),
                        ("NumericFractionalValuesForKLL",
                         Table.from_rows([(str(i), float(i), 0.0) for i in range(1, 31)], ["item", "att1", "att2"],
                                         ["string", "double", "double"]))):
        case = kats[name]
        p = D.ColumnProfiler.profile(table, ["att1"], False, 1, kllParameters=params).profiles["att1"]
        e = case["profile"]
        assert_numeric(p, "att1", e["completeness"], e["approxNumDistinct"], DTI.Fractional, False, {}, None,
                       e["mean"], e["maximum"], e["minimum"], e["sum"], e["stdDev"])
        assert p.kll.buckets == [BucketValue(*b) for b in case["buckets"]]
        assert p.kll.parameters == case["parameters"] and p.kll.data == case["data"]
    # ShortType column with a null (KLLProfileTest.scala:118-155)
    t = Table.from_arrays({"attribute": np.array([1, 2, 3, 4, 5, 6, 0], dtype=np.int16)},
                          validity={"attribute": np.array([1, 1, 1, 1, 1, 1, 0], dtype=bool)})
    p = D.ColumnProfiler.profile(t, kllParameters=params).profiles["attribute"]
    assert p.kll.buckets == [BucketValue(1.0, 3.5, 4), BucketValue(3.5, 6.0, 2)]
    assert p.kll.parameters == [0.64, 2.0] and p.kll.data == [[5.0, 6.0], [1.0, 3.0]]


def test_string_histograms():
    p = D.ColumnProfiler.profile(df_complete_and_incomplete(), ["att2"], False, 10).profiles["att2"]
    want = Distribution({"d": DistributionValue(1, 0.16666666666666666), "f": DistributionValue(3, 0.5),
                         "NullValue": DistributionValue(2, 0.3333333333333333)}, 3)
    assert p == D.StandardColumnProfile("att2", 2.0 / 3.0, 2, DTI.String, True, TYPE_COUNTS_ATT2, want)


@pytest.mark.parametrize("dtype,values,keys", [
    (np.bool_, [True, True, True, False, False], ("true", "false")),
    (np.int32, [2147483647, 2147483647, 2147483647, 2, 2], ("2147483647", "2")),
    (np.int64, [1, 1, 1, 2, 2], ("1", "2")),
    (np.float64, [1.0, 1.0, 1.0, 2.0, 2.0], ("1.0", "2.0")),
    (np.float32, [1.0, 1.0, 1.0, 2.0, 2.0], ("1.0", "2.0")),
    (np.int16, [1, 1, 1, 2, 2], ("1", "2")),
])
def test_typed_histograms(dtype, values, keys):
    # ColumnProfilerTest.scala:228-402: 3 x a, 2 x b, 1 x null; nRows = 6
    vals = np.array(values + [values[0]], dtype=dtype)
    t = Table.from_arrays({"attribute": vals}, validity={"attribute": np.array([1, 1, 1, 1, 1, 0], dtype=bool)})
    h = D.ColumnProfiler.profile(t).profiles["attribute"].histogram
    assert h is not None
    assert h[keys[0]].absolute == 3 and h[keys[0]].ratio == 3.0 / 6
    assert h[keys[1]].absolute == 2 and h[keys[1]].ratio == 2.0 / 6
    assert h["NullValue"].absolute == 1 and h["NullValue"].ratio == 1.0 / 6


def test_titanic_profile():
    # ColumnProfilerTest.scala:406-460 (CSV inferSchema)
    t = Table.from_csv(os.path.join(HERE, "golden", "titanic.csv"))
    profiles = D.ColumnProfiler.profile(t).profiles
    expected = [("PassengerId", 1.0, 891, DTI.Integral, False), ("Survived", 1.0, 2, DTI.Integral, False),
                ("Pclass", 1.0, 3, DTI.Integral, False), ("Name", 1.0, 0, DTI.String, True),
                ("Sex", 1.0, 2, DTI.String, True), ("Ticket", 1.0, 681, DTI.String, True),
                ("Fare", 1.0, 0, DTI.Fractional, False), ("Cabin", 0.22, 0, DTI.String, True)]
    for name, comp, distinct, dtype, inferred in expected:
        a = profiles[name]
        assert a.dataType == dtype and a.completeness >= comp and a.isDataTypeInferred == inferred, name
        if distinct > 0:
            assert 0.9 * distinct <= a.approximateNumDistinctValues <= 1.1 * distinct, name
    # numeric profiles carry the pass-2 statistics
    fare = profiles["Fare"]
    assert isinstance(fare, D.NumericColumnProfile) and fare.minimum == 0.0 and fare.maximum == 512.3292
    assert profiles["Sex"].histogram is not None and profiles["Sex"].histogram["male"].absolute == 577


def test_runner_api_and_json():
    t = df_numeric_fractional()
    res = D.ColumnProfilerRunner().onData(t).restrictToColumns(["att1", "item"]) \
        .withLowCardinalityHistogramThreshold(10).setKLLParameters(D.KLLParameters(2, 0.64, 2)).run()
    assert res.numRecords == 6 and set(res.profiles) == {"att1", "item"}
    js = json.loads(D.ColumnProfiles.toJson(list(res.profiles.values())))
    assert {c["column"] for c in js["columns"]} == {"att1", "item"}
    att1 = [c for c in js["columns"] if c["column"] == "att1"][0]
    assert att1["mean"] == 3.5 and att1["kll"]["buckets"][0]["count"] == 4 and len(att1["histogram"]) == 6
