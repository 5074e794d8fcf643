"""Writes tests/golden/kats.json: the reference's known-answer tests for the AnalysisRunner path.

Inputs are the fixture DataFrames of src/test/scala/com/amazon/deequ/utils/FixtureSupport.scala
(transcribed as data, with the Spark types Scala's `toDF` gives them), expected values are the
assertions of the cited test files (T/ = src/test/scala/com/amazon/deequ/). Run:
    python tests/golden/make_kats.py
"""
import json
import math
import os

HERE = os.path.dirname(os.path.abspath(__file__))

S, I, D, L = "string", "int", "double", "long"

FIXTURES = {
    # FixtureSupport.scala:36-52
    "dfMissing": {"names": ["item", "att1", "att2"], "types": [S, S, S], "rows": [
        ["1", "a", "f"], ["2", "b", "d"], ["3", None, "f"], ["4", "a", None], ["5", "a", "f"], ["6", None, "d"],
        ["7", None, "d"], ["8", "b", None], ["9", "a", "f"], ["10", None, None], ["11", None, "f"],
        ["12", None, "d"]]},
    # FixtureSupport.scala:54-62
    "dfFull": {"names": ["item", "att1", "att2"], "types": [S, S, S], "rows": [
        ["1", "a", "c"], ["2", "a", "c"], ["3", "a", "c"], ["4", "b", "d"]]},
    # FixtureSupport.scala:124-135 (Scala Int literals -> IntegerType)
    "dfWithNumericValues": {"names": ["item", "att1", "att2", "att3"], "types": [S, I, I, I], "rows": [
        ["1", 1, 0, 0], ["2", 2, 0, 0], ["3", 3, 0, 0], ["4", 4, 5, 4], ["5", 5, 6, 6], ["6", 6, 7, 7]]},
    # FixtureSupport.scala:137-147
    "dfWithNumericFractionalValues": {"names": ["item", "att1", "att2"], "types": [S, D, D], "rows": [
        ["1", 1.0, 0.0], ["2", 2.0, 0.0], ["3", 3.0, 0.0], ["4", 4.0, 5.0], ["5", 5.0, 6.0], ["6", 6.0, 7.0]]},
    # FixtureSupport.scala:191-203
    "dfWithUniqueColumns": {"names": ["unique", "nonUnique", "nonUniqueWithNulls", "uniqueWithNulls",
                                      "onlyUniqueWithOtherNonUnique", "halfUniqueCombinedWithNonUnique"],
                            "types": [S, S, S, S, S, S], "rows": [
        ["1", "0", "3", "1", "5", "0"], ["2", "0", "3", "2", "6", "0"], ["3", "0", "3", None, "7", "0"],
        ["4", "5", None, "3", "0", "4"], ["5", "6", None, "4", "0", "5"], ["6", "7", None, "5", "0", "6"]]},
    # FixtureSupport.scala:205-214
    "dfWithDistinctValues": {"names": ["att1", "att2"], "types": [S, S], "rows": [
        ["a", None], ["a", None], [None, "x"], ["b", "x"], ["b", "x"], ["c", "y"]]},
    # FixtureSupport.scala:216-223
    "dfWithConditionallyUninformativeColumns": {"names": ["att1", "att2"], "types": [I, I], "rows": [
        [1, 0], [2, 0], [3, 0]]},
    # FixtureSupport.scala:225-232
    "dfWithConditionallyInformativeColumns": {"names": ["att1", "att2"], "types": [I, I], "rows": [
        [1, 4], [2, 5], [3, 6]]},
    # FixtureSupport.scala:64-72
    "dfWithNegativeNumbers": {"names": ["item", "att1", "att2"], "types": [S, S, S], "rows": [
        ["1", "-1", "-1.0"], ["2", "-2", "-2.0"], ["3", "-3", "-3.0"], ["4", "-4", "-4.0"]]},
    # FixtureSupport.scala:74-84
    "dfCompleteAndInCompleteColumns": {"names": ["item", "att1", "att2"], "types": [S, S, S], "rows": [
        ["1", "a", "f"], ["2", "b", "d"], ["3", "a", None], ["4", "a", "f"], ["5", "b", None], ["6", "a", "f"]]},
    # T/analyzers/AnalyzerTests.scala:488-504 (DecimalType.SYSTEM_DEFAULT, values 123.45, 99, 678)
    "dfDecimal": {"names": ["num"], "types": ["decimal"], "rows": [["123.45"], ["99"], ["678"]]},
    # T/analyzers/NullHandlingTests.scala:40-52: all-null columns of every type, 8 rows
    "dfAllNull": {"names": ["stringCol", "numericCol", "numericCol2", "numericCol3"], "types": [S, D, D, D],
                  "rows": [[None, None, None, float(i)] for i in range(1, 9)]},
    # FixtureSupport.scala:259-268
    "dfWithVariableStringLengthValues": {"names": ["att1"], "types": [S], "rows": [[""], ["a"], ["bb"], ["ccc"],
                                                                                  ["dddd"]]},
    # FixtureSupport.scala:110-135
    "dfFractionalIntegralTypes": {"names": ["item", "att1"], "types": [S, S], "rows": [["1", "1.0"], ["2", "1"]]},
    "dfFractionalStringTypes": {"names": ["item", "att1"], "types": [S, S], "rows": [["1", "1.0"], ["2", "a"]]},
    "dfIntegralStringTypes": {"names": ["item", "att1"], "types": [S, S], "rows": [["1", "1"], ["2", "a"]]},
    # T/analyzers/AnalyzerTests.scala:320-343: att1 cast to FloatType / StringType
    "dfWithNumericValuesCast": {"names": ["item", "att1_float", "att1_str"], "types": [S, "float", S], "rows": [
        [str(i), float(i), str(i)] for i in range(1, 7)]},
    "dfWithNumericFractionalValuesStr": {"names": ["item", "att1_str"], "types": [S, S], "rows": [
        [str(i), "%d.0" % i] for i in range(1, 7)]},
    # T/analyzers/AnalyzerTests.scala:389-420
    "dfBoolean": {"names": ["item", "att1"], "types": [S, S], "rows": [["1", "true"], ["2", "false"]]},
    "dfBooleanAndNull": {"names": ["item", "att1"], "types": [S, S], "rows": [
        ["1", "true"], ["2", "false"], ["3", None], ["4", "2.0"]]},
    # T/analyzers/AnalyzerTests.scala:662-760 (dataFrameWithColumn("some", ...))
    "dfPatternDoubles": {"names": ["some"], "types": [D], "rows": [[1.1], [None], [3.2], [4.4]]},
    "dfPatternInts": {"names": ["some"], "types": [S], "rows": [["1"], ["a"]]},
    "dfPatternEmail": {"names": ["some"], "types": [S], "rows": [["someone@somewhere.org"], ["someone@else"]]},
    "dfPatternCreditCard": {"names": ["some"], "types": [S], "rows": [[x] for x in [
        "378282246310005", "6011111111111117", "6011 1111 1111 1117", "6011-1111-1111-1117", "5555555555554444",
        "5555 5555 5555 4444", "5555-5555-5555-4444", "4111111111111111", "4111 1111 1111 1111",
        "4111-1111-1111-1111", "0000111122223333", "000011112222333", "00001111222233"]]},
    "dfPatternURL": {"names": ["some"], "types": [S], "rows": [[x] for x in [
        "http://foo.com/blah_blah", "http://foo.com/blah_blah_(wikipedia)",
        "http://foo.bar/?q=Test%20URL-encoded%20stuff", "http://\u27a1.ws/\u4a39", "http://\u2318.ws/",
        "http://\u263a.damowmow.com/", "http://\u4f8b\u5b50.\u6d4b\u8bd5", "https://foo_bar.example.com/",
        "http://userid@example.com:8080", "http://foo.com/blah_(wikipedia)#cite-1", "http://../", "h://test",
        "http://.www.foo.bar/"]]},
    "dfPatternSSN": {"names": ["some"], "types": [S], "rows": [[x] for x in [
        "111-05-1130", "111051130", "111-05-000", "111-00-000", "000-05-1130", "666-05-1130", "900-05-1130",
        "999-05-1130"]]},
    # T/analyzers/AnalyzerTests.scala:568-601: sparkContext.range(-1000L, 1000L).toDF("att1")
    "dfRange": {"names": ["att1"], "types": [L], "rows": [[i] for i in range(-1000, 1000)]},
}

ENT = -(0.75 * math.log(0.75) + 0.25 * math.log(0.25))


def dt(**kw):
    """distributionFrom (T/analyzers/AnalyzerTests.scala:271-291): the given classes, zeros elsewhere."""
    return {"datatype": {k: list(v) for k, v in kw.items()}}

# (fixture, analyzer spec, expected) — analyzer spec: [class, args...]; expected: number | "NaN" |
# {"failure": ExceptionName} | {"bins": n, "keys": [...]}
KATS = [
    # T/analyzers/AnalyzerTests.scala:33-42
    ("dfMissing", ["Size"], 12.0, "T/analyzers/AnalyzerTests.scala:37"),
    ("dfFull", ["Size"], 4.0, "T/analyzers/AnalyzerTests.scala:39"),
    # :45-74
    ("dfMissing", ["Completeness", "att1"], 0.5, "T/analyzers/AnalyzerTests.scala:51"),
    ("dfMissing", ["Completeness", "att2"], 0.75, "T/analyzers/AnalyzerTests.scala:53"),
    ("dfMissing", ["Completeness", "someMissingColumn"], {"failure": "NoSuchColumnException"},
     "T/analyzers/AnalyzerTests.scala:57-66"),
    ("dfMissing", ["Completeness", "att1", "item IN ('1', '2')"], 1.0, "T/analyzers/AnalyzerTests.scala:68-73"),
    # :78-131
    ("dfMissing", ["Uniqueness", ["att1"]], 0.0, "T/analyzers/AnalyzerTests.scala:83"),
    ("dfMissing", ["Uniqueness", ["att2"]], 0.0, "T/analyzers/AnalyzerTests.scala:85"),
    ("dfFull", ["Uniqueness", ["att1"]], 0.25, "T/analyzers/AnalyzerTests.scala:89"),
    ("dfFull", ["Uniqueness", ["att2"]], 0.25, "T/analyzers/AnalyzerTests.scala:91"),
    ("dfWithUniqueColumns", ["Uniqueness", ["unique"]], 1.0, "T/analyzers/AnalyzerTests.scala:98"),
    ("dfWithUniqueColumns", ["Uniqueness", ["uniqueWithNulls"]], 1.0, "T/analyzers/AnalyzerTests.scala:100"),
    ("dfWithUniqueColumns", ["Uniqueness", ["unique", "nonUnique"]], 1.0, "T/analyzers/AnalyzerTests.scala:102"),
    ("dfWithUniqueColumns", ["Uniqueness", ["unique", "nonUniqueWithNulls"]], 1.0,
     "T/analyzers/AnalyzerTests.scala:104"),
    ("dfWithUniqueColumns", ["Uniqueness", ["nonUnique", "onlyUniqueWithOtherNonUnique"]], 1.0,
     "T/analyzers/AnalyzerTests.scala:107"),
    ("dfWithUniqueColumns", ["Uniqueness", ["nonExistingColumn"]], {"failure": "NoSuchColumnException"},
     "T/analyzers/AnalyzerTests.scala:116-122"),
    # :133-145
    ("dfFull", ["Entropy", "att1"], ENT, "T/analyzers/AnalyzerTests.scala:137-139"),
    ("dfFull", ["Entropy", "att2"], ENT, "T/analyzers/AnalyzerTests.scala:140-142"),
    # :147-169
    ("dfFull", ["MutualInformation", ["att1", "att2"]], ENT, "T/analyzers/AnalyzerTests.scala:149-152"),
    ("dfWithConditionallyUninformativeColumns", ["MutualInformation", ["att1", "att2"]], 0.0,
     "T/analyzers/AnalyzerTests.scala:155-156"),
    # :171-198
    ("dfWithNumericValues", ["Compliance", "rule1", "att1 > 3"], 3.0 / 6, "T/analyzers/AnalyzerTests.scala:174-175"),
    ("dfWithNumericValues", ["Compliance", "rule2", "att1 > 2"], 4.0 / 6, "T/analyzers/AnalyzerTests.scala:176-177"),
    ("dfWithNumericValues", ["Compliance", "rule1", "att2 = 0", "att1 < 4"], 1.0,
     "T/analyzers/AnalyzerTests.scala:183-185"),
    ("dfWithNumericValues", ["Compliance", "rule1", "attNoSuchColumn > 3"], {"failure": "*"},
     "T/analyzers/AnalyzerTests.scala:188-197"),
    # :201-264
    ("dfMissing", ["Histogram", "att1"], {"bins": 3, "keys": ["a", "b", "NullValue"]},
     "T/analyzers/AnalyzerTests.scala:202-212"),
    ("dfWithNumericValues", ["Histogram", "att2"], {"bins": 4, "nkeys": 4}, "T/analyzers/AnalyzerTests.scala:215-224"),
    ("dfMissing", ["Histogram", "att1", 2], {"bins": 3, "keys": ["a", "NullValue"]},
     "T/analyzers/AnalyzerTests.scala:246-257"),
    ("dfFull", ["Histogram", "att1", 1001], {"failure": "IllegalAnalyzerParameterException"},
     "T/analyzers/AnalyzerTests.scala:259-264"),
    # :423-486 and T/analyzers/AnalysisTest.scala:70-97
    ("dfWithNumericValues", ["Mean", "att1"], 3.5, "T/analyzers/AnalyzerTests.scala:424-428"),
    ("dfFull", ["Mean", "att1"], {"failure": "WrongColumnTypeException"}, "T/analyzers/AnalyzerTests.scala:429-432"),
    ("dfWithNumericValues", ["Mean", "att1", "item != '6'"], 3.0, "T/analyzers/AnalyzerTests.scala:433-438"),
    ("dfWithNumericValues", ["StandardDeviation", "att1"], 1.707825127659933,
     "T/analyzers/AnalyzerTests.scala:440-444"),
    ("dfWithNumericValues", ["Minimum", "att1"], 1.0, "T/analyzers/AnalyzerTests.scala:450-454"),
    ("dfWithNumericValues", ["Maximum", "att1"], 6.0, "T/analyzers/AnalyzerTests.scala:460-464"),
    ("dfWithNumericValues", ["Maximum", "att1", "item != '6'"], 5.0, "T/analyzers/AnalyzerTests.scala:466-471"),
    ("dfWithNumericValues", ["Sum", "att1"], 21.0, "T/analyzers/AnalyzerTests.scala:478-481"),
    ("dfFull", ["Sum", "att1"], {"failure": "WrongColumnTypeException"}, "T/analyzers/AnalyzerTests.scala:483-486"),
    ("dfDecimal", ["Minimum", "num"], 99.0, "T/analyzers/AnalyzerTests.scala:488-504"),
    ("dfWithNumericValues", ["ApproxCountDistinct", "att1"], 6.0, "T/analyzers/AnalysisTest.scala:91-92"),
    ("dfWithNumericValues", ["CountDistinct", ["att1"]], 6.0, "T/analyzers/AnalysisTest.scala:93-94"),
    # :543-565
    ("dfWithUniqueColumns", ["ApproxCountDistinct", "uniqueWithNulls"], 5.0, "T/analyzers/AnalyzerTests.scala:544-548"),
    ("dfWithUniqueColumns", ["ApproxCountDistinct", "uniqueWithNulls", "unique < 4"], 2.0,
     "T/analyzers/AnalyzerTests.scala:550-557"),
    ("dfWithUniqueColumns", ["CountDistinct", ["uniqueWithNulls"]], 5.0, "T/analyzers/AnalyzerTests.scala:560-565"),
    # :638-657
    ("dfWithConditionallyUninformativeColumns", ["Correlation", "att1", "att2"], "NaN",
     "T/analyzers/AnalyzerTests.scala:639-643"),
    ("dfWithConditionallyInformativeColumns", ["Correlation", "att1", "att2"], 1.0,
     "T/analyzers/AnalyzerTests.scala:644-652"),
    ("dfWithConditionallyInformativeColumns", ["Correlation", "att2", "att1"], 1.0,
     "T/analyzers/AnalyzerTests.scala:653-656"),
    # :294-420 DataType
    ("dfFull", ["DataType", "att1"], dt(String=(4, 1.0)), "T/analyzers/AnalyzerTests.scala:294-299"),
    ("dfWithNumericValues", ["DataType", "att1"], dt(Integral=(6, 1.0)), "T/analyzers/AnalyzerTests.scala:301-305"),
    ("dfWithNegativeNumbers", ["DataType", "att1"], dt(Integral=(4, 1.0)), "T/analyzers/AnalyzerTests.scala:307-311"),
    ("dfWithNegativeNumbers", ["DataType", "att2"], dt(Fractional=(4, 1.0)),
     "T/analyzers/AnalyzerTests.scala:313-318"),
    ("dfWithNumericValuesCast", ["DataType", "att1_float"], dt(Fractional=(6, 1.0)),
     "T/analyzers/AnalyzerTests.scala:321-327"),
    ("dfWithNumericValuesCast", ["DataType", "att1_str"], dt(Integral=(6, 1.0)),
     "T/analyzers/AnalyzerTests.scala:329-334"),
    ("dfWithNumericFractionalValuesStr", ["DataType", "att1_str"], dt(Fractional=(6, 1.0)),
     "T/analyzers/AnalyzerTests.scala:336-343"),
    ("dfFractionalIntegralTypes", ["DataType", "att1"], dt(Fractional=(1, 0.5), Integral=(1, 0.5)),
     "T/analyzers/AnalyzerTests.scala:352-360"),
    ("dfFractionalStringTypes", ["DataType", "att1"], dt(Fractional=(1, 0.5), String=(1, 0.5)),
     "T/analyzers/AnalyzerTests.scala:362-370"),
    ("dfIntegralStringTypes", ["DataType", "att1"], dt(Integral=(1, 0.5), String=(1, 0.5)),
     "T/analyzers/AnalyzerTests.scala:372-380"),
    ("dfWithUniqueColumns", ["DataType", "uniqueWithNulls"], dt(Unknown=(1, 1.0 / 6.0), Integral=(5, 5.0 / 6.0)),
     "T/analyzers/AnalyzerTests.scala:382-390"),
    ("dfBoolean", ["DataType", "att1"], dt(Boolean=(2, 1.0)), "T/analyzers/AnalyzerTests.scala:392-402"),
    ("dfBooleanAndNull", ["DataType", "att1"], dt(Fractional=(1, 0.25), Unknown=(1, 0.25), Boolean=(2, 0.5)),
     "T/analyzers/AnalyzerTests.scala:404-420"),
    # :506-540 MinLength / MaxLength
    ("dfWithVariableStringLengthValues", ["MinLength", "att1"], 0.0, "T/analyzers/AnalyzerTests.scala:506-510"),
    ("dfWithVariableStringLengthValues", ["MinLength", "att1", "att1 != ''"], 1.0,
     "T/analyzers/AnalyzerTests.scala:512-517"),
    ("dfWithNumericValues", ["MinLength", "att1"], {"failure": "WrongColumnTypeException"},
     "T/analyzers/AnalyzerTests.scala:519-522"),
    ("dfWithVariableStringLengthValues", ["MaxLength", "att1"], 4.0, "T/analyzers/AnalyzerTests.scala:524-528"),
    ("dfWithVariableStringLengthValues", ["MaxLength", "att1", "att1 != 'dddd'"], 3.0,
     "T/analyzers/AnalyzerTests.scala:530-535"),
    ("dfWithNumericValues", ["MaxLength", "att1"], {"failure": "WrongColumnTypeException"},
     "T/analyzers/AnalyzerTests.scala:537-540"),
    # :662-760 PatternMatch (Patterns = A/PatternMatch.scala:57-72)
    ("dfPatternDoubles", ["PatternMatch", "some", "\\d\\.\\d"], 0.75, "T/analyzers/AnalyzerTests.scala:665-669"),
    ("dfPatternInts", ["PatternMatch", "some", "\\d"], 0.5, "T/analyzers/AnalyzerTests.scala:671-674"),
    ("dfPatternEmail", ["PatternMatch", "some", "@EMAIL"], 0.5, "T/analyzers/AnalyzerTests.scala:676-680"),
    ("dfPatternCreditCard", ["PatternMatch", "some", "@CREDITCARD"], 10.0 / 13.0,
     "T/analyzers/AnalyzerTests.scala:682-707"),
    ("dfPatternURL", ["PatternMatch", "some", "@URL"], 10.0 / 13.0, "T/analyzers/AnalyzerTests.scala:709-736"),
    ("dfPatternSSN", ["PatternMatch", "some", "@SOCIAL_SECURITY_NUMBER_US"], 2.0 / 8.0,
     "T/analyzers/AnalyzerTests.scala:738-754"),
    # :568-601 ApproxQuantile (bounds only: the reference pins no digest values)
    ("dfRange", ["ApproxQuantile", "att1", 0.5], {"between": [-20, 20]}, "T/analyzers/AnalyzerTests.scala:568-579"),
    ("dfRange", ["ApproxQuantile", "att1", 0.25], {"between": [-520, -480]},
     "T/analyzers/AnalyzerTests.scala:581-590"),
    ("dfRange", ["ApproxQuantile", "att1", 0.75], {"between": [480, 520]}, "T/analyzers/AnalyzerTests.scala:592-601"),
    ("dfWithNumericValues", ["ApproxQuantile", "att1", 0.5, 1.1], {"failure": "IllegalAnalyzerParameterException"},
     "T/analyzers/AnalyzerTests.scala:603-610"),
    ("dfWithNumericValues", ["ApproxQuantile", "att1", 0.5, -0.1], {"failure": "IllegalAnalyzerParameterException"},
     "T/analyzers/AnalyzerTests.scala:611-618"),
    ("dfWithNumericValues", ["ApproxQuantile", "att1", -0.1], {"failure": "IllegalAnalyzerParameterException"},
     "T/analyzers/AnalyzerTests.scala:619-627"),
    ("dfWithNumericValues", ["ApproxQuantile", "att1", 1.1], {"failure": "IllegalAnalyzerParameterException"},
     "T/analyzers/AnalyzerTests.scala:628-635"),
    # T/analyzers/NullHandlingTests.scala:54-141 (all-null columns)
    ("dfAllNull", ["Size"], 8.0, "T/analyzers/NullHandlingTests.scala:95"),
    ("dfAllNull", ["Completeness", "stringCol"], 0.0, "T/analyzers/NullHandlingTests.scala:96"),
    ("dfAllNull", ["Mean", "numericCol"], {"failure": "EmptyStateException"}, "T/analyzers/NullHandlingTests.scala:97"),
    ("dfAllNull", ["StandardDeviation", "numericCol"], {"failure": "EmptyStateException"},
     "T/analyzers/NullHandlingTests.scala:98"),
    ("dfAllNull", ["Minimum", "numericCol"], {"failure": "EmptyStateException"},
     "T/analyzers/NullHandlingTests.scala:99"),
    ("dfAllNull", ["Maximum", "numericCol"], {"failure": "EmptyStateException"},
     "T/analyzers/NullHandlingTests.scala:100"),
    ("dfAllNull", ["Sum", "numericCol"], {"failure": "EmptyStateException"}, "T/analyzers/NullHandlingTests.scala:101"),
    ("dfAllNull", ["Correlation", "numericCol", "numericCol2"], {"failure": "EmptyStateException"},
     "T/analyzers/NullHandlingTests.scala:104"),
    ("dfAllNull", ["CountDistinct", ["stringCol"]], 0.0, "T/analyzers/NullHandlingTests.scala:117"),
    ("dfAllNull", ["ApproxCountDistinct", "stringCol"], 0.0, "T/analyzers/NullHandlingTests.scala:119"),
    ("dfAllNull", ["Uniqueness", ["stringCol"]], {"failure": "EmptyStateException"},
     "T/analyzers/NullHandlingTests.scala:120"),
    ("dfAllNull", ["Entropy", "stringCol"], {"failure": "EmptyStateException"},
     "T/analyzers/NullHandlingTests.scala:123"),
    ("dfAllNull", ["MutualInformation", ["numericCol", "numericCol2"]], {"failure": "EmptyStateException"},
     "T/analyzers/NullHandlingTests.scala:124"),
    ("dfAllNull", ["MutualInformation", ["numericCol", "numericCol3"]], {"failure": "EmptyStateException"},
     "T/analyzers/NullHandlingTests.scala:125"),
    ("dfAllNull", ["Correlation", "numericCol", "numericCol3"], {"failure": "EmptyStateException"},
     "T/analyzers/NullHandlingTests.scala:127"),
    ("dfAllNull", ["ApproxQuantile", "numericCol", 0.5], {"failure": "EmptyStateException"},
     "T/analyzers/NullHandlingTests.scala:113"),
    ("dfAllNull", ["MinLength", "stringCol"], {"failure": "EmptyStateException"},
     "T/analyzers/NullHandlingTests.scala:105"),
    ("dfAllNull", ["MaxLength", "stringCol"], {"failure": "EmptyStateException"},
     "T/analyzers/NullHandlingTests.scala:106"),
    ("dfAllNull", ["DataType", "stringCol"], dt(Unknown=(8, 1.0)), "T/analyzers/NullHandlingTests.scala:108-109"),
]

# T/analyzers/IncrementalAnalyzerTest.scala:31-268 — states of two partitions merged.
INCREMENTAL = {
    # initialData (:243-255) / deltaData (:257-268)
    "initial": {"names": ["item", "att1", "count"], "types": [S, S, I], "rows": [
        ["1", "a", 12], ["2", None, 12], ["3", "b", 12]]},
    "delta": {"names": ["item", "att1", "count"], "types": [S, S, I], "rows": [
        ["4", "b", 12], ["5", None, 12]]},
    "cases": [
        (["Size"], 3.0, 2.0, 5.0, "T/analyzers/IncrementalAnalyzerTest.scala:33-52"),
        (["Compliance", "att1", "att1 = 'b'"], 0.3333333333333333, 0.5, 0.4,
         "T/analyzers/IncrementalAnalyzerTest.scala:55-75"),
        (["Completeness", "att1"], 0.6666666666666666, 0.5, 0.6, "T/analyzers/IncrementalAnalyzerTest.scala:78-98"),
        (["Uniqueness", ["att1"]], 1.0, 1.0, 1.0 / 3, "T/analyzers/IncrementalAnalyzerTest.scala:101-121"),
        (["Uniqueness", ["att1", "count"]], 1.0, 1.0, 0.2, "T/analyzers/IncrementalAnalyzerTest.scala:123-145"),
    ],
}


def main():
    doc = {"fixtures": FIXTURES,
           "kats": [{"fixture": f, "analyzer": a, "expected": e, "source": s} for f, a, e, s in KATS],
           "incremental": INCREMENTAL}
    with open(os.path.join(HERE, "kats.json"), "w") as fh:
        json.dump(doc, fh, indent=1)
    print("wrote %d KATs" % len(KATS))


if __name__ == "__main__":
    main()
