"""BASELINE config 1 end to end on the GPU: the reference's BasicExample VerificationSuite
(src/main/scala/com/amazon/deequ/examples/BasicExample.scala:26-72) and the Size / Completeness /
Uniqueness / ApproxQuantile suite on test-data/titanic.csv (tests/golden/titanic.csv), with the
expectations of T/profiles/ColumnProfilerTest.scala:403-460 and SURVEY.md §8c item 3."""
import os

import numpy as np
import pytest

import deequ_amd as D
from deequ_amd.table import Table
import oracle as O

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def items():
    # ExampleUtils.itemsAsDataframe: Item(id: Long, productName, description, priority, numViews: Long)
    rows = [(1, "Thingy A", "awesome thing.", "high", 0),
            (2, "Thingy B", "available at http://thingb.com", None, 0),
            (3, None, None, "low", 5),
            (4, "Thingy D", "checkout https://thingd.ca", "low", 10),
            (5, "Thingy E", None, "high", 12)]
    return Table.from_rows(rows, ["id", "productName", "description", "priority", "numViews"],
                           ["long", "string", "string", "string", "long"])


def test_basic_example_verification():
    result = (D.VerificationSuite().onData(items())
              .addCheck(D.Check(D.CheckLevel.Error, "integrity checks")
                        .hasSize(lambda n: n == 5).isComplete("id").isUnique("id").isComplete("productName")
                        .isContainedIn("priority", ["high", "low"]).isNonNegative("numViews"))
              .addCheck(D.Check(D.CheckLevel.Warning, "distribution checks")
                        .containsURL("description", lambda v: v >= 0.5)
                        .hasApproxQuantile("numViews", 0.5, lambda v: v <= 10))
              .run())
    assert result.status == D.CheckStatus.Error
    failed = sorted((str(r.constraint), r.message) for cr in result.checkResults.values()
                    for r in cr.constraintResults if r.status == D.ConstraintStatus.Failure)
    # the two failures the reference's example prints (deequ README, "Unit tests for data")
    assert failed == [
        ("CompletenessConstraint(Completeness(productName,None))",
         "Value: 0.8 does not meet the constraint requirement!"),
        ("containsURL(description)", "Value: 0.4 does not meet the constraint requirement!")]


def titanic():
    return Table.from_csv(os.path.join(HERE, "golden", "titanic.csv"))


def test_titanic_config1_suite():
    t = titanic()
    assert t.schema["PassengerId"] == "IntegerType" and t.schema["Fare"] == "DoubleType"
    chk = (D.Check(D.CheckLevel.Error, "titanic")
           .hasSize(lambda n: n == 891)
           .isComplete("PassengerId")
           .hasCompleteness("Age", lambda v: v == 714 / 891)
           .hasCompleteness("Cabin", lambda v: v == 204 / 891)
           .hasCompleteness("Embarked", lambda v: v == 889 / 891)
           .isUnique("PassengerId")
           .hasUniqueness(["Ticket"], lambda v: 0.0 < v < 1.0)
           .hasApproxQuantile("Fare", 0.5, lambda v: True)
           .hasApproxQuantile("Age", 0.5, lambda v: True))
    result = D.VerificationSuite().onData(t).addCheck(chk).run()
    bad = [(str(r.constraint), r.message) for r in result.checkResults[chk].constraintResults
           if r.status != D.ConstraintStatus.Success]
    assert not bad, bad
    m = result.metrics
    # ApproxQuantile: Spark's single-partition digest (891 < 50000 rows); within the 1% rank bound of
    # the exact medians (Fare 14.4542, Age 28.0)
    for col, exact in (("Fare", 14.4542), ("Age", 28.0)):
        got = m[D.ApproxQuantile(col, 0.5)].value.get()
        s = O.java_sorted_doubles(t, col)
        lo, hi = O.rank_interval(s, got)
        target = int(np.ceil(0.5 * len(s)))
        assert lo - (np.ceil(0.01 * len(s)) + 1) <= target <= hi + np.ceil(0.01 * len(s)) + 1, (col, got, exact)
    # exact distinct counts of ColumnProfilerTest (±10 % there; exact here through the grouping path)
    ctx = D.AnalysisRunner.onData(t).addAnalyzers(
        [D.CountDistinct(["PassengerId"]), D.CountDistinct(["Ticket"]), D.CountDistinct(["Cabin"]),
         D.CountDistinct(["Sex"]), D.ApproxCountDistinct("Ticket")]).run()
    assert [ctx.metric(D.CountDistinct([c])).value.get() for c in ("PassengerId", "Ticket", "Cabin", "Sex")] == \
        [891.0, 681.0, 147.0, 2.0]
    assert abs(ctx.metric(D.ApproxCountDistinct("Ticket")).value.get() - 681) <= 0.1 * 681
