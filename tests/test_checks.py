"""Check / Constraint evaluation (M/checks/Check.scala, M/constraints/AnalysisBasedConstraint.scala) on
precomputed metrics: host logic only, no GPU. Messages follow the reference's formats."""
import deequ_amd as D
from deequ_amd.checks import AnalysisBasedConstraint, CheckWithLastConstraintFilterable
from deequ_amd.metrics import DoubleMetric, Entity, Success, Failure, EmptyStateException
from deequ_amd.runners import AnalyzerContext


def ctx_of(pairs):
    m = {}
    for a, v in pairs:
        m[a] = DoubleMetric(Entity.Column, type(a).__name__, "x", v if isinstance(v, (Success, Failure)) else Success(v))
    return AnalyzerContext(m)


def test_basic_constraint_results_and_messages():
    chk = (D.Check(D.CheckLevel.Error, "integrity")
           .hasSize(lambda n: n == 5).isComplete("id").isComplete("productName"))
    c = ctx_of([(D.Size(), 5.0), (D.Completeness("id"), 1.0), (D.Completeness("productName"), 0.8)])
    r = chk.evaluate(c)
    assert r.status == D.CheckStatus.Error
    st = [(str(x.constraint), x.status.value, x.message) for x in r.constraintResults]
    assert st[0] == ("SizeConstraint(Size(None))", "Success", None)
    assert st[2] == ("CompletenessConstraint(Completeness(productName,None))", "Failure",
                     "Value: 0.8 does not meet the constraint requirement!")


def test_warning_level_missing_analysis_and_failed_metric():
    chk = D.Check(D.CheckLevel.Warning, "w").hasMean("a", lambda v: v > 0).hasSum("b", lambda v: v > 0, hint="h!")
    c = ctx_of([(D.Mean("a"), Failure(EmptyStateException("Empty state for analyzer Mean(a,None)")))])
    r = chk.evaluate(c)
    assert r.status == D.CheckStatus.Warning
    assert r.constraintResults[0].message == "Empty state for analyzer Mean(a,None)"
    assert r.constraintResults[1].message == AnalysisBasedConstraint.MissingAnalysis


def test_where_replaces_the_last_constraint_and_required_analyzers():
    chk = D.Check(D.CheckLevel.Error, "c").isComplete("a").hasCompleteness("b", lambda v: v > 0.5)
    assert isinstance(chk, CheckWithLastConstraintFilterable)
    chk = chk.where("k > 1")
    assert D.Completeness("b", "k > 1") in chk.requiredAnalyzers()
    assert D.Completeness("a") in chk.requiredAnalyzers()
    assert len(chk.requiredAnalyzers()) == 2


def test_datatype_ratio_picker():
    from deequ_amd.states import DataTypeHistogram
    dist = DataTypeHistogram(2, 1, 3, 0, 0).toDistribution()
    m = {D.DataType("x"): D.HistogramMetric("x", Success(dist))}
    chk = D.Check(D.CheckLevel.Error, "t").hasDataType("x", D.ConstrainableDataTypes.Integral, lambda v: v == 0.75)
    assert chk.evaluate(AnalyzerContext(m)).status == D.CheckStatus.Success
    chk = D.Check(D.CheckLevel.Error, "t").hasDataType("x", D.ConstrainableDataTypes.Null, lambda v: v == 2 / 6)
    assert chk.evaluate(AnalyzerContext(m)).status == D.CheckStatus.Success


def test_contained_in_predicates():
    chk = D.Check(D.CheckLevel.Error, "c").isContainedIn("p", ["high", "lo'w"])
    comp = chk.requiredAnalyzers()[0]
    assert comp.predicate == "`p` IS NULL OR `p` IN ('high','lo''w')"
    chk = D.Check(D.CheckLevel.Error, "c").isContainedIn("v", lowerBound=0, upperBound=10, includeUpperBound=False)
    assert chk.requiredAnalyzers()[0].predicate == "`v` IS NULL OR (`v` >= 0.0 AND `v` < 10.0)"
