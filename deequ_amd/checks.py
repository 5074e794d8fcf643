"""VerificationSuite / Check / Constraint — deequ's declarative layer over the analyzers
(M/VerificationSuite.scala:44-315, M/checks/Check.scala:60-1056, M/constraints/Constraint.scala,
M/constraints/AnalysisBasedConstraint.scala), as a thin host layer: a run collects every check's
required analyzers and hands them to ONE AnalysisRunner.doAnalysisRun (so all scan-shareable
metrics of all checks come from one fused dq_scan), then evaluates the assertions on the metrics.
Anomaly detection, KLL sketches, metrics repositories and file output are out of scope.
"""
import enum

from . import analyzers as A
from .analyzers import _java_double_to_string
from .runners import AnalysisRunner, AnalyzerContext


class CheckLevel(enum.Enum):
    Error = "Error"
    Warning = "Warning"


class CheckStatus(enum.IntEnum):
    Success = 0
    Warning = 1
    Error = 2


class ConstraintStatus(enum.Enum):
    Success = "Success"
    Failure = "Failure"


def is_one(v):
    """Check.IsOne (M/checks/Check.scala: `_ == 1.0`)."""
    return v == 1.0


def _fmt(v):
    if isinstance(v, bool):
        return "true" if v else "false"
    if isinstance(v, float):
        return _java_double_to_string(v)
    return str(v)


class ConstraintResult:
    def __init__(self, constraint, status, message=None, metric=None):
        self.constraint, self.status, self.message, self.metric = constraint, status, message, metric

    def __repr__(self):
        return "ConstraintResult(%s,%s,%r)" % (self.constraint, self.status.value, self.message)


class AnalysisBasedConstraint:
    """M/constraints/AnalysisBasedConstraint.scala:33-110."""
    MissingAnalysis = "Missing Analysis, can't run the constraint!"
    ProblematicMetricPicker = "Can't retrieve the value to assert on"
    AssertionException = "Can't execute the assertion"

    def __init__(self, analyzer, assertion, value_picker=None, hint=None):
        self.analyzer, self.assertion, self.value_picker, self.hint = analyzer, assertion, value_picker, hint

    def evaluate(self, metric_map):
        metric = metric_map.get(self.analyzer)
        if metric is None:
            return ConstraintResult(self, ConstraintStatus.Failure, self.MissingAnalysis, None)
        if metric.value.isFailure:
            return ConstraintResult(self, ConstraintStatus.Failure, str(metric.value.failed), metric)
        try:
            value = self.value_picker(metric.value.get()) if self.value_picker else metric.value.get()
        except Exception as e:
            return ConstraintResult(self, ConstraintStatus.Failure, "%s: %s!" % (self.ProblematicMetricPicker, e),
                                    metric)
        try:
            ok = self.assertion(value)
        except Exception as e:
            return ConstraintResult(self, ConstraintStatus.Failure, "%s: %s!" % (self.AssertionException, e), metric)
        if ok:
            return ConstraintResult(self, ConstraintStatus.Success, None, metric)
        msg = "Value: %s does not meet the constraint requirement!" % _fmt(value)
        if self.hint:
            msg += " " + self.hint
        return ConstraintResult(self, ConstraintStatus.Failure, msg, metric)


class NamedConstraint:
    """M/constraints/Constraint.scala:50-62: the result's constraint is the named decorator."""

    def __init__(self, inner, name):
        self.inner, self.name = inner, name

    def evaluate(self, metric_map):
        r = self.inner.evaluate(metric_map)
        r.constraint = self
        return r

    def __repr__(self):
        return self.name


def _named(analyzer, assertion, name, picker=None, hint=None):
    return NamedConstraint(AnalysisBasedConstraint(analyzer, assertion, picker, hint), name)


def _ratio_types(ignore_unknown, key):
    """Constraint.ratioTypes (M/constraints/Constraint.scala:656-680)."""
    def pick(dist):
        if not ignore_unknown:
            v = dist.values.get(key)
            return 0.0 if v is None else v.ratio
        v = dist.values.get(key)
        count = 0 if v is None else v.absolute
        if count == 0:
            return 0.0
        total = sum(x.absolute for x in dist.values.values())
        unknown = dist.values.get("Unknown")
        return count / (total - (0 if unknown is None else unknown.absolute))
    return pick


class ConstrainableDataTypes(enum.Enum):
    Null = "Null"
    Fractional = "Fractional"
    Integral = "Integral"
    Boolean = "Boolean"
    String = "String"
    Numeric = "Numeric"


class CheckResult:
    def __init__(self, check, status, constraintResults):
        self.check, self.status, self.constraintResults = check, status, constraintResults


class Check:
    """M/checks/Check.scala:60-1056 (anomaly and KLL constraints excluded)."""

    def __init__(self, level, description, constraints=None):
        self.level, self.description = level, description
        self.constraints = list(constraints or [])

    def __repr__(self):
        return "Check(%s,%s,%r)" % (self.level.value, self.description, self.constraints)

    def addConstraint(self, constraint):
        return Check(self.level, self.description, self.constraints + [constraint])

    def _filterable(self, create):
        return CheckWithLastConstraintFilterable(self.level, self.description,
                                                 self.constraints + [create(None)], create)

    # ---- size / completeness / uniqueness ---------------------------------------------------
    def hasSize(self, assertion, hint=None):
        def mk(where):
            size = A.Size(where)
            return _named(size, assertion, "SizeConstraint(%r)" % size, lambda v: int(v), hint)
        return self._filterable(mk)

    def isComplete(self, column, hint=None):
        return self.hasCompleteness(column, is_one, hint)

    def hasCompleteness(self, column, assertion, hint=None):
        def mk(where):
            c = A.Completeness(column, where)
            return _named(c, assertion, "CompletenessConstraint(%r)" % c, hint=hint)
        return self._filterable(mk)

    def isUnique(self, column, hint=None):
        return self.hasUniqueness([column], is_one, hint)

    def isPrimaryKey(self, column, *columns):
        return self.hasUniqueness([column] + list(columns), is_one)

    def hasUniqueness(self, columns, assertion, hint=None):
        u = A.Uniqueness([columns] if isinstance(columns, str) else list(columns))
        return self.addConstraint(_named(u, assertion, "UniquenessConstraint(%r)" % u, hint=hint))

    def hasDistinctness(self, columns, assertion, hint=None):
        d = A.Distinctness(list(columns))
        return self.addConstraint(_named(d, assertion, "DistinctnessConstraint(%r)" % d, hint=hint))

    def hasUniqueValueRatio(self, columns, assertion, hint=None):
        u = A.UniqueValueRatio(list(columns))
        return self.addConstraint(_named(u, assertion, "UniqueValueRatioConstraint(%r" % u, hint=hint))

    def hasNumberOfDistinctValues(self, column, assertion, binningUdf=None,
                                  maxBins=A.Histogram.MaximumAllowedDetailBins, hint=None):
        h = A.Histogram(column, binningUdf, maxBins)
        return self.addConstraint(_named(h, assertion, "HistogramBinConstraint(%r)" % h,
                                         lambda d: d.numberOfBins, hint))

    def hasHistogramValues(self, column, assertion, binningUdf=None,
                           maxBins=A.Histogram.MaximumAllowedDetailBins, hint=None):
        h = A.Histogram(column, binningUdf, maxBins)
        return self.addConstraint(_named(h, assertion, "HistogramConstraint(%r)" % h, hint=hint))

    # ---- information ------------------------------------------------------------------------
    def hasEntropy(self, column, assertion, hint=None):
        e = A.Entropy(column)
        return self.addConstraint(_named(e, assertion, "EntropyConstraint(%r)" % e, hint=hint))

    def hasMutualInformation(self, columnA, columnB, assertion, hint=None):
        m = A.MutualInformation([columnA, columnB])
        return self.addConstraint(_named(m, assertion, "MutualInformationConstraint(%r)" % m, hint=hint))

    def hasApproxQuantile(self, column, quantile, assertion, hint=None):
        q = A.ApproxQuantile(column, quantile)
        return self.addConstraint(_named(q, assertion, "ApproxQuantileConstraint(%r)" % q, hint=hint))

    # ---- per-column statistics (filterable) -------------------------------------------------
    def _stat(self, cls, label, column, assertion, hint):
        def mk(where):
            a = cls(column, where)
            return _named(a, assertion, "%s(%r)" % (label, a), hint=hint)
        return self._filterable(mk)

    def hasMinLength(self, column, assertion, hint=None):
        return self._stat(A.MinLength, "MinLengthConstraint", column, assertion, hint)

    def hasMaxLength(self, column, assertion, hint=None):
        return self._stat(A.MaxLength, "MaxLengthConstraint", column, assertion, hint)

    def hasMin(self, column, assertion, hint=None):
        return self._stat(A.Minimum, "MinimumConstraint", column, assertion, hint)

    def hasMax(self, column, assertion, hint=None):
        return self._stat(A.Maximum, "MaximumConstraint", column, assertion, hint)

    def hasMean(self, column, assertion, hint=None):
        return self._stat(A.Mean, "MeanConstraint", column, assertion, hint)

    def hasSum(self, column, assertion, hint=None):
        return self._stat(A.Sum, "SumConstraint", column, assertion, hint)

    def hasStandardDeviation(self, column, assertion, hint=None):
        return self._stat(A.StandardDeviation, "StandardDeviationConstraint", column, assertion, hint)

    def hasApproxCountDistinct(self, column, assertion, hint=None):
        return self._stat(A.ApproxCountDistinct, "ApproxCountDistinctConstraint", column, assertion, hint)

    def hasCorrelation(self, columnA, columnB, assertion, hint=None):
        def mk(where):
            c = A.Correlation(columnA, columnB, where)
            return _named(c, assertion, "CorrelationConstraint(%r)" % c, hint=hint)
        return self._filterable(mk)

    # ---- predicates -------------------------------------------------------------------------
    def satisfies(self, columnCondition, constraintName, assertion=is_one, hint=None):
        def mk(where):
            c = A.Compliance(constraintName, columnCondition, where)
            return _named(c, assertion, "ComplianceConstraint(%r)" % c, hint=hint)
        return self._filterable(mk)

    def hasPattern(self, column, pattern, assertion=is_one, name=None, hint=None):
        pat = pattern.pattern if hasattr(pattern, "pattern") else str(pattern)

        def mk(where):
            p = A.PatternMatch(column, pat, where)
            return _named(p, assertion, name or "PatternMatchConstraint(%s, %s)" % (column, pat), hint=hint)
        return self._filterable(mk)

    def containsCreditCardNumber(self, column, assertion=is_one, hint=None):
        return self.hasPattern(column, A.Patterns.CREDITCARD, assertion, "containsCreditCardNumber(%s)" % column,
                               hint)

    def containsEmail(self, column, assertion=is_one, hint=None):
        return self.hasPattern(column, A.Patterns.EMAIL, assertion, "containsEmail(%s)" % column, hint)

    def containsURL(self, column, assertion=is_one, hint=None):
        return self.hasPattern(column, A.Patterns.URL, assertion, "containsURL(%s)" % column, hint)

    def containsSocialSecurityNumber(self, column, assertion=is_one, hint=None):
        return self.hasPattern(column, A.Patterns.SOCIAL_SECURITY_NUMBER_US, assertion,
                               "containsSocialSecurityNumber(%s)" % column, hint)

    def hasDataType(self, column, dataType, assertion=is_one, hint=None):
        """Constraint.dataTypeConstraint (M/constraints/Constraint.scala:592-614)."""
        if dataType == ConstrainableDataTypes.Null:
            picker = _ratio_types(False, "Unknown")
        elif dataType == ConstrainableDataTypes.Numeric:
            f, i = _ratio_types(True, "Fractional"), _ratio_types(True, "Integral")

            def picker(d):
                return f(d) + i(d)
        else:
            picker = _ratio_types(True, dataType.value)
        d = A.DataType(column)
        return self.addConstraint(AnalysisBasedConstraint(d, assertion, picker, hint))

    def isNonNegative(self, column, assertion=is_one, hint=None):
        return self.satisfies("COALESCE(%s, 0.0) >= 0" % column, "%s is non-negative" % column, assertion, hint)

    def isPositive(self, column, assertion=is_one, hint=None):
        return self.satisfies("COALESCE(%s, 1.0) > 0" % column, "%s is positive" % column, assertion, hint)

    def isLessThan(self, columnA, columnB, assertion=is_one, hint=None):
        return self.satisfies("%s < %s" % (columnA, columnB), "%s is less than %s" % (columnA, columnB), assertion,
                              hint)

    def isLessThanOrEqualTo(self, columnA, columnB, assertion=is_one, hint=None):
        return self.satisfies("%s <= %s" % (columnA, columnB), "%s is less than or equal to %s" % (columnA, columnB),
                              assertion, hint)

    def isGreaterThan(self, columnA, columnB, assertion=is_one, hint=None):
        return self.satisfies("%s > %s" % (columnA, columnB), "%s is greater than %s" % (columnA, columnB),
                              assertion, hint)

    def isGreaterThanOrEqualTo(self, columnA, columnB, assertion=is_one, hint=None):
        return self.satisfies("%s >= %s" % (columnA, columnB),
                              "%s is greater than or equal to %s" % (columnA, columnB), assertion, hint)

    def isContainedIn(self, column, allowedValues=None, assertion=is_one, hint=None, lowerBound=None,
                      upperBound=None, includeLowerBound=True, includeUpperBound=True):
        """Both isContainedIn variants (M/checks/Check.scala:844-948): a value list, or a numeric interval."""
        if lowerBound is not None or upperBound is not None:
            lo, hi = float(lowerBound), float(upperBound)
            pred = "`%s` IS NULL OR (`%s` %s %s AND `%s` %s %s)" % (
                column, column, ">=" if includeLowerBound else ">", _java_double_to_string(lo), column,
                "<=" if includeUpperBound else "<", _java_double_to_string(hi))
            return self.satisfies(pred, "%s between %s and %s" % (column, _java_double_to_string(lo),
                                                                  _java_double_to_string(hi)), hint=hint)
        values = ",".join("'%s'" % v.replace("'", "''") for v in allowedValues)
        pred = "`%s` IS NULL OR `%s` IN (%s)" % (column, column, values)
        return self.satisfies(pred, "%s contained in %s" % (column, ",".join(allowedValues)), assertion, hint)

    # ---- evaluation -------------------------------------------------------------------------
    def evaluate(self, context):
        """Check.evaluate (M/checks/Check.scala:950-962)."""
        results = [c.evaluate(context.metricMap) for c in self.constraints]
        failed = any(r.status == ConstraintStatus.Failure for r in results)
        if failed:
            status = CheckStatus.Error if self.level == CheckLevel.Error else CheckStatus.Warning
        else:
            status = CheckStatus.Success
        return CheckResult(self, status, results)

    def requiredAnalyzers(self):
        out = []
        for c in self.constraints:
            inner = c.inner if isinstance(c, NamedConstraint) else c
            if isinstance(inner, AnalysisBasedConstraint) and inner.analyzer not in out:
                out.append(inner.analyzer)
        return out


class CheckWithLastConstraintFilterable(Check):
    """M/checks/CheckWithLastConstraintFilterable.scala: `.where(filter)` rebuilds the last constraint."""

    def __init__(self, level, description, constraints, create):
        super().__init__(level, description, constraints)
        self._create = create

    def where(self, filter_):
        return Check(self.level, self.description, self.constraints[:-1] + [self._create(filter_)])


class VerificationResult:
    """M/VerificationResult.scala: overall status, per-check results and all metrics."""

    def __init__(self, status, checkResults, metrics):
        self.status, self.checkResults, self.metrics = status, checkResults, metrics

    @staticmethod
    def successMetricsAsJson(result, forAnalyzers=()):
        return AnalyzerContext.successMetricsAsJson(AnalyzerContext(result.metrics), forAnalyzers)


class VerificationRunBuilder:
    """M/VerificationRunBuilder.scala: onData(..).addCheck(..).addRequiredAnalyzer(..).run()."""

    def __init__(self, data):
        self.data = data
        self.checks = []
        self.requiredAnalyzers = []
        self._aggregateWith = None
        self._saveStatesWith = None

    def addCheck(self, check):
        self.checks.append(check)
        return self

    def addChecks(self, checks):
        self.checks.extend(checks)
        return self

    def addRequiredAnalyzer(self, analyzer):
        self.requiredAnalyzers.append(analyzer)
        return self

    def addRequiredAnalyzers(self, analyzers):
        self.requiredAnalyzers.extend(analyzers)
        return self

    def aggregateWith(self, stateLoader):
        self._aggregateWith = stateLoader
        return self

    def saveStatesWith(self, statePersister):
        self._saveStatesWith = statePersister
        return self

    def run(self):
        return VerificationSuite.doVerificationRun(self.data, self.checks, self.requiredAnalyzers,
                                                   self._aggregateWith, self._saveStatesWith)


class VerificationSuite:
    """M/VerificationSuite.scala:44-315."""

    def onData(self, data):
        return VerificationRunBuilder(data)

    @staticmethod
    def doVerificationRun(data, checks, requiredAnalyzers=(), aggregateWith=None, saveStatesWith=None):
        """M/VerificationSuite.scala:107-144: one analysis run for every check's analyzers."""
        analyzers = list(requiredAnalyzers) + [a for c in checks for a in c.requiredAnalyzers()]
        context = AnalysisRunner.doAnalysisRun(data, analyzers, aggregateWith, saveStatesWith)
        return VerificationSuite.evaluate(checks, context)

    @staticmethod
    def evaluate(checks, context):
        results = {c: c.evaluate(context) for c in checks}
        status = max([r.status for r in results.values()], default=CheckStatus.Success)
        return VerificationResult(status, results, context.metricMap)
