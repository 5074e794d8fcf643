"""deequ_amd — MI355X-native engine for deequ's AnalysisRunner metric computation.

The analyzer / state / metric API mirrors com.amazon.deequ.analyzers; the
per-row work runs in hand-written HIP kernels for gfx950 behind the C-ABI in include/dq.h.
"""
from .metrics import (Entity, DoubleMetric, HistogramMetric, KeyedDoubleMetric, Distribution, DistributionValue, Success, Failure,
                      MetricCalculationException, MetricCalculationRuntimeException, EmptyStateException,
                      NoSuchColumnException, WrongColumnTypeException, NoColumnsSpecifiedException,
                      NumberOfSpecifiedColumnsException, IllegalAnalyzerParameterException)
from .states import (NumMatches, NumMatchesAndCount, MeanState, SumState, MinState, MaxState,
                     StandardDeviationState, CorrelationState, ApproxCountDistinctState,
                     ApproxQuantileState, DataTypeHistogram)
from .analyzers import (Size, Completeness, Compliance, Mean, Sum, Minimum, Maximum, StandardDeviation, Correlation,
                        ApproxCountDistinct, ApproxQuantile, ApproxQuantiles, MinLength, MaxLength, DataType,
                        PatternMatch, Patterns, KLLSketch,
                        Uniqueness, Distinctness, UniqueValueRatio, Entropy, CountDistinct,
                        MutualInformation, Histogram, FrequenciesAndNumRows, Preconditions, computeFrequencies)
from .kll import (KLLParameters, KLLState, KLLMetric, BucketDistribution, BucketValue, QuantileNonSample)
from .runners import (AnalysisRunner, KLLRunner, AnalysisRunBuilder, AnalyzerContext, Analysis, InMemoryStateProvider,
                      ScanBatch)
from .checks import (Check, CheckLevel, CheckStatus, ConstraintStatus, ConstrainableDataTypes, VerificationSuite,
                     VerificationResult)
from .table import ChunkedTable, Table, Column
from .profiles import (ColumnProfiler, ColumnProfilerRunner, ColumnProfilerRunBuilder, ColumnProfiles,
                       StandardColumnProfile, NumericColumnProfile, DataTypeInstances)
from .state_provider import HdfsStateProvider, FileSystemStateProvider
from . import distributed

__all__ = [n for n in dir() if not n.startswith("_")]
