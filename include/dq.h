/*
 * dq.h — C-ABI of the MI355X-native deequ metrics engine (libdq.so).
 *
 * This is the drop-in boundary for deequ's AnalysisRunner hot path. The reference has no native
 * code: the seams replaced here are Scala methods, cited per entry point. A JVM host binds these
 * symbols over JNI; this repository's host mirror binds them over ctypes
 * (deequ_amd/native.py).
 *
 * Conventions
 *   - Plain C types only; no torch / HIP types cross this boundary (streams are `void*`).
 *   - Every call returns 0 (DQ_OK) on success or a negative dq_status; dq_last_error(ctx) then
 *     holds a message. A failed dq_scan fails EVERY op of the batch, mirroring the catch-all in
 *     runScanningAnalyzers (R/AnalysisRunner.scala:320-323).
 *   - A dq_ctx from dq_open is bound to one GPU; one from dq_open_devices spans several GPUs of the node. A ctx
 *     is not re-entrant: one driver thread per ctx. Several contexts of one GPU (each its own stream, scratch
 *     cache and pinned staging) may be driven by different threads at once: independent passes of one analysis
 *     then overlap on the device (the Python host runs grouping builds, histogram builds and the odd row chunks of
 *     a shard on helper contexts this way). Inputs are read-only to every context; a buffer one context's stream
 *     writes must not be read by another before that stream is synchronised.
 *   - States are returned in native byte order (little-endian on x86/MI355X hosts) with the
 *     field order of the reference's HdfsStateProvider layouts (A/StateProvider.scala:187-262).
 *
 * Path abbreviations: A/ = src/main/scala/com/amazon/deequ/analyzers/,
 * R/ = A/runners/, C/ = A/catalyst/ (all under /root/reference).
 */
#ifndef DEEQU_AMD_DQ_H
#define DEEQU_AMD_DQ_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DQ_ABI_VERSION 2

/* ---------------------------------------------------------------------------------------------
 * Status codes
 * ------------------------------------------------------------------------------------------- */
typedef enum dq_status {
    DQ_OK = 0,
    DQ_ERR_INVALID_ARGUMENT = -1,  /* bad op / column index / length mismatch          */
    DQ_ERR_UNSUPPORTED = -2,       /* op not defined for this Spark type               */
    DQ_ERR_DEVICE = -3,            /* HIP runtime error (message in dq_last_error)     */
    DQ_ERR_OUT_OF_MEMORY = -4,
    DQ_ERR_NO_DEVICE = -5,         /* no MI355X visible: the engine never falls back   */
    DQ_ERR_PREDICATE = -6,         /* malformed predicate program                      */
    DQ_ERR_ALIGNMENT = -7          /* device column not 16-B (values) / 8-B (bitmap) aligned */
} dq_status;

/* ---------------------------------------------------------------------------------------------
 * Columns: Arrow-style buffers carrying the *Spark* physical type. The type is mandatory because
 * HLL hashing (C/StatefulHyperloglogPlus.scala:93) and Sum/Min/Max result rules depend on it.
 * ------------------------------------------------------------------------------------------- */
typedef enum dq_spark_type {
    DQ_TYPE_BOOLEAN = 1,    /* uint8 0/1                                 */
    DQ_TYPE_BYTE = 2,       /* int8                                      */
    DQ_TYPE_SHORT = 3,      /* int16                                     */
    DQ_TYPE_INT = 4,        /* int32                                     */
    DQ_TYPE_LONG = 5,       /* int64                                     */
    DQ_TYPE_FLOAT = 6,      /* float32                                   */
    DQ_TYPE_DOUBLE = 7,     /* float64                                   */
    DQ_TYPE_STRING = 8,     /* UTF-8 bytes in `values`, int32 `offsets`  */
    DQ_TYPE_DATE = 9,       /* int32 days since epoch                    */
    DQ_TYPE_TIMESTAMP = 10, /* int64 microseconds since epoch            */
    DQ_TYPE_DECIMAL = 11    /* int64 unscaled value, precision <= 18     */
} dq_spark_type;

#define DQ_COL_DEVICE 0x1u /* values/validity/offsets are device pointers on the ctx's GPU */
/* STRING: `offsets` points to length + 1 int64 offsets (Arrow large_string) -- a column whose UTF-8 bytes pass
 * 2^31, e.g. the row chunks of a shard concatenated in HBM for one grouping build. Accepted by dq_frequencies(_ex)
 * only; every other entry point fails such a column with DQ_ERR_UNSUPPORTED. */
#define DQ_COL_OFFSETS64 0x2u

typedef struct dq_column {
    int32_t spark_type;        /* dq_spark_type                                               */
    uint32_t flags;            /* DQ_COL_*                                                    */
    int64_t length;            /* rows                                                        */
    const void* values;        /* fixed width: `length` elements; STRING: UTF-8 data bytes    */
    const uint8_t* validity;   /* Arrow LSB-first bitmap (bit i set = row i non-null), or NULL */
    const int32_t* offsets;    /* STRING only: length + 1 offsets into `values`                */
    int32_t decimal_precision; /* DECIMAL only                                                 */
    int32_t decimal_scale;     /* DECIMAL only                                                 */
} dq_column;

/* ---------------------------------------------------------------------------------------------
 * Predicates (`where` filters and Compliance predicates). deequ accepts Spark SQL strings
 * (A/Analyzer.scala:409-432, A/Compliance.scala:49-52); the host compiles them to this postfix
 * program, evaluated per row on the GPU with SQL three-valued logic.
 * ------------------------------------------------------------------------------------------- */
typedef enum dq_pred_opcode {
    DQ_P_COL = 1,        /* arg: column index          -> push column value (NULL if invalid) */
    DQ_P_CONST = 2,      /* arg: constant index        -> push constant                       */
    DQ_P_NULL = 3,       /*                            -> push NULL                           */
    DQ_P_EQ = 10, DQ_P_NE = 11, DQ_P_LT = 12, DQ_P_LE = 13, DQ_P_GT = 14, DQ_P_GE = 15,
    DQ_P_EQ_NULLSAFE = 16, /* <=>                                                              */
    DQ_P_AND = 20, DQ_P_OR = 21, DQ_P_NOT = 22,
    DQ_P_IS_NULL = 23, DQ_P_IS_NOT_NULL = 24,
    DQ_P_IN = 25,        /* arg: n                     -> x IN (v1..vn); n+1 operands          */
    DQ_P_COALESCE = 26,  /* arg: n operands                                                    */
    DQ_P_ADD = 30, DQ_P_SUB = 31, DQ_P_MUL = 32, DQ_P_DIV = 33, DQ_P_MOD = 34, DQ_P_NEG = 35,
    DQ_P_LIKE = 40,      /* arg: constant index of the pattern; 1 operand                      */
    DQ_P_LENGTH = 41,    /* UTF-8 character count                                             */
    DQ_P_CAST_DOUBLE = 42, DQ_P_CAST_LONG = 43, DQ_P_CAST_STRING_NUM = 44,
    /* PatternMatch (A/PatternMatch.scala:46-48): arg = index of a STRING constant holding a compiled
     * java.util.regex program (deequ_amd/regex.py image, 4-byte aligned in the pool); 1 operand.
     * TRUE when the first Matcher.find() match of the value's string form is non-empty, FALSE
     * otherwise, also for NULL (`when(regexp_extract(..) != "", 1).otherwise(0)`). Only as the whole
     * program [COL c, REGEX k], over STRING / integral / BOOLEAN columns. */
    DQ_P_REGEX = 45,
    /* str RLIKE regex (Spark RLike: Pattern.compile(regex).matcher(str).find(), any match): arg = index of a STRING
     * constant holding a compiled regex program (as DQ_P_REGEX); 1 operand, a non-string one as its Spark string
     * cast. NULL in -> NULL. */
    DQ_P_RLIKE = 46,
    DQ_P_LOWER = 47, DQ_P_UPPER = 48,  /* lower(str) / upper(str): simple Unicode case mappings                 */
    DQ_P_TRIM = 49,      /* arg 0 trim, 1 ltrim, 2 rtrim (ASCII spaces, Spark 2.2 UTF8String.trim)                 */
    DQ_P_CASE = 50,      /* CASE WHEN c1 THEN v1 .. [ELSE e] END: arg = 2 * #WHEN + has ELSE; operands c1 v1 .. [e] */
    DQ_P_ISNAN = 51,     /* isnan(x): never NULL                                                                  */
    DQ_P_ABS = 52,
    DQ_P_SUBSTR = 53,    /* substring(str, pos, len): 3 operands, UTF8String.substringSQL                          */
    DQ_P_YEAR = 54, DQ_P_MONTH = 55, DQ_P_DAY = 56, /* arg 0: DATE days, 1: TIMESTAMP micros (UTC session zone)  */
    DQ_P_NANVL = 57      /* nanvl(a, b): 2 operands                                                               */
} dq_pred_opcode;

typedef enum dq_value_tag { DQ_V_BOOL = 1, DQ_V_LONG = 2, DQ_V_DOUBLE = 3, DQ_V_STRING = 4 } dq_value_tag;

typedef struct dq_const {
    int32_t tag;           /* dq_value_tag                                         */
    int32_t str_len;       /* STRING: byte length                                  */
    int64_t i64;           /* BOOL / LONG                                          */
    double f64;            /* DOUBLE                                               */
    int64_t str_offset;    /* STRING: offset into dq_predicate.strings             */
} dq_const;

typedef struct dq_predicate {
    const int32_t* code;   /* pairs (opcode, arg)                                  */
    int32_t code_len;      /* number of int32 words (2 per instruction)            */
    int32_t n_consts;
    const dq_const* consts;
    const uint8_t* strings;/* string constant pool                                 */
    int64_t strings_len;
} dq_predicate;

/* ---------------------------------------------------------------------------------------------
 * Scan-shareable ops. One dq_op per deduplicated analyzer (VerificationSuite does not dedupe,
 * M/VerificationSuite.scala:119; the host does).
 * ------------------------------------------------------------------------------------------- */
typedef enum dq_op_kind {
    DQ_OP_SIZE = 1,                 /* A/Size.scala:33-47                    -> num_matches            */
    DQ_OP_COMPLETENESS = 2,         /* A/Completeness.scala:26-46            -> num_matches_and_count  */
    DQ_OP_COMPLIANCE = 3,           /* A/Compliance.scala:37-53              -> num_matches_and_count  */
    DQ_OP_MEAN = 4,                 /* A/Mean.scala:25-54                    -> mean                   */
    DQ_OP_SUM = 5,                  /* A/Sum.scala:25-52                     -> dbl                    */
    DQ_OP_MINIMUM = 6,              /* A/Minimum.scala:25-53                 -> dbl                    */
    DQ_OP_MAXIMUM = 7,              /* A/Maximum.scala:25-53                 -> dbl                    */
    DQ_OP_STANDARD_DEVIATION = 8,   /* A/StandardDeviation.scala:25-73       -> stddev                 */
    DQ_OP_CORRELATION = 9,          /* A/Correlation.scala:26-105            -> corr                   */
    DQ_OP_APPROX_COUNT_DISTINCT = 10,/* A/ApproxCountDistinct.scala:26-64    -> hll                    */
    DQ_OP_MIN_LENGTH = 11,          /* A/MinLength.scala:25-41               -> dbl                    */
    DQ_OP_MAX_LENGTH = 12,          /* A/MaxLength.scala:25-41               -> dbl                    */
    DQ_OP_DATATYPE = 13             /* A/DataType.scala:32-183               -> datatype               */
} dq_op_kind;

typedef struct dq_op {
    int32_t kind;       /* dq_op_kind                                         */
    int32_t column[2];  /* column indices; column[1] only for CORRELATION     */
    int32_t where;      /* predicate index of the `where` filter, -1 = none   */
    int32_t predicate;  /* COMPLIANCE: predicate index; otherwise -1          */
} dq_op;

#define DQ_HLL_NUM_WORDS 52 /* DeequHyperLogLogPlusPlusUtils.NUM_WORDS, C/StatefulHyperloglogPlus.scala:154 */
#define DQ_HLL_REGISTERS 512

/* One state per op. present == 0 encodes `None` (ifNoNullsIn, A/Analyzer.scala:389-403), which
 * the host turns into EmptyStateException (A/Analyzer.scala:444-455). */
typedef struct dq_state {
    int32_t kind;
    int32_t present;
    union {
        struct { int64_t num_matches; } num_matches;                        /* NumMatches          */
        struct { int64_t num_matches; int64_t count; } num_matches_and_count;/* NumMatchesAndCount  */
        /* MeanState / SumState. For integral (non-decimal) columns Spark sums in a Long that wraps around and
         * casts the FINAL sum to Double (A/Sum.scala:34-37): `isum` keeps that exact Long partial and
         * `exact` = 1 so merges of shards / chunks (dq_state_merge, dq_state_fold) add the Longs and re-cast,
         * rather than adding rounded doubles. `sum` / `value` is always (double)isum then. */
        struct { double sum; int64_t count; int64_t isum; int32_t exact; int32_t pad; } mean;
        struct { double value; int64_t isum; int32_t exact; int32_t pad; } dbl;  /* Sum/Min/Max State */
        struct { double n, avg, m2; } stddev;                               /* StandardDeviationState */
        struct { double n, x_avg, y_avg, ck, x_mk, y_mk; } corr;            /* CorrelationState    */
        struct { int64_t words[DQ_HLL_NUM_WORDS]; } hll;                    /* ApproxCountDistinctState */
        struct { int64_t num_null, num_fractional, num_integral, num_boolean, num_string; } datatype;
    } u;
} dq_state;

#define DQ_SCAN_OUT_DEVICE 0x1u /* `out` is a device pointer: dq_scan returns without syncing */

/* ---------------------------------------------------------------------------------------------
 * Frequency tables (grouping analyzers). Replaces FrequencyBasedAnalyzer.computeFrequencies
 * (A/GroupingAnalyzers.scala:53-79) and the fused aggregation over the table in
 * runAnalyzersForParticularGrouping (R/AnalysisRunner.scala:480-548).
 * ------------------------------------------------------------------------------------------- */
typedef struct dq_freq_table dq_freq_table; /* device-resident (key -> count) table */

#define DQ_FREQ_INCLUDE_NULLS 0x1u /* Histogram semantics: null is a key ("NullValue"), all rows count */

typedef struct dq_freq_summary {
    int64_t num_rows;      /* rows with >= 1 non-null grouping column (A/GroupingAnalyzers.scala:73-76) */
    int64_t num_groups;    /* count(*) over the table  (CountDistinct, Distinctness numerator)         */
    int64_t num_unique;    /* sum[count == 1]          (Uniqueness, UniqueValueRatio numerator)        */
    double entropy;        /* sum over groups of -(c/N) ln(c/N), N = entropy_rows                     */
    int64_t entropy_rows;  /* the N used for `entropy`                                                 */
    int64_t max_count;
    int64_t null_count;    /* DQ_FREQ_INCLUDE_NULLS: rows whose keys are all NULL (one extra group)  */
    /* `entropy` exactly as the order-free sum it was rounded from: each group's term rounded once to
     * a signed 128-bit integer of 2^-104 units, the integers added. entropy ==
     * (double)(hi:lo) * 2^-104. Parts of a sharded table (disjoint groups) add these, not `entropy`,
     * so any split of the same groups gives the same bits. */
    uint64_t entropy_fx_lo;
    int64_t entropy_fx_hi;
} dq_freq_summary;

/* ---------------------------------------------------------------------------------------------
 * Entry points
 * ------------------------------------------------------------------------------------------- */
typedef struct dq_ctx dq_ctx;

int dq_abi_version(void);

/* Bind a context to HIP device `device`. Fails with DQ_ERR_NO_DEVICE when no GPU is visible. */
dq_ctx* dq_open(int device, int* status);
void dq_close(dq_ctx* ctx);
const char* dq_last_error(const dq_ctx* ctx);

/* One context over `ndev` GPUs of this node (multi-GPU row): dq_scan over host columns splits the
 * rows into contiguous 2048-row-aligned shards, one per device, scans them concurrently and returns the states
 * folded in device order with the reference merges (the partition merge inside R/AnalysisRunner.scala:313);
 * dq_frequencies pre-aggregates each shard on its device and exchanges the (key, count) groups by owner device
 * over RCCL (ncclSend / ncclRecv all-to-all over xGMI), so each group lives on exactly one device. The context
 * owns one RCCL communicator per device (ncclCommInitAll) when the devices are distinct; a repeated device
 * (several shards on one GPU, e.g. to test the sharded path on one card) moves the groups with device copies
 * instead. ndev == 1 runs the same sharded path with one shard. dq_quantile_summary runs its selection passes on every
 * device's shard and returns the order statistics of the whole column (the same samples as one device); dq_kll_sketch
 * sketches one partition per device and merges them in device order (QuantileNonSample.merge, as KLLRunner's reduce
 * over partitions, R/KLLRunner.scala:104-112); dq_cast_column casts every device's shard into HOST result buffers. */
dq_ctx* dq_open_devices(const int* devices, int ndev, int* status);
int dq_ctx_num_devices(const dq_ctx* ctx);
int dq_ctx_uses_rccl(const dq_ctx* ctx);   /* 1 when the context's exchange runs over RCCL */

/* dq_scan over columns already resident in HBM across the devices of a multi-device context: shard i's columns
 * (shard_columns[i][0..ncols), DQ_COL_DEVICE on device i, or host) hold shard_rows[i] rows. States come back
 * folded in device order (host memory). */
int dq_scan_sharded(dq_ctx* ctx, const dq_column* const* shard_columns, const int64_t* shard_rows, int ncols,
                    const dq_op* ops, int nops, const dq_predicate* preds, int npreds, dq_state* out);

/* Run kernels on this HIP stream (hipStream_t as void*); NULL = the context's own stream. */
int dq_set_stream(dq_ctx* ctx, void* stream);
/* (r06) HIP stream priority of the context's own stream and its internal side streams: 1 high, 0 normal, -1 low
 * (hipDeviceGetStreamPriorityRange's ends). Waits for the context's queued work. A context whose work is on a job's
 * critical path (e.g. a run submitted beside a ColumnProfiler's passes) dispatches ahead of the device's other
 * contexts. No reference counterpart (Spark's scheduler pools are the nearest analogue). */
int dq_set_priority(dq_ctx* ctx, int priority);
int dq_synchronize(dq_ctx* ctx);

/* Release the context's idle cached device scratch (the grouping builds' partition buffers and tables) beyond
 * keep_bytes, oldest first; 0 releases all of it. A context's scratch cache is locked, so this may be called from
 * any thread (a second context of the device that has finished its helper work). When an allocation fails, a
 * context also releases the idle scratch of every other context of its device before it gives up. No reference
 * counterpart: Spark's executors own their memory (host-side bookkeeping of this engine). */
void dq_scratch_trim(dq_ctx* ctx, int64_t keep_bytes);

/* The fused scan: replaces runScanningAnalyzers (R/AnalysisRunner.scala:289-336), i.e. the single
 * `data.agg(...).collect()` of all ScanShareableAnalyzer.aggregationFunctions() (:306-313) plus
 * fromAggregationResult (A/Analyzer.scala:172-175). Every column is read once from HBM.
 * `out` receives nops dq_state records (host memory unless DQ_SCAN_OUT_DEVICE). */
int dq_scan(dq_ctx* ctx, const dq_column* columns, int ncols, int64_t nrows,
            const dq_op* ops, int nops, const dq_predicate* preds, int npreds,
            dq_state* out, uint32_t flags);

/* dq_scan over host columns streamed through HBM in chunks of chunk_rows rows (rounded to 2048): the copy of the
 * next chunk (its own stream, double-buffered device chunks) overlaps the scan of the current one, and the chunks'
 * states are folded in row order with the reference merges — for tables larger than HBM and host-resident batches
 * (end-to-end rate bound by the host link). Host columns only; `out` is host memory. */
int dq_scan_streamed(dq_ctx* ctx, const dq_column* columns, int ncols, int64_t nrows, const dq_op* ops, int nops,
                     const dq_predicate* preds, int npreds, dq_state* out, int64_t chunk_rows);

/* Number of fused-scan kernel launches issued so far (the analogue of the SparkMonitor job count
 * asserted in T/analyzers/runners/AnalysisRunnerTests.scala:50-74). */
int64_t dq_scan_launch_count(const dq_ctx* ctx);

/* Kernel launches of the scan path by kernel (all devices of a multi-device context), so a test can prove which
 * kernel shape evaluated its ops (tests/test_gpu_configs.py). */
typedef enum dq_scan_kernel {
    DQ_KERNEL_STRIPED = 0,        /* scan_values_kernel: count / sum / min / max / moments, striped 16-B loads     */
    DQ_KERNEL_STRIPED_HEAVY = 1,  /* scan_values_kernel HEAVY: HLL / fused compare over 1-, 2-, 4-byte columns    */
    DQ_KERNEL_HEAVY8 = 2,         /* scan_heavy8_kernel: 8-byte HLL / fused compare / Correlation pairs           */
    DQ_KERNEL_HEAVY8_FULL = 3,    /* scan_heavy8_kernel with every flag on and no `where` (the north-star suite)  */
    DQ_KERNEL_BITS = 4,           /* scan_bits_kernel: Size(where), unread Completeness, non-fused Compliance     */
    DQ_KERNEL_PRED_SIMPLE = 5,    /* pred_simple_kernel: a simple predicate into TRUE / NOT-NULL bitmaps          */
    DQ_KERNEL_PRED_VM = 6,        /* predicate_kernel: the general predicate VM                                   */
    DQ_KERNEL_REGEX = 7,          /* regex_match_kernel (PatternMatch)                                            */
    DQ_KERNEL_STRINGS = 8,        /* scan_strings_kernel                                                          */
    DQ_KERNEL_WHERE_FUSED = 9,    /* a value scan that also evaluates a `where` and writes its masks              */
    DQ_KERNEL_WHERE_MASKS = 10,   /* where_masks_kernel: a `where` into per-column masks (no fused producer)       */
    DQ_KERNEL_COUNT = 11
} dq_scan_kernel;
int64_t dq_scan_kernel_launches(const dq_ctx* ctx, int32_t kernel);

/* Which grouping build produced the frequency tables of this context so far (all devices of a multi-device
 * context), so a test can prove which path it checked against the oracle (tests/test_gpu_grouping_oracle.py). */
typedef enum dq_freq_path {
    DQ_FREQ_PATH_FAST = 0,              /* fast build pass 1 (partition1_fast) over 64-bit keys                */
    DQ_FREQ_PATH_FAST_NARROW = 1,       /* fast build pass 1 over 32-bit offsets around a sampled base         */
    DQ_FREQ_PATH_FAST_DONE = 2,         /* fast builds that produced their table (no exact-path fallback)      */
    DQ_FREQ_PATH_EXACT = 3,             /* exactly-counted path (extract_count + digit histograms)             */
    DQ_FREQ_PATH_PARTITIONED = 4,       /* exact path: radix partition passes (partition1 / scatter2)          */
    DQ_FREQ_PATH_SORTED = 5,            /* exact path: keys sorted on the bucket bits                          */
    DQ_FREQ_PATH_SMALL = 6,             /* one-pass small builds launched (sized or optimistic)                */
    DQ_FREQ_PATH_SMALL_OPTIMISTIC = 7,  /* optimistic small builds (no sizing pass) that produced their table  */
    DQ_FREQ_PATH_FAST_SPILL = 8,        /* fast builds whose full buckets spilled keys (inserted after the build) */
    DQ_FREQ_PATH_SPLIT_BUCKETS = 9,     /* builds with buckets split over several work items (atomic merge)    */
    DQ_FREQ_PATH_LONG_TUPLES = 10,      /* general builds of one string key column with keys past 15 bytes     */
                                        /* (two-word tuples for the short keys, byte compares for the rest)    */
    DQ_FREQ_PATH_COUNT = 11
} dq_freq_path;
int64_t dq_freq_path_count(const dq_ctx* ctx, int32_t path);

/* Semigroup merge of two states of the same op kind (State.sum, per analyzer file);
 * also used for the rank-ordered fold after the RCCL all-gather. */
int dq_state_merge(const dq_state* a, const dq_state* b, dq_state* out);

/* Rank-ordered fold of nparts x nops states (part-major, e.g. an all-gather of per-rank dq_scan outputs):
 * out[i] = states[0][i] + states[1][i] + ... with dq_state_merge, deterministic for every rank count. */
int dq_state_fold(const dq_state* states, int nparts, int nops, dq_state* out);

/* DeequHyperLogLogPlusPlusUtils.count (C/StatefulHyperloglogPlus.scala:210-257), including the
 * Java int-shift quirk `1 << Midx` and precision-9 bias correction; returns the rounded estimate. */
double dq_hll_count(const int64_t words[DQ_HLL_NUM_WORDS]);

/* Spark XxHash64Function.hash(value, type, 42) for one fixed-width value (test hook). */
int64_t dq_spark_hash64(int32_t spark_type, const void* value, int64_t len);

/* Build the (key -> count) table of the given key columns (computeFrequencies). */
int dq_frequencies(dq_ctx* ctx, const dq_column* columns, int ncols, int64_t nrows,
                   const int32_t* key_columns, int nkeys, uint32_t flags, dq_freq_table** table);
/* Fused aggregation over the table (Uniqueness/Distinctness/UniqueValueRatio/Entropy/CountDistinct);
 * entropy_rows <= 0 means "use this table's num_rows". */
int dq_freq_summarize(dq_ctx* ctx, const dq_freq_table* table, int64_t entropy_rows, dq_freq_summary* out);
/* How exported groups are identified: DQ_FREQ_KEYS_VALUES = the canonical 64-bit key of the single
 * fixed-width key column (integers sign-extended, FLOAT/DOUBLE bit patterns with NaN canonical),
 * DQ_FREQ_KEYS_ROWS = the smallest row index of the group (multi-column or string keys). */
#define DQ_FREQ_KEYS_VALUES 0
#define DQ_FREQ_KEYS_ROWS 1
int dq_freq_key_kind(const dq_freq_table* table);
/* Export up to k (key, count) pairs with the largest counts (Histogram top-N, A/Histogram.scala:76-78).
 * Ties are broken by slot order (deterministic). Returns the number written, < 0 on error. */
int64_t dq_freq_top(dq_ctx* ctx, const dq_freq_table* table, int64_t k, int64_t* keys, int64_t* counts);
/* Export the whole table (every group's key and count). Returns the number written, < 0 on error. */
int64_t dq_freq_export(dq_ctx* ctx, const dq_freq_table* table, int64_t capacity, int64_t* keys, int64_t* counts);
void dq_freq_free(dq_ctx* ctx, dq_freq_table* table);

/* Build options: Histogram semantics, and pre-aggregated input (each row stands for weights[row] rows: the
 * partial tables of a sharded computeFrequencies, or persisted (key, count) states). */
typedef struct dq_freq_options {
    uint32_t flags;          /* DQ_FREQ_INCLUDE_NULLS                                                  */
    uint32_t weights_device; /* 1: `weights` is a device pointer on the ctx's GPU                       */
    const int64_t* weights;  /* nrows counts (>= 0), NULL = every row counts once                       */
    int32_t key_type;        /* declared Spark type of the single key column's canonical values, 0 = its own */
    int32_t pad;
} dq_freq_options;
int dq_frequencies_ex(dq_ctx* ctx, const dq_column* columns, int ncols, int64_t nrows, const int32_t* key_columns,
                      int nkeys, const dq_freq_options* options, dq_freq_table** table);
/* dq_frequencies_ex over a table held as row-range parts read where they lie (the row chunks of a ChunkedTable, no
 * concatenation): parts[p * ncols + c] is column c's part p, device columns with int32 offsets; the table's rows are
 * the parts in order (exported representative rows are indices into that order). Two parts on a one-device context,
 * unweighted (r06); other shapes return DQ_ERR_UNSUPPORTED and the caller concatenates. The fast fixed-width build
 * reads one part only, so a fixed-width single key takes the general path here. */
int dq_frequencies_parts(dq_ctx* ctx, const dq_column* parts, int nparts, int ncols, const int32_t* key_columns,
                         int nkeys, const dq_freq_options* options, dq_freq_table** table);

/* Every group of a DQ_FREQ_KEYS_VALUES table as (canonical key, count) into device arrays (the NULL group of a
 * DQ_FREQ_INCLUDE_NULLS table is summary.null_count, not exported). Returns the number written or < 0. */
int64_t dq_freq_export_device(dq_ctx* ctx, const dq_freq_table* table, int64_t capacity, int64_t* keys_dev,
                              int64_t* counts_dev);

#define DQ_FREQ_PAIRS_DEVICE 0x1u /* keys / counts of dq_freq_from_pairs are device pointers */
/* A DQ_FREQ_KEYS_VALUES table from (canonical key, count) pairs — duplicates are added — with the state's numRows
 * and NULL-group count: the persisted frequency states of HdfsStateProvider (A/StateProvider.scala:137-160) and
 * the groups exchanged between shards. */
int dq_freq_from_pairs(dq_ctx* ctx, int32_t key_spark_type, const int64_t* keys, const int64_t* counts, int64_t n,
                       uint32_t flags, int64_t num_rows, int64_t null_count, dq_freq_table** table);

/* FrequenciesAndNumRows.sum (A/GroupingAnalyzers.scala:127-147): null-safe full outer join on the key, counts
 * added, numRows added — on the GPU, for two DQ_FREQ_KEYS_VALUES tables of the same key type. */
int dq_freq_merge(dq_ctx* ctx, const dq_freq_table* a, const dq_freq_table* b, dq_freq_table** out);

/* MutualInformation.computeMetricFrom (A/MutualInformation.scala:35-97): joint = the (x, y) table, x / y = the
 * single-column tables of the same rows (their counts are the marginals of the joint table's non-NULL keys).
 * *mi = sum over joint groups with both keys non-NULL of (pxy/N) ln((pxy/N) / ((px/N)(py/N))), N = joint numRows;
 * *present = 0 when no group joins (the reference's NULL sum -> empty state). The three tables are built over the
 * same rows: all unweighted, or all weighted by the same per-row counts (dq_frequencies_ex over a state's groups). */
int dq_freq_mutual_information(dq_ctx* ctx, const dq_freq_table* joint, const dq_freq_table* x,
                               const dq_freq_table* y, double* mi, int32_t* present);

/* Per row of the table's own source (the nrows rows it was built over by dq_frequencies / dq_frequencies_ex): the
 * count of the row's group, 0 for a row that takes no part (all key columns NULL without DQ_FREQ_INCLUDE_NULLS) —
 * the join of the rows with their frequency table, as MutualInformation joins the joint groups with the marginal
 * tables (A/MutualInformation.scala:50-74); the sharded MutualInformation attaches px / py to exchanged groups
 * with it. `counts` holds nrows entries (a device pointer with DQ_FREQ_PAIRS_DEVICE). */
int dq_freq_row_counts(dq_ctx* ctx, const dq_freq_table* table, int64_t* counts, int64_t nrows, uint32_t flags);

/* ApproxQuantile / ApproxQuantiles (A/ApproxQuantile.scala:28-103, A/ApproxQuantiles.scala:39-101): replaces the
 * per-row PercentileDigest.add of StatefulApproxQuantile.update (C/StatefulApproxQuantile.scala:65-72). Computes
 * EXACT order statistics of the column's non-NULL values cast to double, in java.lang.Double.compare order
 * (-0.0 < 0.0, NaN largest), at 1-based ranks 1, n and every max(1, floor(relative_error * n))-th rank in between:
 * the samples (value, g = rank gap, delta = 0) of a Greenwald-Khanna summary with no rank uncertainty, from which
 * the host builds Spark's QuantileSummaries / PercentileDigest (relative_error = 0 returns all n sorted values).
 * Numeric columns only (Preconditions.isNumeric). values_out / ranks_out hold max_samples entries (2/relative_error
 * + 2 always suffices when relative_error * n >= 1; n otherwise). *count receives n. Returns the number of samples
 * written (0 for an empty or all-NULL column), or a negative dq_status. */
int64_t dq_quantile_summary(dq_ctx* ctx, const dq_column* column, int64_t nrows, double relative_error,
                            int64_t max_samples, double* values_out, int64_t* ranks_out, int64_t* count_out);

/* Several ApproxQuantile summaries at once — the ApproxQuantile(s) analyzers of one analysis run over one shard,
 * each column given as one or more consecutive row ranges ("parts": the chunks of a ChunkedTable, read where they
 * lie, no concatenation). Request r summarises parts[part_begin[r] .. part_begin[r+1]) (same type; each part's own
 * `length` rows) at relative_error[r]: values_out / ranks_out + r * max_samples receive exactly the samples
 * dq_quantile_summary returns for those parts concatenated, counts_out[r] = n, samples_out[r] = their number.
 * One host round trip for all requests (A/ApproxQuantile.scala:28-103 via the runner's batched aggregation,
 * R/AnalysisRunner.scala:289-336). A multi-device context takes one part per request. Returns 0 or a negative
 * dq_status. */
int dq_quantile_summaries(dq_ctx* ctx, const dq_column* parts, const int32_t* part_begin, int nreq,
                          const double* relative_error, int64_t max_samples, double* values_out, int64_t* ranks_out,
                          int64_t* counts_out, int64_t* samples_out);

/* KLLSketch (A/KLLSketch.scala:82-176) as KLLRunner.computeKLLSketchesInExtraPass builds it
 * (R/KLLRunner.scala:91-179): replaces the per-row QuantileNonSample.update loop of sketchPartitions for ONE
 * partition whose non-NULL values (cast to double) arrive in row order. Writes the KLLState bytes
 * (A/KLLSketch.scala:56-66: min f64, max f64, then the KLLSketchSerializer layout,
 * A/catalyst/KLLSketchSerializer.scala:60-80; all big-endian) to state_out when they fit in `capacity`, and
 * returns their length (call again with a larger buffer when the return value exceeds capacity), or a negative
 * dq_status. BYTE/SHORT/INT/LONG/FLOAT/DOUBLE columns only (other types: DQ_ERR_UNSUPPORTED, as
 * KLLRunner.emptySketches throws). NaN items are stored canonical. */
int64_t dq_kll_sketch(dq_ctx* ctx, const dq_column* column, int64_t nrows, int32_t sketch_size,
                      double shrinking_factor, uint8_t* state_out, int64_t capacity);

/* The KLL extra pass over several columns of one table at once (R/KLLRunner.scala:91-112 sketches every KLL column
 * in one pass over the partitions): column i's KLLState bytes, exactly those of dq_kll_sketch, go to
 * state_out + (sum of sizes[0..i)) and sizes[i] receives their length. Returns the total length (nothing is written
 * when it exceeds `capacity`: call again with a larger buffer) or a negative dq_status. The columns' compaction
 * schedules are computed on parallel host threads; the NULL-compaction passes and every compaction level (per kernel
 * class) are one launch each over all the columns, with one host round trip for all of them. */
int64_t dq_kll_sketch_columns(dq_ctx* ctx, const dq_column* columns, int32_t ncols, int64_t nrows, int32_t sketch_size,
                              double shrinking_factor, uint8_t* state_out, int64_t capacity, int64_t* sizes);

/* KLLState.sum of two serialized KLLState byte strings (A/KLLSketch.scala:49-54: QuantileNonSample.merge,
 * A/QuantileNonSample.scala:218-234, then condense until the sketch fits; java max / min of the extremes) — the
 * partition sketches of KLLRunner's treeReduce (R/KLLRunner.scala:104-112) and the row chunks of a chunked table.
 * Host only (no context, no device). Writes the merged state to `out` when it fits in `capacity` and returns its
 * length, or DQ_ERR_INVALID_ARGUMENT for malformed input. */
int64_t dq_kll_merge_states(const uint8_t* a, int64_t na, const uint8_t* b, int64_t nb, uint8_t* out, int64_t capacity);

/* ColumnProfiler.castColumn (M/profiles/ColumnProfiler.scala:346-355): Spark 2.2 Cast of a column to LONG or
 * DOUBLE. STRING sources: UTF8String.toLong (no trimming, optional sign, digits, optional '.' + digits truncated,
 * overflow NULL) / java.lang.Double.parseDouble (correctly rounded); strings that do not parse become NULL.
 * Numeric sources: integers sign-extend / convert, FLOAT/DOUBLE -> LONG as Java's (long) (NaN 0, saturating),
 * DECIMAL(p <= 18) -> Decimal.toLong (truncating) / Decimal.toDouble, BOOLEAN -> 0/1. values_dev receives nrows x 8 B,
 * validity_dev ceil(nrows / 64) x 8 B (LSB-first bitmap); both device memory, 8-B aligned. Returns DQ_OK, or
 * DQ_ERR_UNSUPPORTED when a string needs Double.parseDouble's arbitrary-precision path (hexadecimal literal, or
 * more than 19 significant digits on a rounding boundary) — never a silent guess. On a multi-device context
 * (dq_open_devices) the column is a host column and values_dev / validity_dev are HOST buffers of the same sizes. */
int dq_cast_column(dq_ctx* ctx, const dq_column* column, int64_t nrows, int32_t to_type, void* values_dev,
                   uint8_t* validity_dev);

/* Multi-GPU grouping: the canonical 64-bit keys (see DQ_FREQ_KEYS_VALUES) of one
 * fixed-width column's non-NULL rows, bucketed by owner rank = (mix64(key) >> 32) % nparts, written
 * contiguously per rank into keys_dev (capacity nrows, device memory) for an RCCL all-to-all; the
 * owner of a key builds its table from the keys it receives, so every group lives on exactly one
 * rank. part_counts (host, nparts entries) receives the bucket sizes; *null_rows the NULL rows.
 * Returns DQ_OK or an error. */
int dq_partition_keys(dq_ctx* ctx, const dq_column* column, int64_t nrows, int nparts, int64_t* keys_dev,
                      int64_t* part_counts, int64_t* null_rows);

/* Synthetic input generators for benches/tests (counter-based splitmix64). */
typedef enum dq_synth_kind {
    DQ_SYNTH_DYADIC = 1,   /* f64: k * 2^-8, k uniform in [-256, 256]                */
    DQ_SYNTH_UNIFORM = 2,  /* f64: U[0,1) on a 2^-53 grid                            */
    DQ_SYNTH_NORMAL = 3,   /* f64: 100 + 15 * (sum of 12 U[0,1) on a 2^-48 grid - 6)   */
    DQ_SYNTH_INT32R = 4,   /* i64: U[-2^31, 2^31)                                    */
    DQ_SYNTH_KEY30 = 5,    /* i64: splitmix64(row) mod 2^30                          */
    DQ_SYNTH_GAUSS01 = 6,  /* f64: sum of 12 U[0,1) on a 2^-48 grid - 6              */
    DQ_SYNTH_GAUSS_CORR = 7/* f64: 0.6 * GAUSS01(seed) + 0.8 * GAUSS01(seed ^ 0x5A5A5A5A5A5A5A5A):
                            *      correlated (rho ~ 0.6) with the GAUSS01 column of the same seed */
} dq_synth_kind;

int dq_synth_column(dq_ctx* ctx, int32_t kind, uint64_t seed, int64_t row0, int64_t nrows,
                    void* values_dev);
/* Config-C4 frequency keys: row r of a `total_rows` table gets key
 * mix64(j < distinct ? j : (j - distinct) mod (distinct / 2)) with j = (r * 0x9E3779B1) mod total_rows,
 * so exactly `distinct` keys exist when (total_rows - distinct) is a multiple of distinct / 2. */
int dq_synth_freq_keys(dq_ctx* ctx, int64_t total_rows, int64_t distinct, int64_t row0, int64_t nrows,
                       int64_t* keys_dev);
/* UTF-8 string columns of config C5. Two calls: with bytes_dev == NULL, writes the int32 Arrow
 * offsets (nrows + 1 entries, device) and *total_bytes; then with bytes_dev (>= total_bytes + 16 bytes) writes the
 * strings. Kinds: */
#define DQ_SYNTH_STR_CAT50 101  /* "cat_<0..49>"                                           */
#define DQ_SYNTH_STR_BOOL 102   /* "true" / "false"                                        */
#define DQ_SYNTH_STR_CAT100 103 /* "v<00..99>"                                             */
#define DQ_SYNTH_STR_INT 104    /* an integer in [-1e6, 1e6)                               */
#define DQ_SYNTH_STR_DEC 105    /* "<0..999>.<00..99>"                                     */
#define DQ_SYNTH_STR_MIXNUM 106 /* 70 %: an integer in [-5000, 5000); 30 %: "<+-int>.<ddd>" */
#define DQ_SYNTH_STR_TEXT 107   /* 1-20 characters of [a-z0-9 ]                           */
int dq_synth_strings(dq_ctx* ctx, int32_t kind, uint64_t seed, int64_t row0, int64_t nrows, int32_t* offsets_dev,
                     void* bytes_dev, int64_t* total_bytes);
/* Validity bitmap (ceil(nrows/64) words) with P(null) = null_permille / 1000. */
int dq_synth_validity(dq_ctx* ctx, uint64_t seed, int64_t row0, int64_t nrows, int32_t null_permille,
                      uint8_t* validity_dev);

#ifdef __cplusplus
}
#endif

#endif /* DEEQU_AMD_DQ_H */
