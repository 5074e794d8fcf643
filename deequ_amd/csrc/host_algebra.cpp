// host_algebra.cpp — the pure host code of libdq.so: the reference's State.sum per state, the HLL++ estimate,
// Spark's hash of one value, and the row-shard arithmetic of multi-device contexts. No HIP here: the same file is
// compiled with -DDQ_HOST_ONLY under AddressSanitizer / UBSan by tests/sanitize/ (run by the CPU test suite).
#include <math.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <vector>

#include "../../include/dq.h"
#include "dq_common.h"
#include "hll_bias_p9.h"

namespace dq {
// declared in dq_internal.h (HIP builds); restated here so the host-only build needs no HIP header
constexpr int64_t kShardAlign = 2048;  // = kTileRows: a shard starts on a tile (and validity word) boundary
void shard_bounds(int64_t nrows, int ndev, int i, int64_t* row0, int64_t* count);
void shard_columns(const dq_column* columns, int ncols, int64_t row0, int64_t count, dq_column* out,
                   std::vector<std::vector<int32_t>>& scratch);
}  // namespace dq

namespace {

using namespace dq;

// ---- host state algebra (State.sum of each reference state) --------------------------------------
void hll_merge_words(const int64_t* a, const int64_t* b, int64_t* out) {
    // DeequHyperLogLogPlusPlusUtils.merge (C/StatefulHyperloglogPlus.scala:188-208)
    int idx = 0;
    for (int w = 0; w < DQ_HLL_NUM_WORDS; ++w) {
        uint64_t wa = (uint64_t)a[w], wb = (uint64_t)b[w], word = 0;
        uint64_t mask = 63;
        for (int i = 0; idx < DQ_HLL_REGISTERS && i < 10; ++i, ++idx) {
            word |= std::max(wa & mask, wb & mask);
            mask <<= 6;
        }
        out[w] = (int64_t)word;
    }
}

double java_math_min(double a, double b) {
    if (a != a) return a;
    if (b != b) return b;
    if (a == 0.0 && b == 0.0) return signbit(a) ? a : b;
    return a <= b ? a : b;
}
double java_math_max(double a, double b) {
    if (a != a) return a;
    if (b != b) return b;
    if (a == 0.0 && b == 0.0) return signbit(a) ? b : a;
    return a >= b ? a : b;
}


int cell_bytes(int spark_type) {
    switch (spark_type) {
        case DQ_TYPE_BOOLEAN: case DQ_TYPE_BYTE: return 1;
        case DQ_TYPE_SHORT: return 2;
        case DQ_TYPE_INT: case DQ_TYPE_DATE: case DQ_TYPE_FLOAT: return 4;
        default: return 8;
    }
}

}  // namespace

namespace dq {

void shard_bounds(int64_t nrows, int ndev, int i, int64_t* row0, int64_t* count) {
    int64_t per = (nrows + ndev - 1) / std::max(ndev, 1);
    per = (per + kShardAlign - 1) / kShardAlign * kShardAlign;
    const int64_t r0 = std::min<int64_t>((int64_t)i * per, nrows);
    *row0 = r0;
    *count = std::max<int64_t>(0, std::min<int64_t>(nrows, r0 + per) - r0);
}

void shard_columns(const dq_column* columns, int ncols, int64_t row0, int64_t count, dq_column* out,
                   std::vector<std::vector<int32_t>>& scratch) {
    scratch.resize(ncols);
    for (int c = 0; c < ncols; ++c) {
        dq_column col = columns[c];
        col.length = count;
        if (col.validity) col.validity += row0 / 8;  // row0 is a multiple of 2048
        if (col.spark_type == DQ_TYPE_STRING) {
            const int32_t base = col.offsets ? col.offsets[row0] : 0;
            scratch[c].resize((size_t)count + 1);
            for (int64_t k = 0; k <= count; ++k) scratch[c][k] = col.offsets[row0 + k] - base;
            col.offsets = scratch[c].data();
            col.values = static_cast<const uint8_t*>(col.values) + base;
        } else {
            col.values = static_cast<const uint8_t*>(col.values) + row0 * cell_bytes(col.spark_type);
        }
        out[c] = col;
    }
}

}  // namespace dq

extern "C" {

int dq_state_merge(const dq_state* a, const dq_state* b, dq_state* out) {
    if (!a || !b || !out || a->kind != b->kind) return DQ_ERR_INVALID_ARGUMENT;
    // Analyzers.merge (A/Analyzer.scala:367-386): None is the identity.
    if (!a->present) { *out = *b; return DQ_OK; }
    if (!b->present) { *out = *a; return DQ_OK; }
    dq_state r = *a;
    switch (a->kind) {
        case DQ_OP_SIZE:
            r.u.num_matches.num_matches = a->u.num_matches.num_matches + b->u.num_matches.num_matches;
            break;
        case DQ_OP_COMPLETENESS:
        case DQ_OP_COMPLIANCE:
            r.u.num_matches_and_count.num_matches += b->u.num_matches_and_count.num_matches;
            r.u.num_matches_and_count.count += b->u.num_matches_and_count.count;
            break;
        case DQ_OP_MEAN:
            r.u.mean.count = a->u.mean.count + b->u.mean.count;
            if (a->u.mean.exact && b->u.mean.exact) {  // Long partials: wrap-around add, one final cast
                r.u.mean.isum = (int64_t)((uint64_t)a->u.mean.isum + (uint64_t)b->u.mean.isum);
                r.u.mean.sum = (double)r.u.mean.isum;
            } else {
                r.u.mean.sum = a->u.mean.sum + b->u.mean.sum;
                r.u.mean.exact = 0;
            }
            break;
        case DQ_OP_SUM:
            if (a->u.dbl.exact && b->u.dbl.exact) {
                r.u.dbl.isum = (int64_t)((uint64_t)a->u.dbl.isum + (uint64_t)b->u.dbl.isum);
                r.u.dbl.value = (double)r.u.dbl.isum;
            } else {
                r.u.dbl.value = a->u.dbl.value + b->u.dbl.value;
                r.u.dbl.exact = 0;
            }
            break;
        case DQ_OP_MINIMUM:
        case DQ_OP_MIN_LENGTH:
            r.u.dbl.value = java_math_min(a->u.dbl.value, b->u.dbl.value);
            break;
        case DQ_OP_MAXIMUM:
        case DQ_OP_MAX_LENGTH:
            r.u.dbl.value = java_math_max(a->u.dbl.value, b->u.dbl.value);
            break;
        case DQ_OP_STANDARD_DEVIATION: {  // A/StandardDeviation.scala:37-44
            const double n = a->u.stddev.n, on = b->u.stddev.n;
            const double newN = n + on;
            const double delta = b->u.stddev.avg - a->u.stddev.avg;
            const double deltaN = newN == 0.0 ? 0.0 : delta / newN;
            r.u.stddev.n = newN;
            r.u.stddev.avg = a->u.stddev.avg + deltaN * on;
            r.u.stddev.m2 = a->u.stddev.m2 + b->u.stddev.m2 + delta * deltaN * n * on;
            break;
        }
        case DQ_OP_CORRELATION: {  // A/Correlation.scala:37-52
            const double n1 = a->u.corr.n, n2 = b->u.corr.n, newN = n1 + n2;
            const double dx = b->u.corr.x_avg - a->u.corr.x_avg;
            const double dxN = newN == 0.0 ? 0.0 : dx / newN;
            const double dy = b->u.corr.y_avg - a->u.corr.y_avg;
            const double dyN = newN == 0.0 ? 0.0 : dy / newN;
            r.u.corr.n = newN;
            r.u.corr.x_avg = a->u.corr.x_avg + dxN * n2;
            r.u.corr.y_avg = a->u.corr.y_avg + dyN * n2;
            r.u.corr.ck = a->u.corr.ck + b->u.corr.ck + dx * dyN * n1 * n2;
            r.u.corr.x_mk = a->u.corr.x_mk + b->u.corr.x_mk + dx * dxN * n1 * n2;
            r.u.corr.y_mk = a->u.corr.y_mk + b->u.corr.y_mk + dy * dyN * n1 * n2;
            break;
        }
        case DQ_OP_APPROX_COUNT_DISTINCT:
            hll_merge_words(a->u.hll.words, b->u.hll.words, r.u.hll.words);
            break;
        case DQ_OP_DATATYPE:
            r.u.datatype.num_null += b->u.datatype.num_null;
            r.u.datatype.num_fractional += b->u.datatype.num_fractional;
            r.u.datatype.num_integral += b->u.datatype.num_integral;
            r.u.datatype.num_boolean += b->u.datatype.num_boolean;
            r.u.datatype.num_string += b->u.datatype.num_string;
            break;
        default:
            return DQ_ERR_UNSUPPORTED;
    }
    *out = r;
    return DQ_OK;
}

int dq_state_fold(const dq_state* states, int nparts, int nops, dq_state* out) {
    // Rank-ordered semigroup fold (Analyzers.merge per op, A/Analyzer.scala:367-386) of nparts x nops
    // records laid out part-major, as an all-gather of per-rank dq_scan outputs delivers them.
    if ((nparts > 0 && nops > 0 && (!states || !out)) || nparts < 0 || nops < 0) return DQ_ERR_INVALID_ARGUMENT;
    for (int i = 0; i < nops; ++i) {
        dq_state acc = states[i];
        for (int r = 1; r < nparts; ++r) {
            dq_state next;
            const int rc = dq_state_merge(&acc, &states[(size_t)r * nops + i], &next);
            if (rc) return rc;
            acc = next;
        }
        out[i] = acc;
    }
    return DQ_OK;
}

// DeequHyperLogLogPlusPlusUtils.estimateBias (C/StatefulHyperloglogPlus.scala:259-297), P = 9, K = 6.
static double hll_estimate_bias(double e) {
    const double* est = DQ_HLL_P9_RAW;
    const int num = DQ_HLL_P9_N;
    // java.util.Arrays.binarySearch: index if found, else -(insertion point) - 1 -> insertion point
    int lo = 0, hi = num - 1, nearest = -1;
    while (lo <= hi) {
        const int mid = (int)(((unsigned)lo + (unsigned)hi) >> 1);
        const double mv = est[mid];
        if (mv < e) lo = mid + 1;
        else if (mv > e) hi = mid - 1;
        else {
            // Double.compare semantics; the table holds no NaN / signed zeros.
            nearest = mid;
            break;
        }
    }
    if (nearest < 0) nearest = lo;
    auto distance = [&](int i) {
        const double d = e - est[i];
        return d * d;
    };
    const int K = 6;
    int low = std::max(nearest - K + 1, 0);
    int high = std::min(low + K, num);
    while (high < num && distance(high) < distance(low)) {
        ++low;
        ++high;
    }
    double bias = 0.0;
    for (int i = low; i < high; ++i) bias += DQ_HLL_P9_BIAS[i];
    return bias / (high - low);
}

double dq_hll_count(const int64_t words[DQ_HLL_NUM_WORDS]) {
    const int P = 9, M = 512;
    const double alphaM2 = (0.7213 / (1.0 + 1.079 / M)) * M * M;
    double zInverse = 0.0, V = 0.0;
    int idx = 0;
    for (int w = 0; w < DQ_HLL_NUM_WORDS; ++w) {
        const uint64_t word = (uint64_t)words[w];
        int shift = 0;
        for (int i = 0; idx < M && i < 10; ++i, ++idx, shift += 6) {
            const int64_t Midx = (int64_t)((word >> shift) & 63u);
            // Scala `1 << Midx` on an Int: JVM shift distance is Midx & 31, result is a 32-bit int.
            const int32_t pow2 = (int32_t)((uint32_t)1u << (Midx & 31));
            zInverse += 1.0 / (double)pow2;
            if (Midx == 0) V += 1.0;
        }
    }
    auto corrected = [&]() {
        const double e = alphaM2 / zInverse;
        return (P < 19 && e < 5.0 * M) ? e - hll_estimate_bias(e) : e;
    };
    double estimate;
    if (V > 0) {
        const double H = M * log(M / V);
        estimate = H <= DQ_HLL_P9_THRESHOLD ? H : corrected();
    } else {
        estimate = corrected();
    }
    // Math.round(double): floor(x + 0.5) as a long
    return (double)(int64_t)floor(estimate + 0.5);
}

int64_t dq_spark_hash64(int32_t spark_type, const void* value, int64_t len) {
    if (!value) return 0;
    switch (spark_type) {
        case DQ_TYPE_BOOLEAN: return (int64_t)xxh_int(*(const uint8_t*)value ? 1u : 0u, SPARK_HLL_SEED);
        case DQ_TYPE_BYTE: return (int64_t)xxh_int((uint32_t)(int32_t)*(const int8_t*)value, SPARK_HLL_SEED);
        case DQ_TYPE_SHORT: return (int64_t)xxh_int((uint32_t)(int32_t)*(const int16_t*)value, SPARK_HLL_SEED);
        case DQ_TYPE_INT:
        case DQ_TYPE_DATE: return (int64_t)xxh_int((uint32_t)*(const int32_t*)value, SPARK_HLL_SEED);
        case DQ_TYPE_LONG:
        case DQ_TYPE_TIMESTAMP:
        case DQ_TYPE_DECIMAL: return (int64_t)xxh_long((uint64_t)*(const int64_t*)value, SPARK_HLL_SEED);
        case DQ_TYPE_FLOAT: return (int64_t)xxh_int(float_to_int_bits(*(const float*)value), SPARK_HLL_SEED);
        case DQ_TYPE_DOUBLE: return (int64_t)xxh_long(double_to_long_bits(*(const double*)value), SPARK_HLL_SEED);
        case DQ_TYPE_STRING: return (int64_t)xxh_bytes((const uint8_t*)value, len, SPARK_HLL_SEED);
        default: return 0;
    }
}

}  // extern "C"
