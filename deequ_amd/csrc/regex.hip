// regex.hip — PatternMatch on the GPU (gfx950 / CDNA4).
//
// PatternMatch (A/PatternMatch.scala:37-55) sums `when(regexp_extract(col, pattern, 0) != "", 1)
// .otherwise(0)` under `where`: a row matches when the FIRST match of java.util.regex
// Matcher.find() is non-empty; a NULL value counts 0. The host compiles the pattern
// (deequ_amd/regex.py) to the program of a backtracking engine with Java's leftmost-first
// priorities; this kernel runs it with one lane per row (per-lane explicit stack of branch / undo
// frames in private memory) and emits the predicate bitmaps the scan consumes (TRUE rows, and
// NOT-NULL = every row: the expression is never NULL). Numbers are matched against their Spark
// string cast (integral: decimal digits, boolean: "true"/"false").
//
// Program image (little-endian int32): header {magic, ninstr, nclasses, nranges, ngroups, nloops,
// anchored, 0}, ninstr x {op, a, b}, nclasses x {first range, count}, nranges x {lo, hi}.
#include <hip/hip_runtime.h>

#include "dq_common.h"
#include "dq_internal.h"
#include "java_dtoa.h"
#include "rx_engine.h"

namespace dq {

using namespace rx;


__global__ void __launch_bounds__(256)
regex_match_kernel(PredColumn col, const int32_t* __restrict__ image, int64_t nrows, int64_t padded_words,
                   uint64_t* __restrict__ out_t, uint64_t* __restrict__ out_nn, int32_t* __restrict__ status) {
    const int64_t row = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    RxProg p;
    p.ninstr = image[1];
    p.anchored = image[6];
    p.ins = image + 8;
    p.classes = p.ins + 3 * p.ninstr;
    p.ranges = p.classes + 2 * image[2];
    bool t = false;
    if (row < nrows) {
        bool valid = true;
        if (col.validity) valid = (col.validity[row >> 6] >> (row & 63)) & 1ull;
        if (valid) {
            uint8_t buf[32];
            const uint8_t* s;
            int n;
            switch (col.spark_type) {
                case DQ_TYPE_STRING: {
                    const int32_t o0 = col.offsets[row], o1 = col.offsets[row + 1];
                    s = static_cast<const uint8_t*>(col.values) + o0;
                    n = o1 - o0;
                    break;
                }
                case DQ_TYPE_DOUBLE:  // Cast(x AS STRING) = Double.toString / Float.toString (java_dtoa.h)
                    n = java_double_to_chars(static_cast<const double*>(col.values)[row], buf);
                    s = buf;
                    break;
                case DQ_TYPE_FLOAT:
                    n = java_float_to_chars(static_cast<const float*>(col.values)[row], buf);
                    s = buf;
                    break;
                case DQ_TYPE_BOOLEAN: {
                    const bool b = static_cast<const uint8_t*>(col.values)[row] != 0;
                    const char* txt = b ? "true" : "false";
                    n = b ? 4 : 5;
                    for (int k = 0; k < n; ++k) buf[k] = (uint8_t)txt[k];
                    s = buf;
                    break;
                }
                case DQ_TYPE_DECIMAL:
                    n = format_decimal(static_cast<const int64_t*>(col.values)[row], col.decimal_scale, buf);
                    s = buf;
                    break;
                case DQ_TYPE_DATE:
                    n = format_date_days(static_cast<const int32_t*>(col.values)[row], buf);
                    s = buf;
                    break;
                case DQ_TYPE_TIMESTAMP:
                    n = format_timestamp_utc(static_cast<const int64_t*>(col.values)[row], buf);
                    s = buf;
                    break;
                default: {
                    int64_t v;
                    switch (col.spark_type) {
                        case DQ_TYPE_BYTE: v = static_cast<const int8_t*>(col.values)[row]; break;
                        case DQ_TYPE_SHORT: v = static_cast<const int16_t*>(col.values)[row]; break;
                        case DQ_TYPE_INT: v = static_cast<const int32_t*>(col.values)[row]; break;
                        default: v = static_cast<const int64_t*>(col.values)[row]; break;
                    }
                    n = format_long(v, buf);
                    s = buf;
                    break;
                }
            }
            uint64_t stk[kRxStack];
            // Matcher.find(): the first start position (code point boundaries) with a match
            for (int start = 0; start <= n;) {
                const int end = rx_match_at(p, s, n, start, stk);
                if (end == -2) {
                    atomicOr(status, 1);
                    break;
                }
                if (end >= 0) {
                    t = end > start;  // regexp_extract(..., 0) != ""
                    break;
                }
                if (p.anchored || start == n) break;
                int len;
                decode(s, n, start, len);
                start += len;
            }
        }
    }
    const uint64_t bt = __ballot(t);
    const uint64_t bn = __ballot(row < nrows);
    const int64_t w = row >> 6;
    if ((threadIdx.x & 63) == 0 && w < padded_words) {
        out_t[w] = bt;
        out_nn[w] = bn;
    }
}

void launch_regex(const PredColumn& col, const int32_t* image_dev, int64_t nrows, int64_t padded_words,
                  uint64_t* out_t, uint64_t* out_nn, int32_t* status, hipStream_t s) {
    const int64_t rows = padded_words * 64;
    const int64_t blocks = (rows + 255) / 256;
    hipLaunchKernelGGL(regex_match_kernel, dim3((unsigned)blocks), dim3(256), 0, s, col, image_dev, nrows,
                       padded_words, out_t, out_nn, status);
}

}  // namespace dq
