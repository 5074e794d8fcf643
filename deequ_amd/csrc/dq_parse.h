// dq_parse.h — Spark 2.2 / Java string -> number casts on the device.
//
//   spark_string_to_long: UTF8String.toLong as Spark 2.2's Cast(StringType -> LongType) calls it (no
//     trimming; optional sign; digits; an optional '.' followed by digits only, truncated; overflow
//     is NULL) — spark-unsafe 2.2.2, third-party (absent from /root/reference).
//   java_parse_double: java.lang.Double.parseDouble as Cast(StringType -> DoubleType) calls it through
//     `s.toString.toDouble` (String.trim of chars <= ' '; optional sign; "NaN" / "Infinity"; decimal
//     digits with an optional point, an optional exponent and an optional f/F/d/D suffix), CORRECTLY
//     ROUNDED like Java: Eisel-Lemire over a 128-bit powers-of-five table (pow5_table.h), exact for up
//     to 19 significant digits; with more, the truncated significand w and w + 1 must round alike,
//     otherwise `slow` is set (and hexadecimal literals set it too) so the caller can fail loudly.
#pragma once

#include <stdint.h>

#if defined(DQ_HOST_ONLY)  // host-only build (tests/sanitize/): the same parsers, checked by ASan / UBSan
#define DQ_PARSE_FN inline
#define __constant__
#else
#include <hip/hip_runtime.h>
#define DQ_PARSE_FN __host__ __device__ inline
#endif

#include "pow5_table.h"

namespace dq {

DQ_PARSE_FN int parse_clz64(uint64_t w) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __clzll((long long)w);
#else
    return __builtin_clzll(w);
#endif
}
DQ_PARSE_FN double parse_bits_double(uint64_t u) {
    union { uint64_t u; double d; } c;
    c.u = u;
    return c.d;
}
DQ_PARSE_FN uint64_t parse_double_bits(double d) {
    union { uint64_t u; double d; } c;
    c.d = d;
    return c.u;
}
DQ_PARSE_FN uint64_t parse_umulhi64(uint64_t a, uint64_t b) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __umul64hi(a, b);
#else
    return (uint64_t)(((unsigned __int128)a * b) >> 64);
#endif
}

DQ_PARSE_FN bool spark_string_to_long(const uint8_t* s, int n, int64_t& out) {
    if (n == 0) return false;
    uint8_t b = s[0];
    const bool negative = b == '-';
    int offset = 0;
    if (negative || b == '+') {
        ++offset;
        if (n == 1) return false;
    }
    const int64_t stop = INT64_MIN / 10;
    int64_t result = 0;  // accumulated negative, as the reference does
    while (offset < n) {
        b = s[offset++];
        if (b == '.') break;
        if (b < '0' || b > '9') return false;
        if (result < stop) return false;
        result = (int64_t)((uint64_t)result * 10ull - (uint64_t)(b - '0'));  // Java wraps; checked next
        if (result > 0) return false;
    }
    while (offset < n) {
        const uint8_t c = s[offset++];
        if (c < '0' || c > '9') return false;
    }
    if (!negative) {
        result = (int64_t)(0ull - (uint64_t)result);
        if (result < 0) return false;
    }
    out = result;
    return true;
}

struct AdjustedMantissa {
    uint64_t mantissa;
    int32_t power2;
};

// Eisel-Lemire compute_float for binary64 (w != 0 path; see tools/gen_pow5_table.py for references).
DQ_PARSE_FN AdjustedMantissa el_compute_float(int64_t q, uint64_t w) {
    AdjustedMantissa a;
    if (w == 0 || q < DQ_POW5_MIN_Q) {
        a.power2 = 0;
        a.mantissa = 0;
        return a;
    }
    if (q > DQ_POW5_MAX_Q) {
        a.power2 = 0x7FF;
        a.mantissa = 0;
        return a;
    }
    const int lz = parse_clz64(w);
    w <<= lz;
    const int index = 2 * (int)(q - DQ_POW5_MIN_Q);
    const uint64_t precision_mask = 0xFFFFFFFFFFFFFFFFull >> 55;
    uint64_t p_hi = parse_umulhi64(w, dq_pow5_128[index]);
    uint64_t p_lo = w * dq_pow5_128[index];
    if ((p_hi & precision_mask) == precision_mask) {
        const uint64_t s_hi = parse_umulhi64(w, dq_pow5_128[index + 1]);
        p_lo += s_hi;
        if (s_hi > p_lo) ++p_hi;
    }
    const int upperbit = (int)(p_hi >> 63);
    const int shift = upperbit + 64 - 52 - 3;
    a.mantissa = p_hi >> shift;
    a.power2 = (int32_t)((((152170 + 65536) * q) >> 16) + 63 + upperbit - lz + 1023);
    if (a.power2 <= 0) {  // subnormal
        if (-a.power2 + 1 >= 64) {
            a.power2 = 0;
            a.mantissa = 0;
            return a;
        }
        a.mantissa >>= -a.power2 + 1;
        a.mantissa += (a.mantissa & 1);
        a.mantissa >>= 1;
        a.power2 = (a.mantissa < (1ull << 52)) ? 0 : 1;
        return a;
    }
    if (p_lo <= 1 && q >= -4 && q <= 23 && (a.mantissa & 3) == 1) {  // exact halfway: round to even
        if ((a.mantissa << shift) == p_hi) a.mantissa &= ~1ull;
    }
    a.mantissa += (a.mantissa & 1);
    a.mantissa >>= 1;
    if (a.mantissa >= (2ull << 52)) {
        a.mantissa = 1ull << 52;
        ++a.power2;
    }
    a.mantissa &= ~(1ull << 52);
    if (a.power2 >= 0x7FF) {
        a.power2 = 0x7FF;
        a.mantissa = 0;
    }
    return a;
}

DQ_PARSE_FN bool match_word(const uint8_t* s, int i, int n, const char* w, int wl) {
    if (n - i != wl) return false;
    for (int k = 0; k < wl; ++k)
        if (s[i + k] != (uint8_t)w[k]) return false;
    return true;
}

DQ_PARSE_FN bool java_parse_double(const uint8_t* s, int n, double& out, bool& slow) {
    int i = 0;
    while (i < n && s[i] <= ' ') ++i;  // String.trim
    while (n > i && s[n - 1] <= ' ') --n;
    if (i >= n) return false;
    bool neg = false;
    if (s[i] == '+' || s[i] == '-') {
        neg = s[i] == '-';
        ++i;
    }
    if (i < n && s[i] == 'N') {
        if (!match_word(s, i, n, "NaN", 3)) return false;
        out = parse_bits_double(0x7ff8000000000000ULL);
        return true;
    }
    if (i < n && s[i] == 'I') {
        if (!match_word(s, i, n, "Infinity", 8)) return false;
        out = neg ? -parse_bits_double(0x7ff0000000000000ULL) : parse_bits_double(0x7ff0000000000000ULL);
        return true;
    }
    if (i + 1 < n && s[i] == '0' && (s[i + 1] == 'x' || s[i + 1] == 'X')) {
        // hexadecimal floating-point literal: 0x (hex digits [. hex digits] | . hex digits) p [+-] digits [fFdD].
        // A well-formed one is not converted on the device (slow); anything else is a NumberFormatException.
        int j = i + 2, hd = 0;
        bool hdot = false;
        for (; j < n; ++j) {
            const uint8_t c = s[j];
            const bool hex = (c >= '0' && c <= '9') || (c >= 'a' && c <= 'f') || (c >= 'A' && c <= 'F');
            if (hex) ++hd;
            else if (c == '.' && !hdot) hdot = true;
            else break;
        }
        if (hd == 0 || j >= n || (s[j] != 'p' && s[j] != 'P')) return false;
        ++j;
        if (j < n && (s[j] == '+' || s[j] == '-')) ++j;
        int ed = 0;
        for (; j < n && s[j] >= '0' && s[j] <= '9'; ++j) ++ed;
        if (ed == 0) return false;
        if (j < n && !(j + 1 == n && (s[j] == 'd' || s[j] == 'D' || s[j] == 'f' || s[j] == 'F'))) return false;
        slow = true;
        return false;
    }
    uint64_t w = 0;
    int nd = 0;
    int64_t exp_adj = 0;
    bool any = false, dot = false, trunc = false;
    for (; i < n; ++i) {
        const uint8_t c = s[i];
        if (c >= '0' && c <= '9') {
            any = true;
            if (w == 0 && c == '0') {
                if (dot) --exp_adj;
                continue;
            }
            if (nd < 19) {
                w = w * 10 + (c - '0');
                ++nd;
                if (dot) --exp_adj;
            } else {
                if (!dot) ++exp_adj;
                if (c != '0') trunc = true;
            }
        } else if (c == '.' && !dot) {
            dot = true;
        } else {
            break;
        }
    }
    if (!any) return false;
    if (i < n && (s[i] == 'e' || s[i] == 'E')) {
        ++i;
        bool eneg = false;
        if (i < n && (s[i] == '+' || s[i] == '-')) {
            eneg = s[i] == '-';
            ++i;
        }
        int64_t e = 0;
        int ed = 0;
        for (; i < n && s[i] >= '0' && s[i] <= '9'; ++i, ++ed)
            if (e < 100000000) e = e * 10 + (s[i] - '0');
        if (ed == 0) return false;
        exp_adj += eneg ? -e : e;
    }
    if (i < n) {  // one type suffix may follow
        if (!(i + 1 == n && (s[i] == 'd' || s[i] == 'D' || s[i] == 'f' || s[i] == 'F'))) return false;
    }
    uint64_t bits = 0;
    if (w != 0 && !trunc && w <= (1ull << 53) && exp_adj >= -22 && exp_adj <= 22) {
        // Clinger's fast path: w and 10^|e| (<= 10^22 = 2^22 * 5^22, 5^22 < 2^53) are exact doubles, so one IEEE
        // multiplication or division is the correctly rounded result, as Double.parseDouble's
        double p = 1.0;
        for (int k = 0; k < (exp_adj < 0 ? -exp_adj : exp_adj); ++k) p *= 10.0;
        const double d = exp_adj < 0 ? (double)w / p : (double)w * p;
        bits = parse_double_bits(d);
    } else if (w != 0) {
        const AdjustedMantissa a = el_compute_float(exp_adj, w);
        if (trunc) {
            const AdjustedMantissa b = el_compute_float(exp_adj, w + 1);
            if (a.mantissa != b.mantissa || a.power2 != b.power2) {
                slow = true;
                return false;
            }
        }
        bits = a.mantissa | ((uint64_t)a.power2 << 52);
    }
    if (neg) bits |= 0x8000000000000000ull;
    out = parse_bits_double((uint64_t)bits);
    return true;
}

}  // namespace dq
