// java_dtoa.h — java.lang.Double.toString / Float.toString on the device (host + device code).
//
// Spark's Cast(x AS STRING) of a DOUBLE / FLOAT value is the boxed value's toString (spark-catalyst 2.2.2,
// third-party): the shortest decimal digits that round-trip to the value, in plain notation for
// 1e-3 <= |x| < 1e7 ("123.45", "0.001", "1.0") and computerised scientific notation otherwise ("1.0E10",
// "1.234E-5"); "NaN", "Infinity", "-Infinity", "0.0", "-0.0". PatternMatch (A/PatternMatch.scala:46-48) and the
// oracle (oracle/oracle.py java_double_to_string) work on that text.
//
// The shortest digits are computed with Ryu (U. Adams, "Ryu: fast float-to-string conversion", PLDI 2018):
// the rounding interval of the value scaled by an exact 128-bit power of five (ryu_tables.h, generated), then
// digits removed while the interval still separates them. The same routine serves FLOAT: its 24-bit mantissa
// and exponent give the float's own (wider) interval, so the digits are Float.toString's. Java 8's
// FloatingDecimal is not always shortest (JDK-4511638; e.g. Double.MIN_VALUE prints 4.9E-324): those
// documented exceptions are not reproduced — the oracle restates the shortest form too (parity unpinned there).
#pragma once

#include <stdint.h>

#include "ryu_tables.h"

#ifndef DQ_HD
#define DQ_HD __host__ __device__ __forceinline__
#endif

namespace dq {

DQ_HD uint32_t ryu_pow5bits(int32_t e) { return (uint32_t)(((e * 1217359) >> 19) + 1); }
DQ_HD uint32_t ryu_log10pow2(int32_t e) { return (uint32_t)((e * 78913) >> 18); }
DQ_HD uint32_t ryu_log10pow5(int32_t e) { return (uint32_t)((e * 732923) >> 20); }

DQ_HD bool ryu_multiple_of_pow5(uint64_t v, uint32_t p) {
    uint32_t count = 0;
    for (;;) {
        if (v % 5 != 0) break;
        v /= 5;
        ++count;
    }
    return count >= p;
}

// (m * mul) >> j for the 128-bit multiplier mul = (lo, hi), j >= 64.
DQ_HD uint64_t ryu_mul_shift(uint64_t m, uint64_t lo, uint64_t hi, int32_t j) {
    const unsigned __int128 b0 = (unsigned __int128)m * lo;
    const unsigned __int128 b2 = (unsigned __int128)m * hi;
    return (uint64_t)(((b0 >> 64) + b2) >> (j - 64));
}

DQ_HD void ryu_table(bool inverse, int idx, uint64_t& lo, uint64_t& hi) {
#if defined(__HIP_DEVICE_COMPILE__)
    if (inverse) { lo = kPow5InvSplit_d[idx][0]; hi = kPow5InvSplit_d[idx][1]; }
    else { lo = kPow5Split_d[idx][0]; hi = kPow5Split_d[idx][1]; }
#else
    if (inverse) { lo = kPow5InvSplit_h[idx][0]; hi = kPow5InvSplit_h[idx][1]; }
    else { lo = kPow5Split_h[idx][0]; hi = kPow5Split_h[idx][1]; }
#endif
}

// Shortest round-trip decimal of the finite, non-zero binary value m2 * 2^e2 (e2 already including the
// -2 of Ryu's 4x scaling) whose format has the interval flags `mm_shift` / `accept_bounds`: digits `out`,
// decimal exponent `exp10` (value = out * 10^exp10).
DQ_HD void ryu_shortest(uint64_t m2, int32_t e2, bool mm_shift, bool accept_bounds, uint64_t& out, int32_t& exp10) {
    const uint64_t mv = 4 * m2;
    const uint32_t mmShift = mm_shift ? 1u : 0u;
    uint64_t vr, vp, vm;
    int32_t e10;
    bool vmTrailingZeros = false, vrTrailingZeros = false;
    uint64_t lo, hi;
    if (e2 >= 0) {
        const uint32_t q = ryu_log10pow2(e2) - (e2 > 3);
        e10 = (int32_t)q;
        const int32_t k = 125 + (int32_t)ryu_pow5bits((int32_t)q) - 1;
        const int32_t i = -e2 + (int32_t)q + k;
        ryu_table(true, (int)q, lo, hi);
        vr = ryu_mul_shift(4 * m2, lo, hi, i);
        vp = ryu_mul_shift(4 * m2 + 2, lo, hi, i);
        vm = ryu_mul_shift(4 * m2 - 1 - mmShift, lo, hi, i);
        if (q <= 21) {
            if (mv % 5 == 0) vrTrailingZeros = ryu_multiple_of_pow5(mv, q);
            else if (accept_bounds) vmTrailingZeros = ryu_multiple_of_pow5(mv - 1 - mmShift, q);
            else vp -= ryu_multiple_of_pow5(mv + 2, q);
        }
    } else {
        const uint32_t q = ryu_log10pow5(-e2) - (-e2 > 1);
        e10 = (int32_t)q + e2;
        const int32_t i = -e2 - (int32_t)q;
        const int32_t k = (int32_t)ryu_pow5bits(i) - 125;
        const int32_t j = (int32_t)q - k;
        ryu_table(false, i, lo, hi);
        vr = ryu_mul_shift(4 * m2, lo, hi, j);
        vp = ryu_mul_shift(4 * m2 + 2, lo, hi, j);
        vm = ryu_mul_shift(4 * m2 - 1 - mmShift, lo, hi, j);
        if (q <= 1) {
            vrTrailingZeros = true;
            if (accept_bounds) vmTrailingZeros = mmShift == 1;
            else --vp;
        } else if (q < 63) {
            vrTrailingZeros = (mv & ((1ull << q) - 1)) == 0;
        }
    }
    int32_t removed = 0;
    uint8_t lastRemoved = 0;
    uint64_t output;
    if (vmTrailingZeros || vrTrailingZeros) {
        while (vp / 10 > vm / 10) {
            vmTrailingZeros &= vm % 10 == 0;
            vrTrailingZeros &= lastRemoved == 0;
            lastRemoved = (uint8_t)(vr % 10);
            vr /= 10;
            vp /= 10;
            vm /= 10;
            ++removed;
        }
        if (vmTrailingZeros) {
            while (vm % 10 == 0) {
                vrTrailingZeros &= lastRemoved == 0;
                lastRemoved = (uint8_t)(vr % 10);
                vr /= 10;
                vp /= 10;
                vm /= 10;
                ++removed;
            }
        }
        if (vrTrailingZeros && lastRemoved == 5 && vr % 2 == 0) lastRemoved = 4;  // round half to even
        output = vr + ((vr == vm && (!accept_bounds || !vmTrailingZeros)) || lastRemoved >= 5);
    } else {
        bool roundUp = false;
        if (vp / 100 > vm / 100) {
            roundUp = vr % 100 >= 50;
            vr /= 100;
            vp /= 100;
            vm /= 100;
            removed += 2;
        }
        while (vp / 10 > vm / 10) {
            roundUp = vr % 10 >= 5;
            vr /= 10;
            vp /= 10;
            vm /= 10;
            ++removed;
        }
        output = vr + (vr == vm || roundUp);
    }
    out = output;
    exp10 = e10 + removed;
}

// Java's layout of (sign, digits, exponent): plain for 1e-3 <= |x| < 1e7, else d.dddE<exp>. Returns the length.
DQ_HD int java_layout(bool neg, uint64_t digits, int32_t exp10, bool plain, uint8_t* buf) {
    uint8_t d[20];
    int nd = 0;
    do {
        d[nd++] = (uint8_t)('0' + digits % 10);
        digits /= 10;
    } while (digits);
    // d[nd-1] is the most significant digit; value = 0.d1 d2 ... dn * 10^(exp10 + nd)
    int n = 0;
    if (neg) buf[n++] = '-';
    const int point = exp10 + nd;  // digits before the decimal point
    if (plain) {
        if (point <= 0) {
            buf[n++] = '0';
            buf[n++] = '.';
            for (int z = 0; z < -point; ++z) buf[n++] = '0';
            for (int k = nd - 1; k >= 0; --k) buf[n++] = d[k];
        } else if (point >= nd) {
            for (int k = nd - 1; k >= 0; --k) buf[n++] = d[k];
            for (int z = 0; z < point - nd; ++z) buf[n++] = '0';
            buf[n++] = '.';
            buf[n++] = '0';
        } else {
            for (int k = nd - 1; k >= 0; --k) {
                buf[n++] = d[k];
                if (k == nd - point) buf[n++] = '.';
            }
        }
        return n;
    }
    buf[n++] = d[nd - 1];
    buf[n++] = '.';
    if (nd == 1) buf[n++] = '0';
    for (int k = nd - 2; k >= 0; --k) buf[n++] = d[k];
    buf[n++] = 'E';
    int e = point - 1;
    if (e < 0) {
        buf[n++] = '-';
        e = -e;
    }
    uint8_t t[4];
    int nt = 0;
    do {
        t[nt++] = (uint8_t)('0' + e % 10);
        e /= 10;
    } while (e);
    while (nt) buf[n++] = t[--nt];
    return n;
}

DQ_HD int java_special(uint64_t bits, int exp_bits_all_ones, bool mant_zero, bool is_zero, bool neg, uint8_t* buf) {
    const char* s = nullptr;
    if (exp_bits_all_ones) s = !mant_zero ? "NaN" : (neg ? "-Infinity" : "Infinity");
    else if (is_zero) s = neg ? "-0.0" : "0.0";
    if (!s) return -1;
    int n = 0;
    while (s[n]) {
        buf[n] = (uint8_t)s[n];
        ++n;
    }
    (void)bits;
    return n;
}

// java.lang.Double.toString(d) into buf (>= 25 bytes); returns the length.
DQ_HD int java_double_to_chars(double d, uint8_t* buf) {
    union { double d; uint64_t u; } c;
    c.d = d;
    const uint64_t bits = c.u;
    const bool neg = (bits >> 63) != 0;
    const uint32_t ieeeExp = (uint32_t)((bits >> 52) & 0x7FFu);
    const uint64_t ieeeMant = bits & ((1ull << 52) - 1);
    const int sp = java_special(bits, ieeeExp == 0x7FFu, ieeeMant == 0, ieeeExp == 0 && ieeeMant == 0, neg, buf);
    if (sp >= 0) return sp;
    uint64_t m2;
    int32_t e2;
    if (ieeeExp == 0) {
        m2 = ieeeMant;
        e2 = 1 - 1023 - 52 - 2;
    } else {
        m2 = (1ull << 52) | ieeeMant;
        e2 = (int32_t)ieeeExp - 1023 - 52 - 2;
    }
    uint64_t out;
    int32_t e10;
    ryu_shortest(m2, e2, ieeeMant != 0 || ieeeExp <= 1, (m2 & 1) == 0, out, e10);
    const double a = neg ? -d : d;
    return java_layout(neg, out, e10, a >= 1e-3 && a < 1e7, buf);
}

// java.lang.Float.toString(f) into buf (>= 25 bytes); returns the length.
DQ_HD int java_float_to_chars(float f, uint8_t* buf) {
    union { float f; uint32_t u; } c;
    c.f = f;
    const uint32_t bits = c.u;
    const bool neg = (bits >> 31) != 0;
    const uint32_t ieeeExp = (bits >> 23) & 0xFFu;
    const uint32_t ieeeMant = bits & ((1u << 23) - 1);
    const int sp = java_special(bits, ieeeExp == 0xFFu, ieeeMant == 0, ieeeExp == 0 && ieeeMant == 0, neg, buf);
    if (sp >= 0) return sp;
    uint64_t m2;
    int32_t e2;
    if (ieeeExp == 0) {
        m2 = ieeeMant;
        e2 = 1 - 127 - 23 - 2;
    } else {
        m2 = (1u << 23) | ieeeMant;
        e2 = (int32_t)ieeeExp - 127 - 23 - 2;
    }
    uint64_t out;
    int32_t e10;
    ryu_shortest(m2, e2, ieeeMant != 0 || ieeeExp <= 1, (m2 & 1) == 0, out, e10);
    const float a = neg ? -f : f;
    return java_layout(neg, out, e10, a >= 1e-3f && a < 1e7f, buf);
}

}  // namespace dq
