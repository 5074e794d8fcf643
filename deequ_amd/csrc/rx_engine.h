// rx_engine.h — the java.util.regex backtracking engine of the GPU (one lane per value) and Spark's
// Cast(x AS STRING) formatters, shared by PatternMatch (regex.hip: regexp_extract(col, p, 0) != "",
// A/PatternMatch.scala:46-48) and the predicate VM's RLIKE (predicate.hip). The program image comes from
// deequ_amd/regex.py; see that module for the supported syntax.
#pragma once

#include <hip/hip_runtime.h>

#include "dq_common.h"
#include "dq_internal.h"

namespace dq {
namespace rx {

enum RxOp : int32_t {
    RX_CHAR = 1, RX_CLASS, RX_ANY, RX_SPLIT, RX_JMP, RX_SAVE, RX_ASSERT, RX_BACKREF, RX_LOOK, RX_LOOKEND, RX_MARK,
    RX_CHECK, RX_MATCH, RX_ATOMIC, RX_ATOMIC_END, RX_STEPBACK, RX_ATPOS
};
// ^ / $ / \Z without and with MULTILINE, and their UNIX_LINES forms (only '\n' ends a line)
enum RxAssert : int32_t {
    AS_BOL = 0, AS_EOL, AS_WORDB, AS_NWORDB, AS_BEGIN, AS_END, AS_ENDZ, AS_MBOL, AS_MEOL, AS_EOL_UNIX, AS_MBOL_UNIX,
    AS_MEOL_UNIX, AS_ENDZ_UNIX
};
// stack frames: a branch to retry, undo records (capture, empty-loop mark), a lookaround (its start position),
// an atomic group's marker, a lookbehind's next start offset to try
enum RxFrame : uint32_t { FR_BRANCH = 0, FR_CAP = 1, FR_LOOP = 2, FR_LOOK = 3, FR_ATOMIC = 4, FR_STEP = 5 };

constexpr int kRxStack = 512;       // frames per lane
constexpr int kRxSteps = 1 << 20;   // instruction budget per row
constexpr int kRxGroups = 10;       // group 0 unused + 9 capturing groups
constexpr int kRxLoops = 16;

struct RxProg {
    const int32_t* ins;      // 3 words per instruction
    const int32_t* classes;  // (first, count) pairs
    const int32_t* ranges;   // (lo, hi) pairs
    int32_t ninstr;
    int32_t anchored;
};

// One code point at byte i (UTF-8); malformed bytes decode as U+FFFD of length 1.
__device__ __forceinline__ int32_t decode(const uint8_t* s, int n, int i, int& len) {
    const uint8_t c = s[i];
    if (c < 0x80) {
        len = 1;
        return c;
    }
    const int need = c >= 0xF0 ? 3 : (c >= 0xE0 ? 2 : (c >= 0xC0 ? 1 : -1));
    if (need < 0 || i + need >= n) {
        len = 1;
        return 0xFFFD;
    }
    int32_t cp = c & (0x3F >> need);
    for (int k = 1; k <= need; ++k) {
        const uint8_t b = s[i + k];
        if ((b & 0xC0) != 0x80) {
            len = 1;
            return 0xFFFD;
        }
        cp = (cp << 6) | (b & 0x3F);
    }
    len = need + 1;
    return cp;
}

// Character.toLowerCase / toUpperCase (xf = 1 / 2) of one code point: the simple case mappings of US-ASCII, Latin-1,
// Latin Extended-A, Greek, Cyrillic and the fullwidth Latin letters (Spark's lower() / upper() = String.toLowerCase /
// toUpperCase; their context- and locale-dependent forms -- final sigma, 'ß' -> "SS", dotted I -- are not applied).
__device__ __forceinline__ int32_t case_map(int32_t c, int xf) {
    if (xf == 0) return c;
    const bool lo = xf == 1;
    if (c < 0x80) {
        if (lo) return (c >= 'A' && c <= 'Z') ? c + 32 : c;
        return (c >= 'a' && c <= 'z') ? c - 32 : c;
    }
    if (c < 0x100) {
        if (lo) return (c >= 0xC0 && c <= 0xDE && c != 0xD7) ? c + 32 : c;
        if (c >= 0xE0 && c <= 0xFE && c != 0xF7) return c - 32;
        if (c == 0xFF) return 0x178;
        if (c == 0xB5) return 0x39C;
        return c;
    }
    if (c < 0x180) {  // Latin Extended-A: (upper, lower) pairs on even / odd code points, shifted in two stretches
        if (c == 0x130 || c == 0x131 || c == 0x138 || c == 0x149 || c == 0x17F) return c == 0x17F && !lo ? 'S' : c;
        if (c == 0x178) return lo ? 0xFF : c;
        const bool odd_upper = (c >= 0x139 && c <= 0x148) || (c >= 0x179 && c <= 0x17E);
        const bool is_upper = odd_upper ? (c & 1) : !(c & 1);
        if (lo) return is_upper ? (odd_upper ? c + 1 : c + 1) : c;
        return is_upper ? c : c - 1;
    }
    if (c >= 0x391 && c <= 0x3CE) {  // Greek
        if (lo) {
            if (c >= 0x391 && c <= 0x3AB && c != 0x3A2) return c + 32;
            return c;
        }
        if (c >= 0x3B1 && c <= 0x3CB && c != 0x3C2) return c - 32;
        if (c == 0x3C2) return 0x3A3;
        if (c == 0x3AC) return 0x386;
        if (c >= 0x3AD && c <= 0x3AF) return c - 37;
        if (c == 0x3CC) return 0x38C;
        if (c == 0x3CD || c == 0x3CE) return c - 63;
        return c;
    }
    if (c >= 0x386 && c <= 0x38F) {
        if (!lo) return c;
        if (c == 0x386) return 0x3AC;
        if (c >= 0x388 && c <= 0x38A) return c + 37;
        if (c == 0x38C) return 0x3CC;
        if (c == 0x38E || c == 0x38F) return c + 63;
        return c;
    }
    if (c >= 0x400 && c <= 0x45F) {  // Cyrillic
        if (lo) return c < 0x410 ? c + 80 : (c < 0x430 ? c + 32 : c);
        return c >= 0x450 ? c - 80 : (c >= 0x430 ? c - 32 : c);
    }
    if (c >= 0xFF21 && c <= 0xFF3A) return lo ? c + 32 : c;
    if (c >= 0xFF41 && c <= 0xFF5A) return lo ? c : c - 32;
    return c;
}

// One code point of a string read under a case transform (xf: 0 none, 1 lower, 2 upper).
__device__ __forceinline__ int32_t decode_xf(const uint8_t* s, int n, int i, int& len, int xf) {
    return case_map(decode(s, n, i, len), xf);
}

// Start of the code point ending at byte i (exclusive), for look-behind of \b.
__device__ __forceinline__ int32_t decode_prev(const uint8_t* s, int n, int i) {
    int j = i - 1;
    while (j > 0 && (s[j] & 0xC0) == 0x80 && i - j < 4) --j;
    int len;
    return decode(s, n, j, len);
}

__device__ __forceinline__ bool is_line_term(int32_t c) {
    return c == '\n' || c == '\r' || c == 0x85 || c == 0x2028 || c == 0x2029;
}

// Character.isLetterOrDigit || '_' (Java's \b), exact for ASCII and Latin-1, coarse above.
__device__ __forceinline__ bool is_word(int32_t c) {
    if (c < 0x80) return (c >= '0' && c <= '9') || (c >= 'A' && c <= 'Z') || (c >= 'a' && c <= 'z') || c == '_';
    if (c < 0xC0) return c == 0xAA || c == 0xB5 || c == 0xBA;
    if (c == 0xD7 || c == 0xF7) return false;
    if ((c >= 0x2000 && c <= 0x2BFF) || (c >= 0x3000 && c <= 0x303F) || (c >= 0xFE30 && c <= 0xFE4F) ||
        (c >= 0xFF00 && c <= 0xFF0F) || c >= 0x1F000)
        return false;
    return true;
}

__device__ __forceinline__ bool in_class(const RxProg& p, int k, int32_t c) {
    const int first = p.classes[2 * k], cnt = p.classes[2 * k + 1];
    const int32_t* r = p.ranges + 2 * first;
    if (cnt <= 8) {
        for (int i = 0; i < cnt; ++i) {
            if (c < r[2 * i]) return false;  // ranges are sorted and disjoint
            if (c <= r[2 * i + 1]) return true;
        }
        return false;
    }
    int lo = 0, hi = cnt - 1;  // Unicode property classes: hundreds of ranges
    while (lo <= hi) {
        const int mid = (lo + hi) >> 1;
        if (c < r[2 * mid]) hi = mid - 1;
        else if (c > r[2 * mid + 1]) lo = mid + 1;
        else return true;
    }
    return false;
}

// Java's CASE_INSENSITIVE back reference (CIBackRef): code points equal, or equal after toUpperCase / toLowerCase
// (US-ASCII letters; with UNICODE_CASE also Latin-1 and the Greek / Cyrillic blocks' simple +-32 / +-80 pairs).
__device__ __forceinline__ int32_t fold_ci(int32_t c, bool unicode) {
    if (c >= 'A' && c <= 'Z') return c + 32;
    if (!unicode) return c;
    if ((c >= 0xC0 && c <= 0xDE && c != 0xD7) || (c >= 0x391 && c <= 0x3AB && c != 0x3A2) || (c >= 0x410 && c <= 0x42F))
        return c + 32;
    if (c >= 0x400 && c <= 0x40F) return c + 80;
    return c;
}

// $ without MULTILINE: end of input, or before a final line terminator ("\r\n" counts as one).
__device__ __forceinline__ bool at_eol(const uint8_t* s, int n, int i) {
    if (i == n) return true;
    int len;
    const int32_t c = decode(s, n, i, len);
    if (c == '\r' && i + 1 < n && s[i + 1] == '\n') return i + 2 == n;
    if (c == '\n' && i > 0 && s[i - 1] == '\r') return false;  // not between "\r" and "\n"
    return is_line_term(c) && i + len == n;
}

// MULTILINE ^: start of input, or after a line terminator, but never at the end of input ("Perl does not match ^ at
// end of input even after newline", Java's Caret; not between the '\r' and '\n' of "\r\n").
__device__ __forceinline__ bool at_mbol(const uint8_t* s, int n, int i) {
    if (i == n) return false;
    if (i == 0) return true;
    const int32_t p = decode_prev(s, n, i);
    if (p == '\r' && s[i] == '\n') return false;
    return is_line_term(p);
}

// MULTILINE $: end of input, or before any line terminator (not between "\r" and "\n").
__device__ __forceinline__ bool at_meol(const uint8_t* s, int n, int i) {
    if (i == n) return true;
    int len;
    const int32_t c = decode(s, n, i, len);
    if (c == '\n' && i > 0 && s[i - 1] == '\r') return false;
    return is_line_term(c);
}

// The code point position k code points before byte i, or -1.
__device__ __forceinline__ int back_cps(const uint8_t* s, int i, int k) {
    for (; k > 0; --k) {
        if (i <= 0) return -1;
        --i;
        int steps = 0;
        while (i > 0 && (s[i] & 0xC0) == 0x80 && steps < 3) { --i; ++steps; }
    }
    return i;
}

__device__ __forceinline__ uint64_t frame(uint32_t kind, uint32_t a, int32_t pos) {
    return ((uint64_t)((kind << 28) | (a & 0x0FFFFFFFu)) << 32) | (uint32_t)pos;
}

// Backtracking match of the program anchored at byte `start`: end position, -1 = no match,
// -2 = resource limit (stack / step budget).
// xf: the value is read lower- / upper-cased (RLIKE over lower(x) / upper(x), predicate.hip).
__device__ inline int rx_match_at(const RxProg& p, const uint8_t* s, int n, int start, uint64_t* stk, int xf = 0) {
    int32_t caps[2 * kRxGroups];
    int32_t loops[kRxLoops];
    for (int k = 0; k < 2 * kRxGroups; ++k) caps[k] = -1;
    for (int k = 0; k < kRxLoops; ++k) loops[k] = -1;
    int top = 0, pc = 0, pos = start;
    for (int steps = 0; steps < kRxSteps; ++steps) {
        const int op = p.ins[3 * pc], a = p.ins[3 * pc + 1], b = p.ins[3 * pc + 2];
        bool ok = true;
        switch (op) {
            case RX_CHAR: {
                int len;
                if (pos < n && decode_xf(s, n, pos, len, xf) == a) { pos += len; ++pc; } else ok = false;
                break;
            }
            case RX_CLASS: {
                int len;
                if (pos < n && in_class(p, a, decode_xf(s, n, pos, len, xf))) { pos += len; ++pc; } else ok = false;
                break;
            }
            case RX_ANY: {
                int len;
                if (pos < n && !is_line_term(decode(s, n, pos, len))) { pos += len; ++pc; } else ok = false;
                break;
            }
            case RX_SPLIT:
                if (top >= kRxStack) return -2;
                stk[top++] = frame(FR_BRANCH, (uint32_t)b, pos);
                pc = a;
                break;
            case RX_JMP: pc = a; break;
            case RX_SAVE:
                if (top >= kRxStack) return -2;
                stk[top++] = frame(FR_CAP, (uint32_t)a, caps[a]);
                caps[a] = pos;
                ++pc;
                break;
            case RX_ASSERT: {
                bool r;
                switch (a) {
                    case AS_BOL: case AS_BEGIN: r = pos == 0; break;
                    case AS_EOL: case AS_ENDZ: r = at_eol(s, n, pos); break;
                    case AS_END: r = pos == n; break;
                    case AS_MBOL: r = at_mbol(s, n, pos); break;
                    case AS_MEOL: r = at_meol(s, n, pos); break;
                    case AS_EOL_UNIX: case AS_ENDZ_UNIX: r = pos == n || (pos + 1 == n && s[pos] == '\n'); break;
                    case AS_MBOL_UNIX: r = pos < n && (pos == 0 || s[pos - 1] == '\n'); break;
                    case AS_MEOL_UNIX: r = pos == n || s[pos] == '\n'; break;
                    default: {
                        int len;
                        const bool left = pos > 0 && is_word(decode_prev(s, n, pos));
                        const bool right = pos < n && is_word(decode(s, n, pos, len));
                        r = (left != right) == (a == AS_WORDB);
                        break;
                    }
                }
                if (r) ++pc; else ok = false;
                break;
            }
            case RX_BACKREF: {
                const int g0 = caps[2 * a], g1 = caps[2 * a + 1];
                if (g0 < 0 || g1 < 0) { ok = false; break; }  // Java: a reference to an unset group fails
                const int len = g1 - g0;
                if (pos + len > n) { ok = false; break; }
                if (b == 0 && xf == 0) {
                    for (int k = 0; k < len && ok; ++k) ok = s[g0 + k] == s[pos + k];
                } else {  // case-insensitive: code point by code point
                    int i0 = g0, i1 = pos;
                    while (ok && i0 < g1) {
                        int l0, l1;
                        const int32_t c0 = decode_xf(s, n, i0, l0, xf);
                        if (i1 >= n) { ok = false; break; }
                        const int32_t c1 = decode_xf(s, n, i1, l1, xf);
                        ok = c0 == c1 || (b != 0 && fold_ci(c0, b == 2) == fold_ci(c1, b == 2));
                        i0 += l0;
                        i1 += l1;
                    }
                    if (ok) { pos = i1; ++pc; }
                    break;
                }
                if (ok) { pos += len; ++pc; }
                break;
            }
            case RX_LOOK:
                if (top >= kRxStack) return -2;
                stk[top++] = frame(FR_LOOK, (uint32_t)(a | (b << 24)), pos);  // b = 1: negative
                ++pc;
                break;
            case RX_LOOKEND: {
                // The lookahead body matched. Find its LOOK frame, drop the frames above it (for
                // (?!X) undoing X's captures, as the whole lookahead then fails).
                int j = top - 1;
                while (j >= 0 && (uint32_t)(stk[j] >> 60) != FR_LOOK) --j;
                if (j < 0) return -2;
                const uint32_t larg = (uint32_t)(stk[j] >> 32) & 0x0FFFFFFFu;
                const bool neg = (larg >> 24) != 0;
                for (int k = top - 1; k > j; --k) {
                    const uint32_t kind = (uint32_t)(stk[k] >> 60), arg = (uint32_t)(stk[k] >> 32) & 0x0FFFFFFFu;
                    const int32_t fp = (int32_t)(uint32_t)stk[k];
                    if (kind == FR_CAP && neg) caps[arg] = fp;
                    if (kind == FR_LOOP) loops[arg] = fp;
                }
                const int32_t lpos = (int32_t)(uint32_t)stk[j];
                top = j;
                if (neg) ok = false;  // (?!X) and X matched
                else {                // (?=X): continue after the group at the original position
                    pos = lpos;
                    pc = (int)(larg & 0xFFFFFF);
                }
                break;
            }
            case RX_MARK:
                if (top >= kRxStack) return -2;
                stk[top++] = frame(FR_LOOP, (uint32_t)a, loops[a]);
                loops[a] = pos;
                ++pc;
                break;
            case RX_CHECK:
                if (pos == loops[a]) ok = false; else ++pc;  // an empty iteration does not repeat
                break;
            case RX_ATOMIC:
                if (top >= kRxStack) return -2;
                stk[top++] = frame(FR_ATOMIC, 0, pos);
                ++pc;
                break;
            case RX_ATOMIC_END: {
                // (?>X) matched: drop X's untried alternatives (branch / lookbehind-start frames) above the marker, keep
                // the undo records so that backtracking past the group still restores captures and loop marks
                int j = top - 1;
                while (j >= 0 && (uint32_t)(stk[j] >> 60) != FR_ATOMIC) --j;
                if (j < 0) return -2;
                int w = j;
                for (int k = j + 1; k < top; ++k) {
                    const uint32_t kind = (uint32_t)(stk[k] >> 60);
                    if (kind == FR_CAP || kind == FR_LOOP) stk[w++] = stk[k];
                }
                top = w;
                ++pc;
                break;
            }
            case RX_STEPBACK:
            case RX_ATPOS: {
                // lookbehind: the LOOK frame below holds the position the body must end at
                int j = top - 1;
                while (j >= 0 && (uint32_t)(stk[j] >> 60) != FR_LOOK) --j;
                if (j < 0) return -2;
                const int32_t target = (int32_t)(uint32_t)stk[j];
                if (op == RX_ATPOS) {
                    if (pos == target) ++pc; else ok = false;
                    break;
                }
                const int st = back_cps(s, target, a);  // first try: `a` (the minimum length) code points back
                if (st < 0 || a > b) { ok = false; break; }
                if (top >= kRxStack) return -2;
                stk[top++] = frame(FR_STEP, (uint32_t)pc, a + 1);
                pos = st;
                ++pc;
                break;
            }
            case RX_MATCH: return pos;
            default: return -2;
        }
        if (ok) continue;
        // backtrack
        for (;;) {
            if (top == 0) return -1;
            const uint64_t f = stk[--top];
            const uint32_t kind = (uint32_t)(f >> 60), arg = (uint32_t)(f >> 32) & 0x0FFFFFFFu;
            const int32_t fp = (int32_t)(uint32_t)f;
            if (kind == FR_BRANCH) { pc = (int)arg; pos = fp; break; }
            if (kind == FR_CAP) { caps[arg] = fp; continue; }
            if (kind == FR_LOOP) { loops[arg] = fp; continue; }
            if (kind == FR_ATOMIC) continue;
            if (kind == FR_STEP) {  // the lookbehind body failed from this start: one more code point back
                const int k = fp, maxk = p.ins[3 * arg + 2];
                if (k > maxk) continue;
                int j = top - 1;
                while (j >= 0 && (uint32_t)(stk[j] >> 60) != FR_LOOK) --j;
                if (j < 0) return -2;
                const int st = back_cps(s, (int32_t)(uint32_t)stk[j], k);
                if (st < 0) continue;
                stk[top++] = frame(FR_STEP, arg, k + 1);
                pos = st;
                pc = (int)arg + 1;
                break;
            }
            // FR_LOOK: the lookahead body failed
            if (arg >> 24) { pos = fp; pc = (int)(arg & 0xFFFFFF); break; }  // (?!X): succeeds
        }
    }
    return -2;
}

// Spark's cast of an integral value to its decimal string.
__device__ inline int format_long(int64_t v, uint8_t* buf) {
    uint8_t tmp[20];
    uint64_t m = v < 0 ? (uint64_t)0 - (uint64_t)v : (uint64_t)v;
    int k = 0;
    do {
        tmp[k++] = (uint8_t)('0' + m % 10);
        m /= 10;
    } while (m);
    int n = 0;
    if (v < 0) buf[n++] = '-';
    while (k) buf[n++] = tmp[--k];
    return n;
}

// Spark 2.2's Cast(decimal AS STRING) = Decimal.toString = java.math.BigDecimal.toString of the unscaled Long at
// the column scale: plain notation while the adjusted exponent (digits - 1 - scale) is >= -6, scientific below
// ("1E-7", "0E-7", "1.5E-8"); scale >= 0 for every Spark DecimalType, so no "E+".
__device__ inline int format_decimal(int64_t unscaled, int scale, uint8_t* buf) {
    uint8_t d[20];
    uint64_t m = unscaled < 0 ? (uint64_t)0 - (uint64_t)unscaled : (uint64_t)unscaled;
    int k = 0;
    do {
        d[k++] = (uint8_t)('0' + m % 10);
        m /= 10;
    } while (m);  // d[k-1] is the most significant digit
    int n = 0;
    if (unscaled < 0) buf[n++] = '-';
    const int adjusted = k - 1 - scale;
    if (adjusted >= -6) {
        if (scale == 0) {
            for (int i = k - 1; i >= 0; --i) buf[n++] = d[i];
        } else if (k > scale) {
            for (int i = k - 1; i >= scale; --i) buf[n++] = d[i];
            buf[n++] = '.';
            for (int i = scale - 1; i >= 0; --i) buf[n++] = d[i];
        } else {
            buf[n++] = '0';
            buf[n++] = '.';
            for (int i = 0; i < scale - k; ++i) buf[n++] = '0';
            for (int i = k - 1; i >= 0; --i) buf[n++] = d[i];
        }
        return n;
    }
    buf[n++] = d[k - 1];
    if (k > 1) {
        buf[n++] = '.';
        for (int i = k - 2; i >= 0; --i) buf[n++] = d[i];
    }
    buf[n++] = 'E';
    buf[n++] = '-';
    return n + format_long(-(int64_t)adjusted, buf + n);
}

__device__ __forceinline__ int64_t floor_div(int64_t a, int64_t b) {
    const int64_t q = a / b;
    return (a % b != 0 && ((a < 0) != (b < 0))) ? q - 1 : q;
}

// The civil date of a day number (days since 1970-01-01) as java.text.SimpleDateFormat prints it with its default
// GregorianCalendar: Gregorian from 1582-10-15 (Julian Day 2299161), the Julian calendar before the cutover
// (E. G. Richards' day-number conversions). `year` is the year of era (1 BC prints as 1: "yyyy" shows no era).
__device__ inline void civil_from_days(int64_t days, int64_t* year, int* month, int* day) {
    const int64_t J = days + 2440588;
    int64_t f = J + 1401;
    if (J >= 2299161) f += floor_div(floor_div(4 * J + 274277, 146097) * 3, 4) - 38;
    const int64_t e = 4 * f + 3;
    const int64_t g = floor_div(e - floor_div(e, 1461) * 1461, 4);
    const int64_t h = 5 * g + 2;
    *day = (int)(floor_div(h - floor_div(h, 153) * 153, 5) + 1);
    *month = (int)((floor_div(h, 153) + 2) % 12 + 1);
    const int64_t y = floor_div(e, 1461) - 4716 + (12 + 2 - *month) / 12;  // astronomical year
    *year = y >= 1 ? y : 1 - y;
}

__device__ __forceinline__ int put2(int v, uint8_t* b) {
    b[0] = (uint8_t)('0' + v / 10);
    b[1] = (uint8_t)('0' + v % 10);
    return 2;
}

// "yyyy-MM-dd" (at least four year digits, more when needed).
__device__ inline int format_date_days(int64_t days, uint8_t* buf) {
    int64_t y;
    int mo, d;
    civil_from_days(days, &y, &mo, &d);
    int n = 0;
    for (int64_t p = 1000; p > y && p > 1; p /= 10) buf[n++] = '0';
    n += format_long(y, buf + n);
    buf[n++] = '-';
    n += put2(mo, buf + n);
    buf[n++] = '-';
    return n + put2(d, buf + n);
}

// Spark 2.2's Cast(timestamp AS STRING) (DateTimeUtils.timestampToString) in a UTC session time zone:
// "yyyy-MM-dd HH:mm:ss" of the floored second, then java.sql.Timestamp.toString's fraction (the microseconds as
// nanoseconds, trailing zeros dropped) unless it is ".0".
__device__ inline int format_timestamp_utc(int64_t micros, uint8_t* buf) {
    const int64_t secs = floor_div(micros, 1000000);
    const int64_t frac = micros - secs * 1000000;
    const int64_t days = floor_div(secs, 86400);
    const int64_t sod = secs - days * 86400;
    int n = format_date_days(days, buf);
    buf[n++] = ' ';
    n += put2((int)(sod / 3600), buf + n);
    buf[n++] = ':';
    n += put2((int)(sod / 60 % 60), buf + n);
    buf[n++] = ':';
    n += put2((int)(sod % 60), buf + n);
    if (frac) {
        buf[n++] = '.';
        int64_t f = frac, div = 100000;
        while (f) {
            buf[n++] = (uint8_t)('0' + f / div);
            f %= div;
            div /= 10;
        }
    }
    return n;
}

}  // namespace rx
}  // namespace dq
