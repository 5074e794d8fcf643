// predicate.hip — row predicates for `where` filters and Compliance (gfx950).
//
// deequ passes Spark SQL strings: `where` (conditionalSelection / conditionalCount,
// A/Analyzer.scala:409-432) and Compliance predicates (A/Compliance.scala:49-52). The host
// compiles them to a postfix program (dq_pred_opcode, include/dq.h); this kernel evaluates it for
// one row per lane with SQL three-valued logic and emits two bitmaps per 64 rows via wave ballots:
// TRUE rows and NOT-NULL rows. Rows past nrows (up to the padded length) get zero bits.
// The program is wave-uniform, so every dispatch branch below is a uniform (scalar) branch.
#include <hip/hip_runtime.h>

#include <math.h>

#include "dq_common.h"
#include "dq_internal.h"
#include "dq_parse.h"
#include "java_dtoa.h"
#include "rx_engine.h"

namespace dq {

namespace {

struct Val {
    int32_t tag;   // dq_value_tag
    int32_t null;
    int64_t i;     // BOOL / LONG
    double d;      // DOUBLE
    const uint8_t* s;
    int32_t slen;
    int32_t xf;    // STRING read through lower() / upper(): 0 none, 1 lower, 2 upper (rx::case_map)
};

__device__ __forceinline__ Val vnull() {
    Val v;
    v.tag = DQ_V_BOOL;
    v.null = 1;
    v.i = 0;
    v.d = 0.0;
    v.s = nullptr;
    v.slen = 0;
    v.xf = 0;
    return v;
}
__device__ __forceinline__ Val vbool(bool b) {
    Val v = vnull();
    v.null = 0;
    v.i = b ? 1 : 0;
    return v;
}
__device__ __forceinline__ Val vlong(int64_t x) {
    Val v = vnull();
    v.tag = DQ_V_LONG;
    v.null = 0;
    v.i = x;
    return v;
}
__device__ __forceinline__ Val vdouble(double x) {
    Val v = vnull();
    v.tag = DQ_V_DOUBLE;
    v.null = 0;
    v.d = x;
    return v;
}

__device__ __forceinline__ bool is_ws(uint8_t c) { return c == ' ' || c == '\t' || c == '\n' || c == '\r'; }

__device__ const double kPow10[23] = {1e0,  1e1,  1e2,  1e3,  1e4,  1e5,  1e6,  1e7,  1e8,  1e9,  1e10, 1e11,
                                      1e12, 1e13, 1e14, 1e15, 1e16, 1e17, 1e18, 1e19, 1e20, 1e21, 1e22};

// Spark Cast(string -> double) = java.lang.Double.parseDouble, correctly rounded (dq_parse.h). The
// rare literal it cannot round on the device (hexadecimal, or > 19 significant digits on a rounding
// boundary) falls back to a plain decimal scale here: predicates have no per-row error channel.
__device__ bool parse_double_approx(const uint8_t* s, int n, double& out) {
    int i = 0;
    while (i < n && s[i] <= ' ') ++i;
    while (n > i && s[n - 1] <= ' ') --n;
    if (i >= n) return false;
    bool neg = false;
    if (s[i] == '+' || s[i] == '-') {
        neg = s[i] == '-';
        ++i;
    }
    double v = 0.0;
    int exp10 = 0, nd = 0;
    bool seen_dot = false;
    for (; i < n; ++i) {
        const uint8_t c = s[i];
        if (c >= '0' && c <= '9') {
            ++nd;
            v = v * 10.0 + (c - '0');
            if (seen_dot) --exp10;
        } else if (c == '.' && !seen_dot) {
            seen_dot = true;
        } else {
            break;
        }
    }
    if (nd == 0) return false;
    if (i < n && (s[i] == 'e' || s[i] == 'E')) {
        ++i;
        bool eneg = false;
        if (i < n && (s[i] == '+' || s[i] == '-')) {
            eneg = s[i] == '-';
            ++i;
        }
        int e = 0;
        for (; i < n && s[i] >= '0' && s[i] <= '9'; ++i) e = e < 10000 ? e * 10 + (s[i] - '0') : e;
        exp10 += eneg ? -e : e;
    }
    while (exp10 > 22) { v *= 1e22; exp10 -= 22; }
    while (exp10 < -22) { v /= 1e22; exp10 += 22; }
    v = exp10 >= 0 ? v * kPow10[exp10] : v / kPow10[-exp10];
    out = neg ? -v : v;
    return true;
}

__device__ bool parse_double(const uint8_t* s, int n, double& out) {
    bool slow = false;
    if (java_parse_double(s, n, out, slow)) return true;
    return slow ? parse_double_approx(s, n, out) : false;
}

// Spark 2.2 Cast(string -> long) = UTF8String.toLong (dq_parse.h).
__device__ bool parse_long(const uint8_t* s, int n, int64_t& out) { return spark_string_to_long(s, n, out); }

__device__ __forceinline__ bool numeric(const Val& v) { return v.tag == DQ_V_LONG || v.tag == DQ_V_DOUBLE || v.tag == DQ_V_BOOL; }
__device__ __forceinline__ double as_double(const Val& v) { return v.tag == DQ_V_DOUBLE ? v.d : (double)v.i; }

// Spark's NaN-aware double ordering (NaN = NaN, NaN greatest).
__device__ __forceinline__ int cmp_double(double a, double b) {
    const bool an = a != a, bn = b != b;
    if (an && bn) return 0;
    if (an) return 1;
    if (bn) return -1;
    return a < b ? -1 : (a > b ? 1 : 0);
}

__device__ int cmp_bytes(const uint8_t* a, int na, const uint8_t* b, int nb) {
    const int n = na < nb ? na : nb;
    for (int i = 0; i < n; ++i)
        if (a[i] != b[i]) return a[i] < b[i] ? -1 : 1;
    return na < nb ? -1 : (na > nb ? 1 : 0);
}

// Binary (UTF-8 byte) order of two strings, each possibly read through lower() / upper(): UTF-8 preserves code point
// order, so the mapped code point sequences compare like their encodings.
__device__ int cmp_str(const Val& a, const Val& b) {
    if (a.xf == 0 && b.xf == 0) return cmp_bytes(a.s, a.slen, b.s, b.slen);
    int i = 0, j = 0;
    while (i < a.slen && j < b.slen) {
        int la, lb;
        const int32_t ca = rx::decode_xf(a.s, a.slen, i, la, a.xf), cb = rx::decode_xf(b.s, b.slen, j, lb, b.xf);
        if (ca != cb) return ca < cb ? -1 : 1;
        i += la;
        j += lb;
    }
    return (i < a.slen) ? 1 : ((j < b.slen) ? -1 : 0);
}

// The bytes of a string value for the numeric parsers: a transformed value is mapped into `buf` (numbers are ASCII;
// a longer value is parsed as stored -- it cannot be a number whose parse depends on letter case).
__device__ __forceinline__ const uint8_t* str_bytes(const Val& v, uint8_t (&buf)[64], int& n) {
    n = v.slen;
    if (v.xf == 0 || v.slen > 64) return v.s;
    for (int k = 0; k < v.slen; ++k) {
        const uint8_t c = v.s[k];
        buf[k] = c < 0x80 ? (uint8_t)rx::case_map(c, v.xf) : c;
    }
    return buf;
}

__device__ bool parse_double_v(const Val& v, double& out) {
    uint8_t buf[64];
    int n;
    const uint8_t* p = str_bytes(v, buf, n);
    return parse_double(p, n, out);
}

// Coerce a string operand against a numeric one the way Spark 2.x PromoteStrings does
// (string -> double). Returns false when the string does not parse (comparison is NULL).
__device__ bool compare(const Val& a, const Val& b, int& c) {
    if (a.tag == DQ_V_STRING && b.tag == DQ_V_STRING) {
        c = cmp_str(a, b);
        return true;
    }
    if (a.tag == DQ_V_STRING || b.tag == DQ_V_STRING) {
        double x, y;
        if (a.tag == DQ_V_STRING) {
            if (!parse_double_v(a, x)) return false;
        } else {
            x = as_double(a);
        }
        if (b.tag == DQ_V_STRING) {
            if (!parse_double_v(b, y)) return false;
        } else {
            y = as_double(b);
        }
        c = cmp_double(x, y);
        return true;
    }
    if (a.tag != DQ_V_DOUBLE && b.tag != DQ_V_DOUBLE) {
        c = a.i < b.i ? -1 : (a.i > b.i ? 1 : 0);
        return true;
    }
    c = cmp_double(as_double(a), as_double(b));
    return true;
}

// SQL LIKE with % and _ over UTF-8 (one _ = one character); '\' escapes.
__device__ bool like_match(const uint8_t* s, int ns, const uint8_t* p, int np) {
    int si = 0, pi = 0, star_p = -1, star_s = 0;
    while (si < ns) {
        if (pi < np && p[pi] == '%') {
            star_p = ++pi;
            star_s = si;
            continue;
        }
        if (pi < np) {
            bool esc = p[pi] == '\\' && pi + 1 < np;
            const uint8_t pc = esc ? p[pi + 1] : p[pi];
            if (!esc && pc == '_') {
                int len = 1;
                const uint8_t c = s[si];
                if (c >= 0xF0) len = 4;
                else if (c >= 0xE0) len = 3;
                else if (c >= 0xC0) len = 2;
                si += len;
                pi += 1;
                continue;
            }
            if (pc == s[si]) {
                si += 1;
                pi += esc ? 2 : 1;
                continue;
            }
        }
        if (star_p >= 0) {
            pi = star_p;
            si = ++star_s;
            continue;
        }
        return false;
    }
    while (pi < np && p[pi] == '%') ++pi;
    return pi == np;
}

// LIKE over a value read through lower() / upper(): code point by code point ('_' = one character, '%' = any run,
// '\\' escapes), backtracking to the last '%' like like_match.
__device__ bool like_match_xf(const uint8_t* s, int ns, int xf, const uint8_t* p, int np) {
    int si = 0, pi = 0, star_p = -1, star_s = 0;
    while (si < ns) {
        int ls;
        const int32_t c = rx::decode_xf(s, ns, si, ls, xf);
        if (pi < np && p[pi] == '%') {
            star_p = ++pi;
            star_s = si;
            continue;
        }
        if (pi < np) {
            const bool esc = p[pi] == '\\' && pi + 1 < np;
            int lp;
            const int32_t pc = rx::decode(p, np, esc ? pi + 1 : pi, lp);
            if (!esc && pc == '_') {
                si += ls;
                pi += 1;
                continue;
            }
            if (pc == c) {
                si += ls;
                pi += (esc ? 1 : 0) + lp;
                continue;
            }
        }
        if (star_p >= 0) {
            pi = star_p;
            int l0;
            rx::decode(s, ns, star_s, l0);
            star_s += l0;
            si = star_s;
            continue;
        }
        return false;
    }
    while (pi < np && p[pi] == '%') ++pi;
    return pi == np;
}

__device__ __forceinline__ int utf8_chars(const uint8_t* s, int n) {
    int c = 0;
    for (int i = 0; i < n; ++i) c += (s[i] & 0xC0) != 0x80;
    return c;
}

__device__ Val load_col(const PredColumn& c, int64_t row) {
    if (c.validity) {
        const uint8_t* vb = reinterpret_cast<const uint8_t*>(c.validity);
        if (!((vb[row >> 3] >> (row & 7)) & 1)) return vnull();
    }
    switch (c.spark_type) {
        case DQ_TYPE_BOOLEAN: return vbool(static_cast<const uint8_t*>(c.values)[row] != 0);
        case DQ_TYPE_BYTE: return vlong(static_cast<const int8_t*>(c.values)[row]);
        case DQ_TYPE_SHORT: return vlong(static_cast<const int16_t*>(c.values)[row]);
        case DQ_TYPE_INT:
        case DQ_TYPE_DATE: return vlong(static_cast<const int32_t*>(c.values)[row]);
        case DQ_TYPE_LONG:
        case DQ_TYPE_TIMESTAMP: return vlong(static_cast<const int64_t*>(c.values)[row]);
        case DQ_TYPE_DECIMAL: {
            double d = (double)static_cast<const int64_t*>(c.values)[row];
            for (int k = 0; k < c.decimal_scale; ++k) d /= 10.0;
            return vdouble(d);
        }
        case DQ_TYPE_FLOAT: return vdouble((double)static_cast<const float*>(c.values)[row]);
        case DQ_TYPE_DOUBLE: return vdouble(static_cast<const double*>(c.values)[row]);
        case DQ_TYPE_STRING: {
            Val v = vnull();
            v.tag = DQ_V_STRING;
            v.null = 0;
            const int32_t o0 = c.offsets[row], o1 = c.offsets[row + 1];
            v.s = static_cast<const uint8_t*>(c.values) + o0;
            v.slen = o1 - o0;
            return v;
        }
        default: return vnull();
    }
}

__device__ Val arith(int op, const Val& a, const Val& b) {
    if (a.null || b.null) return vnull();
    Val x = a, y = b;
    if (x.tag == DQ_V_STRING) {
        double d;
        if (!parse_double_v(x, d)) return vnull();
        x = vdouble(d);
    }
    if (y.tag == DQ_V_STRING) {
        double d;
        if (!parse_double_v(y, d)) return vnull();
        y = vdouble(d);
    }
    const bool integral = x.tag != DQ_V_DOUBLE && y.tag != DQ_V_DOUBLE;
    switch (op) {
        case DQ_P_ADD: return integral ? vlong((int64_t)((uint64_t)x.i + (uint64_t)y.i)) : vdouble(as_double(x) + as_double(y));
        case DQ_P_SUB: return integral ? vlong((int64_t)((uint64_t)x.i - (uint64_t)y.i)) : vdouble(as_double(x) - as_double(y));
        case DQ_P_MUL: return integral ? vlong((int64_t)((uint64_t)x.i * (uint64_t)y.i)) : vdouble(as_double(x) * as_double(y));
        case DQ_P_DIV: {  // Spark `/` is fractional division; x / 0 is NULL
            const double dy = as_double(y);
            if (dy == 0.0) return vnull();
            return vdouble(as_double(x) / dy);
        }
        case DQ_P_MOD:
            if (integral) {
                if (y.i == 0) return vnull();
                return vlong(x.i % y.i);
            } else {
                const double dy = as_double(y);
                if (dy == 0.0) return vnull();
                return vdouble(fmod(as_double(x), dy));
            }
        default: return vnull();
    }
}

// Spark 2.2 DateTimeUtils.getYear / getMonth / getDayOfMonth of a day number (days since 1970-01-01): the
// proleptic Gregorian civil date of the day number, shifted back 10 days on or before 1582-10-04 (day -141428)
// as getYearAndDayInYear does for the Julian-to-Gregorian gap.
__device__ void spark_ymd(int64_t days, int64_t& y, int& m, int& d) {
    if (days <= -141428) days -= 10;
    const int64_t z = days + 719468;  // H. Hinnant's days_from_civil inverse
    const int64_t era = (z >= 0 ? z : z - 146096) / 146097;
    const int64_t doe = z - era * 146097;
    const int64_t yoe = (doe - doe / 1460 + doe / 36524 - doe / 146096) / 365;
    const int64_t doy = doe - (365 * yoe + yoe / 4 - yoe / 100);
    const int64_t mp = (5 * doy + 2) / 153;
    d = (int)(doy - (153 * mp + 2) / 5 + 1);
    m = (int)(mp < 10 ? mp + 3 : mp - 9);
    y = yoe + era * 400 + (m <= 2 ? 1 : 0);
}

// Spark's Cast(x AS STRING) of a non-string operand of RLIKE into buf (rx_engine.h formatters, java_dtoa.h).
__device__ int value_string(const Val& v, int spark_type, int scale, uint8_t* buf) {
    if (v.tag == DQ_V_BOOL) {
        const char* t = v.i ? "true" : "false";
        const int n = v.i ? 4 : 5;
        for (int k = 0; k < n; ++k) buf[k] = (uint8_t)t[k];
        return n;
    }
    if (v.tag == DQ_V_DOUBLE) return spark_type == DQ_TYPE_FLOAT ? java_float_to_chars((float)v.d, buf)
                                                                 : java_double_to_chars(v.d, buf);
    if (spark_type == DQ_TYPE_DATE) return rx::format_date_days(v.i, buf);
    if (spark_type == DQ_TYPE_TIMESTAMP) return rx::format_timestamp_utc(v.i, buf);
    return rx::format_long(v.i, buf);
}

}  // namespace

// RX: the program holds RLIKE (each lane then carries the regex engine's backtracking stack).
template <bool RX>
__global__ void __launch_bounds__(256)
predicate_kernel(const PredProgram* __restrict__ progp, const PredColumn* __restrict__ cols, int64_t nrows,
                 int64_t padded_words, uint64_t* __restrict__ out_t, uint64_t* __restrict__ out_nn,
                 int32_t* __restrict__ status) {
    const PredProgram prog = *progp;
    const int64_t row = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    bool t = false, nn = false;
    if (row < nrows) {
        Val st[kPredStack];
        int st_type[kPredStack];  // Spark type of a value loaded straight from a column (RLIKE's string cast), else 0
        int sp = 0;
        for (int pc = 0; pc + 1 < prog.code_len; pc += 2) {
            const int op = prog.code[pc];
            const int arg = prog.code[pc + 1];
            switch (op) {
                case DQ_P_COL:
                    st_type[sp] = cols[arg].spark_type;
                    st[sp++] = load_col(cols[arg], row);
                    break;
                case DQ_P_CONST: {
                    const dq_const k = prog.consts[arg];
                    Val v = vnull();
                    v.null = 0;
                    v.tag = k.tag;
                    v.i = k.i64;
                    v.d = k.f64;
                    v.s = prog.strings + k.str_offset;
                    v.slen = k.str_len;
                    st_type[sp] = 0;
                    st[sp++] = v;
                    break;
                }
                case DQ_P_NULL: st_type[sp] = 0; st[sp++] = vnull(); break;
                case DQ_P_EQ: case DQ_P_NE: case DQ_P_LT: case DQ_P_LE: case DQ_P_GT: case DQ_P_GE: {
                    const Val b = st[--sp];
                    const Val a = st[--sp];
                    int c = 0;
                    if (a.null || b.null || !compare(a, b, c)) {
                        st[sp++] = vnull();
                        break;
                    }
                    bool r = false;
                    switch (op) {
                        case DQ_P_EQ: r = c == 0; break;
                        case DQ_P_NE: r = c != 0; break;
                        case DQ_P_LT: r = c < 0; break;
                        case DQ_P_LE: r = c <= 0; break;
                        case DQ_P_GT: r = c > 0; break;
                        default: r = c >= 0; break;
                    }
                    st[sp++] = vbool(r);
                    break;
                }
                case DQ_P_EQ_NULLSAFE: {
                    const Val b = st[--sp];
                    const Val a = st[--sp];
                    int c = 1;
                    if (a.null || b.null) st[sp++] = vbool(a.null && b.null);
                    else st[sp++] = vbool(compare(a, b, c) && c == 0);
                    break;
                }
                case DQ_P_AND: {
                    const Val b = st[--sp];
                    const Val a = st[--sp];
                    const bool af = !a.null && a.i == 0, bf = !b.null && b.i == 0;
                    if (af || bf) st[sp++] = vbool(false);
                    else if (a.null || b.null) st[sp++] = vnull();
                    else st[sp++] = vbool(true);
                    break;
                }
                case DQ_P_OR: {
                    const Val b = st[--sp];
                    const Val a = st[--sp];
                    const bool at = !a.null && a.i != 0, bt = !b.null && b.i != 0;
                    if (at || bt) st[sp++] = vbool(true);
                    else if (a.null || b.null) st[sp++] = vnull();
                    else st[sp++] = vbool(false);
                    break;
                }
                case DQ_P_NOT: {
                    Val a = st[sp - 1];
                    if (!a.null) st[sp - 1] = vbool(a.i == 0);
                    break;
                }
                case DQ_P_IS_NULL: st[sp - 1] = vbool(st[sp - 1].null != 0); break;
                case DQ_P_IS_NOT_NULL: st[sp - 1] = vbool(st[sp - 1].null == 0); break;
                case DQ_P_IN: {
                    const int n = arg;
                    const int base = sp - n - 1;
                    const Val x = st[base];
                    Val r = vbool(false);
                    if (x.null) {
                        r = vnull();
                    } else {
                        bool any_null = false, hit = false;
                        for (int k = 0; k < n; ++k) {
                            const Val& e = st[base + 1 + k];
                            int c = 1;
                            if (e.null) any_null = true;
                            else if (compare(x, e, c) && c == 0) hit = true;
                        }
                        r = hit ? vbool(true) : (any_null ? vnull() : vbool(false));
                    }
                    sp = base;
                    st[sp++] = r;
                    break;
                }
                case DQ_P_COALESCE: {
                    const int n = arg;
                    const int base = sp - n;
                    Val r = vnull();
                    for (int k = n - 1; k >= 0; --k)
                        if (!st[base + k].null) r = st[base + k];
                    sp = base;
                    st[sp++] = r;
                    break;
                }
                case DQ_P_ADD: case DQ_P_SUB: case DQ_P_MUL: case DQ_P_DIV: case DQ_P_MOD: {
                    const Val b = st[--sp];
                    const Val a = st[--sp];
                    st[sp++] = arith(op, a, b);
                    break;
                }
                case DQ_P_NEG: {
                    Val a = st[sp - 1];
                    if (!a.null) {
                        if (a.tag == DQ_V_DOUBLE) a.d = -a.d;
                        else a.i = -a.i;
                        st[sp - 1] = a;
                    }
                    break;
                }
                case DQ_P_LIKE: {
                    const Val a = st[sp - 1];
                    if (!a.null && a.tag == DQ_V_STRING) {
                        const dq_const k = prog.consts[arg];
                        st[sp - 1] = vbool(a.xf ? like_match_xf(a.s, a.slen, a.xf, prog.strings + k.str_offset, k.str_len)
                                                : like_match(a.s, a.slen, prog.strings + k.str_offset, k.str_len));
                    } else {
                        st[sp - 1] = vnull();
                    }
                    break;
                }
                case DQ_P_RLIKE: {
                    // str RLIKE regex = Pattern.compile(regex).matcher(str).find(): any match, also an empty one
                    const Val a = st[sp - 1];
                    if (a.null) break;
                    if (RX) {
                        const dq_const k = prog.consts[arg];
                        const int32_t* image = reinterpret_cast<const int32_t*>(prog.strings + k.str_offset);
                        rx::RxProg rp;
                        rp.ninstr = image[1];
                        rp.anchored = image[6];
                        rp.ins = image + 8;
                        rp.classes = rp.ins + 3 * rp.ninstr;
                        rp.ranges = rp.classes + 2 * image[2];
                        uint8_t buf[40];
                        const uint8_t* sv = a.s;
                        int n = a.slen, xf = a.xf;
                        if (a.tag != DQ_V_STRING) {
                            n = value_string(a, st_type[sp - 1], 0, buf);
                            sv = buf;
                            xf = 0;
                        }
                        uint64_t stk[rx::kRxStack];
                        bool found = false;
                        for (int start = 0; start <= n;) {
                            const int end = rx::rx_match_at(rp, sv, n, start, stk, xf);
                            if (end == -2) {
                                atomicOr(status, 1);
                                break;
                            }
                            if (end >= 0) {
                                found = true;
                                break;
                            }
                            if (rp.anchored || start == n) break;
                            int len;
                            rx::decode(sv, n, start, len);
                            start += len;
                        }
                        st[sp - 1] = vbool(found);
                    }
                    st_type[sp - 1] = 0;
                    break;
                }
                case DQ_P_LOWER: case DQ_P_UPPER: {
                    Val& a = st[sp - 1];
                    // a number / boolean's string form has no letters to map: the value stands (a comparison with it
                    // coerces the same way)
                    if (!a.null && a.tag == DQ_V_STRING) a.xf = op == DQ_P_LOWER ? 1 : 2;
                    st_type[sp - 1] = 0;
                    break;
                }
                case DQ_P_TRIM: {  // Spark 2.2 UTF8String.trim / trimLeft / trimRight: ASCII spaces (0x20) only
                    Val& a = st[sp - 1];
                    if (!a.null && a.tag == DQ_V_STRING) {
                        if (arg != 2) while (a.slen > 0 && a.s[0] == ' ') { ++a.s; --a.slen; }
                        if (arg != 1) while (a.slen > 0 && a.s[a.slen - 1] == ' ') --a.slen;
                    }  // a number's string form has no spaces to trim
                    st_type[sp - 1] = 0;
                    break;
                }
                case DQ_P_SUBSTR: {  // substring(str, pos, len): UTF8String.substringSQL (1-based, 0 = 1, < 0 from the end)
                    const Val ln = st[--sp];
                    const Val ps = st[--sp];
                    Val& a = st[sp - 1];
                    st_type[sp - 1] = 0;
                    if (a.null || ps.null || ln.null || a.tag != DQ_V_STRING) { a = vnull(); break; }
                    const int64_t pos = ps.tag == DQ_V_DOUBLE ? (int64_t)ps.d : ps.i;
                    const int64_t length = ln.tag == DQ_V_DOUBLE ? (int64_t)ln.d : ln.i;
                    const int64_t nch = utf8_chars(a.s, a.slen);
                    const int64_t start = pos > 0 ? pos - 1 : (pos < 0 ? nch + pos : 0);
                    const int64_t until = length >= 2147483647 ? nch : start + length;
                    if (until <= start || start >= a.slen) { a.slen = 0; break; }
                    int i = 0;
                    int64_t c = 0;
                    while (i < a.slen && c < start) { int l; rx::decode(a.s, a.slen, i, l); i += l; ++c; }
                    int j = i;
                    while (j < a.slen && c < until) { int l; rx::decode(a.s, a.slen, j, l); j += l; ++c; }
                    a.s += i;
                    a.slen = j - i;
                    break;
                }
                case DQ_P_CASE: {  // CASE WHEN c1 THEN v1 ... [ELSE e] END: arg = 2 * #WHEN + has ELSE
                    const int nw = arg >> 1, has_else = arg & 1;
                    const int base = sp - 2 * nw - has_else;
                    Val r = has_else ? st[sp - 1] : vnull();
                    int rt = has_else ? st_type[sp - 1] : 0;
                    for (int k = 0; k < nw; ++k) {
                        const Val& c = st[base + 2 * k];
                        if (!c.null && (c.tag == DQ_V_DOUBLE ? c.d != 0.0 : c.i != 0)) {
                            r = st[base + 2 * k + 1];
                            rt = st_type[base + 2 * k + 1];
                            break;
                        }
                    }
                    sp = base;
                    st_type[sp] = rt;
                    st[sp++] = r;
                    break;
                }
                case DQ_P_ISNAN: {  // IsNaN: never NULL (FALSE for NULL), a string operand cast to double
                    const Val a = st[sp - 1];
                    bool r = false;
                    if (!a.null) {
                        if (a.tag == DQ_V_DOUBLE) r = a.d != a.d;
                        else if (a.tag == DQ_V_STRING) { double d; r = parse_double_v(a, d) && d != d; }
                    }
                    st[sp - 1] = vbool(r);
                    st_type[sp - 1] = 0;
                    break;
                }
                case DQ_P_ABS: {
                    Val& a = st[sp - 1];
                    if (!a.null) {
                        if (a.tag == DQ_V_STRING) { double d; a = parse_double_v(a, d) ? vdouble(fabs(d)) : vnull(); }
                        else if (a.tag == DQ_V_DOUBLE) a.d = fabs(a.d);
                        else if (a.i < 0) a.i = (int64_t)(0ull - (uint64_t)a.i);  // Long.MinValue stays (Math.abs)
                    }
                    break;
                }
                case DQ_P_NANVL: {  // nanvl(a, b): b when a is NaN, else a (NULL in -> NULL out)
                    const Val b = st[--sp];
                    const Val a = st[sp - 1];
                    if (a.null || b.null) st[sp - 1] = vnull();
                    else if (a.tag == DQ_V_DOUBLE && a.d != a.d) st[sp - 1] = b;
                    st_type[sp - 1] = 0;
                    break;
                }
                case DQ_P_YEAR: case DQ_P_MONTH: case DQ_P_DAY: {  // arg: 0 = DATE (days), 1 = TIMESTAMP (micros, UTC)
                    Val& a = st[sp - 1];
                    st_type[sp - 1] = 0;
                    if (a.null) break;
                    if (a.tag != DQ_V_LONG) { a = vnull(); break; }
                    const int64_t days = arg == 1 ? rx::floor_div(a.i, 86400000000ll) : a.i;
                    int64_t y;
                    int m, d;
                    spark_ymd(days, y, m, d);
                    a = vlong(op == DQ_P_YEAR ? y : (op == DQ_P_MONTH ? m : d));
                    break;
                }
                case DQ_P_LENGTH: {
                    const Val a = st[sp - 1];
                    if (!a.null && a.tag == DQ_V_STRING) st[sp - 1] = vlong(utf8_chars(a.s, a.slen));
                    else if (!a.null) st[sp - 1] = vnull();
                    break;
                }
                case DQ_P_CAST_DOUBLE: {
                    const Val a = st[sp - 1];
                    if (a.null) break;
                    if (a.tag == DQ_V_STRING) {
                        double d;
                        st[sp - 1] = parse_double(a.s, a.slen, d) ? vdouble(d) : vnull();
                    } else {
                        st[sp - 1] = vdouble(as_double(a));
                    }
                    break;
                }
                case DQ_P_CAST_LONG: {
                    const Val a = st[sp - 1];
                    if (a.null) break;
                    if (a.tag == DQ_V_STRING) {
                        int64_t x;
                        st[sp - 1] = parse_long(a.s, a.slen, x) ? vlong(x) : vnull();
                    } else if (a.tag == DQ_V_DOUBLE) {
                        st[sp - 1] = a.d != a.d ? vlong(0) : vlong((int64_t)a.d);
                    } else {
                        st[sp - 1] = vlong(a.i);
                    }
                    break;
                }
                default: break;
            }
            if (op != DQ_P_COL && op != DQ_P_CASE && sp > 0) st_type[sp - 1] = op == DQ_P_COALESCE ? st_type[sp - 1] : 0;
        }
        if (sp > 0) {
            const Val r = st[sp - 1];
            nn = !r.null;
            t = nn && (r.tag == DQ_V_DOUBLE ? r.d != 0.0 : r.i != 0);
        }
    }
    const uint64_t bt = __ballot(t);
    const uint64_t bn = __ballot(nn);
    const int64_t w = row >> 6;
    if ((threadIdx.x & 63) == 0 && w < padded_words) {
        out_t[w] = bt;
        out_nn[w] = bn;
    }
}

// ---- simple predicates (PredSimple): leaves into bit pairs, the boolean postfix on a per-lane bit stack --------------
namespace {

__device__ __forceinline__ double load_as_double(const PredColumn& c, int64_t row) {
    switch (c.spark_type) {
        case DQ_TYPE_BOOLEAN: return static_cast<const uint8_t*>(c.values)[row] != 0 ? 1.0 : 0.0;
        case DQ_TYPE_BYTE: return (double)static_cast<const int8_t*>(c.values)[row];
        case DQ_TYPE_SHORT: return (double)static_cast<const int16_t*>(c.values)[row];
        case DQ_TYPE_INT: case DQ_TYPE_DATE: return (double)static_cast<const int32_t*>(c.values)[row];
        case DQ_TYPE_FLOAT: return (double)static_cast<const float*>(c.values)[row];
        case DQ_TYPE_DOUBLE: return static_cast<const double*>(c.values)[row];
        default: return (double)static_cast<const int64_t*>(c.values)[row];  // LONG / TIMESTAMP
    }
}
__device__ __forceinline__ int64_t load_as_long(const PredColumn& c, int64_t row) {
    switch (c.spark_type) {
        case DQ_TYPE_BOOLEAN: return static_cast<const uint8_t*>(c.values)[row] != 0 ? 1 : 0;
        case DQ_TYPE_BYTE: return static_cast<const int8_t*>(c.values)[row];
        case DQ_TYPE_SHORT: return static_cast<const int16_t*>(c.values)[row];
        case DQ_TYPE_INT: case DQ_TYPE_DATE: return static_cast<const int32_t*>(c.values)[row];
        default: return static_cast<const int64_t*>(c.values)[row];  // LONG / TIMESTAMP
    }
}

}  // namespace

// One wave evaluates kPredRows x 64 rows: lane L takes rows base + 64 j + L (j < kPredRows), so ballot j is bitmap
// word j of the wave and each term issues kPredRows coalesced loads before it compares (latency hidden by the batch).
constexpr int kPredRows = 8;

template <typename T>
__device__ __forceinline__ void load_rows(const void* values, int64_t row0, int64_t nrows, T (&x)[kPredRows]) {
    const T* v = static_cast<const T*>(values);
#pragma unroll
    for (int j = 0; j < kPredRows; ++j) {
        const int64_t r = row0 + 64 * j;
        x[j] = r < nrows ? v[r] : T(0);
    }
}

__device__ __forceinline__ void term_rows(const PredTerm& q, const PredColumn& c, int64_t row0, int64_t nrows,
                                          uint32_t k, uint32_t (&tb)[kPredRows], uint32_t (&nb)[kPredRows]) {
    bool valid[kPredRows];
#pragma unroll
    for (int j = 0; j < kPredRows; ++j) {
        const int64_t r = row0 + 64 * j;
        valid[j] = r < nrows &&
                   (!c.validity || ((reinterpret_cast<const uint8_t*>(c.validity)[r >> 3] >> (r & 7)) & 1));
    }
    if (q.op == DQ_P_IS_NULL || q.op == DQ_P_IS_NOT_NULL) {
#pragma unroll
        for (int j = 0; j < kPredRows; ++j) {
            const bool in = row0 + 64 * j < nrows;
            tb[j] |= (uint32_t)(in && ((q.op == DQ_P_IS_NULL) != valid[j])) << k;
            nb[j] |= (uint32_t)in << k;
        }
        return;
    }
    int c3[kPredRows];
    if (q.dbl) {
        double x[kPredRows];
        switch (c.spark_type) {  // wave-uniform
            case DQ_TYPE_DOUBLE: load_rows(c.values, row0, nrows, x); break;
            case DQ_TYPE_LONG: case DQ_TYPE_TIMESTAMP: {
                int64_t y[kPredRows];
                load_rows(c.values, row0, nrows, y);
#pragma unroll
                for (int j = 0; j < kPredRows; ++j) x[j] = (double)y[j];
                break;
            }
            case DQ_TYPE_FLOAT: {
                float f[kPredRows];
                load_rows(c.values, row0, nrows, f);
#pragma unroll
                for (int j = 0; j < kPredRows; ++j) x[j] = (double)f[j];
                break;
            }
            default: {
#pragma unroll
                for (int j = 0; j < kPredRows; ++j) x[j] = 0.0;
                for (int j = 0; j < kPredRows; ++j)
                    if (row0 + 64 * j < nrows) x[j] = load_as_double(c, row0 + 64 * j);
                break;
            }
        }
#pragma unroll
        for (int j = 0; j < kPredRows; ++j) c3[j] = cmp_double(x[j], q.cd);
    } else {
        int64_t x[kPredRows];
        switch (c.spark_type) {  // wave-uniform
            case DQ_TYPE_LONG: case DQ_TYPE_TIMESTAMP: load_rows(c.values, row0, nrows, x); break;
            case DQ_TYPE_INT: case DQ_TYPE_DATE: {
                int32_t y[kPredRows];
                load_rows(c.values, row0, nrows, y);
#pragma unroll
                for (int j = 0; j < kPredRows; ++j) x[j] = y[j];
                break;
            }
            default: {
#pragma unroll
                for (int j = 0; j < kPredRows; ++j) x[j] = 0;
                for (int j = 0; j < kPredRows; ++j)
                    if (row0 + 64 * j < nrows) x[j] = load_as_long(c, row0 + 64 * j);
                break;
            }
        }
#pragma unroll
        for (int j = 0; j < kPredRows; ++j) c3[j] = x[j] < q.ci ? -1 : (x[j] > q.ci ? 1 : 0);
    }
#pragma unroll
    for (int j = 0; j < kPredRows; ++j) {
        bool r;
        switch (q.op) {
            case DQ_P_EQ: r = c3[j] == 0; break;
            case DQ_P_NE: r = c3[j] != 0; break;
            case DQ_P_LT: r = c3[j] < 0; break;
            case DQ_P_LE: r = c3[j] <= 0; break;
            case DQ_P_GT: r = c3[j] > 0; break;
            default: r = c3[j] >= 0; break;
        }
        tb[j] |= (uint32_t)(valid[j] && r) << k;
        nb[j] |= (uint32_t)valid[j] << k;
    }
}

__global__ void __launch_bounds__(256)
pred_simple_kernel(const PredSimple P, const PredColumn* __restrict__ cols, int64_t nrows, int64_t padded_words,
                   uint64_t* __restrict__ out_t, uint64_t* __restrict__ out_nn) {
    const int lane = threadIdx.x & 63;
    const int64_t w0 = ((int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)) * kPredRows;  // first word
    const int64_t row0 = w0 * 64 + lane;
    uint32_t tb[kPredRows], nb[kPredRows];
#pragma unroll
    for (int j = 0; j < kPredRows; ++j) tb[j] = nb[j] = 0;
    for (int k = 0; k < P.nterms; ++k) term_rows(P.t[k], cols[P.t[k].col], row0, nrows, (uint32_t)k, tb, nb);
    // SQL three-valued AND / OR / NOT on a per-row bit stack; a TRUE bit always has its NOT-NULL bit
    uint32_t st[kPredRows], sn[kPredRows];
#pragma unroll
    for (int j = 0; j < kPredRows; ++j) st[j] = sn[j] = 0;
    int sp = 0;
    for (int i = 0; i < P.nb; ++i) {  // wave-uniform
        const int o = P.b[i];
        if (o >= 0) {
#pragma unroll
            for (int j = 0; j < kPredRows; ++j) {
                st[j] |= ((tb[j] >> o) & 1u) << sp;
                sn[j] |= ((nb[j] >> o) & 1u) << sp;
            }
            ++sp;
        } else if (o == kPB_NOT) {
            const uint32_t m = 1u << (sp - 1);
#pragma unroll
            for (int j = 0; j < kPredRows; ++j) st[j] ^= sn[j] & m;
        } else {
            const uint32_t keep = (1u << (sp - 2)) - 1u;
#pragma unroll
            for (int j = 0; j < kPredRows; ++j) {
                const uint32_t ta = (st[j] >> (sp - 2)) & 1u, na = (sn[j] >> (sp - 2)) & 1u;
                const uint32_t tc = (st[j] >> (sp - 1)) & 1u, nc = (sn[j] >> (sp - 1)) & 1u;
                uint32_t rt, rn;
                if (o == kPB_AND) {
                    const uint32_t af = na & (ta ^ 1u), cf = nc & (tc ^ 1u);
                    rn = af | cf | (na & nc);
                    rt = (af | cf) ? 0u : (na & nc);
                } else {
                    rt = ta | tc;
                    rn = rt | (na & nc);
                }
                st[j] = (st[j] & keep) | (rt << (sp - 2));
                sn[j] = (sn[j] & keep) | (rn << (sp - 2));
            }
            --sp;
        }
    }
#pragma unroll
    for (int j = 0; j < kPredRows; ++j) {
        const uint64_t bt = __ballot(st[j] & 1u);
        const uint64_t bn = __ballot(sn[j] & 1u);
        if (lane == 0 && w0 + j < padded_words) {
            out_t[w0 + j] = bt;
            out_nn[w0 + j] = bn;
        }
    }
}

// Standalone `where` producer (WhereOut): the simple predicate over kPredRows words per wave as in pred_simple_kernel,
// grid-strided over `gridDim.x` blocks; lane j < kPredRows then writes word j of every consumer mask (valid & TRUE) and,
// if asked, of the bitmaps; the TRUE / NOT-NULL counts go to this block's partial of the filter's SK_WHERE slot.
__device__ __forceinline__ uint64_t valid_word(const uint64_t* v, int64_t w, int64_t nrows) {
    if (v == nullptr) return ~0ull;
    if ((w + 1) * 64 <= nrows) return v[w];
    const uint8_t* b = reinterpret_cast<const uint8_t*>(v);
    const int64_t nb = (nrows + 7) >> 3;
    uint64_t x = 0;
    for (int i = 0; i < 8; ++i)
        if (w * 8 + i < nb) x |= (uint64_t)b[w * 8 + i] << (8 * i);
    return x;
}

__global__ void __launch_bounds__(256)
where_masks_kernel(const PredSimple P, const WhereOut* __restrict__ wo, const PredColumn* __restrict__ cols,
                   int64_t nrows, int64_t padded_words, SlotPartial* __restrict__ partials, int wslot, int gstride) {
    __shared__ int64_t red[2][4];
    __shared__ const uint64_t* valid[kWhereMasks];
    __shared__ uint64_t* mask[kWhereMasks];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int nm = wo->nmasks;
    const bool bitmaps = wo->bitmaps != 0;
    uint64_t* const where_t = wo->where_t;
    uint64_t* const where_nn = wo->where_nn;
    if (threadIdx.x < kWhereMasks) {
        valid[threadIdx.x] = wo->valid[threadIdx.x];
        mask[threadIdx.x] = wo->mask[threadIdx.x];
    }
    __syncthreads();
    int64_t wt = 0, wnn = 0;
    const int64_t nchunks = (padded_words + kPredRows - 1) / kPredRows;  // kPredRows words per wave
    for (int64_t ch = (int64_t)blockIdx.x * 4 + wave; ch < nchunks; ch += (int64_t)gridDim.x * 4) {
        const int64_t w0 = ch * kPredRows;
        const int64_t row0 = w0 * 64 + lane;
        uint32_t tb[kPredRows], nb[kPredRows];
#pragma unroll
        for (int j = 0; j < kPredRows; ++j) tb[j] = nb[j] = 0;
        for (int k = 0; k < P.nterms; ++k) term_rows(P.t[k], cols[P.t[k].col], row0, nrows, (uint32_t)k, tb, nb);
        uint32_t st[kPredRows], sn[kPredRows];
#pragma unroll
        for (int j = 0; j < kPredRows; ++j) st[j] = sn[j] = 0;
        int sp = 0;
        for (int i = 0; i < P.nb; ++i) {
            const int o = P.b[i];
            if (o >= 0) {
#pragma unroll
                for (int j = 0; j < kPredRows; ++j) {
                    st[j] |= ((tb[j] >> o) & 1u) << sp;
                    sn[j] |= ((nb[j] >> o) & 1u) << sp;
                }
                ++sp;
            } else if (o == kPB_NOT) {
                const uint32_t m = 1u << (sp - 1);
#pragma unroll
                for (int j = 0; j < kPredRows; ++j) st[j] ^= sn[j] & m;
            } else {
                const uint32_t keep = (1u << (sp - 2)) - 1u;
#pragma unroll
                for (int j = 0; j < kPredRows; ++j) {
                    const uint32_t ta = (st[j] >> (sp - 2)) & 1u, na = (sn[j] >> (sp - 2)) & 1u;
                    const uint32_t tc = (st[j] >> (sp - 1)) & 1u, nc = (sn[j] >> (sp - 1)) & 1u;
                    uint32_t rt, rn;
                    if (o == kPB_AND) {
                        const uint32_t af = na & (ta ^ 1u), cf = nc & (tc ^ 1u);
                        rn = af | cf | (na & nc);
                        rt = (af | cf) ? 0u : (na & nc);
                    } else {
                        rt = ta | tc;
                        rn = rt | (na & nc);
                    }
                    st[j] = (st[j] & keep) | (rt << (sp - 2));
                    sn[j] = (sn[j] & keep) | (rn << (sp - 2));
                }
                --sp;
            }
        }
        uint64_t mine_t = 0, mine_n = 0;
#pragma unroll
        for (int j = 0; j < kPredRows; ++j) {
            const uint64_t bt = __ballot(st[j] & 1u);
            const uint64_t bn = __ballot(sn[j] & 1u);
            wt += __popcll(bt);
            wnn += __popcll(bn);
            mine_t = lane == j ? bt : mine_t;
            mine_n = lane == j ? bn : mine_n;
        }
        // the chunk's kPredRows words x the consumer masks spread over the 64 lanes (lane L: word L % kPredRows of
        // mask m0 + L / kPredRows): one validity load and one store per lane, the loads of a group all in flight
        // before its stores (pointers from the kernel-start copies, so no store can alias them)
        const int jw = lane % kPredRows;
        const uint64_t word_t = __shfl(mine_t, jw, 64);
        const int64_t w = w0 + jw;
        for (int m0 = 0; m0 < nm; m0 += 64 / kPredRows) {  // wave-uniform
            const int m = m0 + lane / kPredRows;
            const bool on = m < nm && w < padded_words;
            const uint64_t v = on ? valid_word(valid[m], w, nrows) : 0ull;
            if (on) mask[m][w] = v & word_t;
        }
        if (bitmaps && lane < kPredRows && w0 + lane < padded_words) {
            where_t[w0 + lane] = mine_t;
            where_nn[w0 + lane] = mine_n;
        }
    }
    if (lane == 0) {
        red[0][wave] = wt;
        red[1][wave] = wnn;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        SlotPartial& o = partials[(int64_t)wslot * gstride + blockIdx.x];
        SlotPartial z;
        memset(&z, 0, sizeof(z));
        z.c[0].imin = z.c[1].imin = INT64_MAX;
        z.c[0].imax = z.c[1].imax = INT64_MIN;
        z.c[0].dmin = z.c[1].dmin = INFINITY;
        z.c[0].dmax = z.c[1].dmax = -INFINITY;
        z.wt = red[0][0] + red[0][1] + red[0][2] + red[0][3];
        z.wnn = red[1][0] + red[1][1] + red[1][2] + red[1][3];
        o = z;
    }
}

void launch_where_masks(const WhereOut* wo_dev, const PredSimple& prog, const PredColumn* cols_dev, int64_t nrows,
                        int64_t padded_words, SlotPartial* partials, int wslot, int gstride, int grid, hipStream_t s) {
    hipLaunchKernelGGL(where_masks_kernel, dim3((unsigned)grid), dim3(256), 0, s, prog, wo_dev, cols_dev, nrows,
                       padded_words, partials, wslot, gstride);
}

void launch_pred_simple(const PredSimple& prog, const PredColumn* cols_dev, int64_t nrows, int64_t padded_words,
                        uint64_t* out_t, uint64_t* out_nn, hipStream_t s) {
    const int64_t words_per_block = 4 * kPredRows;  // 4 waves
    const int64_t blocks = (padded_words + words_per_block - 1) / words_per_block;
    hipLaunchKernelGGL(pred_simple_kernel, dim3((unsigned)blocks), dim3(256), 0, s, prog, cols_dev, nrows,
                       padded_words, out_t, out_nn);
}

void launch_predicate(const PredProgram* prog_dev, bool rx, int32_t* status, const PredColumn* cols_dev, int64_t nrows,
                      int64_t padded_words, uint64_t* out_t, uint64_t* out_nn, hipStream_t s) {
    const int64_t rows = padded_words * 64;
    const int64_t blocks = (rows + 255) / 256;
    if (rx)
        hipLaunchKernelGGL(predicate_kernel<true>, dim3((unsigned)blocks), dim3(256), 0, s, prog_dev, cols_dev, nrows,
                           padded_words, out_t, out_nn, status);
    else
        hipLaunchKernelGGL(predicate_kernel<false>, dim3((unsigned)blocks), dim3(256), 0, s, prog_dev, cols_dev, nrows,
                           padded_words, out_t, out_nn, status);
}

}  // namespace dq
