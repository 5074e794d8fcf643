// dq_common.h — host+device helpers shared by the HIP kernels and the host runtime.
//
// Spark's XXH64 (org.apache.spark.sql.catalyst.expressions.XXH64, spark-catalyst 2.2.2, called by
// XxHash64Function.hash in C/StatefulHyperloglogPlus.scala:93) is the standard XXH64 over the
// little-endian bytes of the value; hashInt/hashLong are its 4- and 8-byte specialisations.
// The counter-based splitmix64 generator defines the synthetic BASELINE inputs.
#pragma once

#include <stdint.h>

#if defined(DQ_HOST_ONLY)  // host-only builds of the pure host code (the sanitizer build, tests/sanitize/)
#define DQ_HD inline
#else
#include <hip/hip_runtime.h>
#define DQ_HD __host__ __device__ __forceinline__
#endif

namespace dq {

constexpr uint64_t P64_1 = 0x9E3779B185EBCA87ULL;
constexpr uint64_t P64_2 = 0xC2B2AE3D27D4EB4FULL;
constexpr uint64_t P64_3 = 0x165667B19E3779F9ULL;
constexpr uint64_t P64_4 = 0x85EBCA77C2B2AE63ULL;
constexpr uint64_t P64_5 = 0x27D4EB2F165667C5ULL;
constexpr uint64_t SPARK_HLL_SEED = 42;  // C/StatefulHyperloglogPlus.scala:93

DQ_HD uint64_t rotl64(uint64_t x, int r) {
#if defined(__HIP_DEVICE_COMPILE__)
    // two v_alignbit_b32 (funnel shifts of the 32-bit halves) instead of the shift/shift/or sequence
    // the compiler emits for a 64-bit rotate: 1 < r < 32 at every call site (XXH64 uses 1..31)
    const uint32_t lo = (uint32_t)x, hi = (uint32_t)(x >> 32);
    const uint32_t nh = __builtin_amdgcn_alignbit(hi, lo, 32 - r);
    const uint32_t nl = __builtin_amdgcn_alignbit(lo, hi, 32 - r);
    return ((uint64_t)nh << 32) | nl;
#else
    return (x << r) | (x >> (64 - r));
#endif
}

DQ_HD uint64_t xxh_fmix(uint64_t h) {
    h ^= h >> 33;
    h *= P64_2;
    h ^= h >> 29;
    h *= P64_3;
    h ^= h >> 32;
    return h;
}

// XXH64.hashInt: 4-byte input.
DQ_HD uint64_t xxh_int(uint32_t v, uint64_t seed) {
    uint64_t h = seed + P64_5 + 4ULL;
    h ^= (uint64_t)v * P64_1;
    h = rotl64(h, 23) * P64_2 + P64_3;
    return xxh_fmix(h);
}

// XXH64.hashLong: 8-byte input.
DQ_HD uint64_t xxh_long(uint64_t v, uint64_t seed) {
    uint64_t h = seed + P64_5 + 8ULL;
    h ^= rotl64(v * P64_2, 31) * P64_1;
    h = rotl64(h, 27) * P64_1 + P64_4;
    return xxh_fmix(h);
}

DQ_HD uint64_t load_le64(const uint8_t* p) {
    uint64_t v = 0;
    for (int i = 0; i < 8; ++i) v |= (uint64_t)p[i] << (8 * i);
    return v;
}
DQ_HD uint32_t load_le32(const uint8_t* p) {
    return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}

DQ_HD uint64_t xxh_round(uint64_t acc, uint64_t input) {
    acc += input * P64_2;
    acc = rotl64(acc, 31);
    return acc * P64_1;
}
DQ_HD uint64_t xxh_merge_round(uint64_t acc, uint64_t val) {
    val = xxh_round(0, val);
    acc ^= val;
    return acc * P64_1 + P64_4;
}

// XXH64.hashUnsafeBytes: arbitrary byte string (UTF-8 strings, binary).
DQ_HD uint64_t xxh_bytes(const uint8_t* p, int64_t len, uint64_t seed) {
    const uint8_t* end = p + len;
    uint64_t h;
    if (len >= 32) {
        const uint8_t* limit = end - 32;
        uint64_t v1 = seed + P64_1 + P64_2, v2 = seed + P64_2, v3 = seed, v4 = seed - P64_1;
        do {
            v1 = xxh_round(v1, load_le64(p));
            v2 = xxh_round(v2, load_le64(p + 8));
            v3 = xxh_round(v3, load_le64(p + 16));
            v4 = xxh_round(v4, load_le64(p + 24));
            p += 32;
        } while (p <= limit);
        h = rotl64(v1, 1) + rotl64(v2, 7) + rotl64(v3, 12) + rotl64(v4, 18);
        h = xxh_merge_round(h, v1);
        h = xxh_merge_round(h, v2);
        h = xxh_merge_round(h, v3);
        h = xxh_merge_round(h, v4);
    } else {
        h = seed + P64_5;
    }
    h += (uint64_t)len;
    while (p + 8 <= end) {
        h ^= xxh_round(0, load_le64(p));
        h = rotl64(h, 27) * P64_1 + P64_4;
        p += 8;
    }
    if (p + 4 <= end) {
        h ^= (uint64_t)load_le32(p) * P64_1;
        h = rotl64(h, 23) * P64_2 + P64_3;
        p += 4;
    }
    while (p < end) {
        h ^= (uint64_t)(*p) * P64_5;
        h = rotl64(h, 11) * P64_1;
        ++p;
    }
    return xxh_fmix(h);
}

// java.lang.Double.doubleToLongBits / Float.floatToIntBits: NaN canonicalised.
DQ_HD uint64_t double_to_long_bits(double d) {
    if (d != d) return 0x7ff8000000000000ULL;
    union { double d; uint64_t u; } c;
    c.d = d;
    return c.u;
}
DQ_HD uint32_t float_to_int_bits(float f) {
    if (f != f) return 0x7fc00000U;
    union { float f; uint32_t u; } c;
    c.f = f;
    return c.u;
}

// HLL++ register update inputs (C/StatefulHyperloglogPlus.scala:96-100, P = 9):
// idx = x >>> 55; pw = numberOfLeadingZeros((x << 9) | 1 << 8) + 1.
DQ_HD uint32_t hll_index(uint64_t x) { return (uint32_t)(x >> 55); }
DQ_HD uint32_t hll_rank(uint64_t x) {
    uint64_t w = (x << 9) | (1ULL << 8);
#if defined(__HIP_DEVICE_COMPILE__)
    return (uint32_t)__clzll((long long)w) + 1u;
#else
    return (uint32_t)__builtin_clzll(w) + 1u;
#endif
}

// Counter-based splitmix64: output i of the stream seeded by `seed`.
DQ_HD uint64_t splitmix64(uint64_t seed, uint64_t i) {
    uint64_t z = seed + (i + 1) * 0x9E3779B97F4A7C15ULL;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

// ---- exact, order-free sums of fp64 terms (entropy / MutualInformation) ------------------------------
// A Spark `sum` over the groups' terms (A/Entropy.scala:28-42, A/MutualInformation.scala:66-90) has no defined
// order; a GPU table's slot order is decided by atomics, so any fp fold over slots is run-to-run and
// geometry dependent. Each term is instead rounded once to a signed 128-bit fixed-point integer of
// kFxBits fraction bits and the integers are added (associative, exact), so every build / launch
// geometry / device split of the same groups gives the same bits. |term| < 2^22 (an entropy term is
// <= 1/e, a MutualInformation term <= ln(2^63) < 44); the rounding error is <= 2^-105 per term.
constexpr int kFxBits = 104;
typedef __int128 fx128;

DQ_HD fx128 fx_of(double t) {
    union { double d; uint64_t u; } c;
    c.d = t;
    const int e = (int)((c.u >> 52) & 0x7ff);
    const uint64_t m = (c.u & ((1ull << 52) - 1)) | (e ? (1ull << 52) : 0ull);
    const int sh = (e ? e : 1) - 1075 + kFxBits;
    fx128 v;
    if (sh >= 0)
        v = (fx128)m << (sh < 74 ? sh : 74);  // callers keep |t| < 2^22 (sh <= 73); clamp defensively
    else if (sh > -64)
        v = (fx128)((m + (1ull << (-sh - 1))) >> -sh);  // round half up (in magnitude)
    else
        v = 0;
    return (c.u >> 63) ? -v : v;
}

// fx128 -> double: one correctly rounded integer conversion, then an exact power-of-two scale.
inline double fx_to_double(fx128 v) {
    const double d = (double)v;
    return d * (1.0 / 20282409603651670423947251286016.0);  // 2^-104
}

#if !defined(DQ_HOST_ONLY)
__device__ __forceinline__ fx128 fx_shfl_down(fx128 v, int off) {
    const unsigned long long lo = (unsigned long long)v, hi = (unsigned long long)(v >> 64);
    const unsigned long long l2 = __shfl_down(lo, off, 64), h2 = __shfl_down(hi, off, 64);
    return (fx128)(((unsigned __int128)h2 << 64) | l2);
}
#endif

}  // namespace dq
