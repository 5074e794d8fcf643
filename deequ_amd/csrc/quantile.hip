// quantile.hip — exact order statistics behind ApproxQuantile / ApproxQuantiles (gfx950 / CDNA4).
//
// Replaces the per-row PercentileDigest.add of StatefulApproxQuantile.update
// (C/StatefulApproxQuantile.scala:65-72; the Greenwald-Khanna QuantileSummaries of
// spark-catalyst 2.2.2, third-party, restated in deequ_amd/quantiles.py). Instead of streaming
// every value through a GK sketch, the GPU computes the EXACT values at the ranks of a summary
// with zero rank uncertainty (g = rank gap, delta = 0): ranks 1, n and every
// max(1, floor(relativeError * n))-th rank in between. Such a summary satisfies the GK error
// invariant by construction, merges with Spark's QuantileSummaries.merge, and every query lands
// within the declared relativeError rank bound (A/ApproxQuantile.scala:33-35).
//
// Algorithm (HBM-bound integer work, no MFMA): values are cast to double (Spark's implicit cast of
// the child to DoubleType) and mapped to order-preserving u64 keys in java.lang.Double.compare
// order (-0.0 < 0.0, NaN largest — the ordering of `sortBy(_.value)` in QuantileSummaries).
//   1. stratified sample of 64 Ki rows -> host sort -> 4095 equi-depth splitters (data adaptive,
//      so skewed fp64 exponents do not pile rows into a few radix digits);
//   2. histogram pass: per-row branchless binary search over the splitters in LDS (4 rows per
//      lane interleaved for ILP), per-bucket counts and counts of keys EQUAL to the bucket's lower
//      splitter (heavy duplicates are answered from the splitter, never compacted);
//   3. the host maps each target rank to (bucket, residual);
//   4. compaction pass: only rows of target buckets (~#targets / 4096 of the data) are written,
//      bucket-contiguous, to a candidate buffer;
//   5. rocPRIM radix sort of the candidates; 6. gather of the target ranks.
#include <hip/hip_runtime.h>
#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_segmented_radix_sort.hpp>

#include <math.h>
#include <string.h>

#include <algorithm>
#include <string>
#include <thread>
#include <vector>

#include "dq_common.h"
#include "dq_internal.h"

namespace dq {

constexpr int kQBuckets = 4096;          // buckets; kQBuckets - 1 splitters + a +inf sentinel
constexpr int kQSample = 65536;          // stratified sample size
constexpr int kQBlock = 256;
constexpr int kQHistBlock = 1024;      // the batched histogram pass: 32 waves per CU at its 64 KB of LDS
#ifndef DQ_Q_ROWS
#define DQ_Q_ROWS 8
#endif
constexpr int kQRowsPerLane = DQ_Q_ROWS;  // independent loads / tree descents in flight per lane
constexpr uint32_t kQNoTarget = 0xFFFFFFFFu;

__device__ __forceinline__ uint64_t q_f64_bits(double d) { return (uint64_t)__double_as_longlong(d); }
__device__ __forceinline__ double q_as_f64(uint64_t u) { return __longlong_as_double((long long)u); }

// java.lang.Double.compare order as an unsigned key; NaN canonical (largest).
__device__ __forceinline__ uint64_t order_key(double d) {
    uint64_t u = d != d ? 0x7ff8000000000000ULL : q_f64_bits(d);
    return (u >> 63) ? ~u : (u | 0x8000000000000000ULL);
}
__device__ __forceinline__ double key_value(uint64_t k) {
    return q_as_f64((k >> 63) ? (k & 0x7fffffffffffffffULL) : ~k);
}

struct QColumn {
    const void* values;
    const uint64_t* validity;
    int32_t elem;
    int32_t decimal_scale;  // DECIMAL: value = unscaled / 10^scale (Spark Decimal.toDouble, compact form)
    double pow10;
};

__device__ __forceinline__ bool q_valid(const QColumn& c, int64_t r) {
    return c.validity == nullptr || ((c.validity[r >> 6] >> (r & 63)) & 1ull);
}

__device__ __forceinline__ double q_load(const QColumn& c, int64_t r) {
    switch (c.elem) {
        case ET_F64: return static_cast<const double*>(c.values)[r];
        case ET_F32: return (double)static_cast<const float*>(c.values)[r];
        case ET_I64: {
            const int64_t v = static_cast<const int64_t*>(c.values)[r];
            return c.decimal_scale ? (double)v / c.pow10 : (double)v;
        }
        case ET_I32: return (double)static_cast<const int32_t*>(c.values)[r];
        case ET_I16: return (double)static_cast<const int16_t*>(c.values)[r];
        case ET_I8: return (double)static_cast<const int8_t*>(c.values)[r];
        default: return (double)static_cast<const uint8_t*>(c.values)[r];
    }
}

// Global-memory view of a pointer read from a table in memory (a generic pointer would compile to flat loads).
template <typename T>
__device__ __forceinline__ T q_gload(const void* base, int64_t i) {
    return ((const __attribute__((address_space(1))) T*)base)[i];
}

// The element's bits as loaded (no conversion), typed at compile time (one kernel instance per element type: a per-row
// switch over the type made the unrolled loops branchy and spilled), so a row's value and validity loads are issued
// independently and the next rows' loads can be in flight while the current rows are searched.
template <int ET>
__device__ __forceinline__ uint64_t q_load_raw(const void* values, int64_t r) {
    if constexpr (ET == ET_F64 || ET == ET_I64) return q_gload<uint64_t>(values, r);
    else if constexpr (ET == ET_F32 || ET == ET_I32) return q_gload<uint32_t>(values, r);
    else if constexpr (ET == ET_I16) return q_gload<uint16_t>(values, r);
    else return q_gload<uint8_t>(values, r);
}
template <int ET>
__device__ __forceinline__ double q_raw_value(const QColumn& c, uint64_t u) {
    if constexpr (ET == ET_F64) return q_as_f64(u);
    else if constexpr (ET == ET_F32) return (double)__uint_as_float((uint32_t)u);
    else if constexpr (ET == ET_I64) return c.decimal_scale ? (double)(int64_t)u / c.pow10 : (double)(int64_t)u;
    else if constexpr (ET == ET_I32) return (double)(int32_t)(uint32_t)u;
    else if constexpr (ET == ET_I16) return (double)(int16_t)(uint16_t)u;
    else if constexpr (ET == ET_I8) return (double)(int8_t)(uint8_t)u;
    else return (double)(uint8_t)u;
}

// One lane's kQRowsPerLane rows of a block step (row base + j * blockDim.x): raw values and validity words, loaded
// unconditionally (a value load predicated on its validity bit would wait for the bitmap first).
struct QRows {
    uint64_t raw[kQRowsPerLane];
    uint64_t vw[kQRowsPerLane];
};
template <int ET>
__device__ __forceinline__ void q_fetch(const QColumn& c, int64_t nrows, int64_t base, QRows& q) {
#pragma unroll
    for (int j = 0; j < kQRowsPerLane; ++j) {
        const int64_t r = base + (int64_t)j * blockDim.x;
        const bool in = r < nrows;
        q.raw[j] = in ? q_load_raw<ET>(c.values, r) : 0;
        q.vw[j] = in ? (c.validity ? q_gload<uint64_t>(c.validity, r >> 6) : ~0ULL) : 0;
    }
}
template <int ET>
__device__ __forceinline__ void q_keys(const QColumn& c, int64_t base, const QRows& q, uint64_t (&k)[kQRowsPerLane],
                                       bool (&v)[kQRowsPerLane]) {
#pragma unroll
    for (int j = 0; j < kQRowsPerLane; ++j) {
        const int64_t r = base + (int64_t)j * blockDim.x;
        v[j] = (q.vw[j] >> (r & 63)) & 1ULL;
        k[j] = v[j] ? order_key(q_raw_value<ET>(c, q.raw[j])) : 0;
    }
}

// Row i of the stratified sample: row floor((2i + 1) * nrows / (2S)); NULL rows are flagged.
__global__ void q_sample_kernel(QColumn c, int64_t nrows, uint64_t* __restrict__ keys, uint8_t* __restrict__ ok) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= kQSample) return;
    const int64_t r = (int64_t)(((uint64_t)(2 * i + 1) * (uint64_t)nrows) / (2 * kQSample));  // nrows < 2^46
    const bool v = r < nrows && q_valid(c, r);
    ok[i] = v ? 1 : 0;
    keys[i] = v ? order_key(q_load(c, r)) : 0;
}

__device__ void q_load_splitters(uint64_t* spl, const uint64_t* __restrict__ splitters) {
    for (int i = threadIdx.x; i < kQBuckets; i += blockDim.x) spl[i] = splitters[i];
}

// The 4095 splitters as an implicit search tree in breadth-first (Eytzinger) order: node i of level d sits at i =
// 2^d - 1 + p and holds sorted splitter (2p + 1) * 2^(11 - d) - 1. A bisection over the sorted array in LDS probes
// indices that are all congruent mod the bank count at each of its first levels (up to 32-way bank conflicts);
// the nodes of one tree level are consecutive words instead.
__host__ __device__ inline int q_tree_sorted_index(int i) {
    int d = 0;
    while ((2 << d) <= i + 1) ++d;
    const int p = i + 1 - (1 << d);
    return ((2 * p + 1) << (11 - d)) - 1;
}

// bucket = number of splitters <= key (0..4095), kQRowsPerLane descents interleaved; then the largest splitter <= key
// (sorted splitter b - 1, bucket b's lower bound) read from its tree node: tracking it through the descent kept one
// compare mask per level and row live and spilled them.
__device__ __forceinline__ void q_tree_search(const uint64_t* tree, const uint64_t (&k)[kQRowsPerLane],
                                              uint32_t (&b)[kQRowsPerLane], uint64_t (&lo)[kQRowsPerLane]) {
#pragma unroll
    for (int j = 0; j < kQRowsPerLane; ++j) b[j] = 0;
#pragma unroll
    for (int level = 0; level < 12; ++level)
#pragma unroll
        for (int j = 0; j < kQRowsPerLane; ++j) b[j] = 2 * b[j] + 1 + (tree[b[j]] <= k[j] ? 1u : 0u);
#pragma unroll
    for (int j = 0; j < kQRowsPerLane; ++j) {
        b[j] -= kQBuckets - 1;
        // sorted index s = b - 1 sits at level d = 11 - ctz(s + 1), position (s + 1) >> (12 - d) in the level
        const uint32_t s1 = b[j] ? b[j] : 1u;  // b = 0 has no lower splitter (lo unused)
        const uint32_t tz = (uint32_t)__builtin_ctz(s1);
        lo[j] = tree[((1u << (11 - tz)) - 1) + (s1 >> (tz + 1))];
    }
}

// Pass 2 body: bucket counts and counts of keys equal to the bucket's lower splitter, over the rows
// this block takes of a column (block `blk` of `nblk` striding the rows); `splitters` in tree order.
// With `bid`, each row's bucket is also recorded (kQBidNull for NULL, kQBidEq | b for a copy of bucket b's lower
// splitter, else b), so the compaction streams these 2-byte ids instead of searching the tree again.
constexpr uint16_t kQBidNull = 0xFFFF, kQBidEq = 0x8000;
template <int ET>
__device__ __forceinline__ void q_hist_rows(const QColumn& c, int64_t nrows, const uint64_t* __restrict__ splitters,
                                            unsigned long long* __restrict__ hist, unsigned long long* __restrict__ eq,
                                            int64_t blk, int64_t nblk, uint16_t* __restrict__ bid = nullptr) {
    __shared__ uint64_t spl[kQBuckets];
    __shared__ uint32_t h[kQBuckets];
    __shared__ uint32_t e[kQBuckets];
    q_load_splitters(spl, splitters);
    for (int i = threadIdx.x; i < kQBuckets; i += blockDim.x) h[i] = e[i] = 0;
    __syncthreads();
    const int64_t stride = nblk * blockDim.x * kQRowsPerLane;
    int64_t base = blk * blockDim.x * kQRowsPerLane + threadIdx.x;
    QRows q;
    for (; base < nrows; base += stride) {
        uint64_t k[kQRowsPerLane];
        bool v[kQRowsPerLane];
        q_fetch<ET>(c, nrows, base, q);
        q_keys<ET>(c, base, q, k, v);
        uint32_t b[kQRowsPerLane];
        uint64_t lo[kQRowsPerLane];
        q_tree_search(spl, k, b, lo);
#pragma unroll
        for (int j = 0; j < kQRowsPerLane; ++j) {
            const bool is_eq = v[j] && b[j] > 0 && lo[j] == k[j];
            if (bid) {
                const int64_t r = base + (int64_t)j * blockDim.x;
                if (r < nrows) bid[r] = !v[j] ? kQBidNull : (uint16_t)(b[j] | (is_eq ? kQBidEq : 0));
            }
            if (!v[j]) continue;
            atomicAdd(&h[b[j]], 1u);
            if (is_eq) atomicAdd(&e[b[j]], 1u);
        }
    }
    __syncthreads();
    for (int i = threadIdx.x; i < kQBuckets; i += blockDim.x) {
        if (h[i]) atomicAdd(&hist[i], (unsigned long long)h[i]);
        if (e[i]) atomicAdd(&eq[i], (unsigned long long)e[i]);
    }
}

template <int ET>
__global__ void __launch_bounds__(kQBlock)
q_hist_kernel(QColumn c, int64_t nrows, const uint64_t* __restrict__ splitters,
              unsigned long long* __restrict__ hist, unsigned long long* __restrict__ eq) {
    q_hist_rows<ET>(c, nrows, splitters, hist, eq, blockIdx.x, gridDim.x);
}

// Pass 4 body: rows of target buckets (other than copies of the lower splitter) -> candidates, written
// into their bucket's segment through a per-bucket cursor.
template <int ET>
__device__ __forceinline__ void q_compact_rows(const QColumn& c, int64_t nrows, const uint64_t* __restrict__ splitters,
                                               const uint32_t* __restrict__ target,
                                               unsigned long long* __restrict__ cursor, uint64_t* __restrict__ cand,
                                               int64_t blk, int64_t nblk) {
    __shared__ uint64_t spl[kQBuckets];
    __shared__ uint32_t tg[kQBuckets];
    q_load_splitters(spl, splitters);
    for (int i = threadIdx.x; i < kQBuckets; i += blockDim.x) tg[i] = target[i];
    __syncthreads();
    const int64_t stride = nblk * blockDim.x * kQRowsPerLane;
    int64_t base = blk * blockDim.x * kQRowsPerLane + threadIdx.x;
    QRows q;
    for (; base < nrows; base += stride) {
        uint64_t k[kQRowsPerLane];
        bool v[kQRowsPerLane];
        q_fetch<ET>(c, nrows, base, q);
        q_keys<ET>(c, base, q, k, v);
        uint32_t b[kQRowsPerLane];
        uint64_t lo[kQRowsPerLane];
        q_tree_search(spl, k, b, lo);
#pragma unroll
        for (int j = 0; j < kQRowsPerLane; ++j) {
            if (!v[j] || tg[b[j]] == kQNoTarget) continue;
            if (b[j] > 0 && lo[j] == k[j]) continue;
            const unsigned long long pos = atomicAdd(&cursor[b[j]], 1ull);
            cand[pos] = k[j];
        }
    }
}

template <int ET>
__global__ void __launch_bounds__(kQBlock)
q_compact_kernel(QColumn c, int64_t nrows, const uint64_t* __restrict__ splitters, const uint32_t* __restrict__ target,
                 unsigned long long* __restrict__ cursor, uint64_t* __restrict__ cand) {
    q_compact_rows<ET>(c, nrows, splitters, target, cursor, cand, blockIdx.x, gridDim.x);
}

// ---- batched requests (dq_quantile_summaries): several columns, each one or more consecutive row ranges ----------

// One row range (part) of request `req`'s column; row0 = its first row in the request's concatenated row order.
struct QPart {
    QColumn qc;
    int64_t nrows;
    int64_t row0;
    int64_t bid_off;  // first of its rows' bucket ids in the id buffer
    int32_t req;
    int32_t pad;
};

// The stratified sample of every request (blockIdx.y): row floor((2i + 1) * N / (2S)) of the concatenated parts;
// NULL rows get the key ~0 (above every value key, so they sort last) and valid rows are counted.
__global__ void __launch_bounds__(256)
q_sample_multi_kernel(const QPart* __restrict__ parts, const int32_t* __restrict__ part_begin,
                      const int64_t* __restrict__ req_rows, uint64_t* __restrict__ keys,
                      unsigned int* __restrict__ valid_count) {
    const int r = blockIdx.y;
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t n = req_rows[r];
    uint64_t key = ~0ULL;
    bool v = false;
    if (n > 0 && i < kQSample) {
        const int64_t g = (int64_t)(((uint64_t)(2 * i + 1) * (uint64_t)n) / (2 * kQSample));  // n < 2^46
        int p = part_begin[r];
        while (p + 1 < part_begin[r + 1] && g >= parts[p + 1].row0) ++p;
        const int64_t lr = g - parts[p].row0;
        if (lr >= 0 && lr < parts[p].nrows && q_valid(parts[p].qc, lr)) {
            v = true;
            key = order_key(q_load(parts[p].qc, lr));
        }
    }
    if (i < kQSample) keys[(size_t)r * kQSample + i] = key;
    const unsigned long long b = __ballot(v);
    if ((threadIdx.x & 63) == 0 && b) atomicAdd(&valid_count[r], (unsigned int)__popcll(b));
}

// 4095 equi-depth splitters per request from its sorted sample (the m valid keys first) + the +inf sentinel;
// all +inf when no sampled row is valid.
__global__ void __launch_bounds__(256)
q_splitters_kernel(const uint64_t* __restrict__ sorted, const unsigned int* __restrict__ valid_count,
                   uint64_t* __restrict__ spl, uint64_t* __restrict__ tree) {
    const int r = blockIdx.x;
    const size_t m = valid_count[r];
    auto splitter = [&](int j) -> uint64_t {
        if (j >= kQBuckets - 1 || m == 0) return ~0ULL;
        size_t at = (size_t)(j + 1) * m / kQBuckets;
        if (at >= m) at = m - 1;
        return sorted[(size_t)r * kQSample + at];
    };
    for (int j = threadIdx.x; j < kQBuckets; j += blockDim.x) {
        spl[(size_t)r * kQBuckets + j] = splitter(j);
        tree[(size_t)r * kQBuckets + j] = j < kQBuckets - 1 ? splitter(q_tree_sorted_index(j)) : ~0ULL;
    }
}

// Histogram of every part (blockIdx.y) into its request's hist / eq (2 * kQBuckets counters per request).
template <int ET>
__global__ void __launch_bounds__(kQHistBlock)
q_hist_multi_kernel(const QPart* __restrict__ parts, const uint64_t* __restrict__ spl,
                    unsigned long long* __restrict__ hist, uint16_t* __restrict__ bid) {
    const QPart p = parts[blockIdx.y];
    unsigned long long* h = hist + (size_t)p.req * 2 * kQBuckets;
    q_hist_rows<ET>(p.qc, p.nrows, spl + (size_t)p.req * kQBuckets, h, h + kQBuckets, blockIdx.x, gridDim.x,
                    bid ? bid + p.bid_off : nullptr);
}

// Compaction of every part into its request's bucket segments (cursors are absolute candidate offsets).
template <int ET>
__global__ void __launch_bounds__(kQBlock)
q_compact_multi_kernel(const QPart* __restrict__ parts, const uint64_t* __restrict__ spl,
                       const uint32_t* __restrict__ target, unsigned long long* __restrict__ cursor,
                       uint64_t* __restrict__ cand) {
    const QPart p = parts[blockIdx.y];
    q_compact_rows<ET>(p.qc, p.nrows, spl + (size_t)p.req * kQBuckets, target + (size_t)p.req * kQBuckets,
                   cursor + (size_t)p.req * kQBuckets, cand, blockIdx.x, gridDim.x);
}

// Compaction from the recorded bucket ids: a row is read again only when its bucket is a target (a few % of rows).
template <int ET>
__global__ void __launch_bounds__(kQBlock)
q_compact_bid_kernel(const QPart* __restrict__ parts, const uint16_t* __restrict__ bid,
                     const uint32_t* __restrict__ target, unsigned long long* __restrict__ cursor,
                     uint64_t* __restrict__ cand) {
    __shared__ uint8_t tg[kQBuckets];
    const QPart p = parts[blockIdx.y];
    const uint32_t* tgt = target + (size_t)p.req * kQBuckets;
    unsigned long long* cur = cursor + (size_t)p.req * kQBuckets;
    for (int i = threadIdx.x; i < kQBuckets; i += blockDim.x) tg[i] = tgt[i] != kQNoTarget ? 1 : 0;
    __syncthreads();
    const uint16_t* ids = bid + p.bid_off;
    const int64_t nrows = p.nrows;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x * kQRowsPerLane;
    for (int64_t base = (int64_t)blockIdx.x * blockDim.x * kQRowsPerLane + threadIdx.x; base < nrows; base += stride) {
        uint16_t id[kQRowsPerLane];
#pragma unroll
        for (int j = 0; j < kQRowsPerLane; ++j) {
            const int64_t r = base + (int64_t)j * blockDim.x;
            id[j] = r < nrows ? q_gload<uint16_t>(ids, r) : kQBidNull;
        }
#pragma unroll
        for (int j = 0; j < kQRowsPerLane; ++j) {
            if (id[j] & kQBidEq) continue;  // NULL (0xFFFF) or a copy of the lower splitter
            if (!tg[id[j]]) continue;
            const int64_t r = base + (int64_t)j * blockDim.x;
            const uint64_t key = order_key(q_raw_value<ET>(p.qc, q_load_raw<ET>(p.qc.values, r)));
            const unsigned long long pos = atomicAdd(&cur[id[j]], 1ull);
            cand[pos] = key;
        }
    }
}

// One order statistic: the k-th smallest (1-based) of cand[lo, lo + cnt), all known to lie in [lo_key, hi_key];
// `out` is its output slot on the host (the kernel writes out[blockIdx.x]).
struct QSelect {
    uint64_t lo;
    uint64_t cnt;
    uint64_t k;
    uint64_t lo_key;
    uint64_t hi_key;
    int64_t out;
};

constexpr int kQSelBuf = 4096;  // matches staged in LDS once a digit narrows them to this many

// MSB-first radix select, 8 bits per round, starting below the bits the bucket bounds share: every round counts the
// digit of the keys matching the prefix chosen so far (global segment, or its LDS copy once few enough match).
__global__ void __launch_bounds__(256)
q_select_kernel(const uint64_t* __restrict__ cand, const QSelect* __restrict__ sel, double* __restrict__ out) {
    __shared__ unsigned int dh[256];
    __shared__ uint64_t buf[kQSelBuf];
    __shared__ unsigned int nbuf, s_digit, s_cnt;
    __shared__ uint64_t s_k;
    const QSelect q = sel[blockIdx.x];
    const uint64_t diff = q.lo_key ^ q.hi_key;
    int shift = diff ? ((63 - __clzll((long long)diff)) & ~7) : -8;
    const uint64_t top = shift + 8 >= 64 ? 0ULL : ~((1ULL << (shift + 8)) - 1);
    uint64_t prefix = q.lo_key & top, mask = top, k = q.k;
    bool staged = false;
    unsigned int nst = 0;
    for (; shift >= 0; shift -= 8) {
        for (int i = threadIdx.x; i < 256; i += blockDim.x) dh[i] = 0;
        __syncthreads();
        if (!staged) {
            for (uint64_t i = threadIdx.x; i < q.cnt; i += blockDim.x) {
                const uint64_t key = cand[q.lo + i];
                if ((key & mask) == prefix) atomicAdd(&dh[(key >> shift) & 255], 1u);
            }
        } else {
            for (unsigned int i = threadIdx.x; i < nst; i += blockDim.x) {
                const uint64_t key = buf[i];
                if ((key & mask) == prefix) atomicAdd(&dh[(key >> shift) & 255], 1u);
            }
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            uint64_t acc = 0;
            int d = 0;
            for (; d < 255; ++d) {
                if (acc + dh[d] >= k) break;
                acc += dh[d];
            }
            s_digit = (unsigned int)d;
            s_k = k - acc;
            s_cnt = dh[d];
        }
        __syncthreads();
        prefix |= (uint64_t)s_digit << shift;
        mask |= 0xFFULL << shift;
        k = s_k;
        const unsigned int cnt = s_cnt;
        if (shift > 0 && !staged && cnt <= (unsigned int)kQSelBuf) {
            if (threadIdx.x == 0) nbuf = 0;
            __syncthreads();
            for (uint64_t i = threadIdx.x; i < q.cnt; i += blockDim.x) {
                const uint64_t key = cand[q.lo + i];
                if ((key & mask) == prefix) buf[atomicAdd(&nbuf, 1u)] = key;
            }
            __syncthreads();
            nst = nbuf;
            staged = true;
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) out[blockIdx.x] = key_value(prefix);
}

__global__ void q_gather_kernel(const uint64_t* __restrict__ sorted, const int64_t* __restrict__ idx, int n,
                                double* __restrict__ out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = key_value(sorted[idx[i]]);
}

// Host dispatch of a kernel template over the element type: BODY sees the type as the constant E.
#define Q_ET_DISPATCH(et, BODY)                                  \
    switch (et) {                                                \
        case ET_F64: { constexpr int E = ET_F64; BODY; } break;  \
        case ET_F32: { constexpr int E = ET_F32; BODY; } break;  \
        case ET_I64: { constexpr int E = ET_I64; BODY; } break;  \
        case ET_I32: { constexpr int E = ET_I32; BODY; } break;  \
        case ET_I16: { constexpr int E = ET_I16; BODY; } break;  \
        case ET_I8: { constexpr int E = ET_I8; BODY; } break;    \
        default: { constexpr int E = ET_U8; BODY; } break;       \
    }

hipStream_t ctx_stream(dq_ctx* ctx);
int ctx_device(dq_ctx* ctx);
int ctx_fail(dq_ctx* ctx, int code, const char* msg);
int ctx_cus(dq_ctx* ctx);
int ctx_num_subs(dq_ctx* ctx);      // devices of a multi-device context, 0 for a single-device one
dq_ctx* ctx_sub(dq_ctx* ctx, int i);

}  // namespace dq

namespace {

using namespace dq;

// Host mirror of order_key / key_value (splitter values answered without a device gather).
double host_key_value(uint64_t k) {
    uint64_t u = (k >> 63) ? (k & 0x7fffffffffffffffULL) : ~k;
    double d;
    memcpy(&d, &u, 8);
    return d;
}

// Device buffers released on every exit path.
// Device buffers released on every exit path: from the context's scratch cache when `ctx` is set (a one-device
// context: a hipFree waits for the whole device, stalling this call behind other contexts' kernels), else hipMalloc.
struct QBuffers {
    dq_ctx* ctx = nullptr;
    std::vector<std::pair<void*, size_t>> ptrs;
    ~QBuffers() {
        for (const auto& p : ptrs) {
            if (ctx) dq::scratch_release(ctx, p.first, p.second);
            else (void)hipFree(p.first);
        }
    }
    hipError_t alloc(void** p, size_t bytes) {
        bytes = std::max<size_t>(bytes, 16);
        if (ctx) {
            *p = dq::scratch_alloc(ctx, bytes);
            if (!*p) return hipErrorOutOfMemory;
        } else {
            hipError_t e = hipMalloc(p, bytes);
            if (e != hipSuccess) return e;
        }
        ptrs.push_back({*p, bytes});
        return hipSuccess;
    }
};

}  // namespace

#define QT_HIP(ctx, expr)                                                                         \
    do {                                                                                          \
        hipError_t e_ = (expr);                                                                   \
        if (e_ != hipSuccess) return dq::ctx_fail((ctx), DQ_ERR_DEVICE, hipGetErrorString(e_));   \
    } while (0)

namespace {

// One shard of the column on one device: the whole column on a single-device context, one contiguous row range per
// device on a multi-device one (dq_open_devices). Every pass runs per shard on its own device and stream; the host
// adds the shards' histograms, so the order statistics are those of the whole column for any device count.
struct QShard {
    dq_ctx* ctx = nullptr;
    QColumn qc;
    int64_t nrows = 0;
    QBuffers buf;
    uint64_t* dkeys = nullptr;
    uint8_t* dok = nullptr;
    uint64_t* dspl = nullptr;
    unsigned long long* dhist = nullptr;
    uint32_t* dtarget = nullptr;
    unsigned long long* dcursor = nullptr;
    uint64_t* dcand = nullptr;
    int64_t ncand = 0;
    int grid = 1;
    std::vector<uint64_t> sk;
    std::vector<uint8_t> sok;
    std::vector<unsigned long long> hist;
    std::string err;
};

hipError_t q_stage_and_sample(QShard& sh, const dq_column& col) {
    hipError_t e = hipSetDevice(ctx_device(sh.ctx));
    if (e != hipSuccess) return e;
    hipStream_t s = ctx_stream(sh.ctx);
    const int t = col.spark_type;
    memset(&sh.qc, 0, sizeof(sh.qc));
    sh.qc.elem = elem_of(t);
    sh.qc.decimal_scale = t == DQ_TYPE_DECIMAL ? col.decimal_scale : 0;
    sh.qc.pow10 = pow(10.0, (double)sh.qc.decimal_scale);
    const int64_t nrows = sh.nrows;
    const size_t vbytes = (size_t)nrows * elem_size(sh.qc.elem);
    const size_t bbytes = (size_t)(nrows + 63) / 64 * 8;
    if (col.flags & DQ_COL_DEVICE) {
        sh.qc.values = col.values;
        sh.qc.validity = (const uint64_t*)col.validity;
    } else {
        void *v = nullptr, *m = nullptr;
        if ((e = sh.buf.alloc(&v, vbytes)) != hipSuccess) return e;
        if (nrows && (e = hipMemcpyAsync(v, col.values, vbytes, hipMemcpyHostToDevice, s)) != hipSuccess) return e;
        if (col.validity) {
            if ((e = sh.buf.alloc(&m, bbytes)) != hipSuccess) return e;
            if ((e = hipMemsetAsync(m, 0, bbytes, s)) != hipSuccess) return e;
            if (nrows && (e = hipMemcpyAsync(m, col.validity, (size_t)(nrows + 7) / 8, hipMemcpyHostToDevice, s)) != hipSuccess)
                return e;
        }
        sh.qc.values = v;
        sh.qc.validity = (const uint64_t*)m;
    }
    sh.sk.assign(kQSample, 0);
    sh.sok.assign(kQSample, 0);
    if (nrows == 0) return hipSuccess;
    if ((e = sh.buf.alloc((void**)&sh.dkeys, sizeof(uint64_t) * kQSample)) != hipSuccess) return e;
    if ((e = sh.buf.alloc((void**)&sh.dok, kQSample)) != hipSuccess) return e;
    hipLaunchKernelGGL(q_sample_kernel, dim3(kQSample / 256), dim3(256), 0, s, sh.qc, nrows, sh.dkeys, sh.dok);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    if ((e = hipMemcpyAsync(sh.sk.data(), sh.dkeys, sizeof(uint64_t) * kQSample, hipMemcpyDeviceToHost, s)) != hipSuccess)
        return e;
    if ((e = hipMemcpyAsync(sh.sok.data(), sh.dok, kQSample, hipMemcpyDeviceToHost, s)) != hipSuccess) return e;
    return hipStreamSynchronize(s);
}

}  // namespace

#define QS_HIP(ctx, expr)                                                                                  \
    do {                                                                                                   \
        hipError_t e_ = (expr);                                                                            \
        if (e_ != hipSuccess) return dq::ctx_fail((ctx), DQ_ERR_DEVICE, hipGetErrorString(e_));            \
    } while (0)

extern "C" {

int64_t dq_quantile_summary(dq_ctx* ctx, const dq_column* column, int64_t nrows, double relative_error,
                            int64_t max_samples, double* values_out, int64_t* ranks_out, int64_t* count_out) {
    if (!ctx || !column || nrows < 0 || column->length != nrows || !count_out || max_samples < 0 ||
        (max_samples > 0 && (!values_out || !ranks_out)))
        return dq::ctx_fail(ctx, DQ_ERR_INVALID_ARGUMENT, "dq_quantile_summary: invalid arguments");
    if (!(relative_error >= 0.0 && relative_error <= 1.0))
        return dq::ctx_fail(ctx, DQ_ERR_INVALID_ARGUMENT, "dq_quantile_summary: relative error must be in [0, 1]");
    const int t = column->spark_type;
    // Preconditions.isNumeric (A/Analyzer.scala:329-343): the analyzer checks it; the ABI rejects the rest.
    if (!(t == DQ_TYPE_BYTE || t == DQ_TYPE_SHORT || t == DQ_TYPE_INT || t == DQ_TYPE_LONG || t == DQ_TYPE_FLOAT ||
          t == DQ_TYPE_DOUBLE || t == DQ_TYPE_DECIMAL))
        return dq::ctx_fail(ctx, DQ_ERR_UNSUPPORTED, "dq_quantile_summary: column is not numeric");
    if (t == DQ_TYPE_DECIMAL && (column->decimal_precision > 18 || column->decimal_scale < 0 || column->decimal_scale > 18))
        return dq::ctx_fail(ctx, DQ_ERR_UNSUPPORTED, "dq_quantile_summary: decimal precision > 18 unsupported");
    *count_out = 0;
    if (nrows == 0) return 0;
    if (nrows >= (1LL << 46)) return dq::ctx_fail(ctx, DQ_ERR_INVALID_ARGUMENT, "dq_quantile_summary: too many rows");
    const int nsub = dq::ctx_num_subs(ctx);
    if (nsub > 0 && (column->flags & DQ_COL_DEVICE))
        return dq::ctx_fail(ctx, DQ_ERR_UNSUPPORTED, "a multi-device context takes host columns");

    // ---- shards: one per device, staged and sampled concurrently -----------------------------------
    const int ns_dev = nsub > 0 ? nsub : 1;
    std::vector<QShard> sh(ns_dev);
    std::vector<dq_column> cols(ns_dev, *column);
    std::vector<std::vector<std::vector<int32_t>>> scratch(ns_dev);
    for (int i = 0; i < ns_dev; ++i) {
        sh[i].ctx = nsub > 0 ? dq::ctx_sub(ctx, i) : ctx;
        if (nsub == 0) sh[i].buf.ctx = ctx;
        int64_t r0 = 0, cnt = nrows;
        if (nsub > 0) {
            dq::shard_bounds(nrows, nsub, i, &r0, &cnt);
            dq::shard_columns(column, 1, r0, cnt, &cols[i], scratch[i]);
        }
        sh[i].nrows = cnt;
    }
    {
        std::vector<hipError_t> rc(ns_dev, hipSuccess);
        std::vector<std::thread> th;
        for (int i = 0; i < ns_dev; ++i) th.emplace_back([&, i]() { rc[i] = q_stage_and_sample(sh[i], cols[i]); });
        for (auto& x : th) x.join();
        for (int i = 0; i < ns_dev; ++i)
            if (rc[i] != hipSuccess) return dq::ctx_fail(ctx, DQ_ERR_DEVICE, hipGetErrorString(rc[i]));
    }
    // splitters from every shard's stratified sample (equi-depth over the union; exactness does not depend on them)
    std::vector<uint64_t> valid;
    valid.reserve((size_t)kQSample * ns_dev);
    for (int i = 0; i < ns_dev; ++i)
        for (int j = 0; j < kQSample && sh[i].nrows; ++j)
            if (sh[i].sok[j]) valid.push_back(sh[i].sk[j]);
    std::sort(valid.begin(), valid.end());
    std::vector<uint64_t> spl(kQBuckets, ~0ULL);  // entry kQBuckets-1 stays +inf (no key reaches it)
    const size_t m = valid.size();
    if (m > 0)
        for (int j = 0; j < kQBuckets - 1; ++j) spl[j] = valid[(size_t)(j + 1) * m / kQBuckets < m ? (size_t)(j + 1) * m / kQBuckets : m - 1];

    std::vector<uint64_t> tree(kQBuckets, ~0ULL);  // the splitters in search-tree order (the kernels' layout)
    for (int j = 0; j < kQBuckets - 1; ++j) tree[j] = spl[q_tree_sorted_index(j)];

    // ---- 2. histogram per shard, added on the host ------------------------------------------------
    for (QShard& q : sh) {
        if (!q.nrows) continue;
        QS_HIP(ctx, hipSetDevice(dq::ctx_device(q.ctx)));
        hipStream_t s = dq::ctx_stream(q.ctx);
        QS_HIP(ctx, q.buf.alloc((void**)&q.dspl, sizeof(uint64_t) * kQBuckets));
        QS_HIP(ctx, hipMemcpyAsync(q.dspl, tree.data(), sizeof(uint64_t) * kQBuckets, hipMemcpyHostToDevice, s));
        QS_HIP(ctx, q.buf.alloc((void**)&q.dhist, sizeof(unsigned long long) * kQBuckets * 2));
        QS_HIP(ctx, hipMemsetAsync(q.dhist, 0, sizeof(unsigned long long) * kQBuckets * 2, s));
        const int64_t lanes_needed = (q.nrows + kQRowsPerLane - 1) / kQRowsPerLane;
        q.grid = (int)std::max<int64_t>(1, std::min<int64_t>((lanes_needed + kQBlock - 1) / kQBlock,
                                                             (int64_t)dq::ctx_cus(q.ctx) * 2));
        Q_ET_DISPATCH(q.qc.elem, hipLaunchKernelGGL(q_hist_kernel<E>, dim3(q.grid), dim3(kQBlock), 0, s, q.qc, q.nrows,
                                                    (const uint64_t*)q.dspl, q.dhist, q.dhist + kQBuckets));
        QS_HIP(ctx, hipGetLastError());
        q.hist.assign(kQBuckets * 2, 0);
        QS_HIP(ctx, hipMemcpyAsync(q.hist.data(), q.dhist, sizeof(unsigned long long) * kQBuckets * 2,
                                   hipMemcpyDeviceToHost, s));
    }
    std::vector<unsigned long long> hist(kQBuckets * 2, 0);
    for (QShard& q : sh) {
        if (!q.nrows) continue;
        QS_HIP(ctx, hipSetDevice(dq::ctx_device(q.ctx)));
        QS_HIP(ctx, hipStreamSynchronize(dq::ctx_stream(q.ctx)));
        for (int b = 0; b < kQBuckets * 2; ++b) hist[b] += q.hist[b];
    }
    const unsigned long long* eq = hist.data() + kQBuckets;
    int64_t n = 0;
    for (int b = 0; b < kQBuckets; ++b) n += (int64_t)hist[b];
    *count_out = n;
    if (n == 0) return 0;

    // ---- 3. summary ranks -> (bucket, residual) --------------------------------------------------
    const int64_t spacing = std::max<int64_t>(1, (int64_t)floor(relative_error * (double)n));
    const int64_t ns = (n - 1) / spacing + 1 + ((n - 1) % spacing != 0 ? 1 : 0);
    if (ns > max_samples) {
        char msg[160];
        snprintf(msg, sizeof(msg), "dq_quantile_summary: %lld samples needed, capacity %lld", (long long)ns,
                 (long long)max_samples);
        return dq::ctx_fail(ctx, DQ_ERR_INVALID_ARGUMENT, msg);
    }
    std::vector<int64_t> ranks;
    ranks.reserve(ns);
    for (int64_t r = 1; r <= n; r += spacing) ranks.push_back(r);
    if (ranks.back() != n) ranks.push_back(n);
    std::vector<int64_t> cum(kQBuckets + 1, 0);
    for (int b = 0; b < kQBuckets; ++b) cum[b + 1] = cum[b] + (int64_t)hist[b];
    std::vector<uint32_t> target(kQBuckets, kQNoTarget);
    std::vector<int> rank_bucket(ns);
    std::vector<int64_t> rank_resid(ns);
    std::vector<char> from_splitter(ns, 0);
    for (int64_t i = 0; i < ns; ++i) {
        const int64_t r = ranks[i];
        const int b = (int)(std::upper_bound(cum.begin(), cum.end(), r - 1) - cum.begin()) - 1;  // cum[b] < r <= cum[b+1]
        int64_t resid = r - cum[b];
        rank_bucket[i] = b;
        if (b > 0 && resid <= (int64_t)eq[b]) {
            from_splitter[i] = 1;  // a copy of the lower splitter
            values_out[i] = host_key_value(spl[b - 1]);
        } else {
            if (b > 0) resid -= (int64_t)eq[b];
            target[b] = 0;
        }
        rank_resid[i] = resid;
        ranks_out[i] = r;
    }
    // global bucket segments of the sorted candidates; per shard, its own bucket-contiguous layout
    std::vector<unsigned long long> cursor(kQBuckets, 0);
    int64_t ncand = 0;
    for (int b = 0; b < kQBuckets; ++b) {
        if (target[b] == kQNoTarget) continue;
        target[b] = 1;
        cursor[b] = (unsigned long long)ncand;
        ncand += (int64_t)hist[b] - (b > 0 ? (int64_t)eq[b] : 0);
    }
    if (ncand == 0) return ns;

    // ---- 4. compaction per shard, candidates gathered on the first shard's device ------------------
    QShard& s0 = sh[0];
    uint64_t *dall = nullptr, *dsorted = nullptr;
    QS_HIP(ctx, hipSetDevice(dq::ctx_device(s0.ctx)));
    QS_HIP(ctx, s0.buf.alloc((void**)&dall, sizeof(uint64_t) * ncand));
    QS_HIP(ctx, s0.buf.alloc((void**)&dsorted, sizeof(uint64_t) * ncand));
    int64_t at = 0;
    for (QShard& q : sh) {
        if (!q.nrows) continue;
        std::vector<unsigned long long> lcur(kQBuckets, 0);
        int64_t nloc = 0;
        for (int b = 0; b < kQBuckets; ++b) {
            if (target[b] == kQNoTarget) continue;
            lcur[b] = (unsigned long long)nloc;
            nloc += (int64_t)q.hist[b] - (b > 0 ? (int64_t)q.hist[kQBuckets + b] : 0);
        }
        q.ncand = nloc;
        if (nloc == 0) continue;
        QS_HIP(ctx, hipSetDevice(dq::ctx_device(q.ctx)));
        hipStream_t s = dq::ctx_stream(q.ctx);
        QS_HIP(ctx, q.buf.alloc((void**)&q.dtarget, sizeof(uint32_t) * kQBuckets));
        QS_HIP(ctx, q.buf.alloc((void**)&q.dcursor, sizeof(unsigned long long) * kQBuckets));
        QS_HIP(ctx, q.buf.alloc((void**)&q.dcand, sizeof(uint64_t) * nloc));
        QS_HIP(ctx, hipMemcpyAsync(q.dtarget, target.data(), sizeof(uint32_t) * kQBuckets, hipMemcpyHostToDevice, s));
        QS_HIP(ctx, hipMemcpyAsync(q.dcursor, lcur.data(), sizeof(unsigned long long) * kQBuckets, hipMemcpyHostToDevice, s));
        Q_ET_DISPATCH(q.qc.elem, hipLaunchKernelGGL(q_compact_kernel<E>, dim3(q.grid), dim3(kQBlock), 0, s, q.qc,
                                                    q.nrows, (const uint64_t*)q.dspl, (const uint32_t*)q.dtarget,
                                                    q.dcursor, q.dcand));
        QS_HIP(ctx, hipGetLastError());
        QS_HIP(ctx, hipMemcpyPeerAsync(dall + at, dq::ctx_device(s0.ctx), q.dcand, dq::ctx_device(q.ctx),
                                       sizeof(uint64_t) * nloc, s));
        at += nloc;
    }
    for (QShard& q : sh) {
        if (!q.ncand) continue;
        QS_HIP(ctx, hipSetDevice(dq::ctx_device(q.ctx)));
        QS_HIP(ctx, hipStreamSynchronize(dq::ctx_stream(q.ctx)));
    }
    if (at != ncand) return dq::ctx_fail(ctx, DQ_ERR_DEVICE, "dq_quantile_summary: candidate count mismatch");

    // ---- 5. sort all candidates (bucket segments follow key order) --------------------------------
    QS_HIP(ctx, hipSetDevice(dq::ctx_device(s0.ctx)));
    hipStream_t s = dq::ctx_stream(s0.ctx);
    size_t tmp_bytes = 0;
    QS_HIP(ctx, rocprim::radix_sort_keys(nullptr, tmp_bytes, dall, dsorted, (size_t)ncand, 0, 64, s));
    void* dtmp = nullptr;
    QS_HIP(ctx, s0.buf.alloc(&dtmp, tmp_bytes));
    QS_HIP(ctx, rocprim::radix_sort_keys(dtmp, tmp_bytes, dall, dsorted, (size_t)ncand, 0, 64, s));

    // ---- 6. gather -------------------------------------------------------------------------------
    std::vector<int64_t> idx;
    std::vector<int64_t> which;
    for (int64_t i = 0; i < ns; ++i) {
        if (from_splitter[i]) continue;
        idx.push_back((int64_t)cursor[rank_bucket[i]] + rank_resid[i] - 1);
        which.push_back(i);
    }
    const int ng = (int)idx.size();
    int64_t* didx = nullptr;
    double* dvals = nullptr;
    QS_HIP(ctx, s0.buf.alloc((void**)&didx, sizeof(int64_t) * ng));
    QS_HIP(ctx, s0.buf.alloc((void**)&dvals, sizeof(double) * ng));
    QS_HIP(ctx, hipMemcpyAsync(didx, idx.data(), sizeof(int64_t) * ng, hipMemcpyHostToDevice, s));
    hipLaunchKernelGGL(q_gather_kernel, dim3((ng + 255) / 256), dim3(256), 0, s, (const uint64_t*)dsorted,
                       (const int64_t*)didx, ng, dvals);
    QS_HIP(ctx, hipGetLastError());
    std::vector<double> got(ng);
    QS_HIP(ctx, hipMemcpyAsync(got.data(), dvals, sizeof(double) * ng, hipMemcpyDeviceToHost, s));
    QS_HIP(ctx, hipStreamSynchronize(s));
    for (int j = 0; j < ng; ++j) values_out[which[j]] = got[j];
    return ns;
}


// Several summaries in one set of passes (samples, splitters and histograms of every request in one launch each, one
// host round trip, one compaction launch, a radix select per summary rank): the values are exactly those of
// dq_quantile_summary over each request's parts concatenated (exact order statistics do not depend on the
// splitters). Device scratch comes from the context's cache.
int dq_quantile_summaries(dq_ctx* ctx, const dq_column* parts, const int32_t* part_begin, int nreq,
                          const double* relative_error, int64_t max_samples, double* values_out, int64_t* ranks_out,
                          int64_t* counts_out, int64_t* samples_out) {
    if (!ctx || nreq < 0 || (nreq > 0 && (!parts || !part_begin || !relative_error || !counts_out || !samples_out)) ||
        max_samples < 0 || (max_samples > 0 && nreq > 0 && (!values_out || !ranks_out)))
        return dq::ctx_fail(ctx, DQ_ERR_INVALID_ARGUMENT, "dq_quantile_summaries: invalid arguments");
    if (nreq == 0) return 0;
    if (part_begin[0] != 0) return dq::ctx_fail(ctx, DQ_ERR_INVALID_ARGUMENT, "dq_quantile_summaries: part_begin[0] != 0");
    for (int r = 0; r < nreq; ++r) {
        if (part_begin[r + 1] <= part_begin[r])
            return dq::ctx_fail(ctx, DQ_ERR_INVALID_ARGUMENT, "dq_quantile_summaries: a request without parts");
        if (!(relative_error[r] >= 0.0 && relative_error[r] <= 1.0))
            return dq::ctx_fail(ctx, DQ_ERR_INVALID_ARGUMENT, "dq_quantile_summaries: relative error must be in [0, 1]");
        const int t = parts[part_begin[r]].spark_type;
        for (int p = part_begin[r]; p < part_begin[r + 1]; ++p) {
            const dq_column& c = parts[p];
            if (c.spark_type != t || c.length < 0 ||
                (t == DQ_TYPE_DECIMAL && c.decimal_scale != parts[part_begin[r]].decimal_scale))
                return dq::ctx_fail(ctx, DQ_ERR_INVALID_ARGUMENT, "dq_quantile_summaries: parts of one request differ");
        }
        if (!(t == DQ_TYPE_BYTE || t == DQ_TYPE_SHORT || t == DQ_TYPE_INT || t == DQ_TYPE_LONG || t == DQ_TYPE_FLOAT ||
              t == DQ_TYPE_DOUBLE || t == DQ_TYPE_DECIMAL))
            return dq::ctx_fail(ctx, DQ_ERR_UNSUPPORTED, "dq_quantile_summaries: column is not numeric");
        if (t == DQ_TYPE_DECIMAL && (parts[part_begin[r]].decimal_precision > 18 ||
                                     parts[part_begin[r]].decimal_scale < 0 || parts[part_begin[r]].decimal_scale > 18))
            return dq::ctx_fail(ctx, DQ_ERR_UNSUPPORTED, "dq_quantile_summaries: decimal precision > 18 unsupported");
    }
    const int nparts = part_begin[nreq];
    if (dq::ctx_num_subs(ctx) > 0) {
        // multi-device context: its sharded single-column path, one request (of one part) at a time
        for (int r = 0; r < nreq; ++r) {
            if (part_begin[r + 1] - part_begin[r] != 1)
                return dq::ctx_fail(ctx, DQ_ERR_UNSUPPORTED, "a multi-device context takes one part per request");
            const int64_t ns = dq_quantile_summary(ctx, &parts[part_begin[r]], parts[part_begin[r]].length,
                                                   relative_error[r], max_samples, values_out + (size_t)r * max_samples,
                                                   ranks_out + (size_t)r * max_samples, &counts_out[r]);
            if (ns < 0) return (int)ns;
            samples_out[r] = ns;
        }
        return 0;
    }
    QS_HIP(ctx, hipSetDevice(dq::ctx_device(ctx)));
    hipStream_t s = dq::ctx_stream(ctx);

    // scratch blocks handed back to the context's cache on every exit path (their last use is on `s`)
    struct Scratch {
        dq_ctx* ctx;
        std::vector<std::pair<void*, size_t>> blocks;
        ~Scratch() {
            for (auto& b : blocks) dq::scratch_release(ctx, b.first, b.second);
        }
        void* get(size_t bytes) {
            void* p = dq::scratch_alloc(ctx, bytes);
            if (p) blocks.emplace_back(p, bytes);
            return p;
        }
    } scr{ctx, {}};
#define QM_ALLOC(ptr, T, count)                                                                          \
    do {                                                                                                 \
        (ptr) = (T*)scr.get(sizeof(T) * (size_t)std::max<int64_t>((count), 1));                          \
        if (!(ptr)) return dq::ctx_fail(ctx, DQ_ERR_DEVICE, "dq_quantile_summaries: out of device memory"); \
    } while (0)

    // ---- part table (host parts staged into scratch) ------------------------------------------------
    std::vector<QPart> qp(nparts);
    std::vector<int64_t> req_rows(nreq, 0);
    int64_t total_rows = 0;
    for (int r = 0; r < nreq; ++r) {
        int64_t at = 0;
        for (int p = part_begin[r]; p < part_begin[r + 1]; ++p) {
            const dq_column& c = parts[p];
            QPart& q = qp[p];
            memset(&q, 0, sizeof(q));
            q.qc.elem = elem_of(c.spark_type);
            q.qc.decimal_scale = c.spark_type == DQ_TYPE_DECIMAL ? c.decimal_scale : 0;
            q.qc.pow10 = pow(10.0, (double)q.qc.decimal_scale);
            q.nrows = c.length;
            q.row0 = at;
            q.bid_off = total_rows + at;
            q.req = r;
            at += c.length;
            if (c.flags & DQ_COL_DEVICE) {
                q.qc.values = c.values;
                q.qc.validity = (const uint64_t*)c.validity;
            } else if (c.length > 0) {
                const size_t vbytes = (size_t)c.length * elem_size(q.qc.elem);
                const size_t bbytes = (size_t)(c.length + 63) / 64 * 8;
                void* v = scr.get(vbytes);
                if (!v) return dq::ctx_fail(ctx, DQ_ERR_DEVICE, "dq_quantile_summaries: out of device memory");
                QS_HIP(ctx, hipMemcpyAsync(v, c.values, vbytes, hipMemcpyHostToDevice, s));
                q.qc.values = v;
                if (c.validity) {
                    void* m = scr.get(bbytes);
                    if (!m) return dq::ctx_fail(ctx, DQ_ERR_DEVICE, "dq_quantile_summaries: out of device memory");
                    QS_HIP(ctx, hipMemsetAsync(m, 0, bbytes, s));
                    QS_HIP(ctx, hipMemcpyAsync(m, c.validity, (size_t)(c.length + 7) / 8, hipMemcpyHostToDevice, s));
                    q.qc.validity = (const uint64_t*)m;
                }
            }
        }
        if (at >= (1LL << 46)) return dq::ctx_fail(ctx, DQ_ERR_INVALID_ARGUMENT, "dq_quantile_summaries: too many rows");
        req_rows[r] = at;
        total_rows += at;
    }
    QPart* dparts;
    int32_t* dbegin;
    int64_t* drows;
    uint64_t *dkeys, *dsorted, *dspl, *dtree;
    unsigned int* dvalid;
    unsigned long long* dhist;
    QM_ALLOC(dparts, QPart, nparts);
    QM_ALLOC(dbegin, int32_t, nreq + 1);
    QM_ALLOC(drows, int64_t, nreq);
    QM_ALLOC(dkeys, uint64_t, (int64_t)nreq * kQSample);
    QM_ALLOC(dsorted, uint64_t, (int64_t)nreq * kQSample);
    QM_ALLOC(dspl, uint64_t, (int64_t)nreq * kQBuckets);
    QM_ALLOC(dtree, uint64_t, (int64_t)nreq * kQBuckets);
    QM_ALLOC(dvalid, unsigned int, nreq);
    QM_ALLOC(dhist, unsigned long long, (int64_t)nreq * 2 * kQBuckets);
    QS_HIP(ctx, hipMemcpyAsync(dparts, qp.data(), sizeof(QPart) * nparts, hipMemcpyHostToDevice, s));
    QS_HIP(ctx, hipMemcpyAsync(dbegin, part_begin, sizeof(int32_t) * (nreq + 1), hipMemcpyHostToDevice, s));
    QS_HIP(ctx, hipMemcpyAsync(drows, req_rows.data(), sizeof(int64_t) * nreq, hipMemcpyHostToDevice, s));
    QS_HIP(ctx, hipMemsetAsync(dvalid, 0, sizeof(unsigned int) * nreq, s));
    QS_HIP(ctx, hipMemsetAsync(dhist, 0, sizeof(unsigned long long) * nreq * 2 * kQBuckets, s));

    // ---- 1. samples, their per-request sort, splitters: all on the device ----------------------------
    hipLaunchKernelGGL(q_sample_multi_kernel, dim3(kQSample / 256, nreq), dim3(256), 0, s, (const QPart*)dparts,
                       (const int32_t*)dbegin, (const int64_t*)drows, dkeys, dvalid);
    QS_HIP(ctx, hipGetLastError());
    std::vector<unsigned int> seg_off(nreq + 1);
    for (int r = 0; r <= nreq; ++r) seg_off[r] = (unsigned int)r * kQSample;
    unsigned int* dseg;
    QM_ALLOC(dseg, unsigned int, nreq + 1);
    QS_HIP(ctx, hipMemcpyAsync(dseg, seg_off.data(), sizeof(unsigned int) * (nreq + 1), hipMemcpyHostToDevice, s));
    size_t tmp_bytes = 0;
    QS_HIP(ctx, rocprim::segmented_radix_sort_keys(nullptr, tmp_bytes, dkeys, dsorted, (unsigned int)nreq * kQSample,
                                                   (unsigned int)nreq, dseg, dseg + 1, 0, 64, s));
    void* dtmp = scr.get(tmp_bytes);
    if (!dtmp) return dq::ctx_fail(ctx, DQ_ERR_DEVICE, "dq_quantile_summaries: out of device memory");
    QS_HIP(ctx, rocprim::segmented_radix_sort_keys(dtmp, tmp_bytes, dkeys, dsorted, (unsigned int)nreq * kQSample,
                                                   (unsigned int)nreq, dseg, dseg + 1, 0, 64, s));
    hipLaunchKernelGGL(q_splitters_kernel, dim3(nreq), dim3(256), 0, s, (const uint64_t*)dsorted,
                       (const unsigned int*)dvalid, dspl, dtree);
    QS_HIP(ctx, hipGetLastError());

    // ---- 2. histograms of every part ------------------------------------------------------------------
    int64_t max_part = 1;
    for (const QPart& q : qp) max_part = std::max<int64_t>(max_part, q.nrows);
    const int64_t lanes_needed = (max_part + kQRowsPerLane - 1) / kQRowsPerLane;
    // one resident round of workgroups over all parts: 2 per CU in the histogram pass (64 KB of LDS), 3 in the
    // compaction (48 KB)
    auto part_grid = [&](int per_cu, int block) {
        return (int)std::max<int64_t>(1, std::min<int64_t>((lanes_needed + block - 1) / block,
                                                           (int64_t)dq::ctx_cus(ctx) * per_cu / nparts));
    };
    const int gx = part_grid(2, kQHistBlock), gxc = part_grid(3, kQBlock), gxb = part_grid(8, kQBlock);
    // the parts grouped by element type: one launch per type present (blockIdx.y = part of that type)
    std::vector<QPart> typed(qp);
    std::stable_sort(typed.begin(), typed.end(), [](const QPart& a, const QPart& b) { return a.qc.elem < b.qc.elem; });
    QPart* dtyped;
    QM_ALLOC(dtyped, QPart, nparts);
    QS_HIP(ctx, hipMemcpyAsync(dtyped, typed.data(), sizeof(QPart) * nparts, hipMemcpyHostToDevice, s));
    std::vector<std::pair<int, int>> type_runs;  // (first typed part, count)
    for (int i = 0; i < nparts;) {
        int j = i;
        while (j < nparts && typed[j].qc.elem == typed[i].qc.elem) ++j;
        type_runs.emplace_back(i, j - i);
        i = j;
    }
    // every row's bucket id (2 B a row) for the compaction; without room for it the compaction searches again
    uint16_t* dbid = getenv("DQ_Q_NO_BID") ? nullptr : (uint16_t*)scr.get(sizeof(uint16_t) * (size_t)std::max<int64_t>(total_rows, 1));
    for (auto& tr : type_runs) {
        Q_ET_DISPATCH(typed[tr.first].qc.elem,
                      hipLaunchKernelGGL(q_hist_multi_kernel<E>, dim3(gx, tr.second), dim3(kQHistBlock), 0, s,
                                         (const QPart*)(dtyped + tr.first), (const uint64_t*)dtree, dhist, dbid));
        QS_HIP(ctx, hipGetLastError());
    }
    std::vector<unsigned long long> hist((size_t)nreq * 2 * kQBuckets);
    std::vector<uint64_t> spl((size_t)nreq * kQBuckets);
    QS_HIP(ctx, hipMemcpyAsync(hist.data(), dhist, sizeof(unsigned long long) * hist.size(), hipMemcpyDeviceToHost, s));
    QS_HIP(ctx, hipMemcpyAsync(spl.data(), dspl, sizeof(uint64_t) * spl.size(), hipMemcpyDeviceToHost, s));
    QS_HIP(ctx, hipStreamSynchronize(s));

    // ---- 3. ranks -> (bucket, residual); target buckets get absolute candidate segments -----------------
    constexpr int64_t kSelectMaxRanks = 4096;  // more ranks than this (relative_error 0 on small data): sort instead
    std::vector<uint32_t> target((size_t)nreq * kQBuckets, kQNoTarget);
    std::vector<unsigned long long> cursor((size_t)nreq * kQBuckets, 0);
    std::vector<unsigned long long> seg0((size_t)nreq * kQBuckets, 0);
    std::vector<QSelect> sel;
    struct SortReq {
        int r;
        int64_t base, ncand;
        std::vector<int64_t> idx, out;
    };
    std::vector<SortReq> sorts;
    int64_t ncand = 0;
    for (int r = 0; r < nreq; ++r) {
        const unsigned long long* h = hist.data() + (size_t)r * 2 * kQBuckets;
        const unsigned long long* eq = h + kQBuckets;
        const uint64_t* sp = spl.data() + (size_t)r * kQBuckets;
        double* vout = values_out + (size_t)r * max_samples;
        int64_t* rout = ranks_out + (size_t)r * max_samples;
        int64_t n = 0;
        for (int b = 0; b < kQBuckets; ++b) n += (int64_t)h[b];
        counts_out[r] = n;
        samples_out[r] = 0;
        if (n == 0) continue;
        const int64_t spacing = std::max<int64_t>(1, (int64_t)floor(relative_error[r] * (double)n));
        const int64_t ns = (n - 1) / spacing + 1 + ((n - 1) % spacing != 0 ? 1 : 0);
        if (ns > max_samples) {
            char msg[160];
            snprintf(msg, sizeof(msg), "dq_quantile_summaries: %lld samples needed, capacity %lld", (long long)ns,
                     (long long)max_samples);
            return dq::ctx_fail(ctx, DQ_ERR_INVALID_ARGUMENT, msg);
        }
        samples_out[r] = ns;
        std::vector<int64_t> cum(kQBuckets + 1, 0);
        for (int b = 0; b < kQBuckets; ++b) cum[b + 1] = cum[b] + (int64_t)h[b];
        uint32_t* tg = target.data() + (size_t)r * kQBuckets;
        std::vector<int> rb(ns);
        std::vector<int64_t> rres(ns);
        std::vector<char> from_spl(ns, 0);
        for (int64_t i = 0; i < ns; ++i) {
            const int64_t rank = std::min<int64_t>(1 + i * spacing, n);
            const int b = (int)(std::upper_bound(cum.begin(), cum.end(), rank - 1) - cum.begin()) - 1;
            int64_t resid = rank - cum[b];
            rb[i] = b;
            rout[i] = rank;
            if (b > 0 && resid <= (int64_t)eq[b]) {
                from_spl[i] = 1;
                vout[i] = host_key_value(sp[b - 1]);
            } else {
                if (b > 0) resid -= (int64_t)eq[b];
                tg[b] = 1;
            }
            rres[i] = resid;
        }
        const int64_t base = ncand;
        for (int b = 0; b < kQBuckets; ++b) {
            if (tg[b] == kQNoTarget) continue;
            cursor[(size_t)r * kQBuckets + b] = seg0[(size_t)r * kQBuckets + b] = (unsigned long long)ncand;
            ncand += (int64_t)h[b] - (b > 0 ? (int64_t)eq[b] : 0);
        }
        const bool by_sort = ns > kSelectMaxRanks;
        if (by_sort) sorts.push_back(SortReq{r, base, ncand - base, {}, {}});
        for (int64_t i = 0; i < ns; ++i) {
            if (from_spl[i]) continue;
            const int b = rb[i];
            const uint64_t lo = seg0[(size_t)r * kQBuckets + b];
            if (by_sort) {
                sorts.back().idx.push_back((int64_t)lo - base + rres[i] - 1);
                sorts.back().out.push_back((int64_t)r * max_samples + i);
                continue;
            }
            QSelect q;
            q.lo = lo;
            q.cnt = (uint64_t)((int64_t)h[b] - (b > 0 ? (int64_t)eq[b] : 0));
            q.k = (uint64_t)rres[i];
            q.lo_key = b > 0 ? sp[b - 1] : 0ULL;
            q.hi_key = sp[b] - 1;  // keys below the next splitter (every key < the +inf sentinel ~0)
            q.out = (int64_t)r * max_samples + i;
            sel.push_back(q);
        }
    }
    if (ncand == 0) return 0;

    // ---- 4. compaction of every part --------------------------------------------------------------------
    uint32_t* dtarget;
    unsigned long long* dcursor;
    uint64_t* dcand;
    QM_ALLOC(dtarget, uint32_t, (int64_t)nreq * kQBuckets);
    QM_ALLOC(dcursor, unsigned long long, (int64_t)nreq * kQBuckets);
    QM_ALLOC(dcand, uint64_t, ncand);
    QS_HIP(ctx, hipMemcpyAsync(dtarget, target.data(), sizeof(uint32_t) * target.size(), hipMemcpyHostToDevice, s));
    QS_HIP(ctx, hipMemcpyAsync(dcursor, cursor.data(), sizeof(unsigned long long) * cursor.size(), hipMemcpyHostToDevice, s));
    for (auto& tr : type_runs) {
        if (dbid)
            Q_ET_DISPATCH(typed[tr.first].qc.elem,
                          hipLaunchKernelGGL(q_compact_bid_kernel<E>, dim3(gxb, tr.second), dim3(kQBlock), 0, s,
                                             (const QPart*)(dtyped + tr.first), (const uint16_t*)dbid,
                                             (const uint32_t*)dtarget, dcursor, dcand))
        else
            Q_ET_DISPATCH(typed[tr.first].qc.elem,
                          hipLaunchKernelGGL(q_compact_multi_kernel<E>, dim3(gxc, tr.second), dim3(kQBlock), 0, s,
                                             (const QPart*)(dtyped + tr.first), (const uint64_t*)dtree,
                                             (const uint32_t*)dtarget, dcursor, dcand))
        QS_HIP(ctx, hipGetLastError());
    }

    // ---- 5. order statistics: radix select per rank; a sort for requests with very many ranks ------------
    double* dout = nullptr;
    if (!sel.empty()) {
        QSelect* dsel;
        QM_ALLOC(dsel, QSelect, (int64_t)sel.size());
        QM_ALLOC(dout, double, (int64_t)sel.size());
        QS_HIP(ctx, hipMemcpyAsync(dsel, sel.data(), sizeof(QSelect) * sel.size(), hipMemcpyHostToDevice, s));
        hipLaunchKernelGGL(q_select_kernel, dim3((unsigned int)sel.size()), dim3(256), 0, s, (const uint64_t*)dcand,
                           (const QSelect*)dsel, dout);
        QS_HIP(ctx, hipGetLastError());
    }
    std::vector<std::vector<double>> sorted_vals(sorts.size());
    for (size_t j = 0; j < sorts.size(); ++j) {
        SortReq& q = sorts[j];
        if (q.idx.empty()) continue;
        uint64_t* dsrt;
        QM_ALLOC(dsrt, uint64_t, q.ncand);
        size_t tb = 0;
        QS_HIP(ctx, rocprim::radix_sort_keys(nullptr, tb, dcand + q.base, dsrt, (size_t)q.ncand, 0, 64, s));
        void* dt = scr.get(tb);
        if (!dt) return dq::ctx_fail(ctx, DQ_ERR_DEVICE, "dq_quantile_summaries: out of device memory");
        QS_HIP(ctx, rocprim::radix_sort_keys(dt, tb, dcand + q.base, dsrt, (size_t)q.ncand, 0, 64, s));
        const int ng = (int)q.idx.size();
        int64_t* didx;
        double* dv;
        QM_ALLOC(didx, int64_t, ng);
        QM_ALLOC(dv, double, ng);
        QS_HIP(ctx, hipMemcpyAsync(didx, q.idx.data(), sizeof(int64_t) * ng, hipMemcpyHostToDevice, s));
        hipLaunchKernelGGL(q_gather_kernel, dim3((ng + 255) / 256), dim3(256), 0, s, (const uint64_t*)dsrt,
                           (const int64_t*)didx, ng, dv);
        QS_HIP(ctx, hipGetLastError());
        sorted_vals[j].resize(ng);
        QS_HIP(ctx, hipMemcpyAsync(sorted_vals[j].data(), dv, sizeof(double) * ng, hipMemcpyDeviceToHost, s));
    }
    std::vector<double> got(sel.size());
    if (!sel.empty())
        QS_HIP(ctx, hipMemcpyAsync(got.data(), dout, sizeof(double) * got.size(), hipMemcpyDeviceToHost, s));
    QS_HIP(ctx, hipStreamSynchronize(s));
    for (size_t j = 0; j < sel.size(); ++j) values_out[sel[j].out] = got[j];
    for (size_t j = 0; j < sorts.size(); ++j)
        for (size_t i = 0; i < sorts[j].out.size(); ++i) values_out[sorts[j].out[i]] = sorted_vals[j][i];
#undef QM_ALLOC
    return 0;
}

}  // extern "C"
