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
constexpr int kQRowsPerLane = 4;         // independent binary searches in flight per lane
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

// Pass 2: bucket counts and counts of keys equal to the bucket's lower splitter.
__global__ void __launch_bounds__(kQBlock)
q_hist_kernel(QColumn c, int64_t nrows, const uint64_t* __restrict__ splitters,
              unsigned long long* __restrict__ hist, unsigned long long* __restrict__ eq) {
    __shared__ uint64_t spl[kQBuckets];
    __shared__ uint32_t h[kQBuckets];
    __shared__ uint32_t e[kQBuckets];
    q_load_splitters(spl, splitters);
    for (int i = threadIdx.x; i < kQBuckets; i += blockDim.x) h[i] = e[i] = 0;
    __syncthreads();
    const int64_t stride = (int64_t)gridDim.x * blockDim.x * kQRowsPerLane;
    for (int64_t base = (int64_t)blockIdx.x * blockDim.x * kQRowsPerLane + threadIdx.x; base < nrows; base += stride) {
        uint64_t k[kQRowsPerLane];
        bool v[kQRowsPerLane];
#pragma unroll
        for (int j = 0; j < kQRowsPerLane; ++j) {
            const int64_t r = base + (int64_t)j * blockDim.x;
            v[j] = r < nrows && q_valid(c, r);
            k[j] = v[j] ? order_key(q_load(c, r)) : 0;
        }
        uint32_t b[kQRowsPerLane];
#pragma unroll
        for (int j = 0; j < kQRowsPerLane; ++j) b[j] = 0;
        // bucket = number of splitters <= key: branchless binary search over the sorted LDS array
        // (its last entry is +inf, above every key), kQRowsPerLane searches interleaved.
#pragma unroll
        for (uint32_t step = kQBuckets / 2; step > 0; step >>= 1)
#pragma unroll
            for (int j = 0; j < kQRowsPerLane; ++j) b[j] += (spl[b[j] + step - 1] <= k[j]) ? step : 0u;
#pragma unroll
        for (int j = 0; j < kQRowsPerLane; ++j) {
            if (!v[j]) continue;
            atomicAdd(&h[b[j]], 1u);
            if (b[j] > 0 && spl[b[j] - 1] == k[j]) atomicAdd(&e[b[j]], 1u);
        }
    }
    __syncthreads();
    for (int i = threadIdx.x; i < kQBuckets; i += blockDim.x) {
        if (h[i]) atomicAdd(&hist[i], (unsigned long long)h[i]);
        if (e[i]) atomicAdd(&eq[i], (unsigned long long)e[i]);
    }
}

// Pass 4: rows of target buckets (other than copies of the lower splitter) -> candidates, written
// into their bucket's segment through a per-bucket cursor.
__global__ void __launch_bounds__(kQBlock)
q_compact_kernel(QColumn c, int64_t nrows, const uint64_t* __restrict__ splitters, const uint32_t* __restrict__ target,
                 unsigned long long* __restrict__ cursor, uint64_t* __restrict__ cand) {
    __shared__ uint64_t spl[kQBuckets];
    __shared__ uint32_t tg[kQBuckets];
    q_load_splitters(spl, splitters);
    for (int i = threadIdx.x; i < kQBuckets; i += blockDim.x) tg[i] = target[i];
    __syncthreads();
    const int64_t stride = (int64_t)gridDim.x * blockDim.x * kQRowsPerLane;
    for (int64_t base = (int64_t)blockIdx.x * blockDim.x * kQRowsPerLane + threadIdx.x; base < nrows; base += stride) {
        uint64_t k[kQRowsPerLane];
        bool v[kQRowsPerLane];
#pragma unroll
        for (int j = 0; j < kQRowsPerLane; ++j) {
            const int64_t r = base + (int64_t)j * blockDim.x;
            v[j] = r < nrows && q_valid(c, r);
            k[j] = v[j] ? order_key(q_load(c, r)) : 0;
        }
        uint32_t b[kQRowsPerLane];
#pragma unroll
        for (int j = 0; j < kQRowsPerLane; ++j) b[j] = 0;
        // bucket = number of splitters <= key: branchless binary search over the sorted LDS array
        // (its last entry is +inf, above every key), kQRowsPerLane searches interleaved.
#pragma unroll
        for (uint32_t step = kQBuckets / 2; step > 0; step >>= 1)
#pragma unroll
            for (int j = 0; j < kQRowsPerLane; ++j) b[j] += (spl[b[j] + step - 1] <= k[j]) ? step : 0u;
#pragma unroll
        for (int j = 0; j < kQRowsPerLane; ++j) {
            if (!v[j] || tg[b[j]] == kQNoTarget) continue;
            if (b[j] > 0 && spl[b[j] - 1] == k[j]) continue;
            const unsigned long long pos = atomicAdd(&cursor[b[j]], 1ull);
            cand[pos] = k[j];
        }
    }
}

__global__ void q_gather_kernel(const uint64_t* __restrict__ sorted, const int64_t* __restrict__ idx, int n,
                                double* __restrict__ out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = key_value(sorted[idx[i]]);
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
struct QBuffers {
    std::vector<void*> ptrs;
    ~QBuffers() {
        for (void* p : ptrs) (void)hipFree(p);
    }
    hipError_t alloc(void** p, size_t bytes) {
        hipError_t e = hipMalloc(p, std::max<size_t>(bytes, 16));
        if (e == hipSuccess) ptrs.push_back(*p);
        return e;
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

    // ---- 2. histogram per shard, added on the host ------------------------------------------------
    for (QShard& q : sh) {
        if (!q.nrows) continue;
        QS_HIP(ctx, hipSetDevice(dq::ctx_device(q.ctx)));
        hipStream_t s = dq::ctx_stream(q.ctx);
        QS_HIP(ctx, q.buf.alloc((void**)&q.dspl, sizeof(uint64_t) * kQBuckets));
        QS_HIP(ctx, hipMemcpyAsync(q.dspl, spl.data(), sizeof(uint64_t) * kQBuckets, hipMemcpyHostToDevice, s));
        QS_HIP(ctx, q.buf.alloc((void**)&q.dhist, sizeof(unsigned long long) * kQBuckets * 2));
        QS_HIP(ctx, hipMemsetAsync(q.dhist, 0, sizeof(unsigned long long) * kQBuckets * 2, s));
        const int64_t lanes_needed = (q.nrows + kQRowsPerLane - 1) / kQRowsPerLane;
        q.grid = (int)std::max<int64_t>(1, std::min<int64_t>((lanes_needed + kQBlock - 1) / kQBlock,
                                                             (int64_t)dq::ctx_cus(q.ctx) * 2));
        hipLaunchKernelGGL(q_hist_kernel, dim3(q.grid), dim3(kQBlock), 0, s, q.qc, q.nrows, (const uint64_t*)q.dspl,
                           q.dhist, q.dhist + kQBuckets);
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
        hipLaunchKernelGGL(q_compact_kernel, dim3(q.grid), dim3(kQBlock), 0, s, q.qc, q.nrows, (const uint64_t*)q.dspl,
                           (const uint32_t*)q.dtarget, q.dcursor, q.dcand);
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

}  // extern "C"
