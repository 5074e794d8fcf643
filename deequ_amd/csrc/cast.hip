// cast.hip — Spark Cast of a STRING column to LONG / DOUBLE on gfx950 (one lane per row).
//
// Replaces ColumnProfiler.castColumn (M/profiles/ColumnProfiler.scala:346-355, called from
// castNumericStringColumns :427-445 for columns whose DataType pass inferred Integral / Fractional):
// `data(name).cast(LongType | DoubleType)`. The parsers are the device restatements in dq_parse.h;
// NULL rows and strings that do not parse become NULL. HBM-bound byte work: the offsets and bytes are
// read once, 8 B of value + 1 bit of validity written per row; validity words are assembled with a
// wave ballot (64 rows per wave = one 64-bit word, LSB-first).
#include <hip/hip_runtime.h>

#include <string.h>

#include <algorithm>
#include <vector>

#include "dq_common.h"
#include "dq_internal.h"
#include "dq_parse.h"

namespace dq {

constexpr int kCastBlock = 256;

__global__ void __launch_bounds__(kCastBlock)
cast_strings_kernel(const uint8_t* __restrict__ bytes, const int32_t* __restrict__ offsets,
                    const uint64_t* __restrict__ validity, int64_t nrows, int to_double, void* __restrict__ values_out,
                    uint64_t* __restrict__ validity_out, unsigned int* __restrict__ slow_flag) {
    const int64_t stride = (int64_t)gridDim.x * kCastBlock;
    for (int64_t base = (int64_t)blockIdx.x * kCastBlock; base < nrows; base += stride) {
        const int64_t r = base + threadIdx.x;
        bool ok = false;
        if (r < nrows && (validity == nullptr || ((validity[r >> 6] >> (r & 63)) & 1ull))) {
            const int32_t o = offsets[r];
            const int len = offsets[r + 1] - o;
            const uint8_t* s = bytes + o;
            if (to_double) {
                double d = 0.0;
                bool slow = false;
                ok = java_parse_double(s, len, d, slow);
                if (slow) atomicOr(slow_flag, 1u);
                static_cast<double*>(values_out)[r] = ok ? d : 0.0;
            } else {
                int64_t v = 0;
                ok = spark_string_to_long(s, len, v);
                static_cast<int64_t*>(values_out)[r] = ok ? v : 0;
            }
        } else if (r < nrows) {
            if (to_double) static_cast<double*>(values_out)[r] = 0.0;
            else static_cast<int64_t*>(values_out)[r] = 0;
        }
        const unsigned long long ball = __ballot(ok);
        if ((threadIdx.x & 63) == 0 && r < nrows) validity_out[r >> 6] = ball;
    }
}

hipStream_t ctx_stream(dq_ctx* ctx);
int ctx_device(dq_ctx* ctx);
int ctx_fail(dq_ctx* ctx, int code, const char* msg);
int ctx_cus(dq_ctx* ctx);

}  // namespace dq

namespace {
struct CBuffers {
    std::vector<void*> ptrs;
    ~CBuffers() {
        for (void* p : ptrs) (void)hipFree(p);
    }
    hipError_t alloc(void** p, size_t bytes) {
        hipError_t e = hipMalloc(p, std::max<size_t>(bytes, 16));
        if (e == hipSuccess) ptrs.push_back(*p);
        return e;
    }
};
}  // namespace

#define CA_HIP(ctx, expr)                                                                         \
    do {                                                                                          \
        hipError_t e_ = (expr);                                                                   \
        if (e_ != hipSuccess) return dq::ctx_fail((ctx), DQ_ERR_DEVICE, hipGetErrorString(e_));   \
    } while (0)

extern "C" {

int dq_cast_strings(dq_ctx* ctx, const dq_column* column, int64_t nrows, int32_t to_type, void* values_dev,
                    uint8_t* validity_dev) {
    if (!ctx || !column || nrows < 0 || column->length != nrows || (nrows > 0 && (!values_dev || !validity_dev)))
        return dq::ctx_fail(ctx, DQ_ERR_INVALID_ARGUMENT, "dq_cast_strings: invalid arguments");
    if (column->spark_type != DQ_TYPE_STRING || !column->offsets)
        return dq::ctx_fail(ctx, DQ_ERR_UNSUPPORTED, "dq_cast_strings: column is not a string column");
    if (to_type != DQ_TYPE_LONG && to_type != DQ_TYPE_DOUBLE)
        return dq::ctx_fail(ctx, DQ_ERR_UNSUPPORTED, "dq_cast_strings: target type must be LONG or DOUBLE");
    if (((uintptr_t)values_dev & 7) || ((uintptr_t)validity_dev & 7))
        return dq::ctx_fail(ctx, DQ_ERR_ALIGNMENT, "dq_cast_strings: output buffers must be 8-B aligned");
    if (nrows == 0) return DQ_OK;
    CA_HIP(ctx, hipSetDevice(dq::ctx_device(ctx)));
    hipStream_t s = dq::ctx_stream(ctx);
    CBuffers buf;
    const uint8_t* bytes = (const uint8_t*)column->values;
    const int32_t* offs = column->offsets;
    const uint64_t* valid = (const uint64_t*)column->validity;
    if (!(column->flags & DQ_COL_DEVICE)) {
        const int32_t total = column->offsets[nrows];
        void *b = nullptr, *o = nullptr, *m = nullptr;
        CA_HIP(ctx, buf.alloc(&b, (size_t)total + 16));
        CA_HIP(ctx, buf.alloc(&o, sizeof(int32_t) * (size_t)(nrows + 1)));
        if (total > 0) CA_HIP(ctx, hipMemcpyAsync(b, column->values, (size_t)total, hipMemcpyHostToDevice, s));
        CA_HIP(ctx, hipMemcpyAsync(o, column->offsets, sizeof(int32_t) * (size_t)(nrows + 1), hipMemcpyHostToDevice, s));
        if (column->validity) {
            const size_t bb = (size_t)(nrows + 63) / 64 * 8;
            CA_HIP(ctx, buf.alloc(&m, bb));
            CA_HIP(ctx, hipMemsetAsync(m, 0, bb, s));
            CA_HIP(ctx, hipMemcpyAsync(m, column->validity, (size_t)(nrows + 7) / 8, hipMemcpyHostToDevice, s));
        }
        bytes = (const uint8_t*)b;
        offs = (const int32_t*)o;
        valid = (const uint64_t*)m;
    }
    unsigned int* dslow = nullptr;
    CA_HIP(ctx, buf.alloc((void**)&dslow, sizeof(unsigned int)));
    CA_HIP(ctx, hipMemsetAsync(dslow, 0, sizeof(unsigned int), s));
    const int64_t blocks = (nrows + dq::kCastBlock - 1) / dq::kCastBlock;
    const int grid = (int)std::max<int64_t>(1, std::min<int64_t>(blocks, (int64_t)dq::ctx_cus(ctx) * 16));
    hipLaunchKernelGGL(dq::cast_strings_kernel, dim3(grid), dim3(dq::kCastBlock), 0, s, bytes, offs, valid, nrows,
                       to_type == DQ_TYPE_DOUBLE ? 1 : 0, values_dev, (uint64_t*)validity_dev, dslow);
    CA_HIP(ctx, hipGetLastError());
    unsigned int slow = 0;
    CA_HIP(ctx, hipMemcpyAsync(&slow, dslow, sizeof(slow), hipMemcpyDeviceToHost, s));
    CA_HIP(ctx, hipStreamSynchronize(s));
    if (slow)
        return dq::ctx_fail(ctx, DQ_ERR_UNSUPPORTED,
                            "dq_cast_strings: a value needs the arbitrary-precision path of Double.parseDouble "
                            "(hexadecimal literal, or > 19 significant digits on a rounding boundary)");
    return DQ_OK;
}

}  // extern "C"
