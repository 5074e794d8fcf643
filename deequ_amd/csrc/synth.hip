// synth.hip — on-device generators of the synthetic BASELINE inputs.
//
// Counter-based splitmix64 streams, so every rank generates its own shard in HBM and the CPU
// oracle (oracle/dq_oracle.c) regenerates identical values. Floating-point formulas use explicit
// round-to-nearest operations (no FMA contraction) so host and device produce the same bits.
#include <hip/hip_runtime.h>

#include "dq_common.h"
#include "dq_internal.h"

namespace dq {

constexpr uint64_t kSynthCorrNoise = 0x5A5A5A5A5A5A5A5AULL;

__device__ __forceinline__ double sum12_u48(uint64_t seed, uint64_t row) {
    double s = 0.0;
#pragma unroll
    for (int j = 0; j < 12; ++j) {
        const uint64_t h = splitmix64(seed ^ (0xA5A5A5A5ULL * (uint64_t)(j + 1)), row);
        s = __dadd_rn(s, (double)(h >> 16) * 0x1.0p-48);
    }
    return s;
}

__global__ void synth_column_kernel(int kind, uint64_t seed, int64_t row0, int64_t nrows, void* out) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nrows; i += stride) {
        const uint64_t row = (uint64_t)(row0 + i);
        const uint64_t h = splitmix64(seed, row);
        switch (kind) {
            case DQ_SYNTH_DYADIC: {
                const int64_t k = (int64_t)(h % 513ULL) - 256;
                static_cast<double*>(out)[i] = (double)k * 0x1.0p-8;
                break;
            }
            case DQ_SYNTH_UNIFORM:
                static_cast<double*>(out)[i] = (double)(h >> 11) * 0x1.0p-53;
                break;
            case DQ_SYNTH_NORMAL: {
                const double t = __dsub_rn(sum12_u48(seed, row), 6.0);
                static_cast<double*>(out)[i] = __dadd_rn(100.0, __dmul_rn(15.0, t));
                break;
            }
            case DQ_SYNTH_GAUSS01:
                static_cast<double*>(out)[i] = __dsub_rn(sum12_u48(seed, row), 6.0);
                break;
            case DQ_SYNTH_GAUSS_CORR: {
                // y = 0.6 x + 0.8 e: x = GAUSS01(seed), e = GAUSS01(seed ^ kCorrNoise) -> corr(x, y) ~ 0.6
                const double x = __dsub_rn(sum12_u48(seed, row), 6.0);
                const double e = __dsub_rn(sum12_u48(seed ^ kSynthCorrNoise, row), 6.0);
                static_cast<double*>(out)[i] = __dadd_rn(__dmul_rn(0.6, x), __dmul_rn(0.8, e));
                break;
            }
            case DQ_SYNTH_INT32R:
                static_cast<int64_t*>(out)[i] = (int64_t)(int32_t)(uint32_t)(h >> 32);
                break;
            case DQ_SYNTH_KEY30:
                static_cast<int64_t*>(out)[i] = (int64_t)(h & ((1ULL << 30) - 1));
                break;
            default:
                break;
        }
    }
}

// One 64-row validity word per lane: bit r valid iff splitmix64(seed, row) % 1000 >= permille.
__global__ void synth_validity_kernel(uint64_t seed, int64_t row0, int64_t nrows, int permille, uint8_t* out) {
    const int64_t nwords = (nrows + 63) / 64;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t w = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; w < nwords; w += stride) {
        uint64_t bits = 0;
        for (int b = 0; b < 64; ++b) {
            const int64_t i = w * 64 + b;
            if (i >= nrows) break;
            const uint64_t h = splitmix64(seed, (uint64_t)(row0 + i));
            if ((int)(h % 1000ULL) >= permille) bits |= 1ULL << b;
        }
        const int64_t nbytes = (nrows + 7) / 8;
        for (int k = 0; k < 8; ++k)
            if (w * 8 + k < nbytes) out[w * 8 + k] = (uint8_t)(bits >> (8 * k));
    }
}

__global__ void synth_freq_keys_kernel(int64_t total, int64_t distinct, int64_t row0, int64_t nrows, int64_t* out) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    const uint64_t half = (uint64_t)(distinct / 2 > 0 ? distinct / 2 : 1);
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nrows; i += stride) {
        const uint64_t r = (uint64_t)(row0 + i);
        const uint64_t j = (uint64_t)(((unsigned __int128)r * 0x9E3779B1ULL) % (uint64_t)total);
        const uint64_t k = j < (uint64_t)distinct ? j : (j - (uint64_t)distinct) % half;
        uint64_t z = k;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
        out[i] = (int64_t)(z ^ (z >> 31));
    }
}

// ---- UTF-8 string columns of config C5: categories, numeric-looking strings, free text ----------
__device__ __forceinline__ int put_uint(char* out, int at, uint64_t v, int min_digits) {
    char tmp[20];
    int n = 0;
    do {
        tmp[n++] = (char)('0' + v % 10);
        v /= 10;
    } while (v);
    while (n < min_digits) tmp[n++] = '0';
    for (int k = 0; k < n; ++k)
        if (out) out[at + k] = tmp[n - 1 - k];
    return at + n;
}

// Writes the row's string at out (when out != nullptr) and returns its length in bytes.
__device__ int synth_string(int kind, uint64_t seed, uint64_t row, char* out) {
    const uint64_t h = splitmix64(seed, row);
    int n = 0;
    switch (kind) {
        case DQ_SYNTH_STR_CAT50:  // "cat_<0..49>"
            if (out) { out[0] = 'c'; out[1] = 'a'; out[2] = 't'; out[3] = '_'; }
            return put_uint(out, 4, h % 50, 1);
        case DQ_SYNTH_STR_BOOL: {  // "true" / "false"
            const bool t = (h >> 7) & 1;
            const char* w = t ? "true" : "false";
            const int len = t ? 4 : 5;
            for (int k = 0; k < len; ++k)
                if (out) out[k] = w[k];
            return len;
        }
        case DQ_SYNTH_STR_CAT100:  // "v<00..99>"
            if (out) out[0] = 'v';
            return put_uint(out, 1, h % 100, 2);
        case DQ_SYNTH_STR_INT: {  // integer in [-1e6, 1e6)
            const int64_t v = (int64_t)(h % 2000000ULL) - 1000000;
            if (v < 0 && out) out[0] = '-';
            return put_uint(out, v < 0 ? 1 : 0, (uint64_t)(v < 0 ? -v : v), 1);
        }
        case DQ_SYNTH_STR_DEC: {  // "<0..999>.<00..99>"
            const uint64_t c = h % 100000ULL;
            n = put_uint(out, 0, c / 100, 1);
            if (out) out[n] = '.';
            return put_uint(out, n + 1, c % 100, 2);
        }
        case DQ_SYNTH_STR_MIXNUM: {  // 70 %: integer in [-5000, 5000); 30 %: thousandths in (-1000, 1000)
            const bool integral = (h % 10ULL) < 7;
            const int64_t v = (int64_t)((h >> 8) % 10000ULL) - 5000;
            if (integral) {
                if (v < 0 && out) out[0] = '-';
                return put_uint(out, v < 0 ? 1 : 0, (uint64_t)(v < 0 ? -v : v), 1);
            }
            const int64_t m = (int64_t)((h >> 24) % 1999999ULL) - 999999;  // value m / 1000
            const uint64_t a = (uint64_t)(m < 0 ? -m : m);
            if (m < 0 && out) out[0] = '-';
            n = put_uint(out, m < 0 ? 1 : 0, a / 1000, 1);
            if (out) out[n] = '.';
            return put_uint(out, n + 1, a % 1000, 3);
        }
        default: {  // DQ_SYNTH_STR_TEXT: 1-20 characters of [a-z0-9 ]
            const int len = 1 + (int)(h % 20ULL);
            uint64_t z = h;
            for (int k = 0; k < len; ++k) {
                if ((k & 7) == 0) z = splitmix64(seed ^ 0x7E77ULL, row * 4 + (uint64_t)(k >> 3));
                const int c = (int)((z & 0xFF) % 37);
                z >>= 8;
                if (out) out[k] = c < 26 ? (char)('a' + c) : (c < 36 ? (char)('0' + c - 26) : ' ');
            }
            return len;
        }
    }
}

__global__ void synth_string_lengths_kernel(int kind, uint64_t seed, int64_t row0, int64_t nrows, int32_t* lens) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nrows; i += stride)
        lens[i] = synth_string(kind, seed, (uint64_t)(row0 + i), nullptr);
}

__global__ void synth_string_bytes_kernel(int kind, uint64_t seed, int64_t row0, int64_t nrows,
                                          const int32_t* __restrict__ offsets, char* __restrict__ bytes) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nrows; i += stride)
        synth_string(kind, seed, (uint64_t)(row0 + i), bytes + offsets[i]);
}

void launch_synth_string_lengths(int kind, uint64_t seed, int64_t row0, int64_t nrows, int32_t* lens, hipStream_t s) {
    int64_t blocks = (nrows + 255) / 256;
    if (blocks > 65536) blocks = 65536;
    if (blocks < 1) blocks = 1;
    hipLaunchKernelGGL(synth_string_lengths_kernel, dim3((unsigned)blocks), dim3(256), 0, s, kind, seed, row0, nrows, lens);
}

void launch_synth_string_bytes(int kind, uint64_t seed, int64_t row0, int64_t nrows, const int32_t* offsets, void* bytes,
                               hipStream_t s) {
    int64_t blocks = (nrows + 255) / 256;
    if (blocks > 65536) blocks = 65536;
    if (blocks < 1) blocks = 1;
    hipLaunchKernelGGL(synth_string_bytes_kernel, dim3((unsigned)blocks), dim3(256), 0, s, kind, seed, row0, nrows,
                       offsets, (char*)bytes);
}

void launch_synth_freq_keys(int64_t total, int64_t distinct, int64_t row0, int64_t nrows, int64_t* out, hipStream_t s) {
    int64_t blocks = (nrows + 255) / 256;
    if (blocks > 65536) blocks = 65536;
    if (blocks < 1) blocks = 1;
    hipLaunchKernelGGL(synth_freq_keys_kernel, dim3((unsigned)blocks), dim3(256), 0, s, total, distinct, row0, nrows, out);
}

void launch_synth_column(int kind, uint64_t seed, int64_t row0, int64_t nrows, void* out, hipStream_t s) {
    int64_t blocks = (nrows + 255) / 256;
    if (blocks > 65536) blocks = 65536;
    if (blocks < 1) blocks = 1;
    hipLaunchKernelGGL(synth_column_kernel, dim3((unsigned)blocks), dim3(256), 0, s, kind, seed, row0, nrows, out);
}

void launch_synth_validity(uint64_t seed, int64_t row0, int64_t nrows, int permille, uint8_t* out, hipStream_t s) {
    int64_t words = (nrows + 63) / 64;
    int64_t blocks = (words + 255) / 256;
    if (blocks > 65536) blocks = 65536;
    if (blocks < 1) blocks = 1;
    hipLaunchKernelGGL(synth_validity_kernel, dim3((unsigned)blocks), dim3(256), 0, s, seed, row0, nrows, permille, out);
}

}  // namespace dq
