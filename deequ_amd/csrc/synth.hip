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
