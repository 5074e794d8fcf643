// Microbenchmark: XXH64 + HLL register update throughput on MI355X, to find the compute floor of
// ApproxCountDistinct in the fused scan. Standalone: hipcc -O3 --offload-arch=gfx950 hll_micro.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include "../../deequ_amd/csrc/dq_common.h"
using namespace dq;

__global__ void fill(uint64_t* v, int64_t n) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        v[i] = splitmix64(7, i);
}

template <int MODE>  // 0 = load + xor, 1 = hash + xor, 2 = hash + LDS atomics
__global__ void __launch_bounds__(256) k(const uint64_t* __restrict__ v, int64_t n, uint64_t* out) {
    __shared__ uint32_t regs[512];
    for (int i = threadIdx.x; i < 512; i += 256) regs[i] = 0;
    __syncthreads();
    uint64_t acc = 0;
    const int64_t per = 2048;
    for (int64_t t = blockIdx.x; t * per < n; t += gridDim.x) {
        const uint4* p = reinterpret_cast<const uint4*>(v + t * per) + threadIdx.x;
        uint64_t x[8];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            uint4 q = p[j * 256];
            x[2 * j] = ((uint64_t)q.y << 32) | q.x;
            x[2 * j + 1] = ((uint64_t)q.w << 32) | q.z;
        }
        if (MODE == 0) {
#pragma unroll
            for (int j = 0; j < 8; ++j) acc ^= x[j];
        } else {
            uint32_t pk[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                uint64_t h = xxh_long(x[j], SPARK_HLL_SEED);
                pk[j] = hll_index(h) | (hll_rank(h) << 16);
            }
            if (MODE == 1) {
#pragma unroll
                for (int j = 0; j < 8; ++j) acc += pk[j];
            } else {
#pragma unroll
                for (int j = 0; j < 8; ++j) atomicMax(&regs[pk[j] & 0xffff], pk[j] >> 16);
            }
        }
    }
    __syncthreads();
    if (MODE == 2) acc = regs[threadIdx.x];
    if (acc == 0x1234567) out[0] = acc;
}

int main() {
    const int64_t n = 1LL << 30;
    uint64_t *v, *o;
    hipMalloc(&v, n * 8);
    hipMalloc(&o, 8);
    fill<<<4096, 256>>>(v, n);
    hipDeviceSynchronize();
    int cus;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    for (int mode = 0; mode < 3; ++mode)
        for (int occ : {2, 4, 8}) {
            const int grid = cus * occ;
            float best = 1e9;
            for (int r = 0; r < 5; ++r) {
                hipEventRecord(a);
                if (mode == 0) k<0><<<grid, 256>>>(v, n, o);
                if (mode == 1) k<1><<<grid, 256>>>(v, n, o);
                if (mode == 2) k<2><<<grid, 256>>>(v, n, o);
                hipEventRecord(b);
                hipEventSynchronize(b);
                float ms;
                hipEventElapsedTime(&ms, a, b);
                if (ms < best) best = ms;
            }
            printf("mode %d grid %d: %.3f ms  %.1f GB/s  %.2f Gvalues/s\n", mode, grid, best, n * 8 / best / 1e6,
                   n / best / 1e6);
        }
    return 0;
}
