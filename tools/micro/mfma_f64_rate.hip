// Microbenchmark for VERDICT r5 #6 (suite10 / N1): can v_mfma_f64_16x16x4_f64 take the fp64 moment / co-moment sums
// off the VALU? Measures (1) the MFMA f64 instruction rate alone, (2) a VALU chain alone (the XXH64-style 64-bit
// multiply-add the heavy scan is bound by), (3) both interleaved in one wave stream, the mix a fused scan would issue.
// Each MFMA of the per-row form (lane l supplies row l's x as A[l&15][l>>4] and y as B[l>>4][l&15]) yields 64 useful
// products (the 16 diagonal results, 4 rows each) of its 1024 FMAs; a Gram form over 16 features needs the features of
// one row in 16 different lanes (a transpose of the scan's row-per-lane layout).
//   hipcc -O3 --offload-arch=gfx950 mfma_f64_rate.hip -o mfma_f64_rate && ./mfma_f64_rate
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

typedef double d4 __attribute__((ext_vector_type(4)));
constexpr int REPS = 512;

template <int M, int V>  // M MFMAs and V VALU 64-bit mads per iteration, 4 independent MFMA accumulators
__global__ void __launch_bounds__(256) mix(double* out, uint32_t seed) {
    d4 acc[4] = {};
    double a = seed + threadIdx.x * 0.5, b = seed * 0.25 + threadIdx.x;
    uint64_t h[4];
    for (int i = 0; i < 4; ++i) h[i] = seed + i * 977u + threadIdx.x;
    const uint32_t c = seed * 2654435761u + 1u;
    for (int r = 0; r < REPS; ++r) {
#pragma unroll
        for (int m = 0; m < M; ++m) acc[m & 3] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[m & 3], 0, 0, 0);
#pragma unroll
        for (int v = 0; v < V; ++v) asm volatile("v_mad_u64_u32 %0, vcc, %1, %1, %0" : "+v"(h[v & 3]) : "v"(c));
    }
    double s = 0;
    for (int i = 0; i < 4; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3] + (double)h[i];
    if (s == 1.2345) out[0] = s;
}

typedef void (*kfn)(double*, uint32_t);

static float run(kfn f, double* o, int grid) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    f<<<grid, 256>>>(o, 1);
    hipDeviceSynchronize();
    hipEventRecord(e0);
    for (int i = 0; i < 5; ++i) f<<<grid, 256>>>(o, 1);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    return ms / 5;
}

int main() {
    double* o;
    hipMalloc(&o, 8);
    int cus;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    const int grid = cus * 8;  // 8 workgroups of 4 waves per CU: 8 waves per SIMD
    const double waves = grid * 4.0;
    struct { const char* name; kfn f; int m, v; } ks[] = {
        {"mfma x8", mix<8, 0>, 8, 0},         {"valu mad64 x32", mix<0, 32>, 0, 32},
        {"mfma x8 + mad64 x32", mix<8, 32>, 8, 32}, {"mfma x2 + mad64 x32", mix<2, 32>, 2, 32},
        {"mfma x1 + mad64 x32", mix<1, 32>, 1, 32},
    };
    printf("{\"cus\": %d, \"grid\": %d, \"waves\": %.0f, \"reps\": %d, \"runs\": [\n", cus, grid, waves, REPS);
    for (int i = 0; i < 5; ++i) {
        const float ms = run(ks[i].f, o, grid);
        const double mf = waves * REPS * ks[i].m, va = waves * REPS * ks[i].v;
        printf("  {\"kernel\": \"%s\", \"ms\": %.4f, \"mfma_per_s\": %.4g, \"mfma_tflops\": %.2f, "
               "\"valu_wave_insts_per_s\": %.4g, \"useful_row_products_per_s\": %.4g}%s\n",
               ks[i].name, ms, mf / (ms * 1e-3), mf * 2048.0 / (ms * 1e-3) / 1e12, va / (ms * 1e-3),
               mf * 64.0 / (ms * 1e-3), i < 4 ? "," : "");
    }
    printf("]}\n");
    return 0;
}
