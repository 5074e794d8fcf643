// Microbenchmark: VALU issue rates of the instructions XXH64 / HLL / Welford compile to on gfx950,
// so the suite10 kernels can be priced against a measured compute floor.
// Each lane runs 8 independent dependency chains of one instruction, unrolled; the grid fills the
// chip several times over. Reports lane-instructions per second per instruction kind.
//   hipcc -O3 --offload-arch=gfx950 valu_rates.hip -o valu_rates && ./valu_rates
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

#define CH 8
#define REPS 256

#define OP1(name, asmstr)                                                                        \
    __global__ void __launch_bounds__(256) name(uint32_t* out, uint32_t seed) {                  \
        uint32_t a[CH], b = seed * 7u + threadIdx.x;                                             \
        for (int i = 0; i < CH; ++i) a[i] = seed + i * 13u + threadIdx.x;                        \
        for (int r = 0; r < REPS; ++r) {                                                          \
            _Pragma("unroll") for (int i = 0; i < CH; ++i) asm volatile(asmstr : "+v"(a[i]) : "v"(b)); \
        }                                                                                         \
        uint32_t s = 0;                                                                           \
        for (int i = 0; i < CH; ++i) s ^= a[i];                                                   \
        if (s == 0x12345u) out[0] = s;                                                            \
    }

OP1(k_add, "v_add_u32 %0, %0, %1")
OP1(k_xor, "v_xor_b32 %0, %0, %1")
OP1(k_mullo, "v_mul_lo_u32 %0, %0, %1")
OP1(k_mulhi, "v_mul_hi_u32 %0, %0, %1")
OP1(k_alignbit, "v_alignbit_b32 %0, %0, %1, 7")
OP1(k_ffbh, "v_ffbh_u32 %0, %0")

// 64-bit destination ops
#define OP2(name, asmstr)                                                                        \
    __global__ void __launch_bounds__(256) name(uint32_t* out, uint32_t seed) {                  \
        uint64_t a[CH];                                                                           \
        uint32_t b = seed * 7u + threadIdx.x;                                                     \
        for (int i = 0; i < CH; ++i) a[i] = seed + i * 13u + threadIdx.x;                        \
        for (int r = 0; r < REPS; ++r) {                                                          \
            _Pragma("unroll") for (int i = 0; i < CH; ++i) asm volatile(asmstr : "+v"(a[i]) : "v"(b)); \
        }                                                                                         \
        uint64_t s = 0;                                                                           \
        for (int i = 0; i < CH; ++i) s ^= a[i];                                                   \
        if (s == 0x12345u) out[0] = (uint32_t)s;                                                  \
    }

OP2(k_mad64, "v_mad_u64_u32 %0, vcc, %1, %1, %0")
OP2(k_lshl64, "v_lshlrev_b64 %0, 3, %0")
OP2(k_fma64, "v_fma_f64 %0, %0, %0, %0")
OP2(k_add64f, "v_add_f64 %0, %0, %0")
OP2(k_min64f, "v_min_f64 %0, %0, %0")
OP2(k_cvt64, "v_cvt_f64_i32 %0, %1")

typedef void (*kfn)(uint32_t*, uint32_t);

int main() {
    uint32_t* o;
    hipMalloc(&o, 8);
    int cus;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    int clk = 0;
    hipDeviceGetAttribute(&clk, hipDeviceAttributeClockRate, 0);
    printf("CUs %d, clock %d kHz -> lane-slot peak %.3e /s\n", cus, clk, (double)cus * 64 * clk * 1e3);
    struct { const char* name; kfn f; } ks[] = {
        {"v_add_u32", k_add}, {"v_xor_b32", k_xor}, {"v_mul_lo_u32", k_mullo}, {"v_mul_hi_u32", k_mulhi},
        {"v_alignbit_b32", k_alignbit}, {"v_ffbh_u32", k_ffbh}, {"v_mad_u64_u32", k_mad64},
        {"v_lshlrev_b64", k_lshl64}, {"v_fma_f64", k_fma64}, {"v_add_f64", k_add64f}, {"v_min_f64", k_min64f},
        {"v_cvt_f64_i32", k_cvt64}};
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    const int grid = cus * 32;
    for (auto& k : ks) {
        float best = 1e9;
        for (int r = 0; r < 4; ++r) {
            hipEventRecord(a);
            hipLaunchKernelGGL(k.f, dim3(grid), dim3(256), 0, 0, o, (uint32_t)r);
            hipEventRecord(b);
            hipEventSynchronize(b);
            float ms;
            hipEventElapsedTime(&ms, a, b);
            if (r > 0 && ms < best) best = ms;
        }
        const double lane_ops = (double)grid * 256 * CH * REPS;
        printf("%-16s %8.3f ms  %.3e lane-ops/s  (%.2f of 1/clk/lane)\n", k.name, best, lane_ops / (best * 1e-3),
               lane_ops / (best * 1e-3) / ((double)cus * 64 * clk * 1e3));
    }
    return 0;
}
