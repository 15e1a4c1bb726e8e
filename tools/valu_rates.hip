// valu_rates.hip -- issue cost of the integer multiplies Philox can be built from (measurement only).
// Each kernel: every lane runs 8 independent chains of one instruction kind for ITERS rounds; the
// grid fills every SIMD with 8 waves. Prints cycles per wave-instruction per SIMD at the measured
// shader clock (from s_memtime inside the kernel).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

constexpr int ITERS = 4096;

template <int OP>
__global__ __launch_bounds__(256) void k_rate(uint32_t* out, uint32_t m, uint64_t* cyc) {
    uint32_t a[8], b[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        a[k] = threadIdx.x * 2654435761u + k;
        b[k] = a[k] ^ 0x9E3779B9u;
    }
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < ITERS; ++it) {
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            if constexpr (OP == 0) {  // v_mad_u64_u32: both halves of a 32x32 product
                const uint64_t p = (uint64_t)a[k] * m;
                a[k] = (uint32_t)p;
                b[k] ^= (uint32_t)(p >> 32);
            } else if constexpr (OP == 1) {  // v_mul_hi_u32
                a[k] = __umulhi(a[k], m) ^ b[k];
            } else if constexpr (OP == 2) {  // v_mul_lo_u32
                a[k] = a[k] * m + b[k];
            } else if constexpr (OP == 3) {  // v_mul_u32_u24 / v_mad_u32_u24
                a[k] = __umul24(a[k], m) + b[k];
            } else {  // v_xor (reference: full rate)
                a[k] = (a[k] ^ m) + b[k];
            }
        }
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    uint32_t x = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) x ^= a[k] ^ b[k];
    out[blockIdx.x * 256 + threadIdx.x] = x;
    if (threadIdx.x == 0 && blockIdx.x == 0) cyc[0] = t1 - t0;
}

template <int OP>
static void run(const char* name, int n_cu) {
    uint32_t* out;
    uint64_t* cyc;
    const int grid = n_cu * 8;  // 8 WGs x 4 waves = 32 waves per CU = 8 per SIMD
    hipMalloc(&out, 4u * 256u * grid);
    hipMalloc(&cyc, 8);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipLaunchKernelGGL(k_rate<OP>, dim3(grid), dim3(256), 0, 0, out, 0x9E3779B1u, cyc);
    hipEventRecord(e0, 0);
    hipLaunchKernelGGL(k_rate<OP>, dim3(grid), dim3(256), 0, 0, out, 0xD2511F53u, cyc);
    hipEventRecord(e1, 0);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    uint64_t c = 0;
    hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
    // wave-instructions of the measured kind per SIMD: 8 waves x ITERS x 8 chains
    const double per_simd = 8.0 * ITERS * 8;
    printf("{\"op\": \"%s\", \"ms\": %.4f, \"ns_per_wave_inst_per_simd\": %.4f, \"memtime_ticks\": %llu}\n", name, ms,
           ms * 1e6 / per_simd, (unsigned long long)c);
    hipFree(out);
    hipFree(cyc);
}

int main() {
    int n_cu = 0;
    hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, 0);
    run<0>("v_mad_u64_u32 (+1 xor)", n_cu);
    run<1>("v_mul_hi_u32 (+1 xor)", n_cu);
    run<2>("v_mul_lo_u32 (+1 add)", n_cu);
    run<3>("v_mul_u32_u24 (+1 add)", n_cu);
    run<4>("v_xor + v_add", n_cu);
    return 0;
}
