// membench.hip -- memory floor for the step-mode traffic pattern (calibration only, not product).
// Per env: read W=4 u64 (two 16-B loads), write back (all, or a fraction f of 16-B pairs),
// no compute. Also an empty kernel for the launch-to-launch floor. hipEvent timing over K launches.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <stdlib.h>

__global__ void k_copy(uint64_t* s, uint64_t B, int write_pct) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t e = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; e < B; e += stride) {
        ulonglong2* q = reinterpret_cast<ulonglong2*>(s + 4 * e);
        ulonglong2 a = q[0], b = q[1];
        a.x ^= 1;  // touch
        uint32_t h = (uint32_t)(e * 2654435761u) % 100u;
        if ((int)h < write_pct) { q[0] = a; q[1] = b; }
    }
}
__global__ void k_empty() {}

int main(int argc, char** argv) {
    uint64_t B = argc > 1 ? strtoull(argv[1], 0, 10) : (1ull << 20);
    const int K = 200;
    uint64_t* s;
    hipMalloc(&s, 32 * B);
    hipMemset(s, 0, 32 * B);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    int grids[] = {1024, 2048, 4096, (int)((B + 255) / 256)};
    int pcts[] = {100, 45, 0};
    for (int gi = 0; gi < 4; gi++)
        for (int pi = 0; pi < 3; pi++) {
            for (int w = 0; w < 10; w++) k_copy<<<grids[gi], 256>>>(s, B, pcts[pi]);
            hipEventRecord(e0);
            for (int k = 0; k < K; k++) k_copy<<<grids[gi], 256>>>(s, B, pcts[pi]);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            double us = ms * 1e3 / K;
            double bytes = 32.0 * B + 32.0 * B * pcts[pi] / 100.0;
            printf("copy B=%llu grid=%d write%%=%d: %.2f us/launch  %.0f GB/s\n", (unsigned long long)B, grids[gi],
                   pcts[pi], us, bytes / us / 1e3);
        }
    for (int w = 0; w < 10; w++) k_empty<<<2048, 256>>>();
    hipEventRecord(e0);
    for (int k = 0; k < K; k++) k_empty<<<2048, 256>>>();
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    printf("empty 2048x256: %.2f us/launch\n", ms * 1e3 / K);
    return 0;
}
