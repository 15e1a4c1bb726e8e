// Round 6 probe (measurement only): DPP row_shr / row_bcast semantics on gfx950 for the MT map scan --
// what a lane with no source reads, and the scan of k_mt_coop against a serial CPU composition.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>

constexpr uint32_t ID = 36u;
__host__ __device__ inline uint32_t then_plain(uint32_t f, uint32_t g) {
    uint32_t h = 0;
    for (int s = 0; s < 3; ++s) { uint32_t fs = (f >> (2 * s)) & 3u; h |= ((g >> (2 * fs)) & 3u) << (2 * s); }
    return h;
}
__device__ inline uint32_t then_x(uint32_t fx, uint32_t gx) { return then_plain(fx ^ ID, gx ^ ID) ^ ID; }

__global__ void probe(const uint32_t* in, uint32_t* out_raw, uint32_t* out_scan) {
    const uint32_t l = threadIdx.x;
    uint32_t x = in[l];
    out_raw[0 * 64 + l] = (uint32_t)__builtin_amdgcn_update_dpp(777, (int)(l + 1000), 0x111, 0xF, 0xF, false);
    out_raw[1 * 64 + l] = (uint32_t)__builtin_amdgcn_update_dpp(777, (int)(l + 1000), 0x142, 0xA, 0xF, false);
    out_raw[2 * 64 + l] = (uint32_t)__builtin_amdgcn_update_dpp(777, (int)(l + 1000), 0x143, 0xC, 0xF, false);
    out_raw[3 * 64 + l] = (uint32_t)__builtin_amdgcn_update_dpp(777, (int)(l + 1000), 0x138, 0xF, 0xF, false);
    x = then_x((uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xF, 0xF, false), x);
    x = then_x((uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xF, 0xF, false), x);
    x = then_x((uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xF, 0xF, false), x);
    x = then_x((uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xF, 0xF, false), x);
    x = then_x((uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xA, 0xF, false), x);
    x = then_x((uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xC, 0xF, false), x);
    out_scan[l] = x;
}

int main() {
    uint32_t h_in[64], h_raw[256], h_scan[64];
    srand(5);
    for (int l = 0; l < 64; ++l) h_in[l] = (((rand() & 7) ? 1u : 0u) | (2u << 2)) ^ ID;
    uint32_t *d_in, *d_raw, *d_scan;
    hipMalloc(&d_in, 256); hipMalloc(&d_raw, 1024); hipMalloc(&d_scan, 256);
    hipMemcpy(d_in, h_in, 256, hipMemcpyHostToDevice);
    probe<<<1, 64>>>(d_in, d_raw, d_scan);
    hipMemcpy(h_raw, d_raw, 1024, hipMemcpyDeviceToHost);
    hipMemcpy(h_scan, d_scan, 256, hipMemcpyDeviceToHost);
    const char* names[4] = {"row_shr1 old=777 bc=0", "row_bcast15 rm=0xA", "row_bcast31 rm=0xC", "wave_shr1 (0x138) old=777"};
    for (int k = 0; k < 4; ++k) {
        printf("%s:", names[k]);
        for (int l = 0; l < 64; ++l) printf(" %u", h_raw[k * 64 + l]);
        printf("\n");
    }
    // serial reference: prefix maps (plain form), f_0 first
    uint32_t acc = ID;
    int bad = 0;
    for (int l = 0; l < 64; ++l) {
        acc = then_plain(acc, h_in[l] ^ ID);
        if ((h_scan[l] ^ ID) != acc) { if (bad < 8) printf("scan lane %d: got %u want %u\n", l, h_scan[l] ^ ID, acc); ++bad; }
    }
    printf("scan mismatches: %d\n", bad);
    return 0;
}
