// pbn_sync.hip -- synchronous update with optional perturbation.
//
// Reference: Graph.synch_step (gym_PBN/envs/bittner/base.py:286-303): with
// perturbations on, each node is flagged with probability p (base.py:191,288); if
// any flag is set the flagged nodes are flipped and nothing else happens
// (:289-295), otherwise -- and always when perturbations are off -- every node is
// stepped from the same pre-step snapshot (:297-303). (At HEAD the method indexes
// the snapshot tuple by gene ID and cannot run; this is its intended semantics.)
// Truth-table networks use the same scheme with Node.compute_next_value
// (the commented-out synchronous PBN.step, common/pbn.py:135-137).
//
// Each node draws its own random(): nodes 2m and 2m+1 share one Philox call
// (ctr {step_lo, m | step_hi << 16, gid, STREAM_SYNC}; words (0,1) and (2,3)).
// Two LDS planes per lane: the snapshot and the next state, built one dword
// (32 nodes) at a time in a register and written once.
#include <hip/hip_runtime.h>

#include "pbn_device.hpp"
#include "pbn_params.hpp"

namespace pbn {

template <int W, int KIND>
__global__ __launch_bounds__(BLOCK) void k_sync(SyncArgs a) {
    extern __shared__ __align__(16) uint8_t lds[];
    stage_image(reinterpret_cast<const uint4*>(a.img), a.L.bytes / 16, reinterpret_cast<uint4*>(lds));
    const uint32_t N = (uint32_t)a.L.n_nodes;
    uint32_t* gap = reinterpret_cast<uint32_t*>(lds + a.off_gap);
    if (a.gap_thr)
        for (uint32_t k = threadIdx.x; k < N; k += BLOCK) gap[k] = a.gap_thr[k];
    __syncthreads();
    const PlaneT<BLOCK> P0{reinterpret_cast<uint32_t*>(lds + a.off_planes) + threadIdx.x};
    const PlaneT<BLOCK> P1{reinterpret_cast<uint32_t*>(lds + a.off_planes + 8u * W * BLOCK) + threadIdx.x};
    const uint64_t stride = (uint64_t)gridDim.x * BLOCK;
    for (uint64_t e = (uint64_t)blockIdx.x * BLOCK + threadIdx.x; e < a.B; e += stride) {
        uint64_t s[W];
        load_state<W>(a.state + e * W, s);
        to_plane<W>(P0, s);
        const uint64_t g = a.env_base + e;
        for (uint32_t t = 0; t < a.T; ++t) {
            const uint64_t st = a.step_base + t;
            bool flipped = false;
            if (a.gap_thr)
                bernoulli_positions(a.seed, (uint32_t)st, STREAM_SYNC_PERT, g, gap, N, a.gap_inv_log2, [&](uint32_t pos) {
                    const uint32_t d = pos >> 5;
                    P0.put(d, P0.get(d) ^ (1u << (pos & 31u)));
                    flipped = true;
                });
            if (flipped) continue;  // base.py:289-295: a perturbation replaces the update
            const uint32_t c1hi = (uint32_t)(st >> 32) << 16;
            uint32_t w[4];
            for (uint32_t d = 0; d < 2u * W; ++d) {
                const uint32_t self = P0.get(d);
                uint32_t acc = 0;
                for (uint32_t b = 0; b < 32u; ++b) {
                    const uint32_t i = d * 32u + b;
                    if (i >= N) break;
                    if ((i & 1u) == 0) philox_draw(a.seed, (uint32_t)st, (i >> 1) | c1hi, g, STREAM_SYNC, w);
                    const uint64_t k53 = (i & 1u) ? k53_of(w[2], w[3]) : k53_of(w[0], w[1]);
                    uint32_t y;
                    if constexpr (KIND == KIND_PREDICTOR_MIX)
                        y = predictor_eval_lds(P0, i, self, k53, lds, a.L);
                    else
                        y = table_eval_lds(P0, i, k53, lds, a.L);
                    acc |= y << b;
                }
                P1.put(d, acc);
            }
            for (uint32_t d = 0; d < 2u * W; ++d) P0.put(d, P1.get(d));
        }
        from_plane<W>(P0, s);
        store_state<W>(a.state + e * W, s);
    }
}

template <int KIND>
static void* sync_fn(int W) {
    switch (W) {
        case 1: return (void*)k_sync<1, KIND>;
        case 2: return (void*)k_sync<2, KIND>;
        case 3: return (void*)k_sync<3, KIND>;
        case 4: return (void*)k_sync<4, KIND>;
        case 5: return (void*)k_sync<5, KIND>;
        case 6: return (void*)k_sync<6, KIND>;
        case 7: return (void*)k_sync<7, KIND>;
        case 8: return (void*)k_sync<8, KIND>;
    }
    return nullptr;
}

uint32_t sync_layout(int W, uint32_t image_bytes, int n_nodes, SyncArgs* a) {
    a->off_planes = image_bytes;
    a->off_gap = ((a->off_planes + 16u * (uint32_t)W * BLOCK) + 15u) & ~15u;
    return ((a->off_gap + 4u * (uint32_t)n_nodes) + 15u) & ~15u;
}

int launch_sync(int W, const SyncArgs& a, int grid, void* stream) {
    void* fn = a.L.kind == KIND_PREDICTOR_MIX ? sync_fn<KIND_PREDICTOR_MIX>(W) : sync_fn<KIND_PROB_TABLE>(W);
    if (!fn) return (int)hipErrorInvalidValue;
    SyncArgs c = a;
    if (c.lds_bytes > 64u * 1024u) {
        hipError_t e = hipFuncSetAttribute((const void*)fn, hipFuncAttributeMaxDynamicSharedMemorySize,
                                           (int)c.lds_bytes);
        if (e != hipSuccess) return (int)e;
    }
    void* kargs[] = {&c};
    return (int)hipLaunchKernel(fn, dim3((unsigned)grid), dim3(BLOCK), kargs, c.lds_bytes, (hipStream_t)stream);
}

}  // namespace pbn
