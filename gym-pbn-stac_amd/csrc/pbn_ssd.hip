// pbn_ssd.hip -- steady-state-distribution histogram.
//
// Reference: compute_ssd_hist / _ssd_run (gym_PBN/utils/eval.py:20-103): for each
// of R resets, `iters` times: record the bucket of the target genes' values
// (first target = most significant bit, the _state_to_idx convention of
// pbn_target.py:388-391), flip every node independently with probability p
// (np.random.rand(N) < p, eval.py:92-95), then one transition (env.step(0)).
// Here every env of the batch is one "reset"; all run in parallel.
//
// Flips: instead of N Bernoulli draws per iteration, the positions of the flipped
// nodes are generated as successive geometric gaps, P(gap >= k) = (1-p)^k, from
// a host-built table of 32-bit thresholds T_k (gap = #{k >= 1 : u < T_k}, a binary
// search in LDS) -- the same Bernoulli(p) process, ~Np + 1 draws per iteration.
// The bucket is updated incrementally on every change of a target node; counts
// go to an LDS histogram in run-length form (one LDS atomic per bucket change).
#include <hip/hip_runtime.h>

#include "pbn_device.hpp"
#include "pbn_params.hpp"

namespace pbn {

template <int W, int KIND>
__global__ __launch_bounds__(BLOCK) void k_ssd(SSDArgs a) {
    extern __shared__ __align__(16) uint8_t lds[];
    stage_image(reinterpret_cast<const uint4*>(a.img), a.L.bytes / 16, reinterpret_cast<uint4*>(lds));
    const uint32_t N = (uint32_t)a.L.n_nodes;
    const uint32_t nb = 1u << a.n_targets;
    uint32_t* gap = reinterpret_cast<uint32_t*>(lds + a.off_gap);      // T_1..T_N at gap[0..N-1]
    int16_t* tbit = reinterpret_cast<int16_t*>(lds + a.off_tbit);     // bucket bit of node i, or -1
    uint16_t* targets = reinterpret_cast<uint16_t*>(lds + a.off_targets);
    uint32_t* hist = reinterpret_cast<uint32_t*>(lds + a.off_hist);
    for (uint32_t k = threadIdx.x; k < N; k += BLOCK) {
        gap[k] = a.gap_thr ? a.gap_thr[k] : 0xFFFFFFFFu;
        tbit[k] = -1;
    }
    for (uint32_t k = threadIdx.x; k < nb; k += BLOCK) hist[k] = 0;
    __syncthreads();
    for (uint32_t j = threadIdx.x; j < (uint32_t)a.n_targets; j += BLOCK) {
        targets[j] = (uint16_t)a.targets[j];
        tbit[a.targets[j]] = (int16_t)(a.n_targets - 1 - (int)j);
    }
    __syncthreads();
    const PlaneT<BLOCK> P{reinterpret_cast<uint32_t*>(lds + a.off_planes) + threadIdx.x};
    const uint64_t stride = (uint64_t)gridDim.x * BLOCK;
    for (uint64_t e = (uint64_t)blockIdx.x * BLOCK + threadIdx.x; e < a.B; e += stride) {
        uint64_t s[W];
        load_state<W>(a.state + e * W, s);
        to_plane<W>(P, s);
        uint32_t bucket = 0;
        for (int j = 0; j < a.n_targets; ++j) bucket = (bucket << 1) | P.bit(targets[j]);
        uint32_t cur = bucket, run = 0;
        const uint64_t g = a.env_base + e;
        for (uint32_t t = 0; t < a.iters; ++t) {
            const uint64_t it = a.iter_base + t;
            // record (eval.py:88-89)
            if (bucket != cur) {
                atomicAdd(&hist[cur], run);
                cur = bucket;
                run = 0;
            }
            ++run;
            // independent Bernoulli(p) flips (eval.py:92-95) as geometric gaps
            if (a.gap_thr)
                bernoulli_positions(a.seed, (uint32_t)it, STREAM_SSD_FLIP, g, gap, N, a.gap_inv_log2, [&](uint32_t pos) {
                    const uint32_t d = pos >> 5, sh = pos & 31u;
                    P.put(d, P.get(d) ^ (1u << sh));
                    const int tb = tbit[pos];
                    if (tb >= 0) bucket ^= 1u << tb;
                });
            // one transition (env.step(action=0), eval.py:96)
            uint32_t w[4];
            philox_draw(a.seed, (uint32_t)it, (uint32_t)(it >> 32), g, STREAM_SSD, w);
            const uint32_t i = philox_node<KIND>(w[0], N);
            const uint64_t k53 = k53_of(w[1], w[2]);
            uint32_t changed;
            if constexpr (KIND == KIND_PREDICTOR_MIX)
                changed = predictor_update_lds(P, i, k53, lds, a.L);
            else
                changed = table_update_lds(P, i, k53, lds, a.L);
            if (changed) {
                const int tb = tbit[i];
                if (tb >= 0) bucket ^= 1u << tb;
            }
        }
        atomicAdd(&hist[cur], run);
        from_plane<W>(P, s);
        store_state<W>(a.state + e * W, s);
    }
    __syncthreads();
    for (uint32_t k = threadIdx.x; k < nb; k += BLOCK)
        if (hist[k]) atomicAdd(reinterpret_cast<unsigned long long*>(a.hist) + k, (unsigned long long)hist[k]);
}

template <int KIND>
static void* ssd_fn(int W) {
    switch (W) {
        case 1: return (void*)k_ssd<1, KIND>;
        case 2: return (void*)k_ssd<2, KIND>;
        case 3: return (void*)k_ssd<3, KIND>;
        case 4: return (void*)k_ssd<4, KIND>;
        case 5: return (void*)k_ssd<5, KIND>;
        case 6: return (void*)k_ssd<6, KIND>;
        case 7: return (void*)k_ssd<7, KIND>;
        case 8: return (void*)k_ssd<8, KIND>;
    }
    return nullptr;
}

static uint32_t a16(uint32_t x) { return (x + 15u) & ~15u; }

uint32_t ssd_layout(int W, uint32_t image_bytes, int n_nodes, int n_targets, SSDArgs* a) {
    a->off_planes = image_bytes;
    a->off_gap = a16(a->off_planes + 8u * (uint32_t)W * BLOCK);
    a->off_tbit = a16(a->off_gap + 4u * (uint32_t)n_nodes);
    a->off_targets = a16(a->off_tbit + 2u * (uint32_t)n_nodes);
    a->off_hist = a16(a->off_targets + 2u * (uint32_t)n_targets);
    return a16(a->off_hist + 4u * (1u << n_targets));
}

int launch_ssd(int W, const SSDArgs& a, int grid, void* stream) {
    void* fn = a.L.kind == KIND_PREDICTOR_MIX ? ssd_fn<KIND_PREDICTOR_MIX>(W) : ssd_fn<KIND_PROB_TABLE>(W);
    if (!fn) return (int)hipErrorInvalidValue;
    SSDArgs c = a;
    const uint32_t lds = c.lds_bytes;
    if (lds > 64u * 1024u) {
        hipError_t e = hipFuncSetAttribute((const void*)fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) return (int)e;
    }
    void* kargs[] = {&c};
    return (int)hipLaunchKernel(fn, dim3((unsigned)grid), dim3(BLOCK), kargs, lds, (hipStream_t)stream);
}

}  // namespace pbn
