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

// ---------------------------------------------------------------- one wave per env
// At the reference's own size (300 resets) the lane-per-env kernel leaves the chip idle and each
// lane's 4,000 iterations run back to back (~4 us each: two Philox draws, the gap search, the
// update). Here a wave owns an env and works in chunks of 64 iterations: lane k draws iteration
// k's flip positions and transition (they do not depend on the state: Philox counters are the
// iteration index). The chunk is then resolved in parallel (fixed point over the chunk's update
// DAG, see below) for predictor-mix networks and truth-table networks with <= SSD_DAG_KMAX inputs
// per node; otherwise lane 0 applies the 64 iterations in order -- bucket, flips, update -- from
// LDS. Same draws as k_ssd, so the same counts and states.
constexpr int SSD_FMAX = 12;  // serial apply: flip positions kept per iteration; more -> lane 0 redraws them
struct RowT {
    uint32_t* base;  // the env's 2W dwords
    __device__ __forceinline__ uint32_t get(uint32_t d) const { return base[d]; }
    __device__ __forceinline__ void put(uint32_t d, uint32_t v) const { base[d] = v; }
    __device__ __forceinline__ uint32_t bit(uint32_t i) const { return (get(i >> 5) >> (i & 31u)) & 1u; }
};
// per wave: LDS-row path 64*8 + 64*8 + 64*2*SSD_FMAX + 64 + 16*8 = 2,752 B; predictor-mix path
// flips/prefixes [64][17] u32 + writer masks [512] u64 + base row [16] u32 = 8,512 B
constexpr uint32_t SSD_WAVE_BYTES = 64 * 17 * 4 + 512 * 8 + 16 * 4;
constexpr uint32_t SSD_WAVE_MAX_BLOCK = 512;  // shared mode: up to 8 waves on one env

template <int W, int KIND>
__global__ __launch_bounds__(SSD_WAVE_MAX_BLOCK) void k_ssd_wave(SSDArgs a) {
    const uint32_t BLK = blockDim.x;  // 256, or 64 x the waves per env in shared mode
    extern __shared__ __align__(16) uint8_t lds[];
    stage_image(reinterpret_cast<const uint4*>(a.img), a.L.bytes / 16, reinterpret_cast<uint4*>(lds));
    const uint32_t N = (uint32_t)a.L.n_nodes;
    const uint32_t nb = 1u << a.n_targets;
    uint32_t* gap = reinterpret_cast<uint32_t*>(lds + a.off_gap);
    int16_t* tbit = reinterpret_cast<int16_t*>(lds + a.off_tbit);
    uint16_t* targets = reinterpret_cast<uint16_t*>(lds + a.off_targets);
    uint32_t* hist = reinterpret_cast<uint32_t*>(lds + a.off_hist);
    for (uint32_t k = threadIdx.x; k < N; k += BLK) {
        gap[k] = a.gap_thr ? a.gap_thr[k] : 0xFFFFFFFFu;
        tbit[k] = -1;
    }
    for (uint32_t k = threadIdx.x; k < nb; k += BLK) hist[k] = 0;
    __syncthreads();
    for (uint32_t j = threadIdx.x; j < (uint32_t)a.n_targets; j += BLK) {
        targets[j] = (uint16_t)a.targets[j];
        tbit[a.targets[j]] = (int16_t)(a.n_targets - 1 - (int)j);
    }
    __syncthreads();
    const uint32_t lane = __lane_id(), wv = threadIdx.x >> 6;
    uint8_t* wb = lds + a.off_planes + wv * SSD_WAVE_BYTES;
    uint64_t* tr_a = reinterpret_cast<uint64_t*>(wb);                 // [64] record (mix) or k53 (table)
    uint32_t* tr_i = reinterpret_cast<uint32_t*>(wb + 64 * 8);        // [64] node (u32, 8-B slots)
    uint16_t* fpos = reinterpret_cast<uint16_t*>(wb + 64 * 16);       // [64][SSD_FMAX]
    uint8_t* fcnt = wb + 64 * 16 + 64 * 2 * SSD_FMAX;                 // [64], SSD_FMAX + 1 = overflow
    const RowT R{reinterpret_cast<uint32_t*>(wb + 64 * 16 + 64 * 2 * SSD_FMAX + 64)};  // 2W dwords
    auto wave_sync = [] {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    };
    const uint64_t waves = (uint64_t)gridDim.x * (BLK / 64);
    if (a.dag) {
        // Parallel in time: lane c owns iteration t0 + c of a 64-iteration chunk. All draws
        // (flips, node, predictor record) are independent of the state, so lane c has them before
        // any update is applied; only the four operand values of its update depend on earlier
        // iterations of the chunk. With the chunk's flips folded into prefix XORs (P_c = XOR of
        // the flip masks of iterations <= c; the state seen by update c is base ^ P_c, base = the
        // chunk-initial state with the updates < c written as y ^ P at their node), operand n of
        // update c is either the initial bit (no earlier writer of n in the chunk) or the base
        // bit yb_k stored by its last earlier writer k. The writers are known up front (a 64-bit
        // writer mask per node), so the chunk is a DAG of boolean updates: iterate all 64 lanes
        // at once (ballot of the yb bits, one 64-bit shift per operand) until nothing changes --
        // one round per level of the chain instead of one serial step per iteration. The fixed
        // point is unique (update c reads only writers < c), so the result equals the serial
        // order of eval.py:84-96 bit for bit. Truth-table networks (node.py:31-38) take the same
        // route when every node has <= 6 inputs: lane c turns its threshold row and k53 into a
        // 2^k-bit table of y (k53 < thr[x] for every input pattern x), after which both kinds are
        // "y = table bit x of the operand values".
        constexpr int KOP = KIND == KIND_PREDICTOR_MIX ? 4 : SSD_DAG_KMAX;
        uint32_t* fm = reinterpret_cast<uint32_t*>(wb);                                   // [64][17] flips / P
        unsigned long long* wm = reinterpret_cast<unsigned long long*>(wb + 64 * 17 * 4);  // [512] writers
        auto xor_scan = [lane](uint32_t v) {  // inclusive prefix XOR over the wave's lanes
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const uint32_t u = (uint32_t)__shfl_up((int)v, o);
                if (lane >= (uint32_t)o) v ^= u;
            }
            return v;
        };
        const unsigned long long below = (1ull << lane) - 1ull;  // lanes < this one
        auto uni = [](uint32_t v) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)v); };
        auto rl = [](uint32_t v, uint32_t l) { return (uint32_t)__builtin_amdgcn_readlane((int)v, (int)l); };
        const int nt = a.n_targets;  // <= 12 (host check)
        uint32_t tg[12];             // target nodes, wave-uniform
#pragma unroll
        for (int j = 0; j < 12; ++j) tg[j] = j < nt ? uni(targets[j]) : 0u;
        // a.dag == 1: one wave per env (4 envs per workgroup). a.dag == 4: the workgroup's 4 waves
        // share one env -- each draws and prepares its own chunk (iterations t0 + 64 w ..), then
        // they resolve in order, wave w once wave w - 1 has written the state row: the state-free
        // three quarters of the work run on four SIMDs at once. The order is a turn counter in
        // LDS (release / acquire at workgroup scope), not a barrier: a wave that has resolved
        // its chunk goes on drawing its next one while the later waves resolve theirs.
        const uint32_t wpe = (uint32_t)a.dag;                      // waves per env
        // the env's state row (2W dwords): the tail of its first wave's area
        uint32_t* srow = reinterpret_cast<uint32_t*>(lds + a.off_planes + (wpe == 1 ? wv : 0u) * SSD_WAVE_BYTES +
                                                     64 * 17 * 4 + 512 * 8);
        // shared mode's turn counter: the (otherwise unused) row slot of wave 1's area
        uint32_t* turnp = reinterpret_cast<uint32_t*>(lds + a.off_planes + SSD_WAVE_BYTES + 64 * 17 * 4 + 512 * 8);
        const uint64_t env_stride = wpe == 1 ? waves : (uint64_t)gridDim.x;
        auto env_sync = [&] {
            if (wpe == 1)
                wave_sync();
            else
                __syncthreads();
        };
        for (uint64_t e = wpe == 1 ? (uint64_t)blockIdx.x * (BLK / 64) + wv : (uint64_t)blockIdx.x;; e += env_stride) {
            if (e >= a.B) break;  // shared mode: e is the same in all four waves (barriers inside)
            const uint64_t g = a.env_base + e;
            if (lane < 2u * W && (wpe == 1 || wv == 0)) srow[lane] = reinterpret_cast<const uint32_t*>(a.state + e * W)[lane];
            if (wpe > 1 && threadIdx.x == 0) *turnp = 0u;
            env_sync();
            uint32_t round = 0;
            for (uint32_t t00 = 0; t00 < a.iters; t00 += 64u * wpe, ++round) {
                const uint32_t t0 = t00 + 64u * (wpe == 1 ? 0u : wv);  // this wave's chunk
                const uint32_t n = t0 < a.iters ? min(64u, a.iters - t0) : 0u;
                const bool live = lane < n;
                uint32_t* fmr = fm + lane * 17u;  // own row, stride 17 dwords: conflict-free
                for (uint32_t k = lane; k < N; k += 64) wm[k] = 0ull;
#pragma unroll
                for (int q = 0; q < 2 * W; ++q) fmr[q] = 0u;
                // ---- draws of iteration t0 + lane (same counters as k_ssd)
                uint32_t i = 0, nk = 0, nd[KOP];
                uint64_t ytab = 0;  // bit x: y for operand pattern x
#pragma unroll
                for (int k = 0; k < KOP; ++k) nd[k] = 0;
                if (live) {
                    const uint64_t it = a.iter_base + t0 + lane;
                    if (a.gap_thr)
                        bernoulli_positions_x4(a.seed, (uint32_t)it, STREAM_SSD_FLIP, g, gap, N, a.gap_inv_log2,
                                               [&](uint32_t pos) { fmr[pos >> 5] ^= 1u << (pos & 31u); });
                    uint32_t w[4];
                    philox_draw(a.seed, (uint32_t)it, (uint32_t)(it >> 32), g, STREAM_SSD, w);
                    i = philox_node<KIND>(w[0], N);
                    const uint64_t k53 = k53_of(w[1], w[2]);
                    if constexpr (KIND == KIND_PREDICTOR_MIX) {
                        // operands in0, in1, in2, self -> pattern bits 3..0 (predictor_apply)
                        const uint64_t rec = predictor_record(i, k53, lds, a.L);
                        nd[0] = (uint32_t)rec & 0xFFFFu;
                        nd[1] = (uint32_t)(rec >> 16) & 0xFFFFu;
                        nd[2] = (uint32_t)(rec >> 32) & 0xFFFFu;
                        nd[3] = i;
                        nk = 4;
                        ytab = rec >> 48;
                    } else {
                        // operands = the node's inputs, first = MSB (table_eval_lds)
                        const uint64_t info = reinterpret_cast<const uint64_t*>(lds + a.L.off_node)[i];
                        const uint32_t toff = (uint32_t)info, ioff = (uint32_t)(info >> 32) & 0xFFFFu;
                        nk = (uint32_t)(info >> 48) & 0xFFu;  // <= SSD_DAG_KMAX (host check)
                        const uint16_t* in = reinterpret_cast<const uint16_t*>(lds + a.L.off_rec) + ioff;
#pragma unroll
                        for (int k = 0; k < KOP; ++k)
                            if ((uint32_t)k < nk) nd[k] = in[k];
                        const uint64_t* thr = reinterpret_cast<const uint64_t*>(lds + a.L.off_thr) + toff;
                        for (uint32_t x = 0; x < (1u << nk); ++x) ytab |= (uint64_t)(k53 < thr[x]) << x;
                    }
                }
                // ---- own flips -> prefix P (lane-private rows), bucket bits of the own flips
                auto tbits = [&](const uint32_t* r) {  // target bits of a row, first target = MSB
                    uint32_t v = 0;
#pragma unroll
                    for (int j = 0; j < 12; ++j)
                        if (j < nt) v = (v << 1) | ((r[tg[j] >> 5] >> (tg[j] & 31u)) & 1u);
                    return v;
                };
                const uint32_t own_b = tbits(fmr);
#pragma unroll
                for (int q = 0; q < 2 * W; ++q) fmr[q] = xor_scan(fmr[q]);
                if (live) atomicOr(&wm[i], 1ull << lane);
                wave_sync();
                // ---- operands: last earlier writer and the P_c correction (state-free)
                uint32_t lw[KOP], has[KOP], pcs[KOP];
#pragma unroll
                for (int k = 0; k < KOP; ++k) {
                    const unsigned long long m = wm[nd[k]] & below;
                    has[k] = m != 0ull;
                    lw[k] = m ? 63u - (uint32_t)__clzll(m) : 0u;
                    pcs[k] = (fmr[nd[k] >> 5] >> (nd[k] & 31u)) & 1u;
                }
                const uint32_t pself = (fmr[i >> 5] >> (i & 31u)) & 1u;
                const uint32_t p_b = tbits(fmr) ^ own_b;  // targets' flips before iteration c
                const bool last_w = live && (wm[i] >> lane) == 1ull;
                unsigned long long tw[12];  // writer masks of the targets, below this lane
#pragma unroll
                for (int j = 0; j < 12; ++j) tw[j] = j < nt ? wm[tg[j]] & below : 0ull;
                // ---- resolve, in chunk order across the env's waves
                const uint32_t want = round * wpe + (wpe == 1 ? 0u : wv);
                if (wpe > 1) {
                    // the waves of a workgroup are co-resident and wave w - 1 never waits on wave w,
                    // so the turn always comes; the bound only guards against a logic error
                    uint32_t spins = 0;
                    while (__hip_atomic_load(turnp, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) != want &&
                           ++spins < (1u << 24))
                        __builtin_amdgcn_s_sleep(1);
                    if (spins >= (1u << 24) && lane == 0) atomicOr(a.error, 1);
                }
                unsigned long long B = 0ull;  // bit c: base bit stored by update c
                uint32_t tinit = 0;           // the targets' bits at the chunk start (first = MSB)
                if (n) {
                    uint32_t cst[KOP];
#pragma unroll
                    for (int k = 0; k < KOP; ++k) {
                        const uint32_t init = (srow[nd[k] >> 5] >> (nd[k] & 31u)) & 1u;
                        cst[k] = (has[k] ? 0u : init) ^ pcs[k];
                    }
                    const uint32_t sv = lane < 2u * W ? srow[lane] : 0u;
#pragma unroll
                    for (int j = 0; j < 12; ++j)
                        if (j < nt) tinit = (tinit << 1) | ((rl(sv, tg[j] >> 5) >> (tg[j] & 31u)) & 1u);
                    // ---- fixed point over the chunk's updates
                    for (uint32_t r = 0; r <= n; ++r) {
                        uint32_t x = 0;
#pragma unroll
                        for (int k = 0; k < KOP; ++k)
                            if (KIND == KIND_PREDICTOR_MIX || (uint32_t)k < nk)
                                x = (x << 1) | ((((uint32_t)(B >> lw[k]) & has[k]) ^ cst[k]) & 1u);
                        const uint32_t yb = ((uint32_t)(ytab >> x) ^ pself) & 1u;
                        const unsigned long long Bn = __ballot(live && yb);
                        if (Bn == B) break;
                        B = Bn;
                    }
                    wave_sync();  // every lane's row reads before the row is rewritten
                    // ---- the last writer of each node stores its base bit; then base ^ P_{n-1}
                    if (last_w) {
                        const uint32_t bit = 1u << (i & 31u);
                        if ((B >> lane) & 1ull)
                            atomicOr(&srow[i >> 5], bit);
                        else
                            atomicAnd(&srow[i >> 5], ~bit);
                    }
                    wave_sync();
                    if (lane < 2u * W) srow[lane] ^= fm[(n - 1) * 17u + lane];
                }
                wave_sync();
                if (wpe > 1 && lane == 0)  // the next chunk's wave may go (its LDS reads see this chunk's writes)
                    __hip_atomic_store(turnp, want + 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
                // ---- histogram, off the chain of resolutions: the bucket before iteration c's flips
                // = base ^ P_{c-1} on the targets, from the writer masks, B and the chunk-start bits
                if (live) {
                    uint32_t bb = 0;
#pragma unroll
                    for (int j = 0; j < 12; ++j)
                        if (j < nt) {
                            const uint32_t v = tw[j] ? (uint32_t)(B >> (63u - (uint32_t)__clzll(tw[j]))) & 1u
                                                     : (tinit >> (nt - 1 - j)) & 1u;
                            bb = (bb << 1) | v;
                        }
                    atomicAdd(&hist[bb ^ p_b], 1u);
                }
                wave_sync();  // own tables are rewritten by the next round's draws
            }
            env_sync();  // every chunk of the env resolved
            if (lane < 2u * W && (wpe == 1 || wv == 0)) reinterpret_cast<uint32_t*>(a.state + e * W)[lane] = srow[lane];
            env_sync();  // the row is reloaded for the next env
        }
        __syncthreads();
        for (uint32_t k = threadIdx.x; k < nb; k += BLK)
            if (hist[k]) atomicAdd(reinterpret_cast<unsigned long long*>(a.hist) + k, (unsigned long long)hist[k]);
        return;
    }
    for (uint64_t e = (uint64_t)blockIdx.x * (BLK / 64) + wv; e < a.B; e += waves) {
        const uint64_t g = a.env_base + e;
        if (lane < 2u * W) R.put(lane, reinterpret_cast<const uint32_t*>(a.state + e * W)[lane]);
        wave_sync();
        uint32_t bucket = 0, cur = 0, run = 0;
        if (lane == 0) {
            for (int j = 0; j < a.n_targets; ++j) bucket = (bucket << 1) | R.bit(targets[j]);
            cur = bucket;
        }
        for (uint32_t t0 = 0; t0 < a.iters; t0 += 64) {
            const uint32_t n = min(64u, a.iters - t0);
            // ---- draws of iterations t0 .. t0 + n - 1, one per lane
            if (lane < n) {
                const uint64_t it = a.iter_base + t0 + lane;
                uint32_t cnt = 0;
                if (a.gap_thr)
                    bernoulli_positions(a.seed, (uint32_t)it, STREAM_SSD_FLIP, g, gap, N, a.gap_inv_log2,
                                        [&](uint32_t pos) {
                                            if (cnt < (uint32_t)SSD_FMAX) fpos[lane * SSD_FMAX + cnt] = (uint16_t)pos;
                                            ++cnt;
                                        });
                fcnt[lane] = (uint8_t)min(cnt, (uint32_t)SSD_FMAX + 1u);
                uint32_t w[4];
                philox_draw(a.seed, (uint32_t)it, (uint32_t)(it >> 32), g, STREAM_SSD, w);
                const uint32_t i = philox_node<KIND>(w[0], N);
                const uint64_t k53 = k53_of(w[1], w[2]);
                tr_i[2 * lane] = i;
                if constexpr (KIND == KIND_PREDICTOR_MIX)
                    tr_a[lane] = predictor_record(i, k53, lds, a.L);
                else
                    tr_a[lane] = k53;
            }
            wave_sync();
            // ---- lane 0 applies them in order (eval.py:84-96)
            if (lane == 0) {
                for (uint32_t c = 0; c < n; ++c) {
                    if (bucket != cur) {
                        atomicAdd(&hist[cur], run);
                        cur = bucket;
                        run = 0;
                    }
                    ++run;
                    auto flip = [&](uint32_t pos) {
                        const uint32_t d = pos >> 5;
                        R.put(d, R.get(d) ^ (1u << (pos & 31u)));
                        const int tb = tbit[pos];
                        if (tb >= 0) bucket ^= 1u << tb;
                    };
                    const uint32_t fc = fcnt[c];
                    if (fc <= (uint32_t)SSD_FMAX) {
                        for (uint32_t q = 0; q < fc; ++q) flip(fpos[c * SSD_FMAX + q]);
                    } else {  // more flips than the buffer holds: draw them again here
                        bernoulli_positions(a.seed, (uint32_t)(a.iter_base + t0 + c), STREAM_SSD_FLIP, g, gap, N,
                                            a.gap_inv_log2, flip);
                    }
                    const uint32_t i = tr_i[2 * c];
                    uint32_t changed;
                    if constexpr (KIND == KIND_PREDICTOR_MIX) {
                        const uint32_t d = i >> 5, sh = i & 31u;
                        const uint32_t self = R.get(d);
                        const uint32_t y = predictor_apply(R, i, self, tr_a[c]);
                        const uint32_t nv = (self & ~(1u << sh)) | (y << sh);
                        R.put(d, nv);
                        changed = nv != self;
                    } else {
                        changed = table_update_lds(R, i, tr_a[c], lds, a.L);
                    }
                    if (changed) {
                        const int tb = tbit[i];
                        if (tb >= 0) bucket ^= 1u << tb;
                    }
                }
            }
            wave_sync();
        }
        if (lane == 0) atomicAdd(&hist[cur], run);
        if (lane < 2u * W) reinterpret_cast<uint32_t*>(a.state + e * W)[lane] = R.get(lane);
        wave_sync();
    }
    __syncthreads();
    for (uint32_t k = threadIdx.x; k < nb; k += BLK)
        if (hist[k]) atomicAdd(reinterpret_cast<unsigned long long*>(a.hist) + k, (unsigned long long)hist[k]);
}

template <int KIND>
static void* ssd_wave_fn(int W) {
    switch (W) {
        case 1: return (void*)k_ssd_wave<1, KIND>;
        case 2: return (void*)k_ssd_wave<2, KIND>;
        case 3: return (void*)k_ssd_wave<3, KIND>;
        case 4: return (void*)k_ssd_wave<4, KIND>;
        case 5: return (void*)k_ssd_wave<5, KIND>;
        case 6: return (void*)k_ssd_wave<6, KIND>;
        case 7: return (void*)k_ssd_wave<7, KIND>;
        case 8: return (void*)k_ssd_wave<8, KIND>;
    }
    return nullptr;
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

// threads per workgroup: shared mode puts a.dag waves on one env, every other mode runs 256
uint32_t ssd_block(const SSDArgs& a) { return a.wave && a.dag > 1 ? 64u * (uint32_t)a.dag : (uint32_t)BLOCK; }

uint32_t ssd_layout(int W, uint32_t image_bytes, int n_nodes, int n_targets, SSDArgs* a) {
    a->off_planes = image_bytes;  // lane mode: state planes; wave mode: per-wave chunk buffers + row
    const uint32_t per_block = a->wave ? ssd_block(*a) / 64u * SSD_WAVE_BYTES : 8u * (uint32_t)W * BLOCK;
    a->off_gap = a16(a->off_planes + per_block);
    a->off_tbit = a16(a->off_gap + 4u * (uint32_t)n_nodes);
    a->off_targets = a16(a->off_tbit + 2u * (uint32_t)n_nodes);
    a->off_hist = a16(a->off_targets + 2u * (uint32_t)n_targets);
    return a16(a->off_hist + 4u * (1u << n_targets));
}

int launch_ssd(int W, const SSDArgs& a, int grid, void* stream) {
    void* fn = a.wave ? (a.L.kind == KIND_PREDICTOR_MIX ? ssd_wave_fn<KIND_PREDICTOR_MIX>(W)
                                                          : ssd_wave_fn<KIND_PROB_TABLE>(W))
                      : (a.L.kind == KIND_PREDICTOR_MIX ? ssd_fn<KIND_PREDICTOR_MIX>(W) : ssd_fn<KIND_PROB_TABLE>(W));
    if (!fn) return (int)hipErrorInvalidValue;
    SSDArgs c = a;
    const uint32_t lds = c.lds_bytes;
    if (lds > 64u * 1024u) {
        hipError_t e = hipFuncSetAttribute((const void*)fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) return (int)e;
    }
    void* kargs[] = {&c};
    return (int)hipLaunchKernel(fn, dim3((unsigned)grid), dim3(ssd_block(a)), kargs, lds, (hipStream_t)stream);
}

}  // namespace pbn
