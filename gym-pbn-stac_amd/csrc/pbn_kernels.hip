// pbn_kernels.hip -- gfx950 kernels of the vectorised PBN simulator.
//
// Mapping: one lane = one env (state in VGPRs), one 256-thread workgroup stages
// the network image (node info, 53-bit selection thresholds, predictor records
// or probability thresholds) into LDS once, then walks envs in a grid-stride loop.
// The grid is sized to what is resident (CUs x blocks/CU), so the LDS staging is
// paid once per resident workgroup, not once per 256 envs.
//
// Reference semantics implemented (file:line in the reference):
//   k_step    Graph.step base.py:306-312 (+ Node.Predstep :89-119) and
//             PBN.step common/pbn.py:129-133 (+ Node.compute_next_value common/node.py:34-38)
//   k_init    Graph.genRandState base.py:368-370 / PBN.reset(None) pbn.py:105-118 /
//             PBNTargetMultiEnv.reset pbn_target_multi.py:237-249 (Philox streams)
//   k_flip    Graph.flipNode base.py:280-284 over a multi-action row (pbn_target_multi.py:120-131)
//   k_env     PBNTargetMultiEnv.step pbn_target_multi.py:119-154
#include <hip/hip_runtime.h>

#include <algorithm>

#include "pbn_device.hpp"
#include "pbn_params.hpp"

namespace pbn {

// ------------------------------------------------------------------ step
// Layout per workgroup in LDS: [network image][state planes]. The state planes
// hold, for the env each lane is working on, its 2W dwords in planar order
// (dword d of lane l at plane d, column l), so reading node i of the own env is
// one conflict-free ds_read_b32 at plane (i >> 5) and an update is one
// read-modify-write of one dword -- instead of ~20 VALU selects per bit when the
// words sit in VGPRs. Columns are lane-private: no barrier is needed around them.
//
// Each thread walks envs e0, e0 + stride, ... with the next env's state load in
// flight while the current env is computed (software pipeline), so HBM traffic
// of one env overlaps the Philox/LDS work of the previous one.
//
// SB (threads per workgroup) trades LDS staging traffic against scheduling
// granularity: the image is staged once per workgroup, so 1024-thread groups
// read it from L2 4x less often than 256-thread groups.
// One update per env (T == 1), Philox. Envs are taken in pairs (e, e + stride); at the
// bench sizes every thread owns exactly one pair. The pair's draws and (for predictor
// networks) its predictor records depend only on (seed, update counter, env id), so
// they are computed while the pair's state loads are in flight.
template <int W, int KIND, int STORE, int SB>
__device__ __forceinline__ void k_step_single(const StepArgs& a, uint8_t* lds, uint64_t e, uint64_t stride,
                                              uint64_t (&cur)[W], uint32_t N) {
    const uint64_t u = a.update_base;
    const uint64_t po = stride;  // second env of the pair (adjacent envs measured slower: 8.2 vs 7.8 us)
    uint64_t nxt[W];
    uint32_t i0 = 0, i1 = 0;
    uint64_t q0 = 0, q1 = 0;
    auto draws = [&](uint64_t ea) {
        uint32_t w0[4], w1[4];
        philox_draw(a.seed, (uint32_t)u, (uint32_t)(u >> 32), a.env_base + ea, STREAM_STEP, w0);
        philox_draw(a.seed, (uint32_t)u, (uint32_t)(u >> 32), a.env_base + ea + po, STREAM_STEP, w1);
        i0 = philox_node<KIND>(w0[0], N);
        i1 = philox_node<KIND>(w1[0], N);
        q0 = k53_of(w0[1], w0[2]);
        q1 = k53_of(w1[1], w1[2]);
    };
    if (e + po < a.B) load_state<W>(a.state + (e + po) * W, nxt);
    draws(e);
    stage_image(reinterpret_cast<const uint4*>(a.img), a.L.bytes / 16, reinterpret_cast<uint4*>(lds));
    __syncthreads();
    const PlaneT<SB> P{reinterpret_cast<uint32_t*>(lds + a.L.bytes) + threadIdx.x};
    while (e < a.B) {
        const uint64_t e1 = e + po;
        uint64_t r0 = 0, r1 = 0;
        if constexpr (KIND == KIND_PREDICTOR_MIX) {  // state-independent: before the loads land
            r0 = predictor_record(i0, q0, lds, a.L);
            r1 = predictor_record(i1, q1, lds, a.L);
        }
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const uint64_t eh = h ? e1 : e;
            if (eh >= a.B) break;
            uint64_t(&s)[W] = h ? nxt : cur;
            const uint32_t i = h ? i1 : i0;
            const uint32_t d = i >> 5, sh = i & 31u;
            to_plane<W>(P, s);
            const uint32_t self = P.get(d);
            uint32_t y;
            if constexpr (KIND == KIND_PREDICTOR_MIX)
                y = predictor_apply(P, i, self, h ? r1 : r0);
            else
                y = table_eval_lds(P, i, h ? q1 : q0, lds, a.L);
            const uint32_t nv = (self & ~(1u << sh)) | (y << sh);
            if constexpr (STORE == STORE_DIRTY) {
                // store the whole env (32 B at W = 4), and only if its bit changed: a full
                // aligned env write measured faster than writing just the 16-B half that holds
                // node i (7.69 vs 7.93 us at 1M envs), partial sector writes cost extra
                if (nv != self) {
                    P.put(d, nv);
                    uint64_t out[W];
                    from_plane<W>(P, out);
                                        store_state<W>(a.state + eh * W, out);
                }
            } else {
                P.put(d, nv);
                uint64_t out[W];
                from_plane<W>(P, out);
                store_state<W>(a.state + eh * W, out);
            }
        }
        e += 2 * stride;
        if (e < a.B) {
            load_state<W>(a.state + e * W, cur);
            if (e + po < a.B) load_state<W>(a.state + (e + po) * W, nxt);
            draws(e);
        }
    }
}

template <int W, int KIND, int STORE, int REPLAY, int SB>
__global__ __launch_bounds__(SB) void k_step(StepArgs a) {
    extern __shared__ __align__(16) uint8_t lds[];
    const uint64_t stride = (uint64_t)gridDim.x * SB;
    uint64_t e = (uint64_t)blockIdx.x * SB + threadIdx.x;
    const uint32_t N = (uint32_t)a.L.n_nodes;
    uint64_t cur[W];
    if (e < a.B) load_state<W>(a.state + e * W, cur);
    if constexpr (!REPLAY) {
        if (a.T == 1) {
            // Step mode: the draws depend on (seed, update counter, env id) only, so every
            // draw this thread needs is computed while its state loads are in flight.
            k_step_single<W, KIND, STORE, SB>(a, lds, e, stride, cur, N);
            return;
        }
    }
    stage_image(reinterpret_cast<const uint4*>(a.img), a.L.bytes / 16, reinterpret_cast<uint4*>(lds));
    __syncthreads();
    const PlaneT<SB> P{reinterpret_cast<uint32_t*>(lds + a.L.bytes) + threadIdx.x};
    while (e < a.B) {
        const uint64_t en = e + stride;
        uint64_t nxt[W];
        if (en < a.B) load_state<W>(a.state + en * W, nxt);  // prefetch the next env
        to_plane<W>(P, cur);
        uint32_t changed = 0;
        const uint64_t g = a.env_base + e;
        for (uint32_t t = 0; t < a.T; ++t) {
            uint32_t i;
            uint64_t k53;
            if constexpr (REPLAY) {
                i = a.replay_node[(uint64_t)t * a.B + e];
                k53 = a.replay_k53[(uint64_t)t * a.B + e];
            } else {
                const uint64_t u = a.update_base + t;
                uint32_t w[4];
                philox_draw(a.seed, (uint32_t)u, (uint32_t)(u >> 32), g, STREAM_STEP, w);
                i = philox_node<KIND>(w[0], N);
                k53 = k53_of(w[1], w[2]);
            }
            if constexpr (KIND == KIND_PREDICTOR_MIX)
                changed |= predictor_update_lds(P, i, k53, lds, a.L);
            else
                changed |= table_update_lds(P, i, k53, lds, a.L);
        }
        uint64_t out[W];
        from_plane<W>(P, out);
        if constexpr (STORE == STORE_DIRTY) {
            bool diff = false;  // whole env, only if it differs (see k_step_single)
#pragma unroll
            for (int k = 0; k < W; ++k) diff |= out[k] != cur[k];
            if (changed && diff) store_state<W>(a.state + e * W, out);
        } else {
            store_state<W>(a.state + e * W, out);
        }
#pragma unroll
        for (int k = 0; k < W; ++k) cur[k] = nxt[k];
        e = en;
    }
}

// ------------------------------------------------------------------ init / reset
template <int W>
__global__ __launch_bounds__(BLOCK) void k_init(InitArgs a) {
    const uint64_t e = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
    if (e >= a.B) return;
    if (a.mask && !a.mask[e]) return;
    const uint64_t g = a.env_base + e;
    uint64_t s[W];
#pragma unroll
    for (int m = 0; 2 * m < W; ++m) {
        uint32_t w[4];
        philox_draw(a.seed, (uint32_t)m + (a.cube_care ? 1u : 0u), a.reset_count, g,
                    a.cube_care ? STREAM_RESET : STREAM_INIT, w);
        s[2 * m] = ((uint64_t)w[1] << 32) | w[0];
        if (2 * m + 1 < W) s[2 * m + 1] = ((uint64_t)w[3] << 32) | w[2];
    }
    if (a.cube_care) {
        uint32_t w[4];
        philox_draw(a.seed, 0u, a.reset_count, g, STREAM_RESET, w);
        const uint32_t c = __umulhi(w[0], (uint32_t)a.n_cubes);
#pragma unroll
        for (int k = 0; k < W; ++k) {
            const uint64_t care = a.cube_care[(uint64_t)c * W + k];
            s[k] = (a.cube_value[(uint64_t)c * W + k] & care) | (s[k] & ~care);
        }
    }
    const int r = a.n_nodes & 63;
    if (r) s[W - 1] &= (((uint64_t)1 << r) - 1);
    if (a.kind == KIND_PROB_TABLE) s[0] &= ~(uint64_t)1;  // pbn.py:118 state[0] = 0
    store_state<W>(a.state + e * W, s);
    if (a.n_steps) a.n_steps[e] = 0;
}

// Python list indexing of flipNode(a - offset): valid for -N <= idx < N.
__device__ __forceinline__ bool action_node(int32_t a, int32_t offset, int32_t N, uint32_t* node) {
    const int32_t idx = a - offset;
    if (idx >= N || idx < -N) return false;
    *node = (uint32_t)(idx < 0 ? idx + N : idx);
    return true;
}

// Flip every (unique, if dedup) non-zero action of the row; returns the number of
// actions counted by the reference's reward (unique values incl. 0, or A).
template <int W>
__device__ __forceinline__ int apply_actions(uint64_t (&s)[W], const int32_t* row, int32_t A, int32_t offset,
                                             int32_t dedup, int32_t N, bool* bad) {
    int n_act = 0;
    for (int32_t k = 0; k < A; ++k) {
        const int32_t v = row[k];
        bool dup = false;
        if (dedup)
            for (int32_t q = 0; q < k; ++q) dup |= (row[q] == v);
        if (dup) continue;
        ++n_act;
        if (v == 0) continue;
        uint32_t node;
        if (!action_node(v, offset, N, &node)) {
            *bad = true;
            continue;
        }
        setbit<W>(s, node, getbit<W>(s, node) ^ 1u);
    }
    return dedup ? n_act : A;
}

template <int W>
__global__ __launch_bounds__(BLOCK) void k_flip(FlipArgs a) {
    const uint64_t e = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
    if (e >= a.B) return;
    uint64_t s[W];
    load_state<W>(a.state + e * W, s);
    bool bad = false;
    apply_actions<W>(s, a.actions + e * (uint64_t)a.A, a.A, a.offset, a.dedup, a.n_nodes, &bad);
    if (bad) {
        atomicOr(a.error, 1);
        return;  // leave this env untouched
    }
    store_state<W>(a.state + e * W, s);
}

// ------------------------------------------------------------------ R6 env step
template <int W>
__device__ __forceinline__ bool cube_match(const uint64_t (&s)[W], const uint64_t* cv) {
    bool ok = true;
#pragma unroll
    for (int k = 0; k < W; ++k) ok &= ((s[k] & cv[k]) == cv[W + k]);
    return ok;
}

template <int W>
__device__ __forceinline__ bool attracting(const uint64_t (&s)[W], const uint64_t* cubes, int32_t H) {
    bool hit = false;
    for (int32_t h = 0; h < H && !hit; ++h) hit = cube_match<W>(s, cubes + (uint64_t)h * 2 * W);
    return hit;
}

// Mismatch count of a state against one cube: #cared bits that differ from the cube.
template <int W>
__device__ __forceinline__ uint32_t cube_mismatch(const uint64_t (&s)[W], const uint64_t* cv) {
    uint32_t m = 0;
#pragma unroll
    for (int k = 0; k < W; ++k) m += (uint32_t)__popcll((s[k] & cv[k]) ^ cv[W + k]);
    return m;
}

template <int W, class P_t>
__device__ __forceinline__ bool attracting_plane(const P_t& P, const uint64_t* cubes, int32_t H) {
    uint64_t s[W];
    from_plane<W>(P, s);
    return attracting<W>(s, cubes, H);
}

// PBNTargetMultiEnv.step (pbn_target_multi.py:119-154) for every env of the batch.
//
// Persistent waves with lane refill: a lane that finishes its env takes the next
// env index from a global counter (one atomic per wave per refill round), so the
// heavy-tailed until-attractor loops (1 .. 10^4 updates) do not idle the other
// 63 lanes of the wave. The env's state lives in the lane's LDS plane column.
//
// Attractor test (is_attracting_state :489-492 == "matches some cube").
// FAST (<= 8 cubes, each caring about <= 255 nodes): the lane keeps one byte per
// cube counting the cared bits where the state differs from the cube, packed in
// two words; an update that flips node i adds the node's packed delta (or its
// negation), and "some cube matches" is a zero-byte test -- a handful of VALU ops
// per update. Otherwise the state is matched against every cube after a change.
//
// GEN (FAST == 2, predictor-mix networks, Philox): before each chunk the whole wave
// generates the chunk's draws for all its active lanes -- assignment k of
// n_active * ENV_CHUNK goes to lane k % 64 -- and stores (node, chosen predictor) as
// u16 in a per-wave LDS buffer; the lanes then only apply the records. With every lane
// active this is the same Philox work per lane; in the tail, when a few lanes run long
// (capped) loops, idle lanes generate their draws and the per-update cost drops to the
// state read/write.

__device__ __forceinline__ uint32_t has_zero_byte(uint32_t v) { return (v - 0x01010101u) & ~v & 0x80808080u; }

template <int W, int KIND, int REPLAY, int FAST>
__global__ __launch_bounds__(BLOCK) void k_env(EnvArgs a) {
    static_assert(FAST != 2 || (KIND == KIND_PREDICTOR_MIX && !REPLAY), "GEN: predictor mix, Philox");
    extern __shared__ __align__(16) uint8_t lds[];
    stage_image(reinterpret_cast<const uint4*>(a.img), a.L.bytes / 16, reinterpret_cast<uint4*>(lds));
    __syncthreads();
    const PlaneT<BLOCK> P{reinterpret_cast<uint32_t*>(lds + a.L.bytes) + threadIdx.x};
    const uint32_t N = (uint32_t)a.L.n_nodes;
    const uint64_t* cubes = reinterpret_cast<const uint64_t*>(lds + a.off_cubes);
    const uint64_t* target = reinterpret_cast<const uint64_t*>(lds + a.off_target);
    const uint2* ndelta = reinterpret_cast<const uint2*>(lds + a.off_ndelta);
    const int32_t H = a.n_cubes;
    const uint32_t lane = __lane_id();

    int64_t e = -1;
    bool exhausted = false;
    uint64_t o0[W];
    uint32_t m_lo = 0, m_hi = 0;  // FAST: packed per-cube mismatch counters
    bool hit0 = false;            // o0 is attracting (the test made after the first update)
    uint32_t used = 0;
    int64_t nst = 0, dpos = 0, dend = 0;
    int n_act = 0;
    bool capped = false;

    for (;;) {
        // ---- refill idle lanes from the global work counter
        const bool need = e < 0 && !exhausted;
        const uint64_t need_mask = __ballot(need);
        if (need_mask) {
            const uint32_t leader = (uint32_t)__ffsll((unsigned long long)need_mask) - 1u;
            unsigned long long base = 0;
            if (lane == leader) base = atomicAdd(a.counter, (unsigned long long)__popcll(need_mask));
            base = __shfl(base, (int)leader);
            if (need) {
                const uint64_t ne = base + (uint64_t)__popcll(need_mask & ((1ull << lane) - 1ull));
                if (ne >= a.B) {
                    exhausted = true;
                } else {
                    uint64_t s[W];
                    load_state<W>(a.state + ne * W, s);
                    bool bad = false;
                    n_act = apply_actions<W>(s, a.actions + ne * (uint64_t)a.A, a.A, a.offset, a.dedup,
                                             (int32_t)N, &bad);
                    if (bad) {  // reference raises ValueError; this env is left untouched
                        atomicOr(a.error, 1);
                    } else {
                        e = (int64_t)ne;
                        nst = a.n_steps[ne] + 1;  // :123
#pragma unroll
                        for (int k = 0; k < W; ++k) o0[k] = s[k];  // :133 observation before the update
                        to_plane<W>(P, s);
                        if constexpr (FAST >= 1) {
                            uint32_t m[2] = {0x01010101u, 0x01010101u};  // unused cubes: never zero
                            for (int32_t h = 0; h < H; ++h) {
                                const uint32_t c = cube_mismatch<W>(s, cubes + (uint64_t)h * 2 * W);
                                const uint32_t sh = 8u * (uint32_t)(h & 3);
                                m[h >> 2] = (m[h >> 2] & ~(0xFFu << sh)) | (c << sh);
                            }
                            m_lo = m[0];
                            m_hi = m[1];
                            hit0 = (has_zero_byte(m_lo) | has_zero_byte(m_hi)) != 0u;
                        } else {
                            hit0 = attracting<W>(o0, cubes, H);
                        }
                        used = 0;
                        capped = false;
                        if constexpr (REPLAY) {
                            dpos = a.draw_off[ne];
                            dend = a.draw_off[ne + 1];
                        }
                    }
                }
            }
        }
        const uint64_t act = __ballot(e >= 0);
        if (act == 0) {
            if (__ballot(!exhausted) == 0) break;
            continue;
        }
        uint16_t* gbuf = nullptr;
        if constexpr (FAST == 2) {
            // ---- cooperative draw generation for the next ENV_CHUNK updates of every active lane
            uint8_t* gw = lds + a.off_gen + (threadIdx.x >> 6) * ENV_GEN_WAVE_BYTES;
            gbuf = reinterpret_cast<uint16_t*>(gw);                                   // [ENV_CHUNK][64]
            uint8_t* lane_of_rank = gw + ENV_CHUNK * 128;                             // [64]
            uint32_t* used_tab = reinterpret_cast<uint32_t*>(gw + ENV_CHUNK * 128 + 64);  // [64]
            uint64_t* gid_tab = reinterpret_cast<uint64_t*>(gw + ENV_CHUNK * 128 + 64 + 256);  // [64]
            const uint32_t nact = (uint32_t)__popcll(act);
            if (e >= 0) {
                lane_of_rank[__popcll(act & ((1ull << lane) - 1ull))] = (uint8_t)lane;
                used_tab[lane] = used;
                gid_tab[lane] = a.env_base + (uint64_t)e;
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            const uint32_t total = nact * ENV_CHUNK;
            // k / nact as a multiply-high by ceil(2^32 / nact): exact for k < 2^16 (nact == 1 handled apart,
            // its multiplier 2^32 does not fit 32 bits)
            const uint32_t magic = nact > 1 ? (uint32_t)((0x100000000ull + nact - 1) / nact) : 0u;
            for (uint32_t k0 = 0; k0 < total; k0 += 64) {
                const uint32_t k = k0 + lane;
                if (k < total) {
                    const uint32_t sl = nact > 1 ? __umulhi(k, magic) : k, r = k - sl * nact;
                    const uint32_t t = lane_of_rank[r];
                    uint32_t w[4];
                    philox_draw(a.seed, used_tab[t] + sl, a.call_idx, gid_tab[t], STREAM_ENV, w);
                    const uint32_t i = philox_node<KIND>(w[0], N);
                    const uint32_t j = predictor_choice(i, k53_of(w[1], w[2]), lds, a.L);
                    gbuf[sl * 64 + t] = (uint16_t)(i | (j << 9));
                }
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        }
        if (e < 0) continue;

        // ---- up to ENV_CHUNK updates of this lane's env
        const uint64_t g = a.env_base + (uint64_t)e;
        bool done = false;
        if constexpr (FAST == 2) {
            const uint64_t* recs = reinterpret_cast<const uint64_t*>(lds + a.L.off_rec);
            // branch-free per lane: a lane that is done keeps iterating masked (no break, so
            // no per-lane exit bookkeeping); the wave leaves the chunk when no lane is active
            bool act = true;
            for (uint32_t c = 0; c < ENV_CHUNK; ++c) {
                const bool cap_now = used >= a.update_cap;
                capped |= act && cap_now;
                act = act && !cap_now;
                const uint32_t ent = act ? (uint32_t)gbuf[c * 64 + lane] : 0u;
                const uint32_t i = ent & 0x1FFu;
                const uint64_t rec = recs[i * a.L.pmax + (ent >> 9)];
                const uint32_t d = i >> 5, sh = i & 31u;
                const uint32_t self = P.get(d);
                const uint32_t y = predictor_apply(P, i, self, rec);
                const uint32_t nv = (self & ~(1u << sh)) | (y << sh);
                if (act) P.put(d, nv);
                used += act ? 1u : 0u;
                const uint2 nd = ndelta[i];
                const bool changed = act && nv != self;
                m_lo += changed ? (y ? nd.x : 0u - nd.x) : 0u;
                m_hi += changed ? (y ? nd.y : 0u - nd.y) : 0u;
                const bool hit = act && ((used == 1 && !a.first_tested)
                                             ? hit0 : (has_zero_byte(m_lo) | has_zero_byte(m_hi)) != 0u);
                act = act && !hit;
                if (__ballot(act) == 0) break;
            }
            done = !act;
        } else
        for (uint32_t c = 0; c < ENV_CHUNK; ++c) {
            if (used >= a.update_cap) {
                capped = true;
                done = true;
                break;
            }
            uint32_t i;
            uint64_t k53;
            if constexpr (REPLAY) {
                if (dpos >= dend) {
                    capped = true;
                    done = true;
                    break;
                }
                i = a.draws_i[dpos];
                k53 = a.draws_k[dpos];
                ++dpos;
            } else {
                uint32_t w[4];
                philox_draw(a.seed, used, a.call_idx, g, STREAM_ENV, w);
                i = philox_node<KIND>(w[0], N);
                k53 = k53_of(w[1], w[2]);
            }
            uint32_t changed;
            if constexpr (KIND == KIND_PREDICTOR_MIX)
                changed = predictor_update_lds(P, i, k53, lds, a.L);
            else
                changed = table_update_lds(P, i, k53, lds, a.L);
            ++used;
            bool hit;
            if constexpr (FAST == 1) {
                const uint2 d = ndelta[i];
                const uint32_t y = P.bit(i);
                const uint32_t dl = changed ? (y ? d.x : 0u - d.x) : 0u;
                const uint32_t dh = changed ? (y ? d.y : 0u - d.y) : 0u;
                m_lo += dl;
                m_hi += dh;
                // :134 the first update is never tested: the check at used == 1 is on o0
                hit = (used == 1 && !a.first_tested) ? hit0 : (has_zero_byte(m_lo) | has_zero_byte(m_hi)) != 0u;
            } else {
                hit = (used == 1) ? (a.first_tested ? attracting_plane<W>(P, cubes, H) : hit0)
                                  : ((changed || used == 2) && attracting_plane<W>(P, cubes, H));
            }
            if (hit) {
                done = true;
                break;
            }
        }
        if (!done) continue;

        // ---- finish: outputs of step() (:148-154)
        uint64_t s[W];
        from_plane<W>(P, s);
        uint64_t o[W];
#pragma unroll
        for (int k = 0; k < W; ++k) o[k] = (used <= 1 && !a.first_tested) ? o0[k] : s[k];
        const uint64_t eu = (uint64_t)e;
        store_state<W>(a.state + eu * W, s);
        store_state<W>(a.obs + eu * W, o);
        a.n_steps[eu] = nst;
        const bool term = cube_match<W>(o, target);  // :190-199 (target[0] only)
        a.reward[eu] = (term ? a.reward_success : 0) - a.action_cost * n_act;  // :218-222
        a.flags[eu] = (uint8_t)((term ? 1 : 0) | (nst == a.horizon ? 2 : 0) | (capped ? 4 : 0));
        a.n_updates[eu] = used;
        e = -1;
    }
}

// ------------------------------------------------------------------ dispatch
template <int W, int KIND>
static void* step_fn(int store, int replay, int sb) {
    if (replay) return (void*)k_step<W, KIND, STORE_FULL, 1, BLOCK>;
    if (sb == 1024)
        return store == STORE_DIRTY ? (void*)k_step<W, KIND, STORE_DIRTY, 0, 1024>
                                    : (void*)k_step<W, KIND, STORE_FULL, 0, 1024>;
    return store == STORE_DIRTY ? (void*)k_step<W, KIND, STORE_DIRTY, 0, BLOCK>
                                : (void*)k_step<W, KIND, STORE_FULL, 0, BLOCK>;
}

template <int KIND>
static void* step_fn_w(int W, int store, int replay, int sb) {
    switch (W) {
        case 1: return step_fn<1, KIND>(store, replay, sb);
        case 2: return step_fn<2, KIND>(store, replay, sb);
        case 3: return step_fn<3, KIND>(store, replay, sb);
        case 4: return step_fn<4, KIND>(store, replay, sb);
        case 5: return step_fn<5, KIND>(store, replay, sb);
        case 6: return step_fn<6, KIND>(store, replay, sb);
        case 7: return step_fn<7, KIND>(store, replay, sb);
        case 8: return step_fn<8, KIND>(store, replay, sb);
    }
    return nullptr;
}

template <int KIND>
static void* env_fn_w(int W, int replay, int fast) {
#define PBN_ENV_CASE(w)                                                                  \
    case w:                                                                              \
        if (fast == 2 && KIND == KIND_PREDICTOR_MIX && !replay) return (void*)k_env<w, KIND_PREDICTOR_MIX, 0, 2>; \
        if (fast) return replay ? (void*)k_env<w, KIND, 1, 1> : (void*)k_env<w, KIND, 0, 1>; \
        return replay ? (void*)k_env<w, KIND, 1, 0> : (void*)k_env<w, KIND, 0, 0>;
    switch (W) {
        PBN_ENV_CASE(1)
        PBN_ENV_CASE(2)
        PBN_ENV_CASE(3)
        PBN_ENV_CASE(4)
        PBN_ENV_CASE(5)
        PBN_ENV_CASE(6)
        PBN_ENV_CASE(7)
        PBN_ENV_CASE(8)
    }
#undef PBN_ENV_CASE
    return nullptr;
}

static void* init_fn(int W) {
    switch (W) {
        case 1: return (void*)k_init<1>;
        case 2: return (void*)k_init<2>;
        case 3: return (void*)k_init<3>;
        case 4: return (void*)k_init<4>;
        case 5: return (void*)k_init<5>;
        case 6: return (void*)k_init<6>;
        case 7: return (void*)k_init<7>;
        case 8: return (void*)k_init<8>;
    }
    return nullptr;
}

static void* flip_fn(int W) {
    switch (W) {
        case 1: return (void*)k_flip<1>;
        case 2: return (void*)k_flip<2>;
        case 3: return (void*)k_flip<3>;
        case 4: return (void*)k_flip<4>;
        case 5: return (void*)k_flip<5>;
        case 6: return (void*)k_flip<6>;
        case 7: return (void*)k_flip<7>;
        case 8: return (void*)k_flip<8>;
    }
    return nullptr;
}

static int launch(void* fn, int grid, uint32_t lds, void* stream, void* args, size_t args_size) {
    if (!fn) return (int)hipErrorInvalidValue;
    (void)args_size;
    void* kargs[] = {args};
    return (int)hipLaunchKernel(fn, dim3((unsigned)grid), dim3(BLOCK), kargs, lds, (hipStream_t)stream);
}

uint32_t step_lds_bytes(int W, uint32_t image_bytes, int sb) {
    return image_bytes + 8u * (uint32_t)W * (uint32_t)sb;
}

static void* step_kernel(int W, int kind, int store_mode, int replay, int sb) {
    if (replay) sb = BLOCK;
    return kind == KIND_PREDICTOR_MIX ? step_fn_w<KIND_PREDICTOR_MIX>(W, store_mode, replay, sb)
                                      : step_fn_w<KIND_PROB_TABLE>(W, store_mode, replay, sb);
}

int launch_step(int W, const StepArgs& a, int store_mode, int replay, int sb, int grid, void* stream) {
    if (replay) sb = BLOCK;
    void* fn = step_kernel(W, a.L.kind, store_mode, replay, sb);
    if (!fn) return (int)hipErrorInvalidValue;
    const uint32_t lds = step_lds_bytes(W, a.L.bytes, sb);
    if (lds > 64u * 1024u) {
        hipError_t e = hipFuncSetAttribute((const void*)fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) return (int)e;
    }
    StepArgs c = a;
    void* kargs[] = {&c};
    return (int)hipLaunchKernel(fn, dim3((unsigned)grid), dim3((unsigned)sb), kargs, lds, (hipStream_t)stream);
}

int launch_init(int W, const InitArgs& a, int grid, void* stream) {
    InitArgs c = a;
    return launch(init_fn(W), grid, 0, stream, &c, sizeof c);
}

int launch_flip(int W, const FlipArgs& a, int grid, void* stream) {
    FlipArgs c = a;
    return launch(flip_fn(W), grid, 0, stream, &c, sizeof c);
}

int launch_env_multi(int W, const EnvArgs& a, int replay, int grid, void* stream) {
    void* fn = a.L.kind == KIND_PREDICTOR_MIX ? env_fn_w<KIND_PREDICTOR_MIX>(W, replay, a.fast)
                                              : env_fn_w<KIND_PROB_TABLE>(W, replay, a.fast);
    EnvArgs c = a;
    return launch(fn, grid, env_lds_bytes(W, a.L.bytes, replay ? std::min(a.fast, 1) : a.fast), stream, &c, sizeof c);
}

static int occupancy(void* fn, int block, uint32_t lds, int* blocks_per_cu) {
    int nb = 0;
    if (lds > 64u * 1024u) {
        hipError_t e = hipFuncSetAttribute((const void*)fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) return (int)e;
    }
    hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, (const void*)fn, block, lds);
    if (e != hipSuccess) return (int)e;
    *blocks_per_cu = nb < 1 ? 1 : nb;
    return 0;
}

int max_blocks_step(int W, int kind, uint32_t lds_bytes, int sb, int* blocks_per_cu) {
    void* fn = step_kernel(W, kind, STORE_FULL, 0, sb);
    return occupancy(fn, sb, step_lds_bytes(W, lds_bytes, sb), blocks_per_cu);
}

uint32_t env_lds_bytes(int W, uint32_t image_bytes, int fast) {
    const uint32_t planes = image_bytes + 8u * (uint32_t)W * BLOCK;
    return fast == 2 ? planes + (BLOCK / 64) * ENV_GEN_WAVE_BYTES : planes;
}

int max_blocks_env(int W, int kind, int fast, uint32_t lds_bytes, int* blocks_per_cu) {
    void* fn = kind == KIND_PREDICTOR_MIX ? env_fn_w<KIND_PREDICTOR_MIX>(W, 0, fast)
                                          : env_fn_w<KIND_PROB_TABLE>(W, 0, fast);
    return occupancy(fn, BLOCK, env_lds_bytes(W, lds_bytes, fast), blocks_per_cu);
}

}  // namespace pbn
