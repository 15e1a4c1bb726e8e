// pbn_kernels.hip -- gfx950 kernels of the vectorised PBN simulator.
//
// Mapping: one lane owns one env at a time; its state words are loaded into VGPRs and, for the
// node update, spread over the lane's column of LDS state planes. Each workgroup stages the
// network image (thresholds, predictor records or probability tables) into LDS once. Step mode
// (the bench kernel, k_step<.., 1024>): 1024-thread workgroups, two per CU, every thread owning
// one pair of envs (e, e + grid stride) at 1M envs (more pairs per thread, grid-stride, above);
// rollout / R6 / SSD kernels: 256-thread workgroups sized to what is resident, lanes refilled
// from a work counter (R6) or walking envs in a grid-stride loop.
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

#ifdef PBN_STAMPS
// Measurement builds only (tools/build_exp.sh -DPBN_STAMPS): per-wave s_memrealtime stamps (100 MHz)
// of the step kernel's phases, kept in registers and written once at the end of the wave.
__device__ uint64_t g_stamps[16384 * 8];
// k_env (cooperative-draw path): per wave, ENV_STAMPS words (tools/env_stamps.py reads them)
constexpr int ENV_STAMPS = 40;
__device__ uint64_t g_env_stamps[16384 * ENV_STAMPS];
#endif

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
template <int W, int KIND, int STORE, int SB, bool PRE = false>
__device__ __forceinline__ void k_step_single(const StepArgs& a, uint8_t* lds, uint64_t e, uint64_t stride,
                                              uint64_t (&cur)[W], uint32_t N, uint64_t (*pre_nxt)[W] = nullptr) {
    // graph replays read the batch's update counter from device memory (k_bump advances it)
    const uint64_t u = a.update_base + (a.ubase_dev ? *a.ubase_dev : 0ull);
    const uint64_t po = stride;  // second env of the pair (adjacent envs measured slower: 8.2 vs 7.8 us)
    uint64_t nxt[W];
    uint32_t i0 = 0, i1 = 0;
    uint64_t q0 = 0, q1 = 0;
    // envs 2m / 2m + 1 share a Philox call (pbn_device.hpp): with an even env base, lane parity is
    // env parity and the lane pair computes one call per env pair each (step_words_paired). A
    // partner lane that has left the loop holds envs >= B only, so the words it no longer sends
    // belong to envs that are not applied.
    const bool paired = (a.env_base & 1u) == 0u;
    const bool odd = (threadIdx.x & 1u) != 0u;
    auto draws = [&](uint64_t ea) {
        const uint64_t g0 = a.env_base + ea, g1 = g0 + po;
        uint32_t n0, c0, n1, c1;
        if (paired) {
            step_words_paired(a.seed, u, g0, g1, odd, n0, c0, n1, c1);
        } else {
            step_words(a.seed, u, g0, n0, c0);
            step_words(a.seed, u, g1, n1, c1);
        }
        i0 = philox_node<KIND>(n0, N);
        i1 = philox_node<KIND>(n1, N);
        // predictor mix: the choice word itself (compact image, thresholds on the word); tables: k53
        q0 = KIND == KIND_PREDICTOR_MIX ? (uint64_t)c0 : u32_k53(c0);
        q1 = KIND == KIND_PREDICTOR_MIX ? (uint64_t)c1 : u32_k53(c1);
    };
#ifdef PBN_STAMPS
    uint64_t st[8] = {__builtin_amdgcn_s_memrealtime(), 0, 0, 0, 0, 0, 0, 0};
#endif
    const Thr32 X = thr32_layout(a.L);
    if constexpr (PRE) {  // image staged and both loads issued by the caller (k_step)
#pragma unroll
        for (int k = 0; k < W; ++k) nxt[k] = (*pre_nxt)[k];
        draws(e);
#ifdef PBN_STAMPS
        st[2] = st[0];  // the caller's barrier was passed on entry here
        st[1] = __builtin_amdgcn_s_memrealtime();
#endif
    } else {
    if (e + po < a.B) load_state<W>(a.state + (e + po) * W, nxt);
    draws(e);
#ifdef PBN_STAMPS
    st[1] = __builtin_amdgcn_s_memrealtime();
#endif
    if constexpr (KIND == KIND_PREDICTOR_MIX)  // the compact image (thresholds on the choice word)
        stage_image(reinterpret_cast<const uint4*>(reinterpret_cast<const uint8_t*>(a.img) + a.L.bytes), X.bytes / 16,
                    reinterpret_cast<uint4*>(lds));
    else
        stage_image(reinterpret_cast<const uint4*>(a.img), a.L.bytes / 16, reinterpret_cast<uint4*>(lds));
    __syncthreads();
    }
#ifdef PBN_STAMPS
    st[2] = __builtin_amdgcn_s_memrealtime();
#endif
    const PlaneT<SB> P{reinterpret_cast<uint32_t*>(lds + a.L.plane_off) + threadIdx.x};
    while (e < a.B) {
        const uint64_t e1 = e + po;
        uint64_t r0 = 0, r1 = 0;
        if constexpr (KIND == KIND_PREDICTOR_MIX) {  // state-independent: before the loads land
            r0 = predictor_record32(i0, (uint32_t)q0, lds, X);
            r1 = predictor_record32(i1, (uint32_t)q1, lds, X);
        }
#ifdef PBN_STAMPS
        if (!st[3]) {
            __builtin_amdgcn_s_waitcnt(0);  // records read and state landed (measurement build)
            st[3] = __builtin_amdgcn_s_memrealtime();
        }
#endif
        if constexpr (STORE == STORE_DIRTY) {
            // Both envs evaluated first (plane writes and reads of env 1 issued right behind env 0's;
            // LDS runs a wave's operations in order, so reusing the column needs no wait), then both
            // stores: with env 0's store issued before env 1's loads were consumed, the compiler
            // waited for that store to complete (vmcnt(0)) before env 1's plane writes.
            // Env 1 is evaluated unconditionally (past B: junk from a clamped or skipped load,
            // never stored).
            // the plane's last dword holds nodes >= 64W - 32 only: it is written only if N reaches it
            // (Bittner-200: 7 of the 8 dwords, one LDS write of eight saved per env)
            const bool last_dw = N > 64u * W - 32u;
            auto eval = [&](const uint64_t (&s)[W], uint32_t i, uint64_t r, uint64_t q, uint32_t& self) {
#pragma unroll
                for (int k = 0; k < W; ++k) {
                    P.put(2 * k, (uint32_t)s[k]);
                    if (k + 1 < W || last_dw) P.put(2 * k + 1, (uint32_t)(s[k] >> 32));
                }
                self = P.get(i >> 5);
                if constexpr (KIND == KIND_PREDICTOR_MIX)
                    return predictor_apply(P, i, self, r);
                else
                    return table_eval_lds(P, i, q, lds, a.L);
            };
            uint32_t self0, self1;
            const uint32_t y0 = eval(cur, i0, r0, q0, self0);
            const uint32_t y1 = eval(nxt, i1, r1, q1, self1);
            // store the whole env (32 B at W = 4), and only if its bit changed: a full aligned env
            // write measured faster than writing just the 16-B half that holds node i (7.69 vs
            // 7.93 us at 1M envs), partial sector writes cost extra. The env's words are still in
            // registers: bit i is flipped there (one 64-bit select per word) rather than written to
            // the plane and all 2W dwords read back
            auto put = [&](const uint64_t (&s)[W], uint64_t eh, uint32_t i) {
                uint64_t out[W];
                const uint32_t wi = i >> 6;
                const uint64_t m = 1ull << (i & 63u);
#pragma unroll
                for (int k = 0; k < W; ++k) out[k] = s[k] ^ ((uint32_t)k == wi ? m : 0ull);
                store_state<W>(a.state + eh * W, out);
            };
            if (((self0 >> (i0 & 31u)) & 1u) != y0) put(cur, e, i0);
            if (e1 < a.B && ((self1 >> (i1 & 31u)) & 1u) != y1) put(nxt, e1, i1);
        } else {
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
            P.put(d, nv);
            uint64_t out[W];
            from_plane<W>(P, out);
            store_state<W>(a.state + eh * W, out);
        }
        }
#ifdef PBN_STAMPS
        if (!st[4]) st[4] = __builtin_amdgcn_s_memrealtime();  // the first pair's stores issued
#endif
        e += 2 * stride;
        if (e < a.B) {
            load_state<W>(a.state + e * W, cur);
            if (e + po < a.B) load_state<W>(a.state + (e + po) * W, nxt);
            draws(e);
        }
    }
#ifdef PBN_STAMPS
    __builtin_amdgcn_s_waitcnt(0);
    st[5] = __builtin_amdgcn_s_memrealtime();  // every store of the wave done
    const uint32_t wv = blockIdx.x * (SB / 64) + threadIdx.x / 64;
    if ((threadIdx.x & 63) == 0 && wv < 16384) {
        st[6] = blockIdx.x;
        st[7] = __smid();
        for (int k = 0; k < 8; ++k) g_stamps[wv * 8 + k] = st[k];
    }
#endif
}

// The bench shape: every thread owns exactly one env pair (B <= 2 x grid x SB), image staged and both
// loads issued by k_step. Straight-line, so both envs' threshold rows are read in one LDS round trip
// and both records in a second (the looped form read env 0's row, its record, env 1's row, its
// record: three dependent round trips, the uniform tp4 == 4 branch between them), and env 0's plane
// work waits only for env 0's loads.
template <int W, int SB>
__device__ __forceinline__ void k_step_pair(const StepArgs& a, uint8_t* lds, uint64_t e, uint64_t stride,
                                            const uint64_t (&cur)[W], const uint64_t (&nxt)[W], uint32_t N) {
    const uint64_t u = a.update_base + (a.ubase_dev ? *a.ubase_dev : 0ull);
    const uint64_t e1 = e + stride, g0 = a.env_base + e, g1 = g0 + stride;
    uint32_t n0, c0, n1, c1;
    if ((a.env_base & 1u) == 0u) {  // envs 2m / 2m + 1 share a Philox call (k_step_single)
        step_words_paired(a.seed, u, g0, g1, (threadIdx.x & 1u) != 0u, n0, c0, n1, c1);
    } else {
        step_words(a.seed, u, g0, n0, c0);
        step_words(a.seed, u, g1, n1, c1);
    }
    const uint32_t i0 = philox_node<KIND_PREDICTOR_MIX>(n0, N), i1 = philox_node<KIND_PREDICTOR_MIX>(n1, N);
    const Thr32 X = thr32_layout(a.L);
    uint32_t j0, j1;
    if (X.tp4 == 4u) {
        const uint4 t0 = reinterpret_cast<const uint4*>(lds)[i0];
        const uint4 t1 = reinterpret_cast<const uint4*>(lds)[i1];
        j0 = (c0 >= t0.x ? 1u : 0u) + (c0 >= t0.y ? 1u : 0u) + (c0 >= t0.z ? 1u : 0u) + (c0 >= t0.w ? 1u : 0u);
        j1 = (c1 >= t1.x ? 1u : 0u) + (c1 >= t1.y ? 1u : 0u) + (c1 >= t1.z ? 1u : 0u) + (c1 >= t1.w ? 1u : 0u);
    } else {
        j0 = predictor_choice32(i0, c0, lds, X.tp4);
        j1 = predictor_choice32(i1, c1, lds, X.tp4);
    }
    const uint64_t* rec = reinterpret_cast<const uint64_t*>(lds + X.rec_off);
    const uint64_t r0 = rec[__umul24(i0, X.rs) + j0], r1 = rec[__umul24(i1, X.rs) + j1];
    const PlaneT<SB> P{reinterpret_cast<uint32_t*>(lds + a.L.plane_off) + threadIdx.x};
    const bool last_dw = N > 64u * W - 32u;  // the plane's last dword holds nodes >= 64W - 32 only
    auto eval = [&](const uint64_t (&s)[W], uint32_t i, uint64_t r, uint32_t& self) {
#pragma unroll
        for (int k = 0; k < W; ++k) {
            P.put(2 * k, (uint32_t)s[k]);
            if (k + 1 < W || last_dw) P.put(2 * k + 1, (uint32_t)(s[k] >> 32));
        }
        self = P.get(i >> 5);
        return predictor_apply(P, i, self, r);
    };
    auto put = [&](const uint64_t (&s)[W], uint64_t eh, uint32_t i) {  // whole env, bit i flipped
        uint64_t out[W];
        const uint32_t wi = i >> 6;
        const uint64_t m = 1ull << (i & 63u);
#pragma unroll
        for (int k = 0; k < W; ++k) out[k] = s[k] ^ ((uint32_t)k == wi ? m : 0ull);
        store_state<W>(a.state + eh * W, out);
    };
    uint32_t self0, self1;
    const uint32_t y0 = eval(cur, i0, r0, self0);
    // env 0 is stored before env 1 is evaluated; env 1's loads (issued right behind env 0's) are waited
    // for first: after a store that may not have been issued, the compiler can only wait vmcnt(0)
#pragma unroll
    for (int k = 0; k < W; ++k) asm volatile("" ::"v"(nxt[k]));
    if (e < a.B && ((self0 >> (i0 & 31u)) & 1u) != y0) put(cur, e, i0);
    const uint32_t y1 = eval(nxt, i1, r1, self1);  // past B: junk from a clamped load, never stored
    if (e1 < a.B && ((self1 >> (i1 & 31u)) & 1u) != y1) put(nxt, e1, i1);
}

// Step mode (T == 1, Philox; REPLAY == 0) and replay mode (REPLAY == 1: T updates from the
// caller's draws). Rollout (T > 1, Philox) is its own kernel, k_rollout, so that neither
// path's code shapes the other's register allocation and schedule (sharing one kernel cost
// the step path 0.6 us per launch at 1M envs).
template <int W, int KIND, int STORE, int REPLAY, int SB>
// 1024-thread groups, W <= 4: two workgroups per CU = 8 waves per SIMD, so at most 64 VGPRs (every
// instance this bound applies to -- both kinds, both store modes, Philox only: SB = 1024 is never
// launched in replay mode -- compiles without scratch, `make asm`; the stamps build keeps the bound)
__global__ __launch_bounds__(SB, (SB == 1024 && W <= 4) ? 8 : 1)
void k_step(StepArgs a) {
    extern __shared__ __align__(16) uint8_t lds[];
    const uint64_t stride = (uint64_t)gridDim.x * SB;
    uint64_t e = (uint64_t)blockIdx.x * SB + threadIdx.x;
    const uint32_t N = (uint32_t)a.L.n_nodes;
    uint64_t cur[W];
    if constexpr (!REPLAY && KIND == KIND_PREDICTOR_MIX && SB == 1024) {
        // The image's granule (one per thread) is loaded first, then both envs of the pair
        // (unconditional loads, clamped addresses, so the granule's wait counts only itself:
        // vmcnt(4)); the granule is written and the barrier passed while the state is in flight,
        // and the draws follow the barrier. Staged after the draws instead, the barrier waited
        // for every wave's Philox burst and the state loads: 9.21 -> 8.98 us per launch at 1M envs
        // (profiles/r02_step_stage_first_ab.txt; phase stamps r02_step_stamps.json)
        const Thr32 X = thr32_layout(a.L);
        const uint4* src = reinterpret_cast<const uint4*>(reinterpret_cast<const uint8_t*>(a.img) + a.L.bytes);
        const uint32_t n16 = X.bytes / 16;
        uint4 g = make_uint4(0, 0, 0, 0);
        if (threadIdx.x < n16) g = src[threadIdx.x];
        uint64_t nx[W];
        const uint64_t ec = e < a.B ? e : 0, en = e + stride < a.B ? e + stride : 0;
        load_state<W>(a.state + ec * W, cur);
        load_state<W>(a.state + en * W, nx);
        if (threadIdx.x < n16) reinterpret_cast<uint4*>(lds)[threadIdx.x] = g;
        for (uint32_t k = threadIdx.x + SB; k < n16; k += SB) reinterpret_cast<uint4*>(lds)[k] = src[k];
        __syncthreads();
        if (STORE == STORE_DIRTY && 2u * stride >= a.B)
            k_step_pair<W, SB>(a, lds, e, stride, cur, nx, N);  // one pair per thread (the bench shape)
        else
            k_step_single<W, KIND, STORE, SB, true>(a, lds, e, stride, cur, N, &nx);
        return;
    }
    if (e < a.B) load_state<W>(a.state + e * W, cur);
    if constexpr (!REPLAY) {
        // Step mode: the draws depend on (seed, update counter, env id) only, so every
        // draw this thread needs is computed while its state loads are in flight.
        k_step_single<W, KIND, STORE, SB>(a, lds, e, stride, cur, N);
    } else {
        stage_image(reinterpret_cast<const uint4*>(a.img), a.L.bytes / 16, reinterpret_cast<uint4*>(lds));
        __syncthreads();
        const PlaneT<SB> P{reinterpret_cast<uint32_t*>(lds + a.L.bytes) + threadIdx.x};
        while (e < a.B) {
            const uint64_t en = e + stride;
            uint64_t nxt[W];
            if (en < a.B) load_state<W>(a.state + en * W, nxt);  // prefetch the next env
            to_plane<W>(P, cur);
            for (uint32_t t = 0; t < a.T; ++t) {
                const uint32_t i = a.replay_node[(uint64_t)t * a.B + e];
                uint64_t k53;
                if (a.replay_k53) {
                    k53 = a.replay_k53[(uint64_t)t * a.B + e];
                } else {
                    // forced node (Graph.step(i=k), base.py:306-308): the node is the caller's, the
                    // choice word is the env's own Philox step draw of update update_base + t
                    uint32_t wn, wc;
                    step_words(a.seed, a.update_base + t, a.env_base + e, wn, wc);
                    k53 = u32_k53(wc);
                }
                if constexpr (KIND == KIND_PREDICTOR_MIX)
                    predictor_update_lds(P, i, k53, lds, a.L);
                else
                    table_update_lds(P, i, k53, lds, a.L);
            }
            uint64_t out[W];
            from_plane<W>(P, out);
            store_state<W>(a.state + e * W, out);
#pragma unroll
            for (int k = 0; k < W; ++k) cur[k] = nxt[k];
            e = en;
        }
    }
}

// Rollout: T Philox updates per env per launch with the env's state in its LDS plane column;
// the state is read once and written once (only if it changed).
template <int W, int KIND, int SB>
__global__ __launch_bounds__(SB) void k_rollout(StepArgs a) {
    extern __shared__ __align__(16) uint8_t lds[];
    const uint64_t stride = (uint64_t)gridDim.x * SB;
    uint64_t e = (uint64_t)blockIdx.x * SB + threadIdx.x;
    const uint32_t N = (uint32_t)a.L.n_nodes;
    uint64_t cur[W];
    if (e < a.B) load_state<W>(a.state + e * W, cur);
    const Thr32 X = thr32_layout(a.L);
    if constexpr (KIND == KIND_PREDICTOR_MIX)  // the compact image (thresholds on the choice word)
        stage_image(reinterpret_cast<const uint4*>(reinterpret_cast<const uint8_t*>(a.img) + a.L.bytes), X.bytes / 16,
                    reinterpret_cast<uint4*>(lds));
    else
        stage_image(reinterpret_cast<const uint4*>(a.img), a.L.bytes / 16, reinterpret_cast<uint4*>(lds));
    __syncthreads();
    const PlaneT<SB> P{reinterpret_cast<uint32_t*>(lds + a.L.plane_off) + threadIdx.x};
    // Envs 2m / 2m + 1 share their Philox calls (pbn_device.hpp). With an even env base the lane
    // pair holds such a pair, and for updates t, t + 1 the even lane computes the call of t, the
    // odd lane that of t + 1, and they swap the two words the other needs: one call per lane
    // per two updates. Every lane of a wave takes the same trips (lanes past B compute junk
    // and store nothing), so a partner is never missing.
    const bool paired = (a.env_base & 1u) == 0u;
    const bool odd = (threadIdx.x & 1u) != 0u;
    for (;;) {
        const bool live = e < a.B;
        if (__ballot(live) == 0) break;
        const uint64_t en = e + stride;
        uint64_t nxt[W];
        if (en < a.B) load_state<W>(a.state + en * W, nxt);  // prefetch the next env
        to_plane<W>(P, cur);
        uint32_t changed = 0;
        const uint64_t g = a.env_base + e;
        // node / choice words of updates t and t + 1 of this lane's env
        auto words2 = [&](uint32_t t, uint32_t& na, uint32_t& ca, uint32_t& nb, uint32_t& cb) {
            const uint64_t u = a.update_base + t;
            if (paired) {
                uint32_t w[4];
                philox_draw(a.seed, (uint32_t)(u + (odd ? 1u : 0u)), (uint32_t)((u + (odd ? 1u : 0u)) >> 32), g >> 1,
                            STREAM_STEP, w);
                const uint32_t r0 = swap_pair_lanes(odd ? w[0] : w[2]), r1 = swap_pair_lanes(odd ? w[1] : w[3]);
                na = odd ? r0 : w[0];
                ca = odd ? r1 : w[1];
                nb = odd ? w[2] : r0;
                cb = odd ? w[3] : r1;
            } else {
                step_words(a.seed, u, g, na, ca);
                step_words(a.seed, u + 1u, g, nb, cb);
            }
        };
        if constexpr (KIND == KIND_PREDICTOR_MIX) {
            // software pipeline: the draws and predictor records of updates t + 2, t + 3
            // (state-independent) are computed while updates t, t + 1 run -- one env per lane
            // leaves a wave alone on its SIMD at small batches (65,536 envs: one wave per SIMD)
            uint32_t ia, ib;
            uint64_t ra, rb;
            auto draw2 = [&](uint32_t t) {
                uint32_t na, ca, nb, cb;
                words2(t, na, ca, nb, cb);
                ia = philox_node<KIND>(na, N);
                ib = philox_node<KIND>(nb, N);
                ra = predictor_record32(ia, ca, lds, X);
                rb = predictor_record32(ib, cb, lds, X);
            };
            auto apply = [&](uint32_t i, uint64_t rec) {
                const uint32_t d = i >> 5, sh = i & 31u;
                const uint32_t self = P.get(d);
                const uint32_t y = predictor_apply(P, i, self, rec);
                const uint32_t nv = (self & ~(1u << sh)) | (y << sh);
                P.put(d, nv);
                changed |= nv != self;
            };
            draw2(0);
            for (uint32_t t = 0; t < a.T; t += 2) {
                const uint32_t i0 = ia, i1 = ib;
                const uint64_t r0 = ra, r1 = rb;
                draw2(t + 2);  // unconditional (past T: junk, unused): no branch before the plane reads
                apply(i0, r0);
                if (t + 1 < a.T) apply(i1, r1);
            }
        } else {
            for (uint32_t t = 0; t < a.T; t += 2) {
                uint32_t na, ca, nb, cb;
                words2(t, na, ca, nb, cb);
                changed |= table_update_lds(P, philox_node<KIND>(na, N), u32_k53(ca), lds, a.L);
                if (t + 1 < a.T) changed |= table_update_lds(P, philox_node<KIND>(nb, N), u32_k53(cb), lds, a.L);
            }
        }
        uint64_t out[W];
        from_plane<W>(P, out);
        bool diff = false;  // whole env, only if it differs (see k_step_single)
#pragma unroll
        for (int k = 0; k < W; ++k) diff |= out[k] != cur[k];
        if (live && changed && diff) store_state<W>(a.state + e * W, out);
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
// GEN (FAST == 2, or 4 with <= 4 cubes: one counter word; predictor-mix networks, Philox):
// before each chunk the whole wave
// generates the chunk's draws for all its active lanes -- assignment k of
// n_active * ENV_CHUNK goes to lane k % 64 -- and stores (node, chosen predictor) as
// u16 in a per-wave LDS buffer; the lanes then only apply the records. With every lane
// active this is the same Philox work per lane; in the tail, when a few lanes run long
// (capped) loops, idle lanes generate their draws and the per-update cost drops to the
// state read/write.

__device__ __forceinline__ uint32_t has_zero_byte(uint32_t v) { return (v - 0x01010101u) & ~v & 0x80808080u; }

#ifndef PBN_ENV_OWN_DRAWS_MIN
#define PBN_ENV_OWN_DRAWS_MIN 40  // measurement builds (tools/build_exp.sh) change this
#endif
constexpr uint32_t ENV_OWN_DRAWS_MIN = PBN_ENV_OWN_DRAWS_MIN;  // active lanes from which a wave skips the shared draw tables
#ifndef PBN_HELP_SLEEP
#define PBN_HELP_SLEEP 1  // a tail helper's sleep (x 64 cycles) between polls of its ring's consumed count
#endif
constexpr uint32_t ENV_LONG_USED = 1024;  // tail mode: envs past this many updates are resolved longest-first
// grid pool (k_env): global-address-space views, so agent-scope atomics lower to global_ (not flat_) sc1 accesses
typedef __attribute__((address_space(1))) uint32_t gu32;
typedef __attribute__((address_space(1))) unsigned long long gu64;
#ifndef PBN_GPOOL_SLEEP
#define PBN_GPOOL_SLEEP 32  // a workgroup waiting on the pool sleeps this x 64 cycles between polls
#endif
#ifndef PBN_GPOOL_CHECK_TICKS
#define PBN_GPOOL_CHECK_TICKS 500  // a tail wave looks for waiting workgroups at most every 5 us (100 MHz ticks)
#endif
constexpr uint64_t GPOOL_TIMEOUT_TICKS = 200000000ull;  // 2 s: a claimed slot's words never came (error flag 2; never expected)
// a workgroup waiting on the pool this long (20 ms) without an env leaves quietly (its slot given up first), so a
// long launch does not keep idle workgroups resident (measured 3-4 % on the others) or wait on them
constexpr uint64_t GPOOL_GIVE_UP_TICKS = 2000000ull;

// ceil(2^32 / n) for n = 2..63 (0 for n < 2): k / n == umulhi(k, kRankMagic[n]) for k < 2^16
struct RankMagic {
    uint32_t v[64];
    constexpr RankMagic() : v{} {
        for (uint32_t n = 2; n < 64; ++n) v[n] = (uint32_t)((0x100000000ull + n - 1) / n);
    }
};
__constant__ constexpr RankMagic kRankMagic{};

// Inclusive prefix sum over the wave's 64 lanes (row_shr 1/2/4/8 inside each 16-lane row, then
// row_bcast15 / row_bcast31 carry the row totals; lanes without a source add 0).
// Inclusive max over the wave (the same DPP pattern; lanes without a source take 0): lane 63 holds the max.
__device__ __forceinline__ uint32_t wave_inclusive_max(uint32_t x) {
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xF, 0xF, false));
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xF, 0xF, false));
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xF, 0xF, false));
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xF, 0xF, false));
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xA, 0xF, false));
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xC, 0xF, false));
    return x;
}

__device__ __forceinline__ uint32_t wave_inclusive_add(uint32_t x) {
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xF, 0xF, false);
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xF, 0xF, false);
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xF, 0xF, false);
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xF, 0xF, false);
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xA, 0xF, false);
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xC, 0xF, false);
    return x;
}



// A wave's draw buffer (env_gen_wave_bytes(chunk)) in tail mode: the per-node 64-bit writer masks from
// byte 0 (N <= 512 nodes: 4 KiB), the hand-off flag at chunk * 128 and the hand-off box (5 + 2W words)
// 64 B after it; lane mode's draw table [chunk][64] u16 and counter table use the same bytes
static_assert(8u * 512u <= ENV_CHUNK_SMALL * 128u, "tail writer masks (N <= 512) overlap the hand-off flag");
static_assert(ENV_CHUNK_SMALL * 128u + 64u + 8u * (5u + 2u * 8u) <= env_gen_wave_bytes(ENV_CHUNK_SMALL),
              "the hand-off box (W <= 8) overflows the wave's draw buffer");
static_assert(ENV_CHUNK_SMALL % 8u == 0 && ENV_CHUNK_LARGE % 8u == 0 && ENV_UNROLL == 8u,
              "draw-round chunks: multiples of the unroll (and of 4: the own-draw iteration)");

template <int W, int KIND, int REPLAY, int FAST>
__global__ __launch_bounds__(ENV_BLOCK) __attribute__((amdgpu_waves_per_eu(4))) void k_env(EnvArgs a) {
    constexpr bool GEN = FAST == 2 || FAST == 4;
    constexpr bool ONE_WORD = FAST == 4;  // <= 4 cubes: the high counter word is never read
    constexpr bool TAIL = FAST == 4;      // wave-wide tail mode (see below)
    static_assert(!GEN || (KIND == KIND_PREDICTOR_MIX && !REPLAY), "GEN: predictor mix, Philox");
    extern __shared__ __align__(16) uint8_t lds[];
#ifdef PBN_STAMPS
    const uint64_t rt_entry = __builtin_amdgcn_s_memrealtime();
#endif
    const uint32_t N = (uint32_t)a.L.n_nodes;
    const Thr32 X = thr32_layout(a.L);
    if (GEN && a.gen_img) {
        // the host-built LDS image (pbn_abi.cpp env_gen_image): the same bytes as the construction below
        stage_image(reinterpret_cast<const uint4*>(a.gen_img), (a.L.bytes + a.erec_shift) / 16, reinterpret_cast<uint4*>(lds));
    } else if constexpr (GEN) {
        // LDS: the thresholds as staged; in place of the 8-B predictor records, 16-B "env
        // records" (EnvRec) carrying each input's plane offset and bit position, so an update
        // does no index arithmetic; the cubes / target / deltas after them move up by erec_shift
        const uint4* g = reinterpret_cast<const uint4*>(a.img);
        uint4* l = reinterpret_cast<uint4*>(lds);
        // the thresholds re-expressed on the draw word a as the compact image has them (u32, rows
        // of tp4, saturated: thr32_layout), so the choice compares a itself in one 16-B read; env
        // records in rows of rs, slot tp4 holding the record a = 2^32 - 1 selects. Staged once
        // per persistent workgroup, so this computes the conversion instead of reading the
        // compact image (the env config's image does not carry it)
        const uint64_t* gthr = reinterpret_cast<const uint64_t*>(static_cast<const uint8_t*>(a.img) + a.L.off_thr);
        const uint32_t tp = a.L.tp, tp4 = X.tp4, rs = X.rs;
        for (uint32_t k = threadIdx.x; k < N * tp4; k += ENV_BLOCK) {
            const uint32_t i = k / tp4, q = k - i * tp4;
            const uint64_t t = q < tp ? u32_threshold(gthr[i * tp + q]) : (1ull << 32);
            reinterpret_cast<uint32_t*>(lds)[k] = t >> 32 ? 0xFFFFFFFFu : (uint32_t)t;
        }
        const uint32_t tail = a.off_cubes - a.erec_shift;  // the cubes' offset in the device image
        for (uint32_t k = threadIdx.x; k < (a.L.bytes - tail) / 16; k += ENV_BLOCK)
            l[(tail + a.erec_shift) / 16 + k] = g[tail / 16 + k];
        const uint64_t* grec = reinterpret_cast<const uint64_t*>(static_cast<const uint8_t*>(a.img) + a.L.off_rec);
        uint4* erec = reinterpret_cast<uint4*>(lds + a.L.off_rec);
        for (uint32_t r = threadIdx.x; r < N * rs; r += ENV_BLOCK) {
            const uint32_t i = r / rs, q = r - i * rs;
            uint32_t src = q;
            if (q == tp4) {  // the node's thresholds below 2^32 on a (a prefix: non-decreasing)
                src = 0;
                for (uint32_t p = 0; p < tp; ++p) src += (u32_threshold(gthr[i * tp + p]) >> 32) ? 0u : 1u;
            }
            erec[r] = env_record(src < a.L.pmax ? grec[i * a.L.pmax + src] : 0ull, i, a.off_ndelta);
        }
    } else {
        stage_image(reinterpret_cast<const uint4*>(a.img), a.L.bytes / 16, reinterpret_cast<uint4*>(lds));
    }
    // workgroup hand-off (TAIL, steal_local): control words after the draw buffers (busy waves, idle
    // mask); each wave's mailbox flag sits in its own draw buffer's table region (cleared on going idle)
    // the launch's draw-round chunk (GEN) and the per-wave draw buffer it sizes
    const uint32_t CH = GEN ? a.chunk : ENV_CHUNK;
    const uint32_t GWB = env_gen_wave_bytes(CH);
    uint32_t* const wctl = reinterpret_cast<uint32_t*>(lds + a.off_gen + (ENV_BLOCK / 64) * GWB);
    // grid pool words: device memory, every access a global agent-scope atomic (sc1: past the CU's L1)
    auto gctl = [&](int k) { return (gu32*)(a.gpool_ctl + k); };
    const bool GRID = TAIL && a.steal_local && a.gpool_cap != 0u;
    if (TAIL && a.steal_local && threadIdx.x == 0) {
        wctl[0] = ENV_BLOCK / 64;  // busy
        wctl[1] = 0u;          // idle mask
        wctl[2] = 0u;          // grid pool: a wave of this workgroup is waiting on a ticket
        wctl[3] = 0u;          // grid pool: 1 the launch's work is done, leave; 2 this workgroup left its CU's count
        if (GRID) {
            // this workgroup counts as live from its start (a workgroup dispatched late counts from then: a
            // ticket holder that saw the count at 0 gave its slot up, so no env can be pushed to it), and as
            // working on its CU until it first runs out of work
            (void)__hip_atomic_fetch_add(gctl(2), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            (void)__hip_atomic_fetch_add(gctl(GPOOL_CU_WORD + __smid()), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
    }
    __syncthreads();
    const PlaneT<ENV_BLOCK> P{reinterpret_cast<uint32_t*>(lds + a.L.bytes + a.erec_shift) + threadIdx.x};
#ifdef PBN_STAMPS
    // 0 start, 1 first chunk below ENV_OWN_DRAWS_MIN active lanes, 2 first chunk after a lane of the
    // wave found the work queue empty,
    // 3/4/5/6 first chunk with <= 32 / 16 / 8 / 2 active lanes, 7 end; 8 chunks, 9 sum of active
    // lanes over chunks, 10 chunks in the tail (queue empty), 11 sum of active lanes there,
    // 12 block, 13 hw id, 14 env steps of the wave that hit the update cap
    uint64_t est[ENV_STAMPS] = {};
    uint32_t ncapped = 0;
    est[0] = __builtin_amdgcn_s_memrealtime();
    est[33] = rt_entry;  // kernel entry (before the image is staged); est[0] is after the staging barrier
#endif
    const uint64_t* cubes = reinterpret_cast<const uint64_t*>(lds + a.off_cubes);
    const uint64_t* target = reinterpret_cast<const uint64_t*>(lds + a.off_target);
    const uint2* ndelta = reinterpret_cast<const uint2*>(lds + a.off_ndelta);
    const int32_t H = a.n_cubes;
    const uint32_t lane = __lane_id();

    int64_t e = -1;
    uint32_t t = 0;  // env step of this launch the lane is on (a.n_calls steps per env)
    bool exhausted = TAIL && lane >= a.lane_limit;  // lanes past the limit take no env
    uint64_t o0[W];
    uint32_t m_lo = 0, m_hi = 0;  // FAST: packed per-cube mismatch counters
    bool hit0 = false;            // o0 is attracting (the test made after the first update)
    uint32_t used = 0;
    int64_t nst = 0, dpos = 0, dend = 0;
    int n_act = 0;
    bool capped = false;
    bool tmode = false;  // TAIL: this wave resolves its remaining envs one at a time, 64 updates per block
    auto wave_sync = [] {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    };

    // ---- hand-off of tail envs between the waves of a workgroup (TAIL, EnvArgs::steal_local), in LDS.
    // A wave in tail mode resolves its live envs one after another, so a long until-attractor loop
    // (pbn_target_multi.py:135-146) waits behind the others while sibling waves that have run out of
    // envs sit idle. A wave that runs out of envs sets its bit in the workgroup's idle mask and waits
    // on a flag in its own draw buffer (unused while it holds no env); a tail wave holding envs it has
    // not started on (checked when it starts an env and every 16 blocks) claims idle waves (clearing
    // their bits), writes one env per claimed wave (lane registers + state words) into that wave's
    // buffer, counts the claimed wave busy and raises its flag; the claimed wave resumes the env in
    // lane 0. Bit-exact: the env's Philox stream is keyed by its global id, update index and env step,
    // not by the wave. A wave leaves when no wave of its workgroup is busy and it can clear its own
    // idle bit (nobody claimed it). Between workgroups: the grid pool below (round 3's per-wave device
    // mailboxes, where every cross-XCD read was an atomic, measured 7-20x slower).
    const uint32_t wv_in_wg = threadIdx.x >> 6;
    auto box_of = [&](uint32_t w) {
        return reinterpret_cast<uint64_t*>(lds + a.off_gen + w * GWB + CH * 128 + 64);
    };
    auto flag_of = [&](uint32_t w) {
        return reinterpret_cast<uint32_t*>(lds + a.off_gen + w * GWB + CH * 128);
    };
    auto ldl = [](uint32_t* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP); };
    // lane 0 claims up to n idle waves of the workgroup (clears their idle bits); wave-uniform result
    auto claim_idle = [&](uint32_t n) -> uint32_t {
        uint32_t claimed = 0;
        if (lane == 0) {
            uint32_t idle = ldl(&wctl[1]);
            n = min((uint32_t)__popc(idle), n);
            while (idle != 0u && n != 0u) {
                const uint32_t w = (uint32_t)__ffs(idle) - 1u, bit = 1u << w;
                idle &= ~bit;
                // acquire: the claimed wave cleared its flag before setting its idle bit (release), so
                // the flag / box writes that follow are ordered after that clear
                if (__hip_atomic_fetch_and(&wctl[1], ~bit, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) & bit) {
                    claimed |= bit;
                    --n;
                }
            }
        }
        return (uint32_t)__shfl((int)claimed, 0);
    };
    // ---- tail helpers (TAIL, EnvArgs::tail_helpers): the ring a long tail session's blocks are prepared
    // into, in the SESSION wave's draw buffer after its writer-mask table (the session wave, resolving
    // only, does no writer rounds of its own): ring_R slots of one uint2 per lane per block, then the
    // control words -- tags [8] (block index held by each slot), [8] cons (blocks below it are consumed),
    // [9] stop, [10] helpers' acks, [12] u0, [13] c1, [14]/[15] gid, [16] first ring block, [17] helpers
    const uint32_t wm_bytes = ((N + 31u) >> 5) * 256u;
    // ring blocks are 128 updates (two per lane: 16 B per lane, 1 KiB per slot). The ring may run over the
    // session wave's own hand-off flag and box: those are unused while it is in a session (it clears its flag
    // before it next goes idle). Helpers keep a 128-bit writer-mask table (2 x wm_bytes) below their own flag.
    // (the ring's control words end at least 24 B before the draw buffer's end: the grid pool's view is there)
    const uint32_t ring_R = (GWB > wm_bytes + 96u && 2u * wm_bytes <= CH * 128u)
                                ? min(8u, (GWB - wm_bytes - 96u) / 1024u) : 0u;
    auto ring_of = [&](uint32_t w) { return lds + a.off_gen + w * GWB + wm_bytes; };
    auto rctl_of = [&](uint32_t w) { return reinterpret_cast<uint32_t*>(ring_of(w) + ring_R * 1024u); };
    constexpr uint64_t HELP_MARK = 0xFFFFFFFFFFFFFFFEull;  // box[0] of a wave recruited as a helper
    bool helping = false;
    uint32_t help_req = 0;  // session wave | helper index << 8
    auto local_push = [&](uint64_t cand) {
        if constexpr (TAIL) {
            const uint32_t claimed = claim_idle((uint32_t)__popcll(cand));
            if (claimed == 0u) return;
            const uint32_t k = (uint32_t)__popc(claimed);
            const uint32_t above = lane < 63u ? (uint32_t)__popcll(cand >> (lane + 1u)) : 0u;
            const bool mine = ((cand >> lane) & 1ull) != 0ull && above < k;
            uint32_t tw = 0;  // the above-th claimed wave
            if (mine) {
                uint32_t c = claimed;
                for (uint32_t r = 0; r < above; ++r) c &= c - 1u;
                tw = (uint32_t)__ffs(c) - 1u;
                uint64_t* box = box_of(tw);
                uint64_t s[W];
                from_plane<W>(P, s);
                box[0] = (uint64_t)e;
                box[1] = (uint64_t)nst;
                box[2] = (uint64_t)t | (uint64_t)used << 32;
                box[3] = (uint64_t)m_lo | (hit0 ? 1ull << 32 : 0ull);
                box[4] = (uint64_t)(int64_t)n_act;
#pragma unroll
                for (int k2 = 0; k2 < W; ++k2) {
                    box[5 + k2] = o0[k2];
                    box[5 + W + k2] = s[k2];
                }
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
            if (mine) {
                (void)__hip_atomic_fetch_add(&wctl[0], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                __hip_atomic_store(flag_of(tw), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                e = -1;
                exhausted = true;
            }
            if (lane == 0) atomicAdd(a.steal_count, k);  // diagnostics (pbn_env_handoffs)
#ifdef PBN_STAMPS
            est[16] += k;
#endif
        }
    };
    // ---- grid pool: the same hand-off between workgroups. A workgroup whose waves have all run out of work
    // takes a ticket (one wave waits on it for the workgroup); a tail wave that still holds envs it has not
    // started on after the workgroup hand-off, and sees tickets nobody has filled, reserves that many slots
    // and writes one env into each -- the hand-off box's words as 8-B {epoch, value} granules, each one
    // aligned write-through store, so a slot is complete when every granule carries this launch's epoch (no
    // flag, no fence; MI355X_MICROARCH.md "granules"). A slot is claimed by an atomic max on its state word
    // (epoch << 2 | 1) before it is written; a ticket holder that finds the live count at 0 (no workgroup
    // working, no env in the pool) gives its slot up by a max to epoch << 2 | 2 -- whichever lands first
    // tells the other (a late push sees the slot given up and keeps its env; a holder that sees it claimed
    // waits for the granules). Epochs only grow between the pool's zeroings, so older states never match.
    // The waiting wave's siblings stay idle in LDS, so an env received this way gets tail helpers too.
    // Bit-exact like the workgroup hand-off: an env's draws are keyed by its global id, not by the wave.
    constexpr uint32_t NBW = 2u * (5u + 2u * (uint32_t)W);  // hand-off words (u32) per env
    static_assert(NBW <= GPOOL_GRANULES && NBW <= 64u, "grid pool slot: one granule per lane");
    const uint32_t GE = a.gpool_epoch & 0x3FFFFFFFu;
    // The pool as this wave last saw it -- [0] tickets taken, [1] slots reserved, loaded into LDS by an
    // asynchronous LDS-DMA load (global_load_lds, sc1) issued at the previous look, so looking costs no round
    // trip -- and [2] the realtime (low 32 bits) before which the wave does not look again: the last 12 B of its
    // draw buffer (past the ring's control words; unused in tail mode, where the view lives)
    uint32_t* const gview = reinterpret_cast<uint32_t*>(lds + a.off_gen + wv_in_wg * GWB + GWB - 12u);
    auto gview_issue = [&]() {
        if (lane < 2u)
            __builtin_amdgcn_global_load_lds((gu32*)(a.gpool_ctl + 1u - lane),
                                             (__attribute__((address_space(3))) uint32_t*)gview, 4, 0, 16);
    };
    auto grid_push = [&](uint64_t cand) {
        if constexpr (TAIL) {
            if (!GRID || cand == 0ull) return;
            const uint32_t now = (uint32_t)__builtin_amdgcn_s_memrealtime();
            if ((int32_t)(now - gview[2]) < 0) return;
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the view loaded at the last look has landed
            const int32_t waiting = (int32_t)(min(gview[0], a.gpool_cap) - gview[1]);
            wave_sync();
            if (lane == 0) gview[2] = now + PBN_GPOOL_CHECK_TICKS;
            gview_issue();  // for the next look
            if (waiting <= 0) return;
            // one env (the lowest lane of cand): lane 0 reserves a slot and claims it (atomic max of the slot's
            // state: a ticket holder that gave the slot up raised it past this value first); the env's words go
            // through this wave's own hand-off box (unused while it works), then one granule per lane
            int ok = 0;
            uint32_t sl = 0;
            if (lane == 0) {
                (void)__hip_atomic_fetch_add(gctl(2), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // live first
                sl = __hip_atomic_fetch_add(gctl(0), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (sl < a.gpool_cap)
                    ok = (__hip_atomic_fetch_max((gu32*)(a.gpool_state + sl), GE << 2 | 1u, __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_AGENT) >> 2) != GE;
                // given up by its ticket holder, or past the pool: the env stays here
                (void)__hip_atomic_fetch_add(ok ? gctl(3) : gctl(2), ok ? 1u : 0xFFFFFFFFu, __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_AGENT);
            }
            if (!__shfl(ok, 0)) return;
            sl = (uint32_t)__shfl((int)sl, 0);
            uint64_t* box = box_of(wv_in_wg);
            if (lane == (uint32_t)__ffsll((unsigned long long)cand) - 1u) {
                uint64_t s[W];
                from_plane<W>(P, s);
                box[0] = (uint64_t)e;
                box[1] = (uint64_t)nst;
                box[2] = (uint64_t)t | (uint64_t)used << 32;
                box[3] = (uint64_t)m_lo | (hit0 ? 1ull << 32 : 0ull);
                box[4] = (uint64_t)(int64_t)n_act;
#pragma unroll
                for (int k2 = 0; k2 < W; ++k2) {
                    box[5 + k2] = o0[k2];
                    box[5 + W + k2] = s[k2];
                }
                e = -1;
                exhausted = true;
            }
            wave_sync();
            if (lane < NBW) {
                const uint32_t v = reinterpret_cast<const uint32_t*>(box)[lane];
                __hip_atomic_store((gu64*)(a.gpool + (uint64_t)sl * GPOOL_GRANULES) + lane,
                                   (unsigned long long)GE << 32 | v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            wave_sync();  // the box's reads are done before anything reuses it
        }
    };
    // The workgroup's waiting wave (whole wave): a ticket, then its slot's granules swept until every one
    // carries this launch's epoch (true: the env's words are in this wave's box), or the launch is done
    // (false). The workgroup stops counting as live when it takes the ticket.
    // Only a workgroup whose CU has no workgroup still on its own envs takes a ticket: an env moved onto a CU
    // where other waves still work would slow the waves the launch is waiting for (measured: cap 4,096 per
    // step 1.15 -> 1.34 ms when any idle workgroup took envs), while a finished workgroup there leaves the CU
    // to them. Until then it waits (or leaves when nothing is live).
    auto grid_pop = [&]() -> bool {
        uint32_t ticket = 0;
        int leave = 0;
        if (lane == 0) {
            (void)__hip_atomic_fetch_add(gctl(2), 0xFFFFFFFFu, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            gu32* cu = gctl(GPOOL_CU_WORD + __smid());
            if ((ldl(&wctl[3]) & 2u) == 0u) {  // the first time this workgroup runs out of work
                __hip_atomic_store(&wctl[3], 2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                (void)__hip_atomic_fetch_add(cu, 0xFFFFFFFFu, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            const uint64_t ta = __builtin_amdgcn_s_memrealtime();
            while (a.gpool_cu_idle && __hip_atomic_load(cu, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u) {
                if (__hip_atomic_load(gctl(2), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0u ||
                    __builtin_amdgcn_s_memrealtime() - ta > GPOOL_GIVE_UP_TICKS) {
                    leave = 1;  // (no ticket taken yet: nothing to give up)
                    break;
                }
                __builtin_amdgcn_s_sleep(PBN_GPOOL_SLEEP);
            }
            if (!leave) ticket = __hip_atomic_fetch_add(gctl(1), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        if (__shfl(leave, 0)) return false;
        ticket = (uint32_t)__shfl((int)ticket, 0);
        // a ticket past the pool's slots can never receive an env: leave at once (pushers count only the
        // tickets that have slots, so none waits for this one)
        if (ticket >= a.gpool_cap) return false;
        gu64* g = (gu64*)(a.gpool + (uint64_t)ticket * GPOOL_GRANULES);
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        bool claimed = false;  // the quiet give-up found the slot claimed: its words are on their way
        for (uint32_t it = 0;; ++it) {
            // lane 0 polls the slot's last granule; once it carries the epoch, the whole wave sweeps the slot
            int seen = 0;
            if (lane == 0)
                seen = (uint32_t)(__hip_atomic_load(g + (NBW - 1u), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >> 32) == GE;
            if (__shfl(seen, 0)) {
                for (;;) {
                    uint64_t x = 0;
                    if (lane < NBW) x = __hip_atomic_load(g + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    if (__ballot(lane < NBW && (uint32_t)(x >> 32) != GE) == 0ull) {
                        if (lane < NBW) reinterpret_cast<uint32_t*>(box_of(wv_in_wg))[lane] = (uint32_t)x;
                        wave_sync();
                        return true;
                    }
                    __builtin_amdgcn_s_sleep(1);
                }
            }
            if ((it & 1u) == 1u) {
                int leave = 0;
                if (lane == 0) {
                    if (!claimed && __hip_atomic_load(gctl(2), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0u) {
                        // nothing live: no push can come any more -- unless one already claimed this slot
                        leave = (__hip_atomic_fetch_max((gu32*)(a.gpool_state + ticket), GE << 2 | 2u, __ATOMIC_RELAXED,
                                                        __HIP_MEMORY_SCOPE_AGENT) >> 2) != GE;
                        claimed = !leave;
                    }
                    const uint64_t waited = __builtin_amdgcn_s_memrealtime() - t0;
                    if (!leave && !claimed && waited > GPOOL_GIVE_UP_TICKS) {
                        // waited long with no env: give the slot up (as above) and leave, unless a push claimed it
                        if ((__hip_atomic_fetch_max((gu32*)(a.gpool_state + ticket), GE << 2 | 2u, __ATOMIC_RELAXED,
                                                    __HIP_MEMORY_SCOPE_AGENT) >> 2) != GE)
                            leave = 1;
                        else
                            claimed = true;
                    }
                    if (!leave && claimed && waited > GPOOL_TIMEOUT_TICKS) {
                        leave = 1;
                        (void)__hip_atomic_fetch_add(gctl(4), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        atomicOr(a.error, 2);
                        atomicOr(a.error + 1, 2);  // sticky: device-path launches report it at pbn_sync
                    }
                }
                if (__shfl(leave, 0)) return false;
            }
            __builtin_amdgcn_s_sleep(PBN_GPOOL_SLEEP);
        }
    };
    auto local_pop = [&]() -> int {  // 0: leave, 1: an env in lane 0, 2: a helper request (help_req)
        if constexpr (TAIL) {
#ifdef PBN_STAMPS
            const uint64_t t_in = __builtin_amdgcn_s_memrealtime();
            if (!est[18]) est[18] = t_in;
#endif
            int32_t got = 0;
            if (lane == 0) {
                const uint32_t bit = 1u << wv_in_wg;
                // the flag shares bytes with lane mode's draw tables: cleared before the idle bit is set,
                // and the bit set with release semantics, so a pusher that claims the bit (its fetch_and
                // reads it) cannot be ordered before the cleared flag
                __hip_atomic_store(flag_of(wv_in_wg), 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                (void)__hip_atomic_fetch_or(&wctl[1], bit, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
                (void)__hip_atomic_fetch_add(&wctl[0], 0xFFFFFFFFu, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                for (;;) {
                    if (ldl(flag_of(wv_in_wg)) != 0u) {
                        got = 1;
                        break;
                    }
                    if (ldl(&wctl[0]) == 0u) {
                        if (GRID) {
                            // nobody busy: the launch is done (the waiting wave said so) -- leave with the idle
                            // bit set (no wave is busy to claim it); else one wave waits on a ticket for the
                            // workgroup (the others stay idle here)
                            if (ldl(&wctl[3]) & 1u) {
                                got = -1;
                                break;
                            }
                            uint32_t zero = 0u;
                            // acquire: a sibling that got an env from the pool raised the busy count before it
                            // released this word, so the count re-read below sees it (the count
                            // read above may predate that increment)
                            if (__hip_atomic_compare_exchange_strong(&wctl[2], &zero, 1u, __ATOMIC_ACQUIRE,
                                                                     __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) {
                                if (ldl(&wctl[0]) != 0u) {
                                    // the workgroup is busy again: not idle, keep polling
                                    __hip_atomic_store(&wctl[2], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                                    __builtin_amdgcn_s_sleep(2);
                                    continue;
                                }
                                if (__hip_atomic_fetch_and(&wctl[1], ~bit, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) &
                                    bit) {
                                    got = 3;
                                    break;
                                }
                                // claimed meanwhile: an env or a helper request is on its way
                                __hip_atomic_store(&wctl[2], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                                while (ldl(flag_of(wv_in_wg)) == 0u) __builtin_amdgcn_s_sleep(1);
                                got = 1;
                                break;
                            }
                            // a sibling waits on the pool: nothing can arrive here until it has an env, so poll
                            // slowly (this CU's other workgroups may still be working)
                            __builtin_amdgcn_s_sleep(PBN_GPOOL_SLEEP);
                        } else {
                            // nobody busy: leave, unless a pusher claimed this wave before the count reached 0
                            if (__hip_atomic_fetch_and(&wctl[1], ~bit, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) & bit) {
                                got = -1;
                                break;
                            }
                            while (ldl(flag_of(wv_in_wg)) == 0u) __builtin_amdgcn_s_sleep(1);
                            got = 1;
                            break;
                        }
                    }
                    __builtin_amdgcn_s_sleep(2);
                }
            }
            got = __shfl(got, 0);
            if (got == 3) {  // this wave waits on the grid pool for the workgroup
                const bool env = grid_pop();
                if (lane == 0) {
                    if (env) {
                        // busy before the ticket word is released: the siblings never see the workgroup idle
                        (void)__hip_atomic_fetch_add(&wctl[0], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                        __hip_atomic_store(&wctl[2], 0u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
                    } else {
                        (void)__hip_atomic_fetch_or(&wctl[3], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                    }
                }
                got = env ? 1 : -1;
#ifdef PBN_STAMPS
                est[16] += env ? 0x10000u : 0u;  // envs received from the grid pool (high half)
#endif
            }
#ifdef PBN_STAMPS
            est[17] += __builtin_amdgcn_s_memrealtime() - t_in;
            est[15] += got > 0 ? 1u : 0u;
#endif
            if (got < 0) return 0;
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
            if (box_of(wv_in_wg)[0] == HELP_MARK) {  // recruited as a tail helper (every lane reads the box)
                help_req = (uint32_t)box_of(wv_in_wg)[1];
                if (lane == 0) __hip_atomic_store(flag_of(wv_in_wg), 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                return 2;
            }
            if (lane == 0) {
                const uint64_t* box = box_of(wv_in_wg);
                e = (int64_t)box[0];
                nst = (int64_t)box[1];
                const uint64_t tu = box[2], mh = box[3];
                t = (uint32_t)tu;
                used = (uint32_t)(tu >> 32);
                m_lo = (uint32_t)mh;
                hit0 = ((mh >> 32) & 1ull) != 0ull;
                n_act = (int)(int64_t)box[4];
                uint64_t s[W];
#pragma unroll
                for (int k2 = 0; k2 < W; ++k2) {
                    o0[k2] = box[5 + k2];
                    s[k2] = box[5 + W + k2];
                }
                to_plane<W>(P, s);
                capped = false;
                __hip_atomic_store(flag_of(wv_in_wg), 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            }
            return 1;
        }
        return 0;
    };


    // Start env step t (or the first later step whose action row is valid) of lane env e from
    // state s: flips (:120-131), observation before the update (:133), plane, counters. With no
    // step left, write the env's state and step count back and free the lane.
    auto begin_steps = [&](uint64_t (&s)[W]) {
        for (; t < a.n_calls; ++t) {
            uint64_t f[W];
#pragma unroll
            for (int k = 0; k < W; ++k) f[k] = s[k];
            bool bad = false;
            n_act = apply_actions<W>(f, a.actions + ((uint64_t)t * a.B + (uint64_t)e) * (uint64_t)a.A, a.A,
                                     a.offset, a.dedup, (int32_t)N, &bad);
            if (bad) {  // reference raises ValueError; this env step is skipped, the env left untouched
                atomicOr(a.error, 1);
                continue;
            }
            ++nst;  // :123
#pragma unroll
            for (int k = 0; k < W; ++k) o0[k] = f[k];
            to_plane<W>(P, f);
            if constexpr (FAST >= 1) {
                uint32_t m[2] = {0x01010101u, 0x01010101u};  // unused cubes: never zero
                for (int32_t h = 0; h < H; ++h) {
                    const uint32_t c = cube_mismatch<W>(f, cubes + (uint64_t)h * 2 * W);
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
            return;
        }
        store_state<W>(a.state + (uint64_t)e * W, s);
        a.n_steps[e] = nst;
        e = -1;
    };

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
                    e = (int64_t)ne;
                    t = 0;
                    nst = a.n_steps[ne];
                    if constexpr (REPLAY) {
                        dpos = a.draw_off[ne];
                        dend = a.draw_off[ne + 1];
                    }
                    begin_steps(s);
                }
            }
        }
        const uint64_t act = __ballot(e >= 0);
        if (act == 0 && !helping) {
            if (__ballot(!exhausted) == 0) {
                if (TAIL && a.steal_local) {
                    const int r = local_pop();
                    if (r == 1) continue;  // a handed-off env in lane 0
                    if (r == 2) {
                        helping = true;  // prepare another wave's tail blocks (the tail block below)
                    } else {
                        break;
                    }
                } else {
                    break;
                }
            } else {
                continue;
            }
        }
#ifdef PBN_STAMPS
        if constexpr (GEN) {
            const uint64_t now = __builtin_amdgcn_s_memrealtime();
            const uint32_t na = (uint32_t)__popcll(act);
            const bool qe = __ballot(exhausted) != 0;  // a lane of this wave found the queue empty
            if (!est[1] && na < ENV_OWN_DRAWS_MIN) est[1] = now;
            if (!est[2] && qe) est[2] = now;
            if (!est[3] && na <= 32) est[3] = now;
            if (!est[4] && na <= 16) est[4] = now;
            if (!est[5] && na <= 8) est[5] = now;
            if (!est[6] && na <= 2) est[6] = now;
            est[8] += 1;
            est[9] += na;
            if (qe) {
                est[10] += 1;
                est[11] += na;
            }
        }
#endif
        bool done = false;
        bool in_tail = false;
        if constexpr (TAIL) {
            // ---- tail mode: once the work queue has run dry (some lane found it empty) and the wave
            // holds at most a.tail_max envs, the whole wave works on ONE env at a time (the lowest
            // active lane's), resolving 64 consecutive updates per block: lane k takes update used + k
            // (its Philox draw, predictor record and operands are state-independent), finds the last
            // earlier lane of the block that wrote each operand (per-node 64-bit writer masks in the
            // wave's LDS scratch), and the block's outputs are the fixed point of y_k = tt_k(operands
            // from their writers or the block-start state): a DAG, so iterating from the block-start
            // values settles in at most depth + 1 rounds and a round that changes nothing is exact.
            // Packed counter deltas are prefix-summed over the wave; the first update whose counters
            // hit a cube (or update 0 on o0, :134) ends the env step; the last writer of each node in
            // the committed prefix sets its bit in the env's plane column. Bit-exact with lane mode.
            // A long until-attractor loop left alone (the reference's unbounded loop,
            // pbn_target_multi.py:135-146, the per-step launch's last envs) then advances 64 updates
            // per block round trip instead of one per update.
            if (tmode || helping || (__popcll(act) <= a.tail_max && __ballot(exhausted) != 0)) {
                in_tail = true;
                uint64_t* wm = reinterpret_cast<uint64_t*>(lds + a.off_gen + (threadIdx.x >> 6) * GWB);
                if (!tmode) {
                    for (uint32_t k = lane; k < wm_bytes / 8u; k += 64) wm[k] = 0ull;
                    if (GRID) {  // the pool's view: first look after PBN_GPOOL_CHECK_TICKS, its load issued now
                        if (lane == 0) gview[2] = (uint32_t)__builtin_amdgcn_s_memrealtime() + PBN_GPOOL_CHECK_TICKS;
                        wave_sync();
                        gview_issue();
                    }
                    wave_sync();
                    tmode = true;
                }
                // envs beyond the one resolved next go to idle waves, if there are any
                // Which env first: the loop lengths are heavy-tailed (mean ~1,700 updates, longest ~62k at
                // config 5's 2^20 cap), so an env that has already run long is the likeliest to run longest;
                // it goes first (the others are the ones handed to idle waves), so the wave's last env is
                // not the long one queued behind the rest. Lowest lane when none has run past ENV_LONG_USED.
                uint32_t L = act ? (uint32_t)__ffsll((unsigned long long)act) - 1u : 0u;  // (helping: unused)
                if (!helping) {
                    if (__ballot(e >= 0 && used >= ENV_LONG_USED) != 0ull) {
                        const uint32_t mx =
                            (uint32_t)__builtin_amdgcn_readlane((int)wave_inclusive_max(e >= 0 ? used : 0u), 63);
                        L = (uint32_t)__ffsll((unsigned long long)__ballot(e >= 0 && used == mx)) - 1u;
                    }
                    if (a.steal_local && (act & ~(1ull << L)) != 0ull) {
                        local_push(act & ~(1ull << L));
                        grid_push(__ballot(e >= 0) & ~(1ull << L));  // what the workgroup could not take
                    }
                }
                // the env's registers from lane L (wave-uniform index: v_readlane, no LDS permute); a helper
                // takes the session's update base, call index and env id from the session wave's ring control
                auto from_L = [&](uint32_t v) { return (uint32_t)__builtin_amdgcn_readlane((int)v, (int)L); };
                const uint32_t* hrc = rctl_of(help_req & 0xFFu);
                uint32_t u = helping ? hrc[12] : from_L(used);
                uint32_t m = from_L(m_lo);
                const uint32_t h0 = from_L(hit0 ? 1u : 0u);
                const uint64_t gid = helping ? ((uint64_t)hrc[15] << 32 | hrc[14])
                                             : a.env_base + ((uint64_t)from_L((uint32_t)((uint64_t)e >> 32)) << 32 |
                                                             (uint64_t)from_L((uint32_t)(uint64_t)e));
                const uint32_t c1 = helping ? hrc[13] : a.call_idx + from_L(t);
                uint32_t* col = P.base + ((int32_t)L - (int32_t)lane);  // lane L's plane column
                const uint8_t* colb = reinterpret_cast<const uint8_t*>(col);
                const uint4* erec = reinterpret_cast<const uint4*>(lds + a.L.off_rec);
                uint8_t* const wmc = reinterpret_cast<uint8_t*>(wm);
                const uint64_t below = (1ull << lane) - 1ull, upto = (2ull << lane) - 1ull;
                // predictor choice on the draw word (compact u32 thresholds, rows of tp4 <= 16: mode 2/4
                // needs <= 16 predictors per node), as guarded straight-line reads rather than a loop
                const uint32_t nq = X.tp4 >> 2;
                auto tail_session = [&](auto one_row) {
                // one_row: every node's thresholds fit one 16-B row (<= 5 predictors: Bittner-200), so a
                // choice is one ds_read_b128 and the two choices of a Philox pair issue back to back
                constexpr bool ONE_ROW = decltype(one_row)::value;
                auto cnt4 = [](const uint4& t4, uint32_t a32) {
                    return (a32 >= t4.x ? 1u : 0u) + (a32 >= t4.y ? 1u : 0u) + (a32 >= t4.z ? 1u : 0u) +
                           (a32 >= t4.w ? 1u : 0u);
                };
                auto choice = [&](uint32_t i, uint32_t a32) -> uint32_t {
                    const uint4* thr = reinterpret_cast<const uint4*>(lds) + (ONE_ROW ? i : i * nq);
                    uint32_t j = cnt4(thr[0], a32);
                    if (!ONE_ROW && nq > 1u) {
                        j += cnt4(thr[1], a32);
                        if (nq > 2u) {
                            j += cnt4(thr[2], a32);
                            if (nq > 3u) j += cnt4(thr[3], a32);
                        }
                    }
                    return j;
                };
                // Philox with the key schedule recomputed per call (SALU adds): hoisted out of the block
                // loop, its 20 round keys took SGPRs the kernel then spilled to VGPR lanes (v_readlane + nops).
                // the block's calls differ in counter word 0 only (words 1-3: the session's call index and
                // env id), so half of rounds 0 and 1 is the same for every lane: computed once per session
                // (scalar), a block's call is 18 multiplies instead of 20
                const uint32_t sk0 = (uint32_t)a.seed, sk1 = (uint32_t)(a.seed >> 32);
                const uint64_t P1u = (uint64_t)0xCD9E8D57u * (uint32_t)gid;
                const uint32_t A0 = (uint32_t)(P1u >> 32) ^ c1 ^ sk0;
                const uint32_t U0 = (((uint32_t)(gid >> 32) & 0xFFFFFFu) | (STREAM_ENV << 24)) ^ sk1;
                const uint32_t V1 = (uint32_t)P1u ^ (sk0 + 0x9E3779B9u);
                const uint64_t P0u = (uint64_t)0xD2511F53u * A0;
                const uint32_t H1 = (uint32_t)(P0u >> 32) ^ (sk1 + 0xBB67AE85u), L1 = (uint32_t)P0u;
                auto draw = [&](uint32_t c0, uint32_t w4[4]) {
                    const uint64_t p0 = (uint64_t)0xD2511F53u * c0;  // round 0 (its other half: A0, lo(P1u))
                    const uint32_t y = (uint32_t)(p0 >> 32) ^ U0;
                    const uint64_t p1 = (uint64_t)0xCD9E8D57u * y;  // round 1 (its other half: H1, L1)
                    w4[0] = (uint32_t)(p1 >> 32) ^ V1;
                    w4[1] = (uint32_t)p1;
                    w4[2] = (uint32_t)p0 ^ H1;
                    w4[3] = L1;
                    uint32_t k0 = sk0 + 0x9E3779B9u, k1 = sk1 + 0xBB67AE85u;
                    asm volatile("" : "+s"(k0), "+s"(k1));
#pragma unroll
                    for (int r = 2; r < PBN_PHILOX_ROUNDS; ++r) {  // rounds 2.. as philox4x32_10
                        k0 += 0x9E3779B9u;
                        k1 += 0xBB67AE85u;
                        const uint64_t q0 = (uint64_t)0xD2511F53u * w4[0];
                        const uint64_t q1 = (uint64_t)0xCD9E8D57u * w4[2];
                        const uint32_t n0 = __builtin_amdgcn_bitop3_b32(k0, (uint32_t)(q1 >> 32), w4[1], 0x96);
                        const uint32_t n2 = __builtin_amdgcn_bitop3_b32(k1, (uint32_t)(q0 >> 32), w4[3], 0x96);
                        w4[1] = (uint32_t)q1;
                        w4[3] = (uint32_t)q0;
                        w4[0] = n0;
                        w4[2] = n2;
                    }
                };
                // Draws. STREAM_ENV: update U of the env step takes Philox call U >> 1, words 2(U & 1) and
                // 2(U & 1) + 1: lane k of the block starting at update ub makes call (ub + k) >> 1 and uses
                // its update's half (one call per lane per block; pairing two blocks' calls over a
                // ds_bpermute measured no faster, profiles/r04_r6_tail_philox_split_ab.json,
                // tools/patches/r04_variants.patch).
                // The next block is prepared (draw, record, writer round) while the current one resolves;
                // it is speculative (dropped when the current block ends the env step; the writer table is
                // cleared in the same round that sets it, so it is all zero whenever a session ends).
                // Measured and not kept: a three-stage pipeline (block k + 1's writer round, k + 2's record,
                // k + 3's draw issued while k resolves): a lone chain 0.0156 vs 0.0155 us per update, and
                // 2-5 more VGPRs spilled in the lane-mode path (the kernel is at its 128-VGPR bound).
                const uint32_t u0 = u;
                auto draw_idx = [&](uint32_t b) -> uint32_t {  // block b's env-record index
                    const uint32_t U = u0 + 64u * b + lane;
                    uint32_t w4[4];
                    draw(U >> 1, w4);
                    const uint32_t odd = U & 1u;
                    const uint32_t i = philox_node<KIND>(odd ? w4[2] : w4[0], N);
                    uint32_t ir = __umul24(i, X.rs);
                    asm volatile("" : "+v"(ir));  // else folded with the choice into a quarter-rate v_mad_u64_u32
                    return ir + choice(i, odd ? w4[3] : w4[1]);
                };
                auto erec_of = [&](uint32_t E) { return erec[E & 0xFFFFu]; };
                // Writer round of a block (its records q): node n's 64-bit writer mask at wmc + 8n, n = plane
                // offset / 32 | bit (offset = dword * 4 ENV_BLOCK); or, read the four operands' masks, clear.
                struct WRound {
                    uint32_t nd;
                    uint64_t w0, w1, w2, wi;
                };
                auto wround = [&](const uint4& q) {
                    WRound R;
                    R.nd = *reinterpret_cast<const uint32_t*>(lds + (q.w >> 16));
                    auto wadr = [&](uint32_t off, uint32_t bit) {
                        return reinterpret_cast<unsigned long long*>(wmc + (off >> ENV_ROW_SHIFT) + (bit << 3));
                    };
                    const uint32_t z = q.z;
                    unsigned long long* const wi_p = wadr(q.y >> 16, z >> 24);
                    // no wave barrier between the or, the reads and the clear: one wave's LDS operations
                    // complete in issue order, and the compiler keeps these may-alias accesses in program
                    // order (a barrier here also cut the block into scheduling regions)
                    atomicOr(wi_p, 1ull << lane);
                    R.w0 = *wadr(q.x & 0xFFFFu, z & 31u);
                    R.w1 = *wadr(q.x >> 16, (z >> 8) & 31u);
                    R.w2 = *wadr(q.y & 0xFFFFu, (z >> 16) & 31u);
                    R.wi = *wi_p;
                    *wi_p = 0ull;  // the table is all zero again after every round
                    return R;
                };
                //   hm: pattern bits (in0 8, in1 4, in2 2, own 1) whose operand an earlier lane of the
                //       block writes; rr: that lane (the last such) per operand, in0 | in1 << 8 | in2 << 16 |
                //       own << 24, i.e. the shift bringing its output to bit 0 of the block's ballot;
                //   nx: the next lane writing this lane's node (~0: none) -- the commit's last-writer test.
                struct TailDraw {
                    uint4 q;
                    uint32_t nd, hm, rr, nx;
                };
                auto writers = [&](const uint4& q, const WRound& R) {
                    TailDraw D;
                    D.q = q;
                    D.nd = R.nd;
                    uint32_t hm = 0u, rr = 0u;
                    auto lw = [&](uint64_t w, uint32_t pbit, uint32_t sh) {
                        const uint64_t wb = w & below;
                        hm |= (wb != 0ull ? pbit : 0u);
                        rr |= ((63u - (uint32_t)__clzll((long long)wb)) & 63u) << sh;
                    };
                    lw(R.w0, 8u, 0u);
                    lw(R.w1, 4u, 8u);
                    lw(R.w2, 2u, 16u);
                    lw(R.wi, 1u, 24u);
                    D.hm = hm;
                    D.rr = rr;
                    D.nx = (uint32_t)__ffsll((unsigned long long)(R.wi & ~upto)) - 1u;
                    return D;
                };
                bool fin = false, hitf = false;
                uint32_t nblk = 0;
                auto prepare = [&](uint32_t b) {
                    const uint4 qb = erec_of(draw_idx(b));
                    return writers(qb, wround(qb));
                };
                // The next block's preparation in three stages placed between the current block's own, so
                // each stage's LDS round trip (threshold row; env record; writer masks) is in flight while
                // the current block computes (fixed point; prefix and commit) instead of stalling the wave
                // ahead of them (one-row thresholds, one Philox call per lane): lone tail launch 57.9 -> 56.6 us,
                // 131,072 envs per step at cap 2^20 2.11 -> 2.05 ms (profiles/r04_r6_tail_split_ab.json)
                constexpr bool SPLIT = ONE_ROW;
                struct StA {
                    uint32_t ir, a32;
                    uint4 t4;
                };
                auto stageA = [&](uint32_t b) {
                    const uint32_t U = u0 + 64u * b + lane;
                    uint32_t w4[4];
                    draw(U >> 1, w4);
                    const uint32_t odd = U & 1u;
                    const uint32_t i = philox_node<KIND>(odd ? w4[2] : w4[0], N);
                    StA A;
                    A.ir = __umul24(i, X.rs);
                    asm volatile("" : "+v"(A.ir));
                    A.a32 = odd ? w4[3] : w4[1];
                    A.t4 = reinterpret_cast<const uint4*>(lds)[i];
                    return A;
                };
                auto stageB = [&](const StA& A) { return erec[(A.ir + cnt4(A.t4, A.a32)) & 0xFFFFu]; };
                if constexpr (ONE_ROW) {
                    if (helping) {
                        // ---- tail helper: ring blocks hj, hj + H, ... of the session wave's env. A ring block is
                        // 128 updates, lane l taking updates 2l and 2l + 1 of it -- one Philox call (words 0-1
                        // and 2-3) serves both. Each is prepared as the session would (predictor choice, env
                        // record, and a writer round over 128-bit writer masks in this wave's own table: node
                        // n's {even, odd} masks at 16 n) and packed into the session's ring slot, 16 B per lane:
                        // the two record indices | hm bits and next-writer indices | the two updates' last-writer
                        // codes (update t' = 2l' + h' as t', one byte per operand). A slot is written once the
                        // session has consumed the block R earlier (cons); the tag, stored after the slot
                        // (release), tells the session which block it holds
                        const uint32_t sw = help_req & 0xFFu, hj = (help_req >> 8) & 0xFFu;
                        uint8_t* const ring = ring_of(sw);
                        uint32_t* const rcw = rctl_of(sw);
                        const uint32_t H = rcw[17];
                        // zero the 128-bit table (its upper half may hold this wave's own old ring slots)
                        for (uint32_t q2 = lane; q2 < wm_bytes / 8u; q2 += 64u)
                            reinterpret_cast<uint4*>(wmc)[q2] = make_uint4(0u, 0u, 0u, 0u);
                        wave_sync();
                        auto nadr = [&](uint32_t off, uint32_t bit) {  // node entry {even, odd}
                            return reinterpret_cast<unsigned long long*>(wmc + ((off >> ENV_ROW_SHIFT) + (bit << 3)) * 2u);
                        };
                        const uint64_t bl = (1ull << lane) - 1ull, ul = (2ull << lane) - 1ull;
                        // code of the last earlier writer (t' = 2 l' + h', 7 bits) and whether there is one
                        auto lastw = [](const ulonglong2& M, uint64_t bE, uint64_t bO, uint32_t& any) -> uint32_t {
                            const uint64_t E = M.x & bE, O = M.y & bO;
                            const uint32_t te = E ? 2u * (63u - (uint32_t)__clzll((long long)E)) : 0u;
                            const uint32_t to = O ? 2u * (63u - (uint32_t)__clzll((long long)O)) + 1u : 0u;
                            any = (E | O) != 0ull ? 1u : 0u;
                            return max(E ? te : 0u, O ? to : 0u);
                        };
                        auto nextw = [](const ulonglong2& M, uint64_t aE, uint64_t aO) -> uint32_t {  // 128: none
                            const uint64_t E = M.x & aE, O = M.y & aO;
                            const uint32_t te = E ? 2u * (uint32_t)(__ffsll((unsigned long long)E) - 1) : 128u;
                            const uint32_t to = O ? 2u * (uint32_t)(__ffsll((unsigned long long)O) - 1) + 1u : 128u;
                            return min(te, to);
                        };
                        const uint32_t cbase = u0 >> 1;  // the ring's first update is even
                        uint32_t slot = hj % ring_R;
                        for (uint32_t jb = hj;; jb += H) {
                            bool stop = false;
                            for (;;) {
                                if (ldl(&rcw[9]) != 0u) {
                                    stop = true;
                                    break;
                                }
                                if (jb < ldl(&rcw[8]) + ring_R) break;
                                __builtin_amdgcn_s_sleep(PBN_HELP_SLEEP);
                            }
                            if (stop) break;
                            uint32_t w4[4];
                            draw(cbase + 64u * jb + lane, w4);
                            const uint32_t ie = philox_node<KIND>(w4[0], N), io = philox_node<KIND>(w4[2], N);
                            uint32_t ire = __umul24(ie, X.rs), iro = __umul24(io, X.rs);
                            asm volatile("" : "+v"(ire), "+v"(iro));
                            const uint4 te4 = reinterpret_cast<const uint4*>(lds)[ie];
                            const uint4 to4 = reinterpret_cast<const uint4*>(lds)[io];
                            const uint32_t idxe = (ire + cnt4(te4, w4[1])) & 0xFFFFu, idxo = (iro + cnt4(to4, w4[3])) & 0xFFFFu;
                            const uint4 qe = erec[idxe], qo = erec[idxo];
                            unsigned long long* const owe = nadr(qe.y >> 16, qe.z >> 24);
                            unsigned long long* const owo = nadr(qo.y >> 16, qo.z >> 24);
                            atomicOr(owe, 1ull << lane);      // even update 2l: bit l of the node's even mask
                            atomicOr(owo + 1, 1ull << lane);  // odd update 2l + 1: bit l of the odd mask
                            auto rd = [&](unsigned long long* a2) { return *reinterpret_cast<const ulonglong2*>(a2); };
                            const ulonglong2 me0 = rd(nadr(qe.x & 0xFFFFu, qe.z & 31u)), me1 = rd(nadr(qe.x >> 16, (qe.z >> 8) & 31u)),
                                             me2 = rd(nadr(qe.y & 0xFFFFu, (qe.z >> 16) & 31u)), me3 = rd(owe);
                            const ulonglong2 mo0 = rd(nadr(qo.x & 0xFFFFu, qo.z & 31u)), mo1 = rd(nadr(qo.x >> 16, (qo.z >> 8) & 31u)),
                                             mo2 = rd(nadr(qo.y & 0xFFFFu, (qo.z >> 16) & 31u)), mo3 = rd(owo);
                            *reinterpret_cast<ulonglong2*>(owe) = make_ulonglong2(0ull, 0ull);  // all zero after the round
                            *reinterpret_cast<ulonglong2*>(owo) = make_ulonglong2(0ull, 0ull);
                            // earlier than 2l: even l' < l, odd l' < l; earlier than 2l + 1: even l' <= l, odd l' < l
                            uint32_t a0, a1, a2, a3, rre, rro, hme, hmo;
                            rre = lastw(me0, bl, bl, a0) | (lastw(me1, bl, bl, a1) << 8) | (lastw(me2, bl, bl, a2) << 16) |
                                  (lastw(me3, bl, bl, a3) << 24);
                            hme = (a0 << 3) | (a1 << 2) | (a2 << 1) | a3;
                            rro = lastw(mo0, ul, bl, a0) | (lastw(mo1, ul, bl, a1) << 8) | (lastw(mo2, ul, bl, a2) << 16) |
                                  (lastw(mo3, ul, bl, a3) << 24);
                            hmo = (a0 << 3) | (a1 << 2) | (a2 << 1) | a3;
                            // later than 2l: even l' > l, odd l' >= l; later than 2l + 1: even and odd l' > l
                            const uint32_t nxe = nextw(me3, ~ul, ~bl), nxo = nextw(mo3, ~ul, ~ul);
                            reinterpret_cast<uint4*>(ring + slot * 1024u)[lane] =
                                make_uint4(idxe | (idxo << 16), hme | (hmo << 4) | (nxe << 8) | (nxo << 16), rre, rro);
                            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
                            if (lane == 0) __hip_atomic_store(&rcw[slot], jb, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                            slot += H;
                            if (slot >= ring_R) slot -= ring_R;
                        }
                        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
                        if (lane == 0) (void)__hip_atomic_fetch_add(&rcw[10], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                        helping = false;
                        return;
                    }
                }
                // ring mode (helpers recruited): ringH = the session's helpers (0: self-prepared blocks)
                uint32_t ringH = 0;
                uint32_t rblocks = 0, rwaits = 0;  // ring diagnostics (pbn_env_tail_stats)
                uint32_t* const rcs = rctl_of(wv_in_wg);
                TailDraw D = prepare(0u);
#ifdef PBN_STAMPS
                const uint64_t sess_rt = __builtin_amdgcn_s_memrealtime();
                const uint32_t sess_u0 = u;
#endif
                uint32_t k = 0;
                // the self-prepared block loop; when helpers are recruited it returns and ring128 below resolves
                // the rest of the session from their ring (separate code, its own registers)
                auto blocks = [&]() {
                for (; !fin; ++k) {
#ifdef PBN_STAMPS
                    // tail block phases (shader clocks, s_memtime): 19 blocks, 20 cycles per block, 21 fixed-point
                    // rounds, 22 cycles of the resolution (fixed point), 23 cycles from the block's top to the
                    // later blocks' stages issued, 24..31 blocks by rounds (0..6, 7+)
                    const uint64_t c_top = __builtin_amdgcn_s_memtime();
                    const uint64_t r_top = __builtin_amdgcn_s_memrealtime();  // 100 MHz: calibrates s_memtime
                    if (!est[34]) est[34] = r_top;
                    uint32_t nround = 0;
#endif
                    const uint4 q = D.q;
                    const uint32_t U = u + lane;
                    const uint32_t ss = q.z >> 24;
                    // block-start values of the operands (in0, in1, in2, own bit)
                    const uint32_t b0 = *reinterpret_cast<const uint32_t*>(colb + (q.x & 0xFFFFu));
                    const uint32_t b1 = *reinterpret_cast<const uint32_t*>(colb + (q.x >> 16));
                    const uint32_t b2 = *reinterpret_cast<const uint32_t*>(colb + (q.y & 0xFFFFu));
                    const uint32_t b3 = *reinterpret_cast<const uint32_t*>(colb + (q.y >> 16));
                    [[maybe_unused]] StA An;
                    [[maybe_unused]] TailDraw Dn;
                    [[maybe_unused]] uint4 qn;
                    if constexpr (SPLIT)
                        An = stageA(k + 1u);  // while those reads are in flight
                    else
                        Dn = prepare(k + 1u);
#ifdef PBN_STAMPS
                    const uint64_t c_prep = __builtin_amdgcn_s_memtime();
#endif
                    const uint32_t v3 = __builtin_amdgcn_ubfe(b3, ss, 1);
                    const uint32_t p0 = (__builtin_amdgcn_ubfe(b0, q.z, 1) << 3) | (__builtin_amdgcn_ubfe(b1, q.z >> 8, 1) << 2) |
                                        (__builtin_amdgcn_ubfe(b2, q.z >> 16, 1) << 1) | v3;
                    // fixed point: operands with an in-block writer take its output from the ballot of the
                    // previous round (bit rr_j), the others keep their block-start value (pf). The first round
                    // runs unconditionally (no branch before it: one scheduling region with the next block's
                    // draws); 72 % of blocks settle in it, 97 % within two (profiles/r04_tail_stamps_*.json)
                    const uint32_t pf = p0 & ~D.hm;
                    const uint32_t r0 = D.rr & 63u, r1 = (D.rr >> 8) & 63u, r2 = (D.rr >> 16) & 63u, r3 = D.rr >> 24;
                    const uint32_t k0 = (D.hm >> 3) & 1u, k1 = (D.hm >> 2) & 1u, k2 = (D.hm >> 1) & 1u, k3 = D.hm & 1u;
                    uint32_t x3;
                    auto fround = [&](uint32_t yy) {
#ifdef PBN_STAMPS
                        ++nround;
#endif
                        const uint64_t Y = __ballot(yy != 0u);
                        const uint32_t p = pf | (((uint32_t)(Y >> r0) & k0) << 3) | (((uint32_t)(Y >> r1) & k1) << 2) |
                                           (((uint32_t)(Y >> r2) & k2) << 1) | ((uint32_t)(Y >> r3) & k3);
                        x3 = p & 1u;
                        return __builtin_amdgcn_ubfe(q.w, p, 1);
                    };
                    uint32_t y = __builtin_amdgcn_ubfe(q.w, p0, 1);
                    uint32_t yn = fround(y);
                    while (__ballot(yn != y) != 0ull) {
                        y = yn;
                        yn = fround(y);
                    }
                    y = yn;
                    if constexpr (SPLIT) qn = stageB(An);
#ifdef PBN_STAMPS
                    const uint64_t c_fp = __builtin_amdgcn_s_memtime();
#endif
                    // packed counter deltas (+ d for 0 -> 1, - d for 1 -> 0), prefix over the block
                    const uint32_t sg = y - 1u;
                    const uint32_t mk = m + wave_inclusive_add(((D.nd & (0u - (y ^ x3))) ^ sg) - sg);
                    const bool valid = U < a.update_cap;
                    const bool hk = (U == 0u && !a.first_tested) ? h0 != 0u : has_zero_byte(mk) != 0u;
                    const uint64_t SM = __ballot(valid && hk), VM = __ballot(valid);
                    const uint32_t nd = SM ? (uint32_t)__ffsll((unsigned long long)SM) : (uint32_t)__popcll(VM);
                    // commit: the last writer of each node among the first nd updates flips its bit if its
                    // output differs from the block-start value (distinct nodes: distinct bits)
                    if (lane < nd && D.nx >= nd && y != v3)
                        atomicXor(reinterpret_cast<uint32_t*>(const_cast<uint8_t*>(colb) + (q.y >> 16)), 1u << ss);
                    m = (uint32_t)__builtin_amdgcn_readlane((int)mk, (int)(nd - 1u));
                    u += nd;
                    hitf = SM != 0ull;
                    fin = hitf || u >= a.update_cap;
                    if constexpr (SPLIT)
                        D = writers(qn, wround(qn));
                    else
                        D = Dn;  // (the commit above and the next block's plane reads stay in issue order)
#ifdef PBN_STAMPS
                    {
                        const uint64_t c_end = __builtin_amdgcn_s_memtime();
                        const uint64_t r_end = __builtin_amdgcn_s_memrealtime();
                        est[32] += r_end - r_top;  // realtime ticks (10 ns) in tail blocks
                        est[35] = r_end;
                        est[19] += 1;
                        est[20] += c_end - c_top;
                        est[21] += nround;
                        est[22] += c_fp - c_prep;
                        est[23] += c_prep - c_top;
                        est[24 + min(nround, 7u)] += 1;
                    }
#endif
                    // every 16 blocks: idle waves may have appeared since this env was started -- they take
                    // this wave's unstarted envs first, then (a long session: >= 16 blocks) up to three of
                    // the rest become its helpers, preparing the session's updates from u on in 128-update
                    // ring blocks (the self-prepared block k + 1 in D is dropped)
                    if (a.steal_local && (++nblk & 15u) == 0u && !fin) {
                        const uint64_t others = __ballot(e >= 0) & ~(1ull << L);
                        if (others) local_push(others);
                        const bool alone = !(SPLIT && a.tail_helpers && ring_R >= 3u && ldl(&wctl[1]) != 0u);
                        if (others) grid_push(__ballot(e >= 0) & ~(1ull << L));
                        // (a ring starts at an even update: helpers key a pair's Philox call by u >> 1 -- always so
                        // here, lane mode and the hand-offs start sessions at multiples of the draw chunk and a
                        // block advances u by 64 unless the session ends; an odd start keeps self-prepared blocks)
                        if (!alone && (u & 1u) == 0u) {
                            const uint32_t cl = claim_idle(min((uint32_t)a.tail_helpers, 3u));
                            if (cl) {
                                const uint32_t H = (uint32_t)__popc(cl);
                                if (lane < 8u) rcs[lane] = 0xFFFFFFFFu;  // tags: no block
                                if (lane == 0) {
                                    rcs[8] = 0u;   // cons: ring blocks consumed
                                    rcs[9] = 0u;   // stop
                                    rcs[10] = 0u;  // acks
                                    rcs[12] = u;   // the ring's first update (even: a block boundary)
                                    rcs[13] = c1;
                                    rcs[14] = (uint32_t)gid;
                                    rcs[15] = (uint32_t)(gid >> 32);
                                    rcs[17] = H;
                                }
                                uint32_t tw = 0;
                                if (lane < H) {  // the lane-th claimed wave becomes helper `lane`
                                    uint32_t c = cl;
                                    for (uint32_t r = 0; r < lane; ++r) c &= c - 1u;
                                    tw = (uint32_t)__ffs(c) - 1u;
                                    box_of(tw)[0] = HELP_MARK;
                                    box_of(tw)[1] = (uint64_t)(wv_in_wg | (lane << 8));
                                }
                                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
                                if (lane < H) {
                                    (void)__hip_atomic_fetch_add(&wctl[0], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                                    __hip_atomic_store(flag_of(tw), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                                }
                                if (lane == 0) atomicAdd(a.steal_count + 1, H);  // diagnostics (pbn_env_tail_helpers)
                                ringH = H;
                                return;  // on in ring128
                            }
                        }
                    }
                }
                };  // blocks
                // ---- the rest of the session from the helpers' ring, 128 updates per block: lane l resolves updates
                // t = 2l and 2l + 1 (u + t). Per block: the 8 operand reads from the plane, a fixed point over both
                // halves (round: one ballot per half; an operand written earlier in the block reads bit t' >> 1 of
                // the ballot of t''s half), the counter prefix in update order (per lane the pair's sum, one wave
                // prefix), the first update that hits a cube, and the last writers' commits. The ring is read two
                // blocks ahead: block j + 1's records are issued and block j + 2's slot polled while j resolves.
                auto ring128 = [&]() {
                    // wave-uniform column base (an SGPR, not a per-lane VGPR held across the loop) and the lane id
                    // re-formed where it is used: the kernel is at its VGPR bound, and long-lived per-lane values in
                    // this loop were spilled and reloaded from scratch on the block's chain
                    const uint32_t cofs = __builtin_amdgcn_readfirstlane((uint32_t)(colb - lds));
                    const uint8_t* const colr = lds + cofs;
                    const uint32_t rofs = __builtin_amdgcn_readfirstlane((uint32_t)(reinterpret_cast<uint8_t*>(rcs) - lds));
                    uint32_t* const rcr = reinterpret_cast<uint32_t*>(lds + rofs);  // the ring's control words (uniform)
                    auto lane_now = [] {
                        uint32_t v;
                        asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(v));
                        return v;
                    };
                    auto poll = [&](uint32_t jb, uint32_t sl) {
                        if (ldl(&rcr[sl]) != jb) {
                            ++rwaits;  // diagnostics: the block's helper had not written it yet
                            while (ldl(&rcr[sl]) != jb) __builtin_amdgcn_s_sleep(1);
                        }
                        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
                        // the slot's address from the control words' (the ring ends where they start), formed
                        // here: a per-lane ring base held across the loop was spilled to scratch, putting a
                        // scratch round trip between the tag and the slot read (stamps: 820 cycles of a 1,990 block)
                        const uint32_t off = sl * 1024u + lane_now() * 16u;
                        return *reinterpret_cast<const uint4*>(reinterpret_cast<const uint8_t*>(rcr) - ring_R * 1024u + off);
                    };
                    auto nxt_slot = [&](uint32_t sl) { return sl + 1u == ring_R ? 0u : sl + 1u; };
                    auto nd_of = [&](const uint4& qq) { return *reinterpret_cast<const uint32_t*>(lds + (qq.w >> 16)); };
                    uint4 sC = poll(0u, 0u);
                    uint4 sN = poll(1u, nxt_slot(0u));
                    asm volatile("" ::"v"(sN.x), "v"(sN.w) : "memory");
                    if (lane == 0) __hip_atomic_store(&rcr[8], 2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                    uint32_t rsl = nxt_slot(nxt_slot(0u));  // slot of block j + 2
                    uint4 qe = erec[sC.x & 0xFFFFu], qo = erec[sC.x >> 16];
                    uint32_t nde = nd_of(qe), ndo = nd_of(qo), inf = sC.y, rre = sC.z, rro = sC.w;
                    auto look = [](uint64_t Ye, uint64_t Yo, uint32_t c) {  // output of update c (= 2 l' + h')
                        return (uint32_t)(((c & 1u) ? Yo : Ye) >> (c >> 1)) & 1u;
                    };
                    for (uint32_t jb = 0; !fin; ++jb) {
                        ++rblocks;
#ifdef PBN_STAMPS
                        // the same tail-block stamps as the self-prepared loop (est 19-31; rounds count fround calls)
                        const uint64_t c_top = __builtin_amdgcn_s_memtime();
                        const uint64_t r_top = __builtin_amdgcn_s_memrealtime();
                        if (!est[34]) est[34] = r_top;
                        uint32_t nround = 0;
#endif
                        const uint32_t se = qe.z >> 24, so = qo.z >> 24;
                        const uint32_t e0 = *reinterpret_cast<const uint32_t*>(colr + (qe.x & 0xFFFFu));
                        const uint32_t e1 = *reinterpret_cast<const uint32_t*>(colr + (qe.x >> 16));
                        const uint32_t e2 = *reinterpret_cast<const uint32_t*>(colr + (qe.y & 0xFFFFu));
                        const uint32_t e3 = *reinterpret_cast<const uint32_t*>(colr + (qe.y >> 16));
                        const uint32_t o0 = *reinterpret_cast<const uint32_t*>(colr + (qo.x & 0xFFFFu));
                        const uint32_t o1 = *reinterpret_cast<const uint32_t*>(colr + (qo.x >> 16));
                        const uint32_t o2 = *reinterpret_cast<const uint32_t*>(colr + (qo.y & 0xFFFFu));
                        const uint32_t o3 = *reinterpret_cast<const uint32_t*>(colr + (qo.y >> 16));
                        // block j + 1's records, block j + 2's slot (in flight while this block resolves)
                        const uint4 qe2 = erec[sN.x & 0xFFFFu], qo2 = erec[sN.x >> 16];
                        const uint4 sNN = poll(jb + 2u, rsl);
#ifdef PBN_STAMPS
                        const uint64_t c_prep = __builtin_amdgcn_s_memtime();
#endif
                        const uint32_t v3e = __builtin_amdgcn_ubfe(e3, se, 1), v3o = __builtin_amdgcn_ubfe(o3, so, 1);
                        const uint32_t p0e = (__builtin_amdgcn_ubfe(e0, qe.z, 1) << 3) | (__builtin_amdgcn_ubfe(e1, qe.z >> 8, 1) << 2) |
                                             (__builtin_amdgcn_ubfe(e2, qe.z >> 16, 1) << 1) | v3e;
                        const uint32_t p0o = (__builtin_amdgcn_ubfe(o0, qo.z, 1) << 3) | (__builtin_amdgcn_ubfe(o1, qo.z >> 8, 1) << 2) |
                                             (__builtin_amdgcn_ubfe(o2, qo.z >> 16, 1) << 1) | v3o;
                        const uint32_t hme = inf & 15u, hmo = (inf >> 4) & 15u, nxe = (inf >> 8) & 255u, nxo = (inf >> 16) & 255u;
                        const uint32_t pfe = p0e & ~hme, pfo = p0o & ~hmo;
                        uint32_t xe, xo;
                        auto fround = [&](uint32_t ye_, uint32_t yo_, uint32_t& yne, uint32_t& yno) {
#ifdef PBN_STAMPS
                            ++nround;
#endif
                            const uint64_t Ye = __ballot(ye_ != 0u), Yo = __ballot(yo_ != 0u);
                            const uint32_t pe = pfe | ((look(Ye, Yo, rre & 255u) & (hme >> 3)) << 3) |
                                                ((look(Ye, Yo, (rre >> 8) & 255u) & (hme >> 2) & 1u) << 2) |
                                                ((look(Ye, Yo, (rre >> 16) & 255u) & (hme >> 1) & 1u) << 1) |
                                                (look(Ye, Yo, rre >> 24) & hme & 1u);
                            const uint32_t po = pfo | ((look(Ye, Yo, rro & 255u) & (hmo >> 3)) << 3) |
                                                ((look(Ye, Yo, (rro >> 8) & 255u) & (hmo >> 2) & 1u) << 2) |
                                                ((look(Ye, Yo, (rro >> 16) & 255u) & (hmo >> 1) & 1u) << 1) |
                                                (look(Ye, Yo, rro >> 24) & hmo & 1u);
                            xe = pe & 1u;
                            xo = po & 1u;
                            yne = __builtin_amdgcn_ubfe(qe.w, pe, 1);
                            yno = __builtin_amdgcn_ubfe(qo.w, po, 1);
                        };
                        uint32_t ye = __builtin_amdgcn_ubfe(qe.w, p0e, 1), yo = __builtin_amdgcn_ubfe(qo.w, p0o, 1);
                        uint32_t yne, yno;
                        fround(ye, yo, yne, yno);
                        while (__ballot(yne != ye || yno != yo) != 0ull) {
                            ye = yne;
                            yo = yno;
                            fround(ye, yo, yne, yno);
                        }
                        ye = yne;
                        yo = yno;
#ifdef PBN_STAMPS
                        const uint64_t c_fp = __builtin_amdgcn_s_memtime();
#endif
                        // block j + 2's slot is in registers: it is free (the asm keeps the store after the read)
                        asm volatile("" ::"v"(sNN.x), "v"(sNN.w) : "memory");
                        if (lane == 0) __hip_atomic_store(&rcr[8], jb + 3u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                        rsl = nxt_slot(rsl);
                        // packed counter deltas in update order: the pair's sum prefixed over the lanes
                        const uint32_t sge = ye - 1u, sgo = yo - 1u;
                        const uint32_t de = ((nde & (0u - (ye ^ xe))) ^ sge) - sge;
                        const uint32_t dodd = ((ndo & (0u - (yo ^ xo))) ^ sgo) - sgo;
                        const uint32_t pro = m + wave_inclusive_add(de + dodd), pre = pro - dodd;
                        const uint32_t nvalid = a.update_cap > u ? min(128u, a.update_cap - u) : 0u;
                        const uint32_t t2 = 2u * lane_now();  // this lane's even update
                        const bool ve = t2 < nvalid, vo = t2 + 1u < nvalid;
                        // (no first-update test here: a ring starts 16 blocks into a session, u > 0)
                        const uint64_t SMe = __ballot(ve && has_zero_byte(pre) != 0u);
                        const uint64_t SMo = __ballot(vo && has_zero_byte(pro) != 0u);
                        const uint32_t te = SMe ? 2u * (uint32_t)(__ffsll((unsigned long long)SMe) - 1) : 256u;
                        const uint32_t to = SMo ? 2u * (uint32_t)(__ffsll((unsigned long long)SMo) - 1) + 1u : 256u;
                        const uint32_t ts = min(te, to);
                        const uint32_t nd = ts < 256u ? ts + 1u : nvalid;
                        // commit: the last writer of each node among the first nd updates (both halves of a lane may
                        // write; nx says whether a later update of the prefix writes the same node)
                        if (t2 < nd && nxe >= nd && ye != v3e)
                            atomicXor(reinterpret_cast<uint32_t*>(const_cast<uint8_t*>(colr) + (qe.y >> 16)), 1u << se);
                        if (t2 + 1u < nd && nxo >= nd && yo != v3o)
                            atomicXor(reinterpret_cast<uint32_t*>(const_cast<uint8_t*>(colr) + (qo.y >> 16)), 1u << so);
                        m = (uint32_t)__builtin_amdgcn_readlane((int)(((nd - 1u) & 1u) ? pro : pre), (int)((nd - 1u) >> 1));
                        u += nd;
                        hitf = ts < 256u;
                        fin = hitf || u >= a.update_cap;
                        qe = qe2;
                        qo = qo2;
                        nde = nd_of(qe);
                        ndo = nd_of(qo);
                        inf = sN.y;
                        rre = sN.z;
                        rro = sN.w;
                        sN = sNN;
#ifdef PBN_STAMPS
                        {
                            const uint64_t c_end = __builtin_amdgcn_s_memtime();
                            const uint64_t r_end = __builtin_amdgcn_s_memrealtime();
                            est[32] += r_end - r_top;
                            est[35] = r_end;
                            est[19] += 1;
                            est[20] += c_end - c_top;
                            est[21] += nround;
                            est[22] += c_fp - c_prep;
                            est[23] += c_prep - c_top;
                            est[24 + min(nround, 7u)] += 1;
                        }
#endif
                        // every 8 ring blocks (1,024 updates): idle waves may take this wave's unstarted envs
                        if ((jb & 7u) == 7u && !fin) {
                            const uint64_t others = __ballot(e >= 0) & ~(1ull << L);
                            if (others) local_push(others);
                        }
                    }
                };
                blocks();
                if (ringH) {
                    ring128();
                    // release the helpers: stop, then wait until each has acknowledged (the ring lives in this
                    // wave's draw buffer, which its next session reuses)
                    if (lane == 0) {
                        __hip_atomic_store(&rcs[9], 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
                        while (ldl(&rcs[10]) != ringH) __builtin_amdgcn_s_sleep(1);
                    }
                    wave_sync();
                    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
                    if (lane == 0) {
                        atomicAdd(a.steal_count + 2, rblocks);
                        atomicAdd(a.steal_count + 3, rwaits);
                    }
                }
#ifdef PBN_STAMPS
                if ((u - sess_u0) / 64u > est[37]) {  // the wave's longest session: start, blocks, end, prior updates
                    est[36] = sess_rt;
                    est[37] = (u - sess_u0) / 64u;
                    est[38] = __builtin_amdgcn_s_memrealtime();
                    est[39] = sess_u0;
                }
#endif
                if (lane == L) {
                    used = u;
                    m_lo = m;
                    capped = !hitf;
                    done = true;
                }
                };  // tail_session
                if (nq == 1u)
                    tail_session(std::true_type{});
                else
                    tail_session(std::false_type{});
            }
        }
        uint16_t* gbuf = nullptr;
        if (!in_tail) {
        if constexpr (GEN) {
            // ---- cooperative draw generation for the next CH updates of every active lane
            uint8_t* gw = lds + a.off_gen + (threadIdx.x >> 6) * GWB;
            gbuf = reinterpret_cast<uint16_t*>(gw);                                   // [CH][64]
            uint4* ctr_tab = reinterpret_cast<uint4*>(gw + CH * 128 + 64);  // [64] by rank
            auto cnt4 = [](const uint4& t4, uint32_t a32) {
                return (a32 >= t4.x ? 1u : 0u) + (a32 >= t4.y ? 1u : 0u) + (a32 >= t4.z ? 1u : 0u) + (a32 >= t4.w ? 1u : 0u);
            };
            const uint32_t nact = (uint32_t)__popcll(act);
            if (nact >= ENV_OWN_DRAWS_MIN) {
                // (nearly) every lane active: each lane draws its own entries from its registers
                // -- no rank / counter tables; an idle lane's draws are junk nobody reads. Fewer
                // rounds shared over the wave stop paying off below ~40 active lanes (a shared
                // round costs two dependent LDS round trips more)
                // (a chunk starts at an even update index: one Philox call per pair of updates)
                const uint64_t gid = a.env_base + (uint64_t)e;
                if (X.tp4 == 4u) {
                    // one threshold row per node (<= 5 predictors: Bittner-200): four updates (two Philox
                    // calls) per iteration with their four 16-B rows read back to back, so one LDS wait
                    // serves four choices (the generic loop below waited once per choice), and the round
                    // keys recomputed per call by SALU adds (hoisted, the 20 keys took SGPRs the kernel
                    // spilled to VGPR lanes: a v_readlane and s_nop per round)
                    const uint4* thr = reinterpret_cast<const uint4*>(lds);
                    const uint32_t c1 = a.call_idx + t;
                    for (uint32_t sl = 0; sl < CH; sl += 4) {
                        uint32_t w[8];
                        philox_draw_sk(a.seed, (used + sl) >> 1, c1, gid, STREAM_ENV, w);
                        philox_draw_sk(a.seed, ((used + sl) >> 1) + 1u, c1, gid, STREAM_ENV, w + 4);
                        uint32_t i[4];
                        uint4 t4[4];
#pragma unroll
                        for (uint32_t h = 0; h < 4; ++h) i[h] = philox_node<KIND>(w[2 * h], N);
#pragma unroll
                        for (uint32_t h = 0; h < 4; ++h) t4[h] = thr[i[h]];
#pragma unroll
                        for (uint32_t h = 0; h < 4; ++h) {
                            const uint32_t j = cnt4(t4[h], w[2 * h + 1]);
                            uint32_t ir = __umul24(i[h], X.rs);
                            asm volatile("" : "+v"(ir));  // else folded with + j into a quarter-rate v_mad_u64_u32
                            gbuf[(sl + h) * 64 + lane] = (uint16_t)(ir + j);
                        }
                    }
                } else
                for (uint32_t sl = 0; sl < CH; sl += 2) {
                    uint32_t w[4];
                    philox_draw_sk(a.seed, (used + sl) >> 1, a.call_idx + t, gid, STREAM_ENV, w);
#pragma unroll
                    for (uint32_t h = 0; h < 2; ++h) {
                        const uint32_t i = philox_node<KIND>(w[2 * h], N);
                        const uint32_t j = predictor_choice32(i, w[2 * h + 1], lds, X.tp4);
                        gbuf[(sl + h) * 64 + lane] = (uint16_t)(__umul24(i, X.rs) + j);  // EnvRec index
                    }
                }
            } else {
            // shared rounds: the active lanes' Philox counters in a table by rank (the lane id in the
            // stream byte, which is the constant STREAM_ENV), so a round's counter is one 16-B read
            // (before: the rank's lane, then its used / call / gid entries: two dependent round trips)
            if (e >= 0) {
                const uint64_t gid = a.env_base + (uint64_t)e;
                ctr_tab[__popcll(act & ((1ull << lane) - 1ull))] =
                    make_uint4(used >> 1, a.call_idx + t, (uint32_t)gid, ((uint32_t)(gid >> 32) & 0xFFFFFFu) | (lane << 24));
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            const uint32_t total = nact * (CH / 2);  // pairs of updates: one Philox call each
            // k / nact as a multiply-high by ceil(2^32 / nact): exact for k < 2^16 (nact == 1 handled apart,
            // its multiplier 2^32 does not fit 32 bits)
            const uint32_t magic = kRankMagic.v[nact];  // a 64-bit divide here was ~120 scalar instructions
            auto rounds = [&](auto one_row, uint32_t kstart) {
                for (uint32_t k0 = kstart; k0 < total; k0 += 64) {
                    const uint32_t k = k0 + lane;
                    if (k < total) {
                        const uint32_t sp = nact > 1 ? __umulhi(k, magic) : k, r = k - sp * nact;
                        const uint4 cr = ctr_tab[r];
                        const uint32_t q = cr.w >> 24;
                        uint32_t w[4];
                        philox_draw_sk(a.seed, cr.x + sp, cr.y, (uint64_t)(cr.w & 0xFFFFFFu) << 32 | cr.z, STREAM_ENV, w);
                        const uint32_t i0 = philox_node<KIND>(w[0], N), i1 = philox_node<KIND>(w[2], N);
                        uint32_t j0, j1;
                        if constexpr (decltype(one_row)::value) {
                            const uint4* thr = reinterpret_cast<const uint4*>(lds);
                            const uint4 t0 = thr[i0], t1 = thr[i1];  // both rows in flight: one LDS wait
                            j0 = cnt4(t0, w[1]);
                            j1 = cnt4(t1, w[3]);
                        } else {
                            j0 = predictor_choice32(i0, w[1], lds, X.tp4);
                            j1 = predictor_choice32(i1, w[3], lds, X.tp4);
                        }
                        uint32_t r0 = __umul24(i0, X.rs), r1 = __umul24(i1, X.rs);
                        asm volatile("" : "+v"(r0), "+v"(r1));  // else folded with + j into v_mad_u64_u32
                        gbuf[(2 * sp) * 64 + q] = (uint16_t)(r0 + j0);
                        gbuf[(2 * sp + 1) * 64 + q] = (uint16_t)(r1 + j1);
                    }
                }
            };
            // one-row thresholds: two rounds per iteration, their counter entries and then their four rows
            // read together, so each LDS wait serves two rounds (a round waited twice: entry, then rows)
            auto rounds2 = [&]() {
                const uint4* thr = reinterpret_cast<const uint4*>(lds);
                uint32_t k0 = 0;
                for (; k0 + 64u < total; k0 += 128) {  // (a last lone round goes to the one-round loop)
                    const uint32_t ka = k0 + lane, kb = ka + 64u;
                    const bool va = ka < total, vb = kb < total;
                    const uint32_t kac = va ? ka : 0u, kbc = vb ? kb : 0u;  // clamped: reads stay in the table
                    const uint32_t spa = nact > 1 ? __umulhi(kac, magic) : kac, ra = kac - spa * nact;
                    const uint32_t spb = nact > 1 ? __umulhi(kbc, magic) : kbc, rb = kbc - spb * nact;
                    const uint4 ca = ctr_tab[ra], cb = ctr_tab[rb];
                    uint32_t wa[4], wb[4];
                    philox_draw_sk(a.seed, ca.x + spa, ca.y, (uint64_t)(ca.w & 0xFFFFFFu) << 32 | ca.z, STREAM_ENV, wa);
                    philox_draw_sk(a.seed, cb.x + spb, cb.y, (uint64_t)(cb.w & 0xFFFFFFu) << 32 | cb.z, STREAM_ENV, wb);
                    const uint32_t ia0 = philox_node<KIND>(wa[0], N), ia1 = philox_node<KIND>(wa[2], N);
                    const uint32_t ib0 = philox_node<KIND>(wb[0], N), ib1 = philox_node<KIND>(wb[2], N);
                    const uint4 ta0 = thr[ia0], ta1 = thr[ia1], tb0 = thr[ib0], tb1 = thr[ib1];
                    uint32_t ra0 = __umul24(ia0, X.rs), ra1 = __umul24(ia1, X.rs);
                    uint32_t rb0 = __umul24(ib0, X.rs), rb1 = __umul24(ib1, X.rs);
                    asm volatile("" : "+v"(ra0), "+v"(ra1), "+v"(rb0), "+v"(rb1));
                    if (va) {
                        const uint32_t q = ca.w >> 24;
                        gbuf[(2 * spa) * 64 + q] = (uint16_t)(ra0 + cnt4(ta0, wa[1]));
                        gbuf[(2 * spa + 1) * 64 + q] = (uint16_t)(ra1 + cnt4(ta1, wa[3]));
                    }
                    if (vb) {
                        const uint32_t q = cb.w >> 24;
                        gbuf[(2 * spb) * 64 + q] = (uint16_t)(rb0 + cnt4(tb0, wb[1]));
                        gbuf[(2 * spb + 1) * 64 + q] = (uint16_t)(rb1 + cnt4(tb1, wb[3]));
                    }
                }
                rounds(std::true_type{}, k0);
            };
            if (X.tp4 == 4u)
                rounds2();
            else
                rounds(std::false_type{}, 0u);
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        }
        if (e < 0) continue;

        // ---- up to CH updates of this lane's env
        const uint64_t g = a.env_base + (uint64_t)e;
        if constexpr (GEN) {
            const uint4* erec = reinterpret_cast<const uint4*>(lds + a.L.off_rec);
            const uint8_t* pb = reinterpret_cast<const uint8_t*>(P.base);  // this lane's plane column
            // branch-free per lane: a lane that is done keeps iterating masked (no break, so
            // no per-lane exit bookkeeping); the wave leaves the chunk when no lane is active.
            // Entries, records and counter deltas do not depend on the state: the entry is read
            // three updates ahead, its EnvRec two ahead and the node's counter deltas one ahead, so
            // an update's only LDS round trip on the dependent chain is its state-plane read.
            bool act = true, hitf = false;
            const uint32_t lim = a.update_cap > used ? a.update_cap - used : 0u;  // updates left
            uint4 q0 = erec[gbuf[lane]];
            uint4 q1 = erec[gbuf[64 + lane]];
            // the node's counter deltas at the LDS address the record carries (no index arithmetic)
            auto nd_at = [&](const uint4& q) { return *reinterpret_cast<const uint2*>(lds + (q.w >> 16)); };
            uint2 n0 = nd_at(q0);
            uint32_t e2 = gbuf[128 + lane];
            // Update c's counter update and attractor test are made after update c + 1's plane
            // reads are issued, while they are in flight: they only decide whether c + 1 is
            // applied (its act), so the dependent chain from one plane write to the next is the
            // LDS round trip and the y / write work, not also the counters (in source order the
            // wave issues them in between). pfl / psg / pnd carry update c's outcome.
            uint32_t pfl = 0u, psg = 0u;
            uint2 pnd = make_uint2(0u, 0u);
            // packed mismatch counters: node i went to y, d = its delta, + d for 0 -> 1, - d for 1 -> 0;
            // then the test after that update (bitwise, no exec-mask branch around it)
            // (the select between the first-update test and the counters' test is written as
            // bit arithmetic: as a ?: the compiler branched around the counters' test)
            // :134 the first update of an env step is tested on o0: "first" is 1 when the update
            // being settled is it (used == 1 after it; in the chunk, update 1's settle with used 0
            // at the chunk's start)
            // lane flags as 32-bit masks (0 / all ones): the bit operations below are single v_bitop3 /
            // v_and, the counter step an AND with the changed-bit mask, used -= the active mask (as
            // bools they took 16-bit selects, a compare and a select per update: 261 -> 249 VALU and
            // 39 -> 24 SALU per 8 updates; 131,072 envs per step 1.37 -> 1.31 ms,
            // profiles/r03_r6_settle_mask_ab.txt)
            const uint32_t h0 = hit0 ? ~0u : 0u;
            const uint32_t f1 = (used == 0u && !a.first_tested) ? ~0u : 0u;
            uint32_t actm = ~0u, hitm = 0u;
            auto settle = [&](uint32_t pending, uint32_t first) {
                m_lo += ((pnd.x & pfl) ^ psg) - psg;
                uint32_t zb = has_zero_byte(m_lo);
                if constexpr (!ONE_WORD) {
                    m_hi += ((pnd.y & pfl) ^ psg) - psg;
                    zb |= has_zero_byte(m_hi);
                }
                const uint32_t z = zb != 0u ? ~0u : 0u;
                const uint32_t t = (z ^ (first & (z ^ h0))) & pending;  // the test's outcome (o0's on :134)
                hitm |= actm & t;  // one v_bitop3 each: no separate hit mask
                actm &= ~t;
            };
            // the wave tests for "no lane active" once per ENV_UNROLL updates, not per update: the
            // per-update ballot + branch made every update wait for the whole previous one (the
            // wave cannot issue past an unresolved branch). Lanes that finish inside a block run
            // its remaining updates masked (act = 0: nothing is written); the test sees act before
            // the block's last update is settled, so a wave may run one masked block more.
            // The cap test is compiled in only for chunks where some lane of the wave can reach
            // the cap (lim < CH); the other chunks run the loop without it.
            auto chunk = [&](auto cap_near) {
            for (uint32_t c0 = 0; c0 < CH; c0 += ENV_UNROLL) {
#pragma unroll
            for (uint32_t u = 0; u < ENV_UNROLL; ++u) {
                const uint32_t c = c0 + u;
                const uint4 q = q0;
                const uint2 nd = n0;
                // unconditional (clamped) prefetches: no branch, so no wait before the plane reads
                n0 = nd_at(q1);
                q0 = q1;
                q1 = erec[e2];
                e2 = gbuf[min(c + 3, CH - 1) * 64 + lane];
                // Predstep (base.py:100-118): Y = tt[x_in0 x_in1 x_in2 x_self] from the plane
                const uint32_t b0 = *reinterpret_cast<const uint32_t*>(pb + (q.x & 0xFFFFu));
                const uint32_t b1 = *reinterpret_cast<const uint32_t*>(pb + (q.x >> 16));
                const uint32_t b2 = *reinterpret_cast<const uint32_t*>(pb + (q.y & 0xFFFFu));
                const uint32_t self = *reinterpret_cast<const uint32_t*>(pb + (q.y >> 16));
                settle(c != 0 ? ~0u : 0u, c == 1 ? f1 : 0u);  // update c - 1 (nothing pending before the chunk's first)
                if constexpr (decltype(cap_near)::value)
                    actm &= c < lim ? ~0u : 0u;  // the update cap (pbn_target_multi.py's loop is unbounded)
                const uint32_t shs = q.z >> 24;
                const uint32_t xs = __builtin_amdgcn_ubfe(self, shs, 1);
                const uint32_t p = (__builtin_amdgcn_ubfe(b0, q.z, 1) << 3) |
                                   (__builtin_amdgcn_ubfe(b1, q.z >> 8, 1) << 2) |
                                   (__builtin_amdgcn_ubfe(b2, q.z >> 16, 1) << 1) | xs;
                const uint32_t y = __builtin_amdgcn_ubfe(q.w, p, 1);
                const uint32_t fl = (xs ^ y) & actm;  // the bit changes (and is applied)
                *reinterpret_cast<uint32_t*>(const_cast<uint8_t*>(pb) + (q.y >> 16)) = self ^ (fl << (shs & 31u));
                used -= actm;
                pfl = 0u - fl;
                psg = y - 1u;  // 0 (y = 1) or all ones (y = 0)
                pnd = nd;
            }
            if (__ballot(actm != 0u) == 0) break;
            }
            };

            if (__ballot(lim < CH) != 0)
                chunk(std::true_type{});
            else
                chunk(std::false_type{});
            settle(~0u, (used == 1u && !a.first_tested) ? ~0u : 0u);  // the last update made
            act = actm != 0u;
            hitf = hitm != 0u;
            capped = !hitf && used >= a.update_cap;
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
                philox_draw(a.seed, used >> 1, a.call_idx + t, g, STREAM_ENV, w);
                const bool odd = (used & 1u) != 0u;
                i = philox_node<KIND>(odd ? w[2] : w[0], N);
                k53 = u32_k53(odd ? w[3] : w[1]);
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
        }  // !in_tail
        if (!done) continue;

        // ---- finish: outputs of step() (:148-154) into step t's slot, then the env's next step
        uint64_t s[W];
        from_plane<W>(P, s);
        uint64_t o[W];
#pragma unroll
        for (int k = 0; k < W; ++k) o[k] = (used <= 1 && !a.first_tested) ? o0[k] : s[k];
        const uint64_t eo = (uint64_t)t * a.B + (uint64_t)e;
        store_state<W>(a.obs + eo * W, o);
        const bool term = cube_match<W>(o, target);  // :190-199 (target[0] only)
        a.reward[eo] = (term ? a.reward_success : 0) - a.action_cost * n_act;  // :218-222
        a.flags[eo] = (uint8_t)((term ? 1 : 0) | (nst == a.horizon ? 2 : 0) | (capped ? 4 : 0));
        a.n_updates[eo] = used;
#ifdef PBN_STAMPS
        ncapped += capped ? 1u : 0u;
#endif
        ++t;
        begin_steps(s);
    }
#ifdef PBN_STAMPS
    est[7] = __builtin_amdgcn_s_memrealtime();
    for (uint32_t k = 0; k < 64; ++k) est[14] += (uint32_t)__shfl((int)ncapped, (int)k);
    est[12] = blockIdx.x;
    est[13] = __smid();
    const uint32_t wv = blockIdx.x * (ENV_BLOCK / 64) + threadIdx.x / 64;
    if (lane == 0 && wv < 16384)
        for (int k = 0; k < ENV_STAMPS; ++k) g_env_stamps[(uint64_t)wv * ENV_STAMPS + k] = est[k];
#endif
}

// ------------------------------------------------------------------ R6, group mode
// The same env step with G lanes per env: a block of G consecutive updates of one env is
// evaluated by the G lanes at once (parallel in time), so one env advances G updates per
// round trip instead of one. The draws of the block do not depend on the state (Philox
// counter = update index), so lane k knows its node i_k and predictor record up front;
// what it needs are the values of its 4 input nodes at time k, i.e. the output of the
// last update j < k in the block that wrote each input, or the block-start value. The
// writers are found from the byte-packed node list of the group; the outputs y_k are
// then the fixed point of y_k = tt_k(inputs from writers), a DAG of depth < G: every
// round that changes nothing is exact. Per-update mismatch deltas are prefix-summed
// across the group (packed byte counters, as in k_env), the first update whose counters
// hit a cube ends the env step, and the final writer of each node in the committed
// prefix sets its bit in the env's LDS row (ds_or / ds_and: distinct nodes, possibly one
// dword). Same Philox counters as k_env, so the results are bit-identical to lane mode.
//
// Used where the batch is small against the chip (BASELINE config 5: 131,072 envs per
// GPU): there lane mode is latency-bound on the tail of long until-attractor loops.
// Requirements: predictor mix, N <= 256 (byte-packed node list), fast byte counters.

template <int G>
__device__ __forceinline__ uint32_t grp_bcast(uint32_t v, uint32_t j) {
    static_assert(G == 2 || G == 4 || G == 8, "group size");
    if constexpr (G <= 4) {
        // quad_perm [j,j,j,j] (G == 2: lanes 0/1 and 2/3 of each quad form two groups)
        switch (j) {
            case 0: return G == 2 ? (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xA0, 0xF, 0xF, false)   // [0,0,2,2]
                                  : (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x00, 0xF, 0xF, false);  // [0,0,0,0]
            case 1: return G == 2 ? (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xF5, 0xF, 0xF, false)   // [1,1,3,3]
                                  : (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x55, 0xF, 0xF, false);  // [1,1,1,1]
            case 2: return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xAA, 0xF, 0xF, false);
            default: return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xFF, 0xF, 0xF, false);
        }
    } else {
        // ds_swizzle bit-mask mode within 32 lanes: src = (lane & 0x18) | j
        switch (j) {
            case 0: return (uint32_t)__builtin_amdgcn_ds_swizzle((int)v, 0x18 | (0 << 5));
            case 1: return (uint32_t)__builtin_amdgcn_ds_swizzle((int)v, 0x18 | (1 << 5));
            case 2: return (uint32_t)__builtin_amdgcn_ds_swizzle((int)v, 0x18 | (2 << 5));
            case 3: return (uint32_t)__builtin_amdgcn_ds_swizzle((int)v, 0x18 | (3 << 5));
            case 4: return (uint32_t)__builtin_amdgcn_ds_swizzle((int)v, 0x18 | (4 << 5));
            case 5: return (uint32_t)__builtin_amdgcn_ds_swizzle((int)v, 0x18 | (5 << 5));
            case 6: return (uint32_t)__builtin_amdgcn_ds_swizzle((int)v, 0x18 | (6 << 5));
            default: return (uint32_t)__builtin_amdgcn_ds_swizzle((int)v, 0x18 | (7 << 5));
        }
    }
}

// value of lane (lane - n) of the same 16-lane row, 0 where that lane is outside the row
template <int N_>
__device__ __forceinline__ uint32_t row_shr(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x110 + N_, 0xF, 0xF, true);
}

// 0x80 in every byte of v that is zero (exact, no false positives)
__device__ __forceinline__ uint32_t zero_bytes(uint32_t v) {
    return ~(((v & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | v | 0x7F7F7F7Fu);
}

// Byte-packed node list of a group (G <= 8: two words). match(x) -> 0x80 per byte j with i_j == x.
template <int G>
struct GroupNodes {
    uint32_t lo = 0, hi = 0;
    __device__ __forceinline__ explicit GroupNodes(uint32_t i) {
#pragma unroll
        for (int j = 0; j < G; ++j) {
            const uint32_t v = grp_bcast<G>(i, (uint32_t)j);
            if (j < 4)
                lo |= v << (8 * j);
            else
                hi |= v << (8 * (j - 4));
        }
        if (G < 4) lo |= 0xFFFFFFFFu << (8 * G);  // unused bytes never match (node < 256)
        if (G <= 4) hi = 0xFFFFFFFFu;
    }
    // bytes j in [j0, j1) of the list equal to x, as a bit mask over j
    __device__ __forceinline__ uint32_t match(uint32_t x, uint32_t j0, uint32_t j1) const {
        const uint32_t xx = x * 0x01010101u;
        const uint32_t zl = zero_bytes(lo ^ xx), zh = zero_bytes(hi ^ xx);
        // compress 0x80 per byte to one bit per byte
        uint32_t m = ((zl >> 7) & 1u) | ((zl >> 14) & 2u) | ((zl >> 21) & 4u) | ((zl >> 28) & 8u);
        if (G > 4) m |= (((zh >> 7) & 1u) | ((zh >> 14) & 2u) | ((zh >> 21) & 4u) | ((zh >> 28) & 8u)) << 4;
        const uint32_t rng = ((1u << j1) - 1u) & ~((1u << j0) - 1u);
        return m & rng;
    }
};

// One block of G consecutive updates of a group's env, lane k holding update k: node i, its
// predictor record and the block-start values v of its operands (in0, in1, in2, self). Returns
// y (node i's new value) and old (its value right before update k), exact in every lane.
template <int G>
struct GrpBlock {
    uint32_t y = 0, old = 0;
    uint32_t ip = 0;  // G == 2: the partner lane's node
    GroupNodes<G> nodes;
    __device__ __forceinline__ explicit GrpBlock(uint32_t i) : nodes(G == 2 ? 0u : i) {}
    // update k is the last writer of node i among the first n_done updates of the block
    __device__ __forceinline__ bool last(uint32_t i, uint32_t k, uint32_t n_done) const {
        return G == 2 ? (k == 1 || n_done < 2 || ip != i) : nodes.match(i, k + 1, n_done) == 0u;
    }
};

template <int G>
__device__ __forceinline__ GrpBlock<G> grp_resolve(uint32_t i, uint64_t rec, const uint32_t (&in)[4],
                                                   const uint32_t (&v)[4], uint32_t k, uint32_t gbase,
                                                   uint32_t gmask) {
    GrpBlock<G> b(i);
    const uint32_t tt = (uint32_t)(rec >> 48);
    auto tt_of = [&](const uint32_t (&x)[4]) { return (tt >> ((x[0] << 3) | (x[1] << 2) | (x[2] << 1) | x[3])) & 1u; };
    if constexpr (G == 2) {
        // pairs: lane 1 depends on lane 0 only where an input is lane 0's node
        b.ip = (uint32_t)__builtin_amdgcn_mov_dpp((int)i, 0xB1, 0xF, 0xF, false);  // quad_perm [1,0,3,2]
        const uint32_t y0 = tt_of(v);  // exact in lane 0
        const uint32_t yb = (uint32_t)__builtin_amdgcn_mov_dpp((int)y0, 0xA0, 0xF, 0xF, false);  // [0,0,2,2]
        uint32_t x[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) x[q] = (k == 1 && in[q] == b.ip) ? yb : v[q];
        b.y = tt_of(x);
        b.old = x[3];
    } else {
        int32_t wr[4];  // last writer j < k of each input, or -1
        bool dep = false;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const uint32_t mm = b.nodes.match(in[q], 0, k);
            wr[q] = mm ? 31 - __clz((int)mm) : -1;
            dep |= mm != 0;
        }
        auto eval = [&](uint32_t Y, uint32_t* self_old) {
            uint32_t x[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) x[q] = wr[q] >= 0 ? (Y >> wr[q]) & 1u : v[q];
            *self_old = x[3];
            return tt_of(x);
        };
        b.y = eval(0u, &b.old);  // exact where no input has an in-block writer
        if (__ballot(dep) != 0) {
            // after round r lanes 0..r are exact, so round G - 1 at the latest changes nothing;
            // a round that changes nothing has `old` computed from the final outputs
#pragma unroll 1
            for (int r = 0; r < G; ++r) {
                const uint32_t Y = (uint32_t)(__ballot(b.y != 0u) >> gbase) & gmask;
                const uint32_t yn = eval(Y, &b.old);
                if (__ballot(yn != b.y) == 0) break;
                b.y = yn;
            }
        }
    }
    return b;
}

template <int W, int G>
__global__ __launch_bounds__(BLOCK) void k_env_grp(EnvArgs a) {
    extern __shared__ __align__(16) uint8_t lds[];
    stage_image(reinterpret_cast<const uint4*>(a.img), a.L.bytes / 16, reinterpret_cast<uint4*>(lds));
    __syncthreads();
    const uint32_t N = (uint32_t)a.L.n_nodes;
    const uint64_t* cubes = reinterpret_cast<const uint64_t*>(lds + a.off_cubes);
    const uint64_t* target = reinterpret_cast<const uint64_t*>(lds + a.off_target);
    const uint2* ndelta = reinterpret_cast<const uint2*>(lds + a.off_ndelta);
    const uint64_t* recs = reinterpret_cast<const uint64_t*>(lds + a.L.off_rec);
    const int32_t H = a.n_cubes;
    const uint32_t lane = __lane_id();
    const uint32_t k = lane & (G - 1);                     // position in the group = update slot
    const uint32_t gbase = lane & ~(uint32_t)(G - 1);
    const uint32_t gmask = (1u << G) - 1u;
    // the env's 2W dwords, one row per group (bank = group * 2W + dword: 8 groups of W = 4 fill 64 banks)
    uint32_t* row = reinterpret_cast<uint32_t*>(lds + a.off_gen) + (threadIdx.x / G) * (2 * W);
    auto wave_sync = [] {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    };

    // per-env registers, identical in every lane of the group
    int64_t e = -1;
    uint32_t t = 0;  // env step of this launch
    bool exhausted = false;
    uint64_t o0[W];
    uint32_t m_lo = 0, m_hi = 0, used = 0;
    bool hit0 = false;
    int64_t nst = 0;
    int n_act = 0;
    uint64_t gid = 0;

    // step t (or the first later step with a valid action row) of env e from state s; with no
    // step left, write the env back and free the group (as begin_steps in k_env)
    auto begin_steps = [&](uint64_t (&s)[W]) {
        for (; t < a.n_calls; ++t) {
            uint64_t f[W];
#pragma unroll
            for (int q = 0; q < W; ++q) f[q] = s[q];
            bool bad = false;
            n_act = apply_actions<W>(f, a.actions + ((uint64_t)t * a.B + (uint64_t)e) * (uint64_t)a.A, a.A,
                                     a.offset, a.dedup, (int32_t)N, &bad);
            if (bad) {  // reference raises ValueError; this env step is skipped, the env left untouched
                if (k == 0) atomicOr(a.error, 1);
                continue;
            }
            ++nst;  // :123
#pragma unroll
            for (int q = 0; q < W; ++q) o0[q] = f[q];  // :133 observation before the update
            if (k == 0) {
#pragma unroll
                for (int q = 0; q < W; ++q) {
                    row[2 * q] = (uint32_t)f[q];
                    row[2 * q + 1] = (uint32_t)(f[q] >> 32);
                }
            }
            uint32_t m[2] = {0x01010101u, 0x01010101u};  // unused cubes: never zero
            for (int32_t h = 0; h < H; ++h) {
                const uint32_t c = cube_mismatch<W>(f, cubes + (uint64_t)h * 2 * W);
                const uint32_t sh = 8u * (uint32_t)(h & 3);
                m[h >> 2] = (m[h >> 2] & ~(0xFFu << sh)) | (c << sh);
            }
            m_lo = m[0];
            m_hi = m[1];
            hit0 = (has_zero_byte(m_lo) | has_zero_byte(m_hi)) != 0u;
            used = 0;
            return;
        }
        if (k == 0) {
            store_state<W>(a.state + (uint64_t)e * W, s);
            a.n_steps[e] = nst;
        }
        e = -1;
    };

    for (;;) {
        // ---- refill groups without an env: one atomic per wave, ranks over the groups' leaders
        const bool need = e < 0 && !exhausted;
        const uint64_t need_lead = __ballot(need && k == 0);
        if (need_lead) {
            const uint32_t leader = (uint32_t)__ffsll((unsigned long long)need_lead) - 1u;
            unsigned long long base = 0;
            if (lane == leader) base = atomicAdd(a.counter, (unsigned long long)__popcll(need_lead));
            base = __shfl(base, (int)leader);
            if (need) {
                const uint64_t ne = base + (uint64_t)__popcll(need_lead & ((1ull << gbase) - 1ull));
                if (ne >= a.B) {
                    exhausted = true;
                } else {
                    uint64_t s[W];
                    load_state<W>(a.state + ne * W, s);  // every lane of the group: one request
                    e = (int64_t)ne;
                    gid = a.env_base + ne;
                    t = 0;
                    nst = a.n_steps[ne];
                    begin_steps(s);
                }
            }
            wave_sync();
        }
        if (__ballot(e >= 0) == 0) {
            if (__ballot(!exhausted) == 0) break;
            continue;
        }

        // ---- one block: update used + k of this group's env in lane k (idle groups compute junk)
        // (a block starts at a multiple of G: lanes 2m and 2m + 1 share Philox call (used >> 1) + m)
        uint32_t w4[4];
        philox_draw(a.seed, (used + k) >> 1, a.call_idx + t, gid, STREAM_ENV, w4);
        const uint32_t i = philox_node<KIND_PREDICTOR_MIX>((k & 1u) ? w4[2] : w4[0], N);
        const uint64_t rec = recs[i * a.L.pmax + predictor_choice(i, u32_k53((k & 1u) ? w4[3] : w4[1]), lds, a.L)];
        const uint2 nd = ndelta[i];
        const uint32_t in[4] = {(uint32_t)rec & 0xFFFFu, (uint32_t)(rec >> 16) & 0xFFFFu,
                                (uint32_t)(rec >> 32) & 0xFFFFu, i};
        uint32_t v[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) v[q] = (row[in[q] >> 5] >> (in[q] & 31u)) & 1u;  // block-start values
        const GrpBlock<G> blk = grp_resolve<G>(i, rec, in, v, k, gbase, gmask);
        const uint32_t y = blk.y, old = blk.old;
        // mismatch counters after each update of the block (inclusive prefix over the group)
        const bool changed = y != old;
        uint32_t dl = changed ? (y ? nd.x : 0u - nd.x) : 0u;
        uint32_t dh = changed ? (y ? nd.y : 0u - nd.y) : 0u;
        {
            uint32_t tl = row_shr<1>(dl), th = row_shr<1>(dh);
            dl += k >= 1 ? tl : 0u;
            dh += k >= 1 ? th : 0u;
            if constexpr (G >= 4) {
                tl = row_shr<2>(dl);
                th = row_shr<2>(dh);
                dl += k >= 2 ? tl : 0u;
                dh += k >= 2 ? th : 0u;
            }
            if constexpr (G >= 8) {
                tl = row_shr<4>(dl);
                th = row_shr<4>(dh);
                dl += k >= 4 ? tl : 0u;
                dh += k >= 4 ? th : 0u;
            }
        }
        const uint32_t ml = m_lo + dl, mh = m_hi + dh;
        const bool valid = used + k < a.update_cap;
        const bool hit = (used + k == 0 && !a.first_tested) ? hit0 : (has_zero_byte(ml) | has_zero_byte(mh)) != 0u;
        const uint32_t SM = (uint32_t)(__ballot(valid && hit) >> gbase) & gmask;
        const uint32_t VM = (uint32_t)(__ballot(valid) >> gbase) & gmask;
        const uint32_t n_done = SM ? (uint32_t)__ffs((int)SM) : (uint32_t)__popc(VM);
        const bool done = SM != 0u || used + n_done >= a.update_cap;
        const bool capped = SM == 0u;  // only meaningful when done
        // commit: the last writer of each node among the first n_done updates sets its bit
        const bool last = blk.last(i, k, n_done);
        if (e >= 0 && k < n_done && y != v[3] && last) {
            if (y)
                atomicOr(&row[i >> 5], 1u << (i & 31u));
            else
                atomicAnd(&row[i >> 5], ~(1u << (i & 31u)));
        }
        uint32_t nl, nh;  // counters after the last committed update
        if constexpr (G == 2) {
            const uint32_t l1 = (uint32_t)__builtin_amdgcn_mov_dpp((int)ml, 0xF5, 0xF, 0xF, false);  // [1,1,3,3]
            const uint32_t h1 = (uint32_t)__builtin_amdgcn_mov_dpp((int)mh, 0xF5, 0xF, 0xF, false);
            const uint32_t l0 = (uint32_t)__builtin_amdgcn_mov_dpp((int)ml, 0xA0, 0xF, 0xF, false);  // [0,0,2,2]
            const uint32_t h0 = (uint32_t)__builtin_amdgcn_mov_dpp((int)mh, 0xA0, 0xF, 0xF, false);
            nl = n_done == 2 ? l1 : l0;
            nh = n_done == 2 ? h1 : h0;
        } else {
            const uint32_t src = gbase + (n_done ? n_done - 1u : 0u);
            nl = (uint32_t)__shfl((int)ml, (int)src);
            nh = (uint32_t)__shfl((int)mh, (int)src);
        }
        if (e >= 0 && n_done) {
            m_lo = nl;
            m_hi = nh;
        }
        wave_sync();
        if (e < 0) continue;
        used += n_done;
        if (!done) continue;

        // ---- finish: outputs of step() (:148-154) into step t's slot (group leader), next step
        uint64_t s[W];
#pragma unroll
        for (int q = 0; q < W; ++q) s[q] = (uint64_t)row[2 * q] | ((uint64_t)row[2 * q + 1] << 32);
        if (k == 0) {
            uint64_t o[W];
#pragma unroll
            for (int q = 0; q < W; ++q) o[q] = (used <= 1 && !a.first_tested) ? o0[q] : s[q];
            const uint64_t eo = (uint64_t)t * a.B + (uint64_t)e;
            store_state<W>(a.obs + eo * W, o);
            const bool term = cube_match<W>(o, target);  // :190-199 (target[0] only)
            a.reward[eo] = (term ? a.reward_success : 0) - a.action_cost * n_act;  // :218-222
            a.flags[eo] = (uint8_t)((term ? 1 : 0) | (nst == a.horizon ? 2 : 0) | (capped ? 4 : 0));
            a.n_updates[eo] = used;
        }
        wave_sync();  // every lane's row reads before the next step rewrites the row
        ++t;
        begin_steps(s);
        wave_sync();
    }
}

// ------------------------------------------------------------------ rollout, group mode
// k_rollout with G lanes per env (predictor mix, N <= 256): each block of G consecutive updates
// is resolved at once by grp_resolve (the same machinery as k_env_grp), the env's state kept as
// one LDS row per group. Same Philox counters as k_rollout, so the same states. For batches too
// small to give every SIMD several waves in lane mode (BASELINE config 2: 65,536 envs = one
// wave per SIMD), where one env per lane is latency-bound on its own update chain.
template <int W, int G>
__global__ __launch_bounds__(BLOCK) void k_rollout_grp(StepArgs a) {
    extern __shared__ __align__(16) uint8_t lds[];
    const Thr32 X = thr32_layout(a.L);  // the compact image (thresholds on the choice word)
    stage_image(reinterpret_cast<const uint4*>(reinterpret_cast<const uint8_t*>(a.img) + a.L.bytes), X.bytes / 16,
                reinterpret_cast<uint4*>(lds));
    __syncthreads();
    const uint32_t N = (uint32_t)a.L.n_nodes;
    const uint32_t lane = __lane_id();
    const uint32_t k = lane & (G - 1);
    const uint32_t gbase = lane & ~(uint32_t)(G - 1);
    const uint32_t gmask = (1u << G) - 1u;
    uint32_t* row = reinterpret_cast<uint32_t*>(lds + a.L.plane_off) + (threadIdx.x / G) * (2 * W);
    auto wave_sync = [] {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    };
    const uint64_t groups = (uint64_t)gridDim.x * (BLOCK / G);
    // every group of a wave takes the same number of trips (ballots and wave syncs inside)
    for (uint64_t e = (uint64_t)blockIdx.x * (BLOCK / G) + threadIdx.x / G;; e += groups) {
        const bool live = e < a.B;
        if (__ballot(live) == 0) break;
        uint64_t s[W];
        if (live) {
            load_state<W>(a.state + e * W, s);
            if (k == 0) {
#pragma unroll
                for (int q = 0; q < W; ++q) {
                    row[2 * q] = (uint32_t)s[q];
                    row[2 * q + 1] = (uint32_t)(s[q] >> 32);
                }
            }
        }
        wave_sync();
        const uint64_t g = a.env_base + e;
        for (uint32_t used = 0; used < a.T; used += G) {
            uint32_t nw, cw;
            step_words(a.seed, a.update_base + used + k, g, nw, cw);
            const uint32_t i = philox_node<KIND_PREDICTOR_MIX>(nw, N);
            const uint64_t rec = predictor_record32(i, cw, lds, X);
            const uint32_t in[4] = {(uint32_t)rec & 0xFFFFu, (uint32_t)(rec >> 16) & 0xFFFFu,
                                    (uint32_t)(rec >> 32) & 0xFFFFu, i};
            uint32_t v[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) v[q] = (row[in[q] >> 5] >> (in[q] & 31u)) & 1u;  // block-start values
            const GrpBlock<G> blk = grp_resolve<G>(i, rec, in, v, k, gbase, gmask);
            const uint32_t n_done = min((uint32_t)G, a.T - used);
            // the last writer of each node among the block's valid updates sets its bit
            if (live && k < n_done && blk.y != v[3] && blk.last(i, k, n_done)) {
                if (blk.y)
                    atomicOr(&row[i >> 5], 1u << (i & 31u));
                else
                    atomicAnd(&row[i >> 5], ~(1u << (i & 31u)));
            }
            wave_sync();
        }
        if (live && k == 0) {
            uint64_t out[W];
            bool diff = false;  // whole env, only if it differs (see k_step_single)
#pragma unroll
            for (int q = 0; q < W; ++q) {
                out[q] = (uint64_t)row[2 * q] | ((uint64_t)row[2 * q + 1] << 32);
                diff |= out[q] != s[q];
            }
            if (diff) store_state<W>(a.state + e * W, out);
        }
        wave_sync();  // the row is rewritten by the group's next env
    }
}

// ------------------------------------------------------------------ dispatch
template <int W, int KIND>
static void* step_fn(int store, int replay, int sb, int rollout, int grp) {
    if (replay) return (void*)k_step<W, KIND, STORE_FULL, 1, BLOCK>;
    if constexpr (KIND == KIND_PREDICTOR_MIX && W <= 4) {
        if (rollout && grp == 2) return (void*)k_rollout_grp<W, 2>;
        if (rollout && grp == 4) return (void*)k_rollout_grp<W, 4>;
        if (rollout && grp == 8) return (void*)k_rollout_grp<W, 8>;
    }
    if (grp > 1) return nullptr;
    if (rollout) return sb == 1024 ? (void*)k_rollout<W, KIND, 1024> : (void*)k_rollout<W, KIND, BLOCK>;
    if (sb == 1024)
        return store == STORE_DIRTY ? (void*)k_step<W, KIND, STORE_DIRTY, 0, 1024>
                                    : (void*)k_step<W, KIND, STORE_FULL, 0, 1024>;
    return store == STORE_DIRTY ? (void*)k_step<W, KIND, STORE_DIRTY, 0, BLOCK>
                                : (void*)k_step<W, KIND, STORE_FULL, 0, BLOCK>;
}

template <int KIND>
static void* step_fn_w(int W, int store, int replay, int sb, int rollout, int grp) {
    switch (W) {
        case 1: return step_fn<1, KIND>(store, replay, sb, rollout, grp);
        case 2: return step_fn<2, KIND>(store, replay, sb, rollout, grp);
        case 3: return step_fn<3, KIND>(store, replay, sb, rollout, grp);
        case 4: return step_fn<4, KIND>(store, replay, sb, rollout, grp);
        case 5: return step_fn<5, KIND>(store, replay, sb, rollout, grp);
        case 6: return step_fn<6, KIND>(store, replay, sb, rollout, grp);
        case 7: return step_fn<7, KIND>(store, replay, sb, rollout, grp);
        case 8: return step_fn<8, KIND>(store, replay, sb, rollout, grp);
    }
    return nullptr;
}

template <int G>
static void* env_grp_fn(int W) {
    switch (W) {
        case 1: return (void*)k_env_grp<1, G>;
        case 2: return (void*)k_env_grp<2, G>;
        case 3: return (void*)k_env_grp<3, G>;
        case 4: return (void*)k_env_grp<4, G>;
    }
    return nullptr;  // N <= 256
}

template <int KIND>
static void* env_fn_w(int W, int replay, int fast, int grp) {
    if (fast == 3) {
        if (KIND != KIND_PREDICTOR_MIX || replay) return nullptr;
        return grp == 2 ? env_grp_fn<2>(W) : grp == 4 ? env_grp_fn<4>(W) : grp == 8 ? env_grp_fn<8>(W) : nullptr;
    }
#define PBN_ENV_CASE(w)                                                                  \
    case w:                                                                              \
        if (fast == 2 && KIND == KIND_PREDICTOR_MIX && !replay) return (void*)k_env<w, KIND_PREDICTOR_MIX, 0, 2>; \
        if (fast == 4 && KIND == KIND_PREDICTOR_MIX && !replay) return (void*)k_env<w, KIND_PREDICTOR_MIX, 0, 4>; \
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

static int launch(void* fn, int grid, uint32_t lds, void* stream, void* args, size_t args_size, int block = BLOCK) {
    if (!fn) return (int)hipErrorInvalidValue;
    (void)args_size;
    void* kargs[] = {args};
    return (int)hipLaunchKernel(fn, dim3((unsigned)grid), dim3((unsigned)block), kargs, lds, (hipStream_t)stream);
}

uint32_t step_lds_bytes(int W, uint32_t image_bytes, int sb, int grp) {
    if (grp > 1) return image_bytes + 8u * (uint32_t)W * (BLOCK / (uint32_t)grp);  // one row per group
    return image_bytes + 8u * (uint32_t)W * (uint32_t)sb;
}

static void* step_kernel(int W, int kind, int store_mode, int replay, int sb, int rollout, int grp) {
    if (replay) sb = BLOCK;
    return kind == KIND_PREDICTOR_MIX ? step_fn_w<KIND_PREDICTOR_MIX>(W, store_mode, replay, sb, rollout, grp)
                                      : step_fn_w<KIND_PROB_TABLE>(W, store_mode, replay, sb, rollout, grp);
}

int launch_step(int W, const StepArgs& a, int store_mode, int replay, int sb, int grid, void* stream) {
    if (replay) sb = BLOCK;
    const bool rollout = !replay && a.T > 1;
    const int grp = rollout && a.grp > 1 ? a.grp : 1;
    if (grp > 1) sb = BLOCK;
    void* fn = step_kernel(W, a.L.kind, store_mode, replay, sb, rollout, grp);
    if (!fn) return (int)hipErrorInvalidValue;
    const uint32_t lds = step_lds_bytes(W, replay ? a.L.bytes : a.L.plane_off, sb, grp);
    if (lds > 64u * 1024u) {
        hipError_t e = hipFuncSetAttribute((const void*)fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) return (int)e;
    }
    StepArgs c = a;
    void* kargs[] = {&c};
    return (int)hipLaunchKernel(fn, dim3((unsigned)grid), dim3((unsigned)sb), kargs, lds, (hipStream_t)stream);
}

#ifdef PBN_STAMPS
}  // namespace pbn
extern "C" int pbn_exp_stamps(void* out, size_t bytes) {
    return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(pbn::g_stamps), bytes, 0, hipMemcpyDeviceToHost);
}
extern "C" int pbn_exp_stamps_clear() {
    static uint64_t z[16384 * pbn::ENV_STAMPS];
    int rc = (int)hipMemcpyToSymbol(HIP_SYMBOL(pbn::g_stamps), z, 16384 * 8 * 8, 0, hipMemcpyHostToDevice);
    if (!rc) rc = (int)hipMemcpyToSymbol(HIP_SYMBOL(pbn::g_env_stamps), z, sizeof z, 0, hipMemcpyHostToDevice);
    return rc;
}
extern "C" int pbn_exp_env_stamps(void* out, size_t bytes) {
    return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(pbn::g_env_stamps), bytes, 0, hipMemcpyDeviceToHost);
}
namespace pbn {
#endif

// Advances the device-side update counter by k at the end of a captured run of step launches.
__global__ void k_bump(uint64_t* p, uint64_t k) {
    if (threadIdx.x == 0) p[threadIdx.x] += k;
}

int launch_bump(uint64_t* p, uint64_t k, void* stream) {
    void* kargs[] = {(void*)&p, (void*)&k};
    return (int)hipLaunchKernel((const void*)k_bump, dim3(1), dim3(64), kargs, 0, (hipStream_t)stream);
}

int launch_init(int W, const InitArgs& a, int grid, void* stream) {
    InitArgs c = a;
    return launch(init_fn(W), grid, 0, stream, &c, sizeof c);
}

int launch_flip(int W, const FlipArgs& a, int grid, void* stream) {
    FlipArgs c = a;
    return launch(flip_fn(W), grid, 0, stream, &c, sizeof c);
}

// Packed state words [B][W] -> one byte per node [B][N] (Graph.getState as bytes, base.py:320-324):
// one thread per output byte, so consecutive lanes write consecutive bytes (the rows of N bytes
// are not 4-byte aligned) and read the same few words through L1/L2.
__global__ __launch_bounds__(BLOCK) void k_unpack(const uint64_t* __restrict__ words, uint8_t* __restrict__ out,
                                                  uint64_t total, uint32_t N, uint32_t W) {
    if (total <= 0xFFFFFFFFull) {  // 32-bit index math (a 64-bit divide is a long software sequence)
        for (uint32_t k = blockIdx.x * BLOCK + threadIdx.x; k < (uint32_t)total; k += gridDim.x * BLOCK) {
            const uint32_t e = k / N, n = k - e * N;
            out[k] = (uint8_t)((words[(uint64_t)e * W + (n >> 6)] >> (n & 63u)) & 1u);
        }
        return;
    }
    for (uint64_t k = (uint64_t)blockIdx.x * BLOCK + threadIdx.x; k < total; k += (uint64_t)gridDim.x * BLOCK) {
        const uint64_t e = k / N;
        const uint32_t n = (uint32_t)(k - e * N);
        out[k] = (uint8_t)((words[e * W + (n >> 6)] >> (n & 63u)) & 1u);
    }
}

int launch_unpack(const uint64_t* words, uint8_t* out, uint64_t B, uint32_t N, uint32_t W, int grid, void* stream) {
    const uint64_t total = B * N;
    void* kargs[] = {(void*)&words, (void*)&out, (void*)&total, (void*)&N, (void*)&W};
    return (int)hipLaunchKernel((const void*)k_unpack, dim3((unsigned)grid), dim3(BLOCK), kargs, 0,
                                (hipStream_t)stream);
}

int launch_env_multi(int W, const EnvArgs& a, int replay, int grid, void* stream) {
    void* fn = a.L.kind == KIND_PREDICTOR_MIX ? env_fn_w<KIND_PREDICTOR_MIX>(W, replay, a.fast, a.grp)
                                              : env_fn_w<KIND_PROB_TABLE>(W, replay, a.fast, a.grp);
    EnvArgs c = a;
    return launch(fn, grid, env_lds_bytes(W, a.L.bytes + a.erec_shift, replay ? std::min(a.fast, 1) : a.fast, a.grp,
                                          a.L.n_nodes, a.chunk),
                  stream, &c, sizeof c, env_block(a.fast));
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

int max_blocks_step(int W, int kind, uint32_t lds_bytes, int sb, int* blocks_per_cu, int rollout, int grp) {
    if (grp > 1) sb = BLOCK;
    void* fn = step_kernel(W, kind, STORE_FULL, 0, sb, rollout, grp);
    if (!fn) return (int)hipErrorInvalidValue;
    return occupancy(fn, sb, step_lds_bytes(W, lds_bytes, sb, grp), blocks_per_cu);
}

uint32_t env_lds_bytes(int W, uint32_t image_bytes, int fast, int grp, int n_nodes, uint32_t chunk) {
    if (fast == 3) return image_bytes + 8u * (uint32_t)W * (BLOCK / (uint32_t)grp);  // one row per group
    const uint32_t planes = image_bytes + 8u * (uint32_t)W * ENV_BLOCK;
    (void)n_nodes;
    // fast == 4: 16 B of workgroup hand-off control after the per-wave draw buffers
    return fast == 2 || fast == 4 ? planes + (ENV_BLOCK / 64) * env_gen_wave_bytes(chunk) + (fast == 4 ? 16u : 0u) : planes;
}

int max_blocks_env(int W, int kind, int fast, int grp, uint32_t lds_bytes, int* blocks_per_cu, int n_nodes, uint32_t chunk) {
    void* fn = kind == KIND_PREDICTOR_MIX ? env_fn_w<KIND_PREDICTOR_MIX>(W, 0, fast, grp)
                                          : env_fn_w<KIND_PROB_TABLE>(W, 0, fast, grp);
    return occupancy(fn, env_block(fast), env_lds_bytes(W, lds_bytes, fast, grp, n_nodes, chunk), blocks_per_cu);
}

}  // namespace pbn
