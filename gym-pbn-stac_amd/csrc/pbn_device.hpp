// pbn_device.hpp -- device-side building blocks of the gfx950 PBN kernels.
//
// One lane owns one env: its W = ceil(N/64) state words live in VGPRs for the
// whole launch; the network tables live in LDS (staged once per workgroup from
// a packed "image" built on the host, see pbn_abi.cpp: build_image()).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "pbn_params.hpp"

namespace pbn {

// ---------------------------------------------------------------- Philox4x32-10
// Random123's Philox4x32 with 10 rounds (KAT-checked in tests/test_oracle.py and
// tests/test_gpu_parity.py). Each round is two 32x32->64 multiplies
// (v_mad_u64_u32) and four XORs.
#ifndef PBN_PHILOX_ROUNDS
#define PBN_PHILOX_ROUNDS 10  // only measurement builds (tools/) change this
#endif
__device__ __forceinline__ void philox4x32_10(uint32_t c[4], uint32_t k0, uint32_t k1) {
#pragma unroll
    for (int r = 0; r < PBN_PHILOX_ROUNDS; ++r) {
        if (r) {
            k0 += 0x9E3779B9u;
            k1 += 0xBB67AE85u;
        }
        const uint64_t p0 = (uint64_t)0xD2511F53u * c[0];
        const uint64_t p1 = (uint64_t)0xCD9E8D57u * c[2];
        // three-input XOR in one gfx950 v_bitop3_b32 (truth table 0x96), the key from an SGPR;
        // the compiler only forms a few of these on its own
        const uint32_t n0 = __builtin_amdgcn_bitop3_b32(k0, (uint32_t)(p1 >> 32), c[1], 0x96);
        const uint32_t n2 = __builtin_amdgcn_bitop3_b32(k1, (uint32_t)(p0 >> 32), c[3], 0x96);
        c[1] = (uint32_t)p1;
        c[3] = (uint32_t)p0;
        c[0] = n0;
        c[2] = n2;
    }
}

// Counter layout (shared with oracle/pbn_oracle.c philox_draw):
//   ctr = {c0, c1, gid_lo, (gid_hi & 0xFFFFFF) | stream << 24}, key = {seed_lo, seed_hi}
__device__ __forceinline__ void philox_draw(uint64_t seed, uint32_t c0, uint32_t c1, uint64_t gid, uint32_t stream,
                                            uint32_t w[4]) {
    w[0] = c0;
    w[1] = c1;
    w[2] = (uint32_t)gid;
    w[3] = ((uint32_t)(gid >> 32) & 0xFFFFFFu) | (stream << 24);
    philox4x32_10(w, (uint32_t)seed, (uint32_t)(seed >> 32));
}

// The same with the round keys recomputed by SALU adds at the call (seed must be wave-uniform): in a
// kernel short of SGPRs, 20 hoisted round keys are spilled to VGPR lanes and every round pays a
// v_readlane and a wait state (k_env's draw loops)
__device__ __forceinline__ void philox_draw_sk(uint64_t seed, uint32_t c0, uint32_t c1, uint64_t gid, uint32_t stream,
                                               uint32_t w[4]) {
    uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
    asm volatile("" : "+s"(k0), "+s"(k1));
    w[0] = c0;
    w[1] = c1;
    w[2] = (uint32_t)gid;
    w[3] = ((uint32_t)(gid >> 32) & 0xFFFFFFu) | (stream << 24);
    philox4x32_10(w, k0, k1);
}

// Draws of the step and R6 streams use two 32-bit words per update: the node word and the
// predictor-choice uniform a, taken as k53 = a << 21 | a >> 11 (32 random bits spread over the
// 53-bit grid, monotone in a, so the integer thresholds decide the choice exactly; choice
// probabilities exact to 2^-32). One Philox call (four words) thus serves two updates:
//   STREAM_STEP: update u of env g takes call {u, g >> 1}, words 2(g & 1) and 2(g & 1) + 1 (envs
//                2m and 2m + 1 share a call);
//   STREAM_ENV:  update u of an env step takes call {u >> 1, call index}, words 2(u & 1), +1.
// Shared with oracle/pbn_oracle.c (u32_k53, step_words).
__device__ __forceinline__ uint64_t u32_k53(uint32_t a) { return ((uint64_t)a << 21) | (uint64_t)(a >> 11); }

// Threshold T re-expressed on a: the smallest a with u32_k53(a) >= T (2^32 = never), so that
// u32_k53(a) >= T <=> a >= u32_threshold(T) (u32_k53 is monotone; u32_k53(T >> 21 - 1) < T).
__device__ __forceinline__ uint64_t u32_threshold(uint64_t T) {
    const uint64_t a0 = T >> 21;
    if (a0 >= (1ull << 32)) return 1ull << 32;
    return u32_k53((uint32_t)a0) >= T ? a0 : a0 + 1u;
}

// Lanes 2k and 2k + 1 swap a word (DPP quad_perm [1,0,3,2]). A lane whose partner is inactive
// gets its own value back.
__device__ __forceinline__ uint32_t swap_pair_lanes(uint32_t x) {
    return (uint32_t)__builtin_amdgcn_update_dpp((int)x, (int)x, 0xB1, 0xF, 0xF, false);
}

// STREAM_STEP words of update u for this lane's env g and env g + 2j (same parity), when lanes
// 2k / 2k + 1 hold envs 2m / 2m + 1 (even env base): each lane computes ONE call -- the even lane
// the call of its first env's pair, the odd lane that of its second env's pair -- and the pair
// swaps the two words the other needs. n*/c* = node word / choice word of the two envs.
__device__ __forceinline__ void step_words_paired(uint64_t seed, uint64_t u, uint64_t g0, uint64_t g1, bool odd,
                                                  uint32_t& n0, uint32_t& c0, uint32_t& n1, uint32_t& c1) {
    uint32_t w[4];
    philox_draw(seed, (uint32_t)u, (uint32_t)(u >> 32), (odd ? g1 : g0) >> 1, STREAM_STEP, w);
    const uint32_t r0 = swap_pair_lanes(odd ? w[0] : w[2]), r1 = swap_pair_lanes(odd ? w[1] : w[3]);
    n0 = odd ? r0 : w[0];
    c0 = odd ? r1 : w[1];
    n1 = odd ? w[2] : r0;
    c1 = odd ? w[3] : r1;
}

// STREAM_STEP words of update u for env g alone (one call per env).
__device__ __forceinline__ void step_words(uint64_t seed, uint64_t u, uint64_t g, uint32_t& n, uint32_t& c) {
    uint32_t w[4];
    philox_draw(seed, (uint32_t)u, (uint32_t)(u >> 32), g >> 1, STREAM_STEP, w);
    const bool h = (g & 1u) != 0u;
    n = h ? w[2] : w[0];
    c = h ? w[3] : w[1];
}

// random() == k53 * 2^-53, built CPython-style from two words (a>>5, b>>6).
__device__ __forceinline__ uint64_t k53_of(uint32_t a, uint32_t b) {
    return ((uint64_t)(a >> 5) << 26) | (uint64_t)(b >> 6);
}

// ---------------------------------------------------------------- packed state
// The state words must stay in VGPRs: a select chain over s[k] is recognised by
// the compiler as s[i >> 6] and demoted to a scratch array, so word selection is
// written as bitwise masks over 32-bit halves (no indexing).
__device__ __forceinline__ uint32_t lane_mask(uint32_t a, uint32_t b) { return 0u - (uint32_t)(a == b); }

template <int W>
__device__ __forceinline__ uint32_t getbit(const uint64_t (&s)[W], uint32_t i) {
    const uint32_t wi = i >> 6, sh = i & 31u, hi = (i >> 5) & 1u;
    uint32_t x = 0;
#pragma unroll
    for (int k = 0; k < W; ++k) {
        const uint32_t m = lane_mask(wi, (uint32_t)k);
        x |= ((uint32_t)(s[k] >> 32) & m & (0u - hi)) | ((uint32_t)s[k] & m & (hi - 1u));
    }
    return (x >> sh) & 1u;
}

template <int W>
__device__ __forceinline__ void setbit(uint64_t (&s)[W], uint32_t i, uint32_t v) {
    const uint64_t bit = (uint64_t)1 << (i & 63u);
    const uint64_t val = (uint64_t)(v & 1u) << (i & 63u);
    const uint32_t wi = i >> 6;
#pragma unroll
    for (int k = 0; k < W; ++k) {
        const uint64_t m = (uint64_t)(int64_t)(int32_t)lane_mask(wi, (uint32_t)k);
        s[k] = (s[k] & ~(bit & m)) | (val & m);
    }
}

template <int W>
__device__ __forceinline__ void load_state(const uint64_t* __restrict__ p, uint64_t (&s)[W]) {
    if constexpr (W % 2 == 0) {
        const ulonglong2* q = reinterpret_cast<const ulonglong2*>(p);
#pragma unroll
        for (int k = 0; k < W / 2; ++k) {
            ulonglong2 v = q[k];
            s[2 * k] = v.x;
            s[2 * k + 1] = v.y;
        }
    } else {
#pragma unroll
        for (int k = 0; k < W; ++k) s[k] = p[k];
    }
}

template <int W>
__device__ __forceinline__ void store_state(uint64_t* __restrict__ p, const uint64_t (&s)[W]) {
    if constexpr (W % 2 == 0) {
        ulonglong2* q = reinterpret_cast<ulonglong2*>(p);
#pragma unroll
        for (int k = 0; k < W / 2; ++k) q[k] = make_ulonglong2(s[2 * k], s[2 * k + 1]);
    } else {
#pragma unroll
        for (int k = 0; k < W; ++k) p[k] = s[k];
    }
}

// ---------------------------------------------------------------- LDS staging
// Copy the network image (16-byte granules) into LDS; every thread participates.
__device__ __forceinline__ void stage_image(const uint4* __restrict__ img, uint32_t n16, uint4* lds) {
    for (uint32_t k = threadIdx.x; k < n16; k += blockDim.x) lds[k] = img[k];
}

// ---------------------------------------------------------------- node updates
// Philox (node, k53) for update counter c0/c1 of env gid.
//   Bittner: node in [0, N-1] (base.py:308); PBN: node in [1, N-1] (pbn.py:131).
template <int KIND>
__device__ __forceinline__ uint32_t philox_node(uint32_t w0, uint32_t N) {
    if constexpr (KIND == KIND_PREDICTOR_MIX)
        return __umulhi(w0, N);
    else
        return 1u + __umulhi(w0, N - 1u);
}

// ---------------------------------------------------------------- LDS state planes
// SB = lanes per workgroup = the plane's row stride (dword d of lane l at d*SB + l).
template <int SB>
struct PlaneT {
    uint32_t* base;  // &planes[0][tid]
    __device__ __forceinline__ uint32_t get(uint32_t d) const { return base[d * SB]; }
    __device__ __forceinline__ void put(uint32_t d, uint32_t v) const { base[d * SB] = v; }
    __device__ __forceinline__ uint32_t bit(uint32_t i) const { return (get(i >> 5) >> (i & 31u)) & 1u; }
};
using Plane = PlaneT<BLOCK>;

// Bittner Predstep (base.py:89-119) evaluated on the LDS plane: the new value of node i.
// `self` is the dword holding node i (already read by the caller). Predictor choice
// (base.py:94-97): j = #{q : k53 >= thr[i][q]} over the padded thresholds (the padding
// never counts, so j <= count - 1: Python's for/break falling through to the last one).
// Thresholds and record are both addressed by i alone, and the threshold loop has a
// wave-uniform trip count (L.tp), so lanes do not diverge on per-node predictor counts.
__device__ __forceinline__ uint32_t predictor_choice(uint32_t i, uint64_t k53, const uint8_t* tbl,
                                                     const NetLayout& L) {
    const ulonglong2* thr = reinterpret_cast<const ulonglong2*>(tbl + L.off_thr) + (i * L.tp >> 1);
    const uint32_t n2 = L.tp >> 1;
    uint32_t j = 0;
    // up to 8 thresholds (Bittner-200: 4): every read issued before the first compare, so one LDS
    // round trip; n2 is wave-uniform (scalar branches). Reads past the node's row stay inside the
    // image / planes and are masked out.
    if (n2 == 2) {
        const ulonglong2 t0 = thr[0], t1 = thr[1];
        return (k53 >= t0.x ? 1u : 0u) + (k53 >= t0.y ? 1u : 0u) + (k53 >= t1.x ? 1u : 0u) +
               (k53 >= t1.y ? 1u : 0u);
    }
    if (n2 <= 4) {
        ulonglong2 t[4];
#pragma unroll
        for (uint32_t q = 0; q < 4; ++q) t[q] = thr[q];
#pragma unroll
        for (uint32_t q = 0; q < 4; ++q)
            j += q < n2 ? (k53 >= t[q].x ? 1u : 0u) + (k53 >= t[q].y ? 1u : 0u) : 0u;
        return j;
    }
#pragma unroll 4  // several independent 16-B reads in flight (Bittner-28: 7 per update)
    for (uint32_t q = 0; q < n2; ++q) {
        const ulonglong2 t = thr[q];
        j += (k53 >= t.x ? 1u : 0u) + (k53 >= t.y ? 1u : 0u);
    }
    return j;
}

__device__ __forceinline__ uint64_t predictor_record(uint32_t i, uint64_t k53, const uint8_t* tbl,
                                                     const NetLayout& L) {
    return reinterpret_cast<const uint64_t*>(tbl + L.off_rec)[i * L.pmax + predictor_choice(i, k53, tbl, L)];
}

// Compact LDS image of the Philox-driven predictor-mix kernels (k_step, k_rollout), whose choice
// uniform is a 32-bit word a (k53 = u32_k53(a)): thresholds re-expressed on a (u32_threshold)
// and stored as u32, rows padded to tp4 (a multiple of 4) so one ds_read_b128 serves 4 of them
// -- half the LDS bytes of the u64 thresholds, whose random-node reads are the most
// bank-conflicted reads of an update. u32_threshold can be 2^32 ("never": the u64 padding, or
// a threshold above k53(2^32 - 1)); it is stored saturated to 2^32 - 1, which a = 2^32 - 1
// passes. Thresholds are non-decreasing, so the never-entries of a node are its last tp - m_i;
// record slots q >= m_i all hold record m_i (slot rs >= tp4 + 1 per node), and the count's
// overshoot at a = 2^32 - 1 lands on the same record. Bit-exact with predictor_record(i, u32_k53(a)).
// Layout: thr32 [N][tp4] at 0, records u64 [N][rs] at rec_off (16-aligned). For pmax <= 3 it is
// larger than the u64 image, so the kernels that stage it place their planes at L.plane_off =
// max(L.bytes, its size); L.bytes itself stays the u64 image's size (what every other kernel and
// the env config stage). The host builds it (build_predictor_image, pbn_abi.cpp) and appends it
// to the device image at offset L.bytes.
struct Thr32 {
    uint32_t tp4, rs, rec_off, bytes;
};

__device__ __forceinline__ Thr32 thr32_layout(const NetLayout& L) {
    Thr32 X;
    X.tp4 = (L.tp + 3u) & ~3u;
    X.rs = X.tp4 + 1u > L.pmax ? X.tp4 + 1u : L.pmax;
    X.rec_off = ((uint32_t)L.n_nodes * X.tp4 * 4u + 15u) & ~15u;
    X.bytes = (X.rec_off + (uint32_t)L.n_nodes * X.rs * 8u + 15u) & ~15u;
    return X;
}

// Record slot of node i's row chosen by the choice word a (compact thresholds at lds[0]).
__device__ __forceinline__ uint32_t predictor_choice32(uint32_t i, uint32_t a, const uint8_t* lds, uint32_t tp4) {
    const uint4* thr = reinterpret_cast<const uint4*>(lds) + i * (tp4 >> 2);
    uint32_t j = 0;
    if (tp4 == 4) {
        const uint4 t = thr[0];
        j = (a >= t.x ? 1u : 0u) + (a >= t.y ? 1u : 0u) + (a >= t.z ? 1u : 0u) + (a >= t.w ? 1u : 0u);
    } else {
#pragma unroll 4
        for (uint32_t q = 0; q < (tp4 >> 2); ++q) {
            const uint4 t = thr[q];
            j += (a >= t.x ? 1u : 0u) + (a >= t.y ? 1u : 0u) + (a >= t.z ? 1u : 0u) + (a >= t.w ? 1u : 0u);
        }
    }
    return j;
}

__device__ __forceinline__ uint64_t predictor_record32(uint32_t i, uint32_t a, const uint8_t* lds,
                                                       const Thr32& X) {
    // 24-bit multiply (full rate; v_mul_lo_u32 is quarter rate): i < 512, rs <= 17
    return reinterpret_cast<const uint64_t*>(lds + X.rec_off)[__umul24(i, X.rs) + predictor_choice32(i, a, lds, X.tp4)];
}

// Y = rec.tt[x_in0 x_in1 x_in2 x_self] (base.py:100-118 via the exported truth table).
template <class P_t>
__device__ __forceinline__ uint32_t predictor_apply(const P_t& P, uint32_t i, uint32_t self, uint64_t rec) {
    const uint32_t p = (P.bit((uint32_t)rec & 0xFFFFu) << 3) | (P.bit((uint32_t)(rec >> 16) & 0xFFFFu) << 2) |
                       (P.bit((uint32_t)(rec >> 32) & 0xFFFFu) << 1) | ((self >> (i & 31u)) & 1u);
    return (uint32_t)(rec >> (48 + p)) & 1u;
}

template <class P_t>
__device__ __forceinline__ uint32_t predictor_eval_lds(const P_t& P, uint32_t i, uint32_t self, uint64_t k53,
                                                       const uint8_t* tbl, const NetLayout& L) {
    return predictor_apply(P, i, self, predictor_record(i, k53, tbl, L));
}

// PBN Node.compute_next_value (common/node.py:31-38) evaluated on the LDS plane.
template <class P_t>
__device__ __forceinline__ uint32_t table_eval_lds(const P_t& P, uint32_t i, uint64_t k53, const uint8_t* tbl,
                                                   const NetLayout& L) {
    const uint64_t info = reinterpret_cast<const uint64_t*>(tbl + L.off_node)[i];
    const uint32_t toff = (uint32_t)info, ioff = (uint32_t)(info >> 32) & 0xFFFFu, k = (uint32_t)(info >> 48) & 0xFFu;
    const uint16_t* in = reinterpret_cast<const uint16_t*>(tbl + L.off_rec) + ioff;
    uint32_t idx = 0;
#pragma unroll 4
    for (uint32_t q = 0; q < k; ++q) idx = (idx << 1) | P.bit(in[q]);
    const uint64_t t = reinterpret_cast<const uint64_t*>(tbl + L.off_thr)[toff + idx];
    return k53 < t ? 1u : 0u;
}

// Env record (k_env, cooperative-draw mode): predictor record rec (in0 | in1<<16 | in2<<32 | tt<<48)
// of node i re-encoded for the LDS state planes of k_env's workgroups (ENV_BLOCK lanes): byte offsets of the plane
// dwords holding in0 / in1 (x), in2 / node i (y), tt | i << 16
// (w): the bit positions of in0, in1, in2, i in those dwords (one byte each). An update then reads
// its four plane dwords with no index arithmetic. Inputs are < 512 (W <= 8), so every offset is
// < 16 KiB.
// w: the truth table | the LDS byte address of node i's counter deltas (nd_off = the table's offset,
// 8 B per node; the R6 kernel's LDS stays below 64 KiB) << 16
__device__ __forceinline__ uint4 env_record(uint64_t rec, uint32_t i, uint32_t nd_off) {
    const uint32_t x0 = (uint32_t)rec & 0xFFFFu, x1 = (uint32_t)(rec >> 16) & 0xFFFFu,
                   x2 = (uint32_t)(rec >> 32) & 0xFFFFu;
    auto off = [](uint32_t x) { return (x >> 5) * (uint32_t)(ENV_BLOCK * 4); };
    return make_uint4(off(x0) | (off(x1) << 16), off(x2) | (off(i) << 16),
                      (x0 & 31u) | ((x1 & 31u) << 8) | ((x2 & 31u) << 16) | ((i & 31u) << 24),
                      (uint32_t)(rec >> 48) | ((nd_off + 8u * i) << 16));
}

// Async update of node i in place on the plane; returns 1 if the bit changed.
template <class P_t>
__device__ __forceinline__ uint32_t predictor_update_lds(const P_t& P, uint32_t i, uint64_t k53,
                                                         const uint8_t* tbl, const NetLayout& L) {
    const uint32_t d = i >> 5, sh = i & 31u;
    const uint32_t self = P.get(d);
    const uint32_t y = predictor_eval_lds(P, i, self, k53, tbl, L);
    const uint32_t nv = (self & ~(1u << sh)) | (y << sh);
    P.put(d, nv);
    return nv != self;
}

template <class P_t>
__device__ __forceinline__ uint32_t table_update_lds(const P_t& P, uint32_t i, uint64_t k53, const uint8_t* tbl,
                                                     const NetLayout& L) {
    const uint32_t y = table_eval_lds(P, i, k53, tbl, L);
    const uint32_t d = i >> 5, sh = i & 31u;
    const uint32_t self = P.get(d);
    const uint32_t nv = (self & ~(1u << sh)) | (y << sh);
    P.put(d, nv);
    return nv != self;
}

// gap(u) = #{k >= 1 : u < T_k} for the non-increasing table gap[k-1] = T_k = floor((1-p)^k 2^32).
// T_k > u  <=>  k <= log((u+1) 2^-32) / log(1-p), so a float estimate e of that bound is within
// one of the answer; three table entries around e settle it (one LDS round trip), and a result
// that fails the bracket check -- only if the estimate was off by more than one -- falls back to
// a binary search. inv_log2q = 1 / log2(1-p) (from the table, host side); 0 when p == 1.
__device__ __forceinline__ uint32_t geo_gap(uint32_t u, const uint32_t* gap, uint32_t N, float inv_log2q) {
    const float x = ((float)u + 1.0f) * 2.3283064365386963e-10f;
    const float L = __log2f(x) * inv_log2q;
    const uint32_t e = L >= (float)N ? N : (uint32_t)fmaxf(L, 0.0f);
    // gt(k) = "T_k > u", with T_0 = +inf and T_k = 0 past N
    auto rd = [&](uint32_t k) -> uint32_t { return (k >= 1 && k <= N) ? gap[k - 1] : 0u; };
    const uint32_t vm = rd(e - 1), v0 = rd(e), v1 = rd(e + 1), v2 = rd(e + 2);
    const bool bm = e == 1 || (e >= 2 && vm > u);
    const bool b0 = e == 0 || v0 > u;
    const bool b1 = e + 1 <= N && v1 > u;
    const bool b2 = e + 2 <= N && v2 > u;
    const uint32_t g = e + (b1 ? 1u : 0u) - (b0 ? 0u : 1u);  // e - 1, e or e + 1
    const bool bg = g == e + 1 ? b1 : (g == e ? b0 : bm);
    const bool bg1 = g == e + 1 ? b2 : (g == e ? b1 : b0);
    if (bg && !bg1) return g;  // T_g > u >= T_{g+1}: g is the count
    uint32_t lo = 0, hi = N;  // largest k in [0, N] with u < T_k
    while (lo < hi) {
        const uint32_t mid = (lo + hi + 1) >> 1;
        if (u < gap[mid - 1])
            lo = mid;
        else
            hi = mid - 1;
    }
    return lo;
}

// Independent Bernoulli(p) events over positions [0, N) generated as successive
// geometric gaps: gap = #{k >= 1 : u < T_k}, T_k = floor((1-p)^k 2^32) (LDS table
// gap[0..N-1] = T_1..T_N), u = 32-bit Philox words from ctr {c0, m, gid, stream}
// with m = 0, 1, ... Calls on_pos(pos) for every event position in increasing order.
template <class F>
__device__ __forceinline__ void bernoulli_positions(uint64_t seed, uint32_t c0, uint32_t stream, uint64_t gid,
                                                    const uint32_t* gap, uint32_t N, float inv_log2q,
                                                    F&& on_pos) {
    uint32_t w[4];
    uint32_t m = 0, wi = 4, pos = 0;
    bool first = true;
    for (;;) {
        if (wi == 4) {
            philox_draw(seed, c0, m++, gid, stream, w);
            wi = 0;
        }
        const uint32_t lo = geo_gap(w[wi++], gap, N, inv_log2q);
        pos = first ? lo : pos + 1u + lo;
        first = false;
        if (pos >= N) break;
        on_pos(pos);
    }
}

// Same positions as bernoulli_positions, four gaps per Philox draw resolved together: the gap
// searches of one draw are independent (only the running position is a prefix sum), so their
// LDS round trips overlap. For flip rates where several flips per call are common (SSD noise).
template <class F>
__device__ __forceinline__ void bernoulli_positions_x4(uint64_t seed, uint32_t c0, uint32_t stream, uint64_t gid,
                                                       const uint32_t* gap, uint32_t N, float inv_log2q,
                                                       F&& on_pos) {
    uint32_t pos = 0;
    bool first = true;
    for (uint32_t m = 0;; ++m) {
        uint32_t w[4], gp[4];
        philox_draw(seed, c0, m, gid, stream, w);
#pragma unroll
        for (int k = 0; k < 4; ++k) gp[k] = geo_gap(w[k], gap, N, inv_log2q);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            pos = first ? gp[k] : pos + 1u + gp[k];
            first = false;
            if (pos >= N) return;
            on_pos(pos);
        }
    }
}

template <int W, class P_t>
__device__ __forceinline__ void to_plane(const P_t& P, const uint64_t (&s)[W]) {
#pragma unroll
    for (int k = 0; k < W; ++k) {
        P.put(2 * k, (uint32_t)s[k]);
        P.put(2 * k + 1, (uint32_t)(s[k] >> 32));
    }
}

template <int W, class P_t>
__device__ __forceinline__ void from_plane(const P_t& P, uint64_t (&s)[W]) {
#pragma unroll
    for (int k = 0; k < W; ++k) s[k] = (uint64_t)P.get(2 * k) | ((uint64_t)P.get(2 * k + 1) << 32);
}

}  // namespace pbn
