// pbn_mt.hip -- MT mode: every env runs the reference's own RNG streams on the device.
//
// The reference draws from CPython's global `random` (MT19937; base.py:7,94,308,370,
// common/pbn.py:131) and, for truth-table networks, numpy's legacy global RandomState
// (common/node.py:2,37; pbn.py:106). Seeding an env with s here reproduces
// `random.seed(s)` (init_by_array over the 32-bit words of s) and `np.random.seed(s)`
// (init_genrand(s)); consumption reproduces `_randbelow_with_getrandbits` (rejection on
// bit_length(n) bits) and `random()` = ((a>>5)*2^26 + (b>>6)) * 2^-53. So
//   random.seed(s); graph.genRandState(); [graph.step() for _ in range(T)]
// yields the same states on the GPU as in Python, from the seed alone.
//
// Layout: one row of 624 u32 per env per generator, env-major ([B][MT_ROW]), plus the
// row's read position. A lane's successive words share cache lines; a row that runs out is
// twisted in place by the whole wave (k_mt_step below).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <type_traits>

#include "pbn_device.hpp"
#include "pbn_params.hpp"

namespace pbn {

constexpr uint32_t MT_N = 624;  // (M = 397: the twist's offset, mt_twist_coop)

__device__ __forceinline__ uint32_t mt_temper(uint32_t y) {
    y ^= (y >> 11);
    // y ^ (s & B) in one gfx950 v_bitop3_b32 (truth table 0x78) instead of an AND and an XOR (+2 %, 1M envs)
    y = __builtin_amdgcn_bitop3_b32(y, y << 7, 0x9d2c5680u, 0x78);
    y = __builtin_amdgcn_bitop3_b32(y, y << 15, 0xefc60000u, 0x78);
    y ^= (y >> 18);
    return y;
}

__device__ void mt_init_genrand(uint32_t* mt, uint32_t s) {
    mt[0] = s;
    for (uint32_t i = 1; i < MT_N; ++i) {
        s = 1812433253u * (s ^ (s >> 30)) + i;
        mt[i] = s;
    }
}

// CPython random_seed(): init_by_array(key = 32-bit chunks of |s|), key = [0] for s == 0
__device__ void mt_seed_python(uint32_t* mt, uint64_t seed) {
    uint32_t key[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
    const uint32_t klen = key[1] ? 2u : 1u;
    mt_init_genrand(mt, 19650218u);
    uint32_t i = 1, j = 0;
    uint32_t prev = mt[0];
    for (uint32_t k = MT_N; k; --k) {
        const uint32_t v = (mt[i] ^ ((prev ^ (prev >> 30)) * 1664525u)) + (j ? key[1] : key[0]) + j;
        mt[i] = v;
        prev = v;
        ++i;
        ++j;
        if (i >= MT_N) {
            mt[0] = mt[MT_N - 1];
            prev = mt[0];
            i = 1;
        }
        if (j >= klen) j = 0;
    }
    for (uint32_t k = MT_N - 1; k; --k) {
        const uint32_t v = (mt[i] ^ ((prev ^ (prev >> 30)) * 1566083941u)) - i;
        mt[i] = v;
        prev = v;
        ++i;
        if (i >= MT_N) {
            mt[0] = mt[MT_N - 1];
            prev = mt[0];
            i = 1;
        }
    }
    mt[0] = 0x80000000u;
}

__device__ __forceinline__ uint32_t kshift_of(uint32_t n) { return (uint32_t)__clz(n); }  // 32 - bit_length(n)

// Seed every env's generators (random.seed(s): init_by_array; np.random.seed(s): init_genrand); the row
// is left untwisted (pos 624: CPython's first draw twists). Graph.genRandState (base.py:368-370:
// N x randint(0, 1)) / PBN.reset(None) (pbn.py:105-118: np.random.rand(N) > 0.5; state[0] = 0) then run as
// k_mt_step with init_state = 1.
template <int KIND>
__global__ __launch_bounds__(BLOCK) void k_mt_seed(MTArgs a) {
    const uint64_t e = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
    if (e >= a.B) return;
    const uint64_t s = a.seeds[e];
    mt_seed_python(a.mt_py + e * MT_ROW, s);
    a.pos_py[e] = MT_N;
    if constexpr (KIND == KIND_PROB_TABLE) {
        mt_init_genrand(a.mt_np + e * MT_ROW, (uint32_t)s);
        a.pos_np[e] = MT_N;
    }
}

// T reference transitions per env from its own generators:
//   Bittner Graph.step (base.py:306-312): i = randint(0, N-1); r = random() * CODsum
//   PBN.step (pbn.py:129-133): i = randint(1, N-1) [stdlib]; u = np.random.uniform() [numpy]
//
// Each wave owns a tile of 64 envs (grid-stride over tiles). Per chunk of MT_CHUNK updates the wave first
// GENERATES every lane's draws -- one MT word per lane per iteration through a small state machine
// (node word with _randbelow's rejection, then the two words of random(); the truth-table network takes
// its node from the `random` stream and its uniform from numpy's) -- into a per-lane LDS draw buffer,
// then APPLIES them, every lane the same number of steps (no divergence on the rejection loop). A lane
// reads its 2,496-B table row 16 B at a time (a window of the next 4 words, the following 4 prefetched).
// The twist (every 624 words) is done by the whole wave for each row that needs it, 10 words per lane
// in three phases (new[k] needs new[k - 227]: with k = 227 * phase + lane + 64 j that word is the same
// lane's result of the previous phase), coalesced: lanes reach the end of their rows at different times
// (rejection), and the in-lane twist this replaces serialised the wave on every one of them
// (MT mode ran at ~1 % of its memory roofline).
// draws per lane per generation pass. The draw entries are 2 B for predictor mix (round 6: the predictor choice is
// resolved in the generation pass, MTDraw), so the buffer is 4 KiB and 6 workgroups fit a CU instead of 4:
// 54.7 vs 50.0 G node-updates/s at 1M envs (profiles/r06_mt_mode_ab.json)
constexpr uint32_t MT_CHUNK = 8;
// s_waitcnt immediates (gfx9 encoding: vmcnt [3:0] + [15:14], expcnt [6:4], lgkmcnt [11:8])
constexpr int WAIT_VM0 = 0x0F70, WAIT_VM0_LGKM0 = 0x0070, WAIT_LGKM0 = 0xC07F;
constexpr uint32_t MT_UPPER = 0x80000000u, MT_A = 0x9908b0dfu;  // (lower mask: ~MT_UPPER)

__device__ __forceinline__ uint32_t mt_mix(uint32_t a, uint32_t b, uint32_t m) {
    // (a & UPPER) | (b & LOWER) and (y >> 1) ^ (A if y odd) as two v_bitop3 (0xE4: S0 where S2 else S1; 0x78:
    // S0 ^ (S1 & S2)); y's low bit is b's
    const uint32_t y = __builtin_amdgcn_bitop3_b32(a, b, MT_UPPER, 0xE4);
    const uint32_t odd = 0u - (b & 1u);
    return m ^ __builtin_amdgcn_bitop3_b32(y >> 1, odd, MT_A, 0x78);
}

// Twist one row in place, all 64 lanes of the wave active (row: wave-uniform). Returns new word `lane` of the row.
__device__ __forceinline__ uint32_t mt_twist_coop(uint32_t* __restrict__ row, uint32_t lane) {
    uint32_t o1[4], p1[4], m1[4], o2[4], p2[4], o3[3], p3[3];
    // every load unconditional and at a fixed offset from one address (row + lane), so all 26 are in flight
    // together without per-load address arithmetic (conditional loads became a branch and a round trip each).
    // Lanes past a phase's range read up to 29 words past the row -- the next env's row, or the table's tail pad
    // (MT_TAIL_PAD) after the last -- and never store them.
    const uint32_t* const r = row + lane;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        o1[j] = r[64 * j];
        p1[j] = r[64 * j + 1];
        m1[j] = r[64 * j + 397];
        o2[j] = r[64 * j + 227];
        p2[j] = r[64 * j + 228];
    }
#pragma unroll
    for (int j = 0; j < 3; ++j) {
        o3[j] = r[454 + 64 * j];
        p3[j] = r[455 + 64 * j];
    }
    // every old word is read before any new word is written (other lanes read what this lane overwrites). As the
    // builtin, so the compiler knows every load before it (LDS-DMA windows too) is done and adds no wait for them
    // ahead of later LDS reads (an asm wait is opaque to it)
    __builtin_amdgcn_s_waitcnt(WAIT_VM0);
    asm volatile("" ::: "memory");
    uint32_t n1[4], n2[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        n1[j] = mt_mix(o1[j], p1[j], m1[j]);
        n2[j] = mt_mix(o2[j], p2[j], n1[j]);
    }
    const uint32_t new0 = (uint32_t)__builtin_amdgcn_readlane((int)n1[0], 0);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const uint32_t k1 = lane + 64u * j;
        if (k1 < 227u) {
            row[k1] = n1[j];
            row[227u + k1] = n2[j];
        }
    }
#pragma unroll
    for (int j = 0; j < 3; ++j) {
        const uint32_t k3 = 454u + lane + 64u * j;
        // k3 = 623 (lane 41, j = 2): mt[623] = mt[396] ^ f(mt[623], mt[0]) with mt[0], mt[396] already new
        if (k3 < 624u) row[k3] = mt_mix(o3[j], k3 == 623u ? new0 : p3[j], n2[j]);
    }
    return n1[0];
}

// One MT stream of one lane: row, next word index (624: twist first), 4-word window + prefetch
struct MTWin {
    uint32_t* row;
    uint32_t pos;
    uint4 cur, nxt;
    __device__ __forceinline__ void load() {  // window at pos (pos < 624), prefetch of the next 4 words
        const uint32_t g = pos & ~3u;
        cur = *reinterpret_cast<const uint4*>(row + g);
        if (g + 4u < MT_N) nxt = *reinterpret_cast<const uint4*>(row + g + 4u);
    }
    __device__ __forceinline__ uint32_t take() {  // the word at pos (tempered), pos + 1
        const uint32_t q = pos & 3u;
        const uint32_t w = q == 0u ? cur.x : q == 1u ? cur.y : q == 2u ? cur.z : cur.w;
        ++pos;
        if (q == 3u) {
            cur = nxt;
            if ((pos & ~3u) + 4u < MT_N) nxt = *reinterpret_cast<const uint4*>(row + (pos & ~3u) + 4u);
        }
        return mt_temper(w);
    }
};

// Draw entry of the per-lane LDS buffer: truth tables keep k53 | node << 53 (the threshold row depends on the
// state at the update); predictor mix (N <= 512, <= 128 predictors per node) resolves the predictor choice in
// the generation pass (the thresholds depend on node and k53 only) and keeps node | choice << 9 in 16 bits --
// a quarter of the LDS, so 6 workgroups per CU fit instead of 4 (the kernel waits on its rows' round trips)
// (WIDE: a node with more than 128 predictors -- u32 entries, node | choice << 9)
template <int KIND, bool WIDE>
using MTDraw = typename std::conditional<KIND == KIND_PROB_TABLE, uint64_t,
                                         typename std::conditional<WIDE, uint32_t, uint16_t>::type>::type;

template <int W, int KIND, bool WIDE>
__global__ __launch_bounds__(BLOCK) void k_mt_step(MTArgs a) {
    extern __shared__ __align__(16) uint8_t lds[];
    stage_image(reinterpret_cast<const uint4*>(a.img), a.L.bytes / 16, reinterpret_cast<uint4*>(lds));
    __syncthreads();
    const Plane P{reinterpret_cast<uint32_t*>(lds + a.L.bytes) + threadIdx.x};
    // per-lane draw buffer: [MT_CHUNK][BLOCK] entries (MTDraw)
    MTDraw<KIND, WIDE>* const dbuf = reinterpret_cast<MTDraw<KIND, WIDE>*>(lds + a.L.bytes + 8u * W * BLOCK) + threadIdx.x;
    const uint32_t N = (uint32_t)a.L.n_nodes;
    const uint32_t lane = __lane_id();
    constexpr bool TABLE = KIND == KIND_PROB_TABLE;
    // node draw: randint(0, N-1) / randint(1, N-1) / the init bits (randint(0, 1) for Bittner)
    const uint32_t nn = a.init_state ? 2u : (TABLE ? N - 1u : N);
    const uint32_t ks = (uint32_t)__clz(nn);
    const uint64_t stride = (uint64_t)gridDim.x * BLOCK;
    for (uint64_t e0 = (uint64_t)blockIdx.x * BLOCK + (threadIdx.x & ~63u); e0 < a.B; e0 += stride) {
        const uint64_t e = e0 + lane;
        const bool valid = e < a.B;
        const uint64_t ec = valid ? e : e0;  // lanes past B mirror lane 0's row (read only)
        uint64_t st[W];
        if (valid && !a.init_state) {
            load_state<W>(a.state + e * W, st);
        } else {
#pragma unroll
            for (int k = 0; k < W; ++k) st[k] = 0;
        }
        to_plane<W>(P, st);
        MTWin py{a.mt_py + ec * MT_ROW, a.pos_py[ec], {}, {}};
        MTWin np_{TABLE ? a.mt_np + ec * MT_ROW : nullptr, TABLE ? a.pos_np[ec] : 0u, {}, {}};
        if (py.pos < MT_N) py.load();
        if (TABLE && np_.pos < MT_N) np_.load();
        // draws this launch: T updates, or N init draws (Bittner: N x randint(0, 1) from `random`;
        // table: N x random_sample() from numpy, > 0.5)
        uint32_t left = valid ? (a.init_state ? N : a.T) : 0u;
        uint32_t done = 0;  // draws applied (init: the node index)
        // machine: 0 node word (rejection), 1 first word of random(), 2 second word
        uint32_t stt = (TABLE && a.init_state) ? 1u : 0u, node = 0, wa = 0;
        while (__ballot(left > 0u) != 0ull) {
            const uint32_t tgt = min(left, MT_CHUNK);
            uint32_t cnt = 0;
            for (;;) {
                const bool want = cnt < tgt;
                if (__ballot(want) == 0ull) break;
                // the stream the next word comes from: `random` for the node word (and Bittner's random()),
                // numpy for the table network's uniform
                const bool from_np = TABLE && stt != 0u;
                const bool tw_py = want && !from_np && py.pos >= MT_N;
                const bool tw_np = TABLE && want && from_np && np_.pos >= MT_N;
                uint64_t mask = __ballot(tw_py);
                while (mask) {  // twist every row that has run out, one row per round, the whole wave
                    const uint32_t L = (uint32_t)__ffsll((unsigned long long)mask) - 1u;
                    mask &= mask - 1ull;
                    const uint64_t eL = e0 + L;
                    mt_twist_coop(a.mt_py + eL * MT_ROW, lane);
                }
                if constexpr (TABLE) {
                    mask = __ballot(tw_np);
                    while (mask) {
                        const uint32_t L = (uint32_t)__ffsll((unsigned long long)mask) - 1u;
                        mask &= mask - 1ull;
                        mt_twist_coop(a.mt_np + (e0 + L) * MT_ROW, lane);
                    }
                }
                if (__ballot(tw_py || tw_np) != 0ull) {
                    // the twisted rows' new words (written by other lanes of this wave) are read next: workgroup
                    // scope (the wave's own CU, whose L1 the stores went through) -- an agent-scope fence here
                    // wrote back and invalidated the L2 (buffer_wbl2 / buffer_inv sc1) at every twist
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
                    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                    if (tw_py) {
                        py.pos = 0;
                        py.load();
                    }
                    if (tw_np) {
                        np_.pos = 0;
                        np_.load();
                    }
                }
                if (want) {
                    const uint32_t w = from_np ? np_.take() : py.take();
                    if (stt == 0u) {
                        const uint32_t r = w >> ks;  // _randbelow: getrandbits(bit_length(n)), rejected if >= n
                        if (r < nn) {
                            node = r;
                            stt = a.init_state && !TABLE ? 3u : 1u;  // Bittner init: the draw is the bit itself
                        }
                    } else if (stt == 1u) {
                        wa = w;
                        stt = 2u;
                    } else {
                        const uint64_t k53 = k53_of(wa, w);
                        if constexpr (TABLE)
                            dbuf[cnt * BLOCK] = k53 | ((uint64_t)node << 53);
                        else  // (the init draws of Bittner are single bits, stt 3 below)
                            dbuf[cnt * BLOCK] = (MTDraw<KIND, WIDE>)(node | (predictor_choice(node, k53, lds, a.L) << 9));
                        ++cnt;
                        stt = (TABLE && a.init_state) ? 1u : 0u;
                    }
                    if (stt == 3u) {  // Bittner init bit
                        dbuf[cnt * BLOCK] = (MTDraw<KIND, WIDE>)node;
                        ++cnt;
                        stt = 0u;
                    }
                }
            }
            // apply the chunk: every lane its cnt draws (cnt == tgt: each lane finished its chunk)
            for (uint32_t c = 0; c < tgt; ++c) {
                const MTDraw<KIND, WIDE> d = dbuf[c * BLOCK];
                if constexpr (TABLE) {
                    const uint64_t k53 = d & ((1ull << 53) - 1ull);
                    const uint32_t r = (uint32_t)(d >> 53);
                    if (a.init_state) {
                        const uint32_t i = done + c;
                        const uint32_t dw = i >> 5, sh = i & 31u;
                        P.put(dw, (P.get(dw) & ~(1u << sh)) | ((k53 > (1ull << 52) ? 1u : 0u) << sh));
                    } else {
                        table_update_lds(P, 1u + r, k53, lds, a.L);
                    }
                } else if (a.init_state) {
                    const uint32_t i = done + c;
                    const uint32_t dw = i >> 5, sh = i & 31u;
                    P.put(dw, (P.get(dw) & ~(1u << sh)) | ((uint32_t)d << sh));
                } else {
                    const uint32_t i = (uint32_t)d & 511u, dw = i >> 5, sh = i & 31u;
                    const uint64_t rec = reinterpret_cast<const uint64_t*>(lds + a.L.off_rec)[i * a.L.pmax + ((uint32_t)d >> 9)];
                    const uint32_t self = P.get(dw);
                    P.put(dw, (self & ~(1u << sh)) | (predictor_apply(P, i, self, rec) << sh));
                }
            }
            done += tgt;
            left -= tgt;
        }
        if (valid) {
            if (TABLE && a.init_state) P.put(0, P.get(0) & ~1u);  // pbn.py reset: state[0] = 0
            from_plane<W>(P, st);
            store_state<W>(a.state + e * W, st);
            a.pos_py[e] = py.pos;
            if constexpr (TABLE) a.pos_np[e] = np_.pos;
        }
    }
}

// ---- MT mode, predictor-mix steps (Bittner Graph.step; round 6): the per-lane walk with staged windows.
// k_mt_step reads each lane's row 16 B at a time as it walks, and since any lane may move to its next 16 B in any
// iteration, its loop waits for all its loads (s_waitcnt vmcnt(0)) every iteration: a memory round trip per word
// (the SQ counters: 75 % of its cycles waiting, profiles/r06_mt_lanes_sq_pmc.csv). Here a lane's next MT_WIN words
// (from pos rounded down to 16 B) are brought into the wave's LDS by asynchronous LDS-DMA loads (global_load_lds,
// 16 B per lane per instruction, no VGPRs), ONE wait for the whole window, and the walk then reads its words from
// LDS, each one prefetched an iteration ahead; a lane whose window runs out takes the next window in the next pass.
// Windows outlive the apply phases (restaging at every phase cost a round trip each). The draws wait in a per-lane ring
// of MT_RING entries and a phase applies MT_APPLY per lane: a lane that has its draws keeps walking until its ring
// is full instead of idling while the wave's slowest lane catches up (a draw takes 2 + a variable number of node
// words: rejection). The twist's 26 loads are all in flight at once; a run-out row is twisted while the other lanes'
// windows are in flight and its first words go to its owner's window from registers. The machine runs as selects.
// Same draws, same state machine, same entries, same rows and positions as k_mt_step (bit-exact; the tests run both
// walks). Bench workload (1M envs, T = 256): 89 G node-updates/s vs 54.8 (k_mt_step) and 50.0 (round 5); the steps
// are in profiles/r06_mt_mode_ab.json.
#ifndef PBN_MT_WIN
#define PBN_MT_WIN 16  // 12 / 16 / 20: 86.5 / 89.2 / 87.6 G (3 workgroups per CU for all three)
#endif
constexpr uint32_t MT_WIN = PBN_MT_WIN;  // words per staged window: MT_WIN / 4 DMA loads per lane
static_assert(MT_WIN % 4u == 0 && MT_WIN >= 8u, "windows of 16-B granules");
#ifndef PBN_MT_APPLY
#define PBN_MT_APPLY 8
#endif
// draws applied per lane per phase; a lane that has them keeps walking until its ring (MT_RING) is full instead of
// idling while the wave's slowest lane catches up (a draw takes a variable number of words: rejection)
constexpr uint32_t MT_APPLY = PBN_MT_APPLY;
#ifndef PBN_MT_RING
#define PBN_MT_RING 16  // ring / apply 8 / 8: 78.6 G, 16 / 8: 85.8, 16 / 4: 84.7, 16 / 12: 82.4, 32 / 16: 85.6 (W 12)
#endif
constexpr uint32_t MT_RING = PBN_MT_RING;  // draw entries per lane in the ring
#ifndef PBN_MT_WALK_UNROLL
#define PBN_MT_WALK_UNROLL 4  // 1 / 2 / 3 / 4: 94.1 / 94.3 / 92.5 / 94.2 G at 1M envs, 51.4 / 53.9 / 51.7 / 54.9 G at 65k
#endif
static_assert(MT_APPLY >= 1u && MT_APPLY <= MT_RING && MT_RING >= MT_CHUNK && (MT_RING & (MT_RING - 1u)) == 0u,
              "ring of a power of two");

// TP4: every node's thresholds padded to 4 (Bittner-199), read an iteration ahead (loop-carried) so that their LDS
// round trip overlaps the next iteration's temper
template <int W, bool WIDE, bool TP4>
__global__ __launch_bounds__(BLOCK) void k_mt_staged(MTArgs a) {
    using D = MTDraw<KIND_PREDICTOR_MIX, WIDE>;
    typedef __attribute__((address_space(3))) uint32_t l32;
    extern __shared__ __align__(16) uint8_t lds[];
    if constexpr (TP4) {
        // the thresholds re-expressed on X = wa << 32 | w, the draw's two words as they come: k53(X) = (wa >> 5) 2^26 +
        // (w >> 6) is monotone in X, so k53 >= T <=> X >= X_T, X_T = (T >> 26) << 37 | (T mod 2^26) << 6 (the smallest
        // such X); a threshold past every k53 (padding, T >= 2^53) becomes 2^64 - 1, above every X the walk forms (its
        // bit 0 cleared: same k53). The compare then needs no k53 (three ops per draw)
        stage_image(reinterpret_cast<const uint4*>(a.img) + a.L.off_rec / 16, (a.L.bytes - a.L.off_rec) / 16,
                    reinterpret_cast<uint4*>(lds) + a.L.off_rec / 16);
        const uint64_t* const gthr = reinterpret_cast<const uint64_t*>(reinterpret_cast<const uint8_t*>(a.img) + a.L.off_thr);
        uint64_t* const xthr = reinterpret_cast<uint64_t*>(lds + a.L.off_thr);
        for (uint32_t k = threadIdx.x; k < 4u * (uint32_t)a.L.n_nodes; k += BLOCK) {
            const uint64_t t = gthr[k];
            xthr[k] = t >= (1ull << 53) ? ~0ull : ((t >> 26) << 37) | ((t & 0x3FFFFFFull) << 6);
        }
    } else {
        stage_image(reinterpret_cast<const uint4*>(a.img), a.L.bytes / 16, reinterpret_cast<uint4*>(lds));
    }
    __syncthreads();
    const Plane P{reinterpret_cast<uint32_t*>(lds + a.L.bytes) + threadIdx.x};
    D* const dbuf = reinterpret_cast<D*>(lds + a.L.bytes + 8u * W * BLOCK) + threadIdx.x;  // [MT_RING][BLOCK]
    // the wave's windows: granule j (16 B) of lane l at j * 1 KiB + l * 16
    uint8_t* const win = lds + a.L.bytes + 8u * W * BLOCK + (uint32_t)sizeof(D) * MT_RING * BLOCK + (threadIdx.x >> 6) * (MT_WIN * 256u);
    const uint32_t lane = __lane_id();
    const uint32_t* const mine = reinterpret_cast<const uint32_t*>(win + lane * 16u);
    const uint32_t win_ofs = (uint32_t)(reinterpret_cast<const uint8_t*>(mine) - lds);  // this lane's granule 0
    const uint32_t win_lds = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(l32*)win);
    const uint64_t* const recs = reinterpret_cast<const uint64_t*>(lds + a.L.off_rec);
    const ulonglong2* const thr4 = reinterpret_cast<const ulonglong2*>(lds + a.L.off_thr);
    const uint32_t N = (uint32_t)a.L.n_nodes;
    const uint32_t ks = (uint32_t)__clz(N);  // randint(0, N - 1): _randbelow(N), getrandbits(bit_length(N)) < N
    const uint64_t stride = (uint64_t)gridDim.x * BLOCK;
    for (uint64_t e0 = (uint64_t)blockIdx.x * BLOCK + (threadIdx.x & ~63u); e0 < a.B; e0 += stride) {
        const uint64_t e = e0 + lane;
        const bool valid = e < a.B;
        uint32_t* const row = a.mt_py + (valid ? e : e0) * MT_ROW;  // lanes past B stage lane 0's row (unused)
        uint64_t st[W];
        if (valid) {
            load_state<W>(a.state + e * W, st);
        } else {
#pragma unroll
            for (int k = 0; k < W; ++k) st[k] = 0;
        }
        to_plane<W>(P, st);
        uint32_t pos = valid ? a.pos_py[e] : 0u, left = valid ? a.T : 0u;
        uint32_t stt = 0, node = 0, wa = 0;  // machine: 0 node word (rejection), 1 random()'s first word, 2 its second
        // the draws wait in a per-lane ring of MT_RING entries: `pend` made and not yet applied, the next one written
        // to slot `wr`; every phase applies MT_APPLY per lane, oldest first (slot `rd`, the same in every lane)
        uint32_t pend = 0, wr = 0, rd = 0;
        uint32_t base = pos & ~3u, end = 0;  // the lane's window [base, end) of its row; none staged yet
        // row word p of the window at LDS byte wc + 4 p + 1008 (p >> 2) (granule (p - base) / 4 at 1 KiB steps, the
        // word at 4 B): three ops per word from pos, no clamp (p = end reads the pad granule after the windows)
        uint32_t wc = 0;
        auto wword = [&](uint32_t p) {
            return *reinterpret_cast<const uint32_t*>(lds + (__umul24(p >> 2, 1008u) + wc + (p << 2)));
        };
        while (__ballot(left > 0u) != 0ull) {
            const uint32_t tgt = min(left, MT_APPLY);
            const uint32_t cap = min(left, MT_RING);  // never a draw past this launch's T
            for (;;) {
                bool need = pend < tgt;
                if (__ballot(need) == 0ull) break;
                bool can = pend < cap;
                // a new window only when no lane that needs draws has words left in its window (windows outlive the
                // phases: restaging at every phase cost a round trip per phase)
                if (__ballot(need && pos < end) == 0ull) {
                    // stage words [base, base + MT_WIN) of every lane's row, base = pos rounded down to 16 B; granules
                    // past the row's end repeat its last one (never read: a lane stops at the row's end). The window's
                    // previous reads are done first (an LDS-DMA write does not wait for them). A row that has run out
                    // is twisted by the whole wave while the other lanes' windows are in flight, and its first MT_WIN
                    // new words go to its owner's window from the twisting lanes' registers.
                    const bool tw = need && pos >= MT_N;
                    uint64_t mask = __ballot(tw);
                    const bool twisted = mask != 0ull;
                    if (tw) pos = 0;
                    base = pos & ~3u;
                    // the window's previous reads done; a previous pass's twist stores done before any row is read
                    __builtin_amdgcn_s_waitcnt(WAIT_VM0_LGKM0);
                    asm volatile("" ::: "memory");
                    if (!tw) {
#pragma unroll
                        for (uint32_t j = 0; j < MT_WIN / 4u; ++j)
                            // the LDS-DMA as asm (m0 = the granule row's LDS address): for the builtin the compiler
                            // waited vmcnt(0) ahead of the walk's threshold reads (LDS it could not prove disjoint), i.e.
                            // for a twist's stores left in flight (+1 %, profiles/r06_mt_valu_trim_ab.json); the kernel
                            // waits for these itself (the refill's and the twist's s_waitcnt)
                            asm volatile("s_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(row + min(base + 4u * j, MT_N - 4u)),
                                         "{m0}"(win_lds + j * 1024u)
                                         : "memory");
                    }
                    if (twisted) {
                        // (a do-while: the compiler then knows a twist's wait retired the windows' loads)
                        do {
                            const uint32_t L = (uint32_t)__ffsll((unsigned long long)mask) - 1u;
                            mask &= mask - 1ull;
                            const uint32_t nw = mt_twist_coop(a.mt_py + (e0 + L) * MT_ROW, lane);
                            if (lane < MT_WIN)
                                *reinterpret_cast<uint32_t*>(win + (lane >> 2) * 1024u + L * 16u + (lane & 3u) * 4u) = nw;
                            // the row's later windows are staged from what the other lanes wrote (k_mt_step's fence)
                            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
                            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
                        } while (mask);
                        // the windows' loads are done (the twist waited for them before its stores); its stores are
                        // left in flight until the next pass, which waits for them before it reads a row
                        __builtin_amdgcn_s_waitcnt(WAIT_LGKM0);
                    } else {
                        __builtin_amdgcn_s_waitcnt(WAIT_VM0_LGKM0);
                    }
                    asm volatile("" ::: "memory");
                    end = min(base + MT_WIN, MT_N);
                    wc = win_ofs - (base << 2) - (base >> 2) * 1008u;
                }
                uint32_t wn = wword(pos);  // the next word, read an iteration ahead
                ulonglong2 t0{}, t1{};
                if constexpr (TP4) {
                    t0 = thr4[2u * node];
                    t1 = thr4[2u * node + 1u];
                }
                // walk while a lane that needs draws has words; a lane with room in its ring walks along (as the AND
                // of two compares' lane masks: __ballot(need && pos < end) turned the mask into 0 / 1 and back)
                // (PBN_MT_WALK_UNROLL words per test: a word walked after the wave's last needy lane ran out is a lane
                // with ring room walking along, or no lane at all -- the same draws, made earlier)
                auto walk1 = [&]() {
                    // the machine as selects (one divergent branch, the draw's store, instead of three)
                    const bool act = can && pos < end;
                    const uint32_t w = mt_temper(wn);
                    pos += act ? 1u : 0u;
                    wn = wword(pos);
                    const uint32_t r = w >> ks;  // _randbelow: rejected if >= N
                    const bool take_node = act && stt == 0u && r < N, take_wa = act && stt == 1u, emit = act && stt == 2u;
                    uint32_t choice;
                    if constexpr (TP4) {  // the X-space thresholds (prologue)
                        const uint64_t X = ((uint64_t)wa << 32) | (w & ~1u);
                        choice = (X >= t0.x ? 1u : 0u) + (X >= t0.y ? 1u : 0u) + (X >= t1.x ? 1u : 0u) + (X >= t1.y ? 1u : 0u);
                    } else {
                        // k53 = (wa >> 5) << 26 | w >> 6 as its two halves, the low one ({wa >> 5, w} >> 6) by v_alignbit
                        const uint64_t k53 = ((uint64_t)(wa >> 11) << 32) | __builtin_amdgcn_alignbit(wa >> 5, w, 6);
                        choice = predictor_choice(node, k53, lds, a.L);
                    }
                    const uint32_t ent = node | (choice << 9);
                    if (emit) dbuf[wr * BLOCK] = (D)ent;  // (unconditional, into a spare slot: 84.6 vs 87.3 G)
                    node = take_node ? r : node;
                    wa = take_wa ? w : wa;
                    stt = take_node ? 1u : take_wa ? 2u : emit ? 0u : stt;
                    pend += emit ? 1u : 0u;
                    wr = (wr + (emit ? 1u : 0u)) & (MT_RING - 1u);
                    can = pend < cap;
                    if constexpr (TP4) {  // the next iteration's thresholds, read an iteration ahead like its word
                        t0 = thr4[2u * node];
                        t1 = thr4[2u * node + 1u];
                    }
                };
                while ((__builtin_amdgcn_ballot_w64(pos < end) & __builtin_amdgcn_ballot_w64(pend < tgt)) != 0ull) {
#pragma unroll
                    for (int k = 0; k < PBN_MT_WALK_UNROLL; ++k) walk1();
                }
            }
            // apply the phase: every lane its tgt oldest draws
            for (uint32_t c = 0; c < tgt; ++c) {
                const uint32_t d = dbuf[((rd + c) & (MT_RING - 1u)) * BLOCK];
                const uint32_t i = d & 511u, dw = i >> 5, sh = i & 31u;
                const uint64_t rec = recs[__umul24(i, a.L.pmax) + (d >> 9)];  // 24-bit multiply: full rate
                const uint32_t self = P.get(dw);
                P.put(dw, (self & ~(1u << sh)) | (predictor_apply(P, i, self, rec) << sh));
            }
            rd = (rd + tgt) & (MT_RING - 1u);
            pend -= tgt;
            left -= tgt;
        }
        if (valid) {
            from_plane<W>(P, st);
            store_state<W>(a.state + e * W, st);
            a.pos_py[e] = pos;
        }
    }
}

template <bool WIDE, bool TP4>
static void* mt_staged_fn(int W) {
    switch (W) {
        case 1: return (void*)k_mt_staged<1, WIDE, TP4>;
        case 2: return (void*)k_mt_staged<2, WIDE, TP4>;
        case 3: return (void*)k_mt_staged<3, WIDE, TP4>;
        case 4: return (void*)k_mt_staged<4, WIDE, TP4>;
        case 5: return (void*)k_mt_staged<5, WIDE, TP4>;
        case 6: return (void*)k_mt_staged<6, WIDE, TP4>;
        case 7: return (void*)k_mt_staged<7, WIDE, TP4>;
        case 8: return (void*)k_mt_staged<8, WIDE, TP4>;
    }
    return nullptr;
}

template <int KIND, bool WIDE>
static void* mt_step_fn(int W) {
    switch (W) {
        case 1: return (void*)k_mt_step<1, KIND, WIDE>;
        case 2: return (void*)k_mt_step<2, KIND, WIDE>;
        case 3: return (void*)k_mt_step<3, KIND, WIDE>;
        case 4: return (void*)k_mt_step<4, KIND, WIDE>;
        case 5: return (void*)k_mt_step<5, KIND, WIDE>;
        case 6: return (void*)k_mt_step<6, KIND, WIDE>;
        case 7: return (void*)k_mt_step<7, KIND, WIDE>;
        case 8: return (void*)k_mt_step<8, KIND, WIDE>;
    }
    return nullptr;
}

static bool mt_wide(const NetLayout& L) { return L.kind == KIND_PREDICTOR_MIX && L.pmax > 128u; }

int launch_mt_seed(int W, const MTArgs& a, int grid, void* stream) {
    (void)W;
    void* fn = a.L.kind == KIND_PREDICTOR_MIX ? (void*)k_mt_seed<KIND_PREDICTOR_MIX> : (void*)k_mt_seed<KIND_PROB_TABLE>;
    MTArgs c = a;
    void* kargs[] = {&c};
    return (int)hipLaunchKernel(fn, dim3((unsigned)grid), dim3(BLOCK), kargs, 0, (hipStream_t)stream);
}

uint32_t mt_lds_bytes(int W, const NetLayout& L) {
    const uint32_t entry = L.kind == KIND_PROB_TABLE ? 8u : mt_wide(L) ? 4u : 2u;  // MTDraw
    return L.bytes + 8u * (uint32_t)W * BLOCK + entry * MT_CHUNK * BLOCK;
}

// grid: the resident workgroups (every wave walks 64-env tiles), capped by the tiles there are
int launch_mt_step(int W, const MTArgs& a, int n_cu, void* stream) {
    // predictor-mix steps: the staged walk (genRandState's init draws and truth tables: k_mt_step)
    const bool staged = a.L.kind == KIND_PREDICTOR_MIX && !a.init_state && !a.lane_walk;
    const bool tp4 = a.L.tp == 4u;
    void* fn = staged ? (mt_wide(a.L) ? (tp4 ? mt_staged_fn<true, true>(W) : mt_staged_fn<true, false>(W))
                                      : (tp4 ? mt_staged_fn<false, true>(W) : mt_staged_fn<false, false>(W)))
               : a.L.kind != KIND_PREDICTOR_MIX ? mt_step_fn<KIND_PROB_TABLE, false>(W)
               : mt_wide(a.L)                  ? mt_step_fn<KIND_PREDICTOR_MIX, true>(W)
                                               : mt_step_fn<KIND_PREDICTOR_MIX, false>(W);
    if (!fn) return (int)hipErrorInvalidValue;
    const uint32_t entry = mt_wide(a.L) ? 4u : 2u;  // staged: MT_WIN-word windows, a ring of MT_RING entries
    // (staged: + one granule row after the last wave's windows, read by a lane at the end of its window)
    const uint32_t lds = mt_lds_bytes(W, a.L) + (staged ? MT_WIN * 4u * BLOCK + (MT_RING - MT_CHUNK) * entry * BLOCK + 1024u : 0u);
    int bpc = 0;
    if (hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&bpc, reinterpret_cast<const void*>(fn), BLOCK, lds))
        return (int)e;
    const uint64_t want = (a.B + BLOCK - 1) / BLOCK;
    const int grid = (int)std::max<uint64_t>(1, std::min<uint64_t>(want, (uint64_t)n_cu * (uint64_t)std::max(bpc, 1)));
    MTArgs c = a;
    void* kargs[] = {&c};
    return (int)hipLaunchKernel(fn, dim3((unsigned)grid), dim3(BLOCK), kargs, lds, (hipStream_t)stream);
}

}  // namespace pbn
