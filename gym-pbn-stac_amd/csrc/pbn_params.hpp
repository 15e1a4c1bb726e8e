// pbn_params.hpp -- plain structs shared by the host ABI (g++) and the kernels (hipcc).
#pragma once
#include <stdint.h>

namespace pbn {

enum { KIND_PREDICTOR_MIX = 1, KIND_PROB_TABLE = 2 };
enum {
    STREAM_STEP = 1,
    STREAM_INIT = 2,
    STREAM_ENV = 3,
    STREAM_RESET = 4,
    STREAM_SSD = 5,
    STREAM_SSD_FLIP = 6,
    STREAM_SYNC = 7,
    STREAM_SYNC_PERT = 8
};
enum { STORE_FULL = 0, STORE_DIRTY = 1 };

constexpr int BLOCK = 256;          // 4 wave64 per workgroup
#ifndef PBN_ENV_BLOCK
#define PBN_ENV_BLOCK 256
#endif
// k_env's workgroup (lane / tail / hand-off modes; group mode k_env_grp keeps BLOCK): the workgroup is the
// tail hand-off's and the helpers' domain
constexpr int ENV_BLOCK = PBN_ENV_BLOCK;
static_assert(ENV_BLOCK % 64 == 0 && ENV_BLOCK / 64 <= 16, "k_env: whole waves, idle mask / helper codes fit");
// k_env's LDS budget per workgroup: 64 KiB at 256 threads (two workgroups per CU), the CU's 160 KiB above
constexpr uint32_t ENV_LDS_MAX = ENV_BLOCK > 256 ? 160u * 1024u : 64u * 1024u;
// a plane byte offset (dword * 4 * ENV_BLOCK) >> ENV_ROW_SHIFT = dword * 256: the tail writer-mask tables' row
constexpr uint32_t ENV_ROW_SHIFT = __builtin_ctz((unsigned)ENV_BLOCK / 64u);
constexpr int MAX_WORDS = 8;        // N <= 512
constexpr uint32_t MAX_IMAGE = 48 * 1024;  // LDS bytes for the network image (state planes come on top)

// Byte offsets of the tables inside the LDS image (16-byte aligned image).
// Predictor-mix networks use a padded per-node layout so that both table reads of an
// update are addressed by the node index alone (no dependent "node info" read):
//   thr [N][tp]   u64 selection thresholds, tp = max predictors - 1 rounded up to even,
//                 padding = UINT64_MAX (never reached: k53 < 2^53)
//   rec [N][pmax] u64 records in0 | in1<<16 | in2<<32 | tt<<48
struct NetLayout {
    uint32_t off_node;  // per-node info (truth-table networks)
    uint32_t off_thr;   // u64 thresholds
    uint32_t off_rec;   // predictor records (u64) or input lists (u16)
    uint32_t bytes;     // total, multiple of 16
    int32_t kind;
    int32_t n_nodes;
    uint32_t tp;        // predictor mix: thresholds per node (even)
    uint32_t pmax;      // predictor mix: record slots per node
    // LDS offset of the state planes of k_step / k_rollout / k_rollout_grp: max(bytes, the compact
    // image's size) for predictor mix (those kernels stage the compact image, which for pmax <= 3
    // is larger than the u64 one), bytes for tables. Every other kernel places its planes at bytes.
    uint32_t plane_off;
};

struct StepArgs {
    uint64_t* state;             // [B][W]
    const void* img;             // network image (device, 16-B aligned)
    NetLayout L;
    uint64_t B;
    uint64_t env_base;           // global id of env 0 of this batch
    uint64_t seed;
    uint64_t update_base;        // Philox update counter of the first update
    uint32_t T;                  // updates per launch
    const uint32_t* replay_node; // [T][B] (replay mode)
    const uint64_t* replay_k53;  // [T][B]; null: forced nodes, choice words from the Philox step stream
    int32_t grp;                 // rollout: lanes per env (1 = k_rollout; 2/4/8 = k_rollout_grp)
    const uint64_t* ubase_dev;   // step mode in a HIP graph: update counter = *ubase_dev + update_base
};

struct InitArgs {
    uint64_t* state;
    uint64_t B, env_base, seed;
    uint32_t reset_count;
    int32_t n_nodes, kind;
    // env reset (R6): choose a cube among n_cubes, keep its cared bits, draw the rest
    const uint64_t* cube_care;   // [n_cubes][W] or null (plain randomize)
    const uint64_t* cube_value;
    int32_t n_cubes;
    const uint8_t* mask;         // [B] or null
    int64_t* n_steps;            // zeroed for reset envs, if non-null
};

struct FlipArgs {
    uint64_t* state;
    const int32_t* actions;  // [B][A]
    uint64_t B;
    int32_t A, offset, dedup, n_nodes;
    int32_t* error;          // set to 1 on an out-of-range action (device path)
};

struct EnvArgs {
    uint64_t* state;         // [B][W]
    int64_t* n_steps;        // [B]
    const int32_t* actions;  // [B][A]
    uint64_t* obs;           // [B][W]
    int32_t* reward;         // [B]
    uint8_t* flags;          // [B]
    uint32_t* n_updates;     // [B]
    int32_t* error;
    const void* img;         // network image + cubes appended
    NetLayout L;
    uint32_t off_cubes;      // care/value pairs [H][2][W] u64 inside the LDS image
    uint32_t off_target;     // target care/value [2][W]
    uint32_t off_ndelta;     // per node: uint2 packed mismatch-counter deltas (fast attractor test)
    unsigned long long* counter;  // work-queue head (zeroed per launch)
    int32_t n_cubes;
    int32_t fast;            // 1: <= 8 cubes, each caring about <= 255 nodes (byte counters);
                             // 2: and predictor mix with <= 16 predictors per node, Philox: the
                             //    draws are generated cooperatively by the whole wave;
                             // 3: group mode (k_env_grp); 4: as 2 with <= 4 cubes (one counter word)
    uint32_t off_gen;        // fast == 2 / 4: per-wave draw buffers (ENV_GEN_WAVE_BYTES each);
                             // fast == 3: per-group env rows (2W dwords per group of grp lanes)
    uint64_t B, env_base, seed;
    uint32_t call_idx, update_cap;
    int32_t A, offset, dedup, horizon, reward_success, action_cost;
    int32_t first_tested;     // 1: test the state after the first update too (pbn_target.py R5)
    const int64_t* draw_off;  // replay mode: [B+1]
    const uint32_t* draws_i;
    const uint64_t* draws_k;
    int32_t grp;              // fast == 3: lanes per env (2, 4 or 8), k_env_grp
    uint32_t n_calls;         // env steps per env in this launch: actions [n_calls][B][A], outputs
                              // [n_calls][B]...; step t draws with Philox c1 = call_idx + t
    uint32_t erec_shift;      // fast == 2: LDS bytes the 16-B env records add over the 8-B records
                              // (off_cubes / off_target / off_ndelta / off_gen are LDS offsets)
    uint32_t tail_max;        // fast == 4: a wave whose queue ran dry resolves its envs one at a time,
                              // 64 updates per block, once it holds at most this many (0 = never)
    uint32_t lane_limit;      // fast == 4: lanes per wave that take envs from the work queue (64 = all;
                              // <= tail_max: every wave in tail mode from its first env)
    int32_t steal_local;      // fast == 4: hand-off of tail envs between the waves of a workgroup (LDS)
    uint32_t* steal_count;    // envs handed off in this launch (diagnostics), zeroed per launch
    const void* gen_img;      // fast == 2 / 4: the LDS image as staged (host-built, pbn_abi.cpp env_gen_image);
                              // null: the kernel builds it from img
    uint32_t chunk;           // fast == 2 / 4: updates per lane between draw rounds (ENV_CHUNK_SMALL / _LARGE)
    int32_t tail_helpers;     // fast == 4 (with steal_local): up to this many (<= 3) idle waves of the workgroup prepare a long tail
                              // session's blocks ahead (draws, records, writer masks) into the session wave's
                              // LDS ring, so the session wave only resolves (k_env, tail helpers)
    // fast == 4 (with steal_local): grid-wide hand-off of tail envs to workgroups that have run out of work
    // (k_env, "grid pool"). Device memory, control words zeroed per launch:
    uint32_t* gpool_ctl;      // [0] slots reserved by pushers, [1] tickets taken by idle workgroups, [2] live:
                              // workgroups working + envs in the pool, [3] envs pushed, [4] waits given up,
                              // [5] of the pushed, sessions moved mid-way (a long session no sibling could help)
    uint32_t* gpool_state;    // [gpool_cap] per slot: epoch << 2 | 1 (a pusher claimed it) or | 2 (its ticket
                              // holder gave up on it); any other epoch: unclaimed
    uint64_t* gpool;          // [gpool_cap][GPOOL_GRANULES] 8-B {epoch, value} granules: one env's hand-off words
    uint32_t gpool_cap;       // slots; 0 = grid hand-off off
    uint32_t gpool_epoch;     // this launch's tag (1 .. 2^30 - 1, a new one per launch)
    uint32_t gpool_cu_idle;   // 1: a workgroup takes tickets only once no workgroup of its CU is on its own envs;
                              // 0: as soon as its own waves have run out of work
};

constexpr uint32_t GPOOL_GRANULES = 64;  // per slot: the hand-off box as u32 words (10 + 4W <= 64 for W <= 13)
constexpr uint32_t GPOOL_CAP = 8192;     // grid pool slots (4 MiB); envs past them stay with their wave
// control words: [0, 16) counters, [GPOOL_CU_WORD + __smid()] workgroups on that CU still on their own envs
// (__smid() < 1024: XCC, SE, CU id bits); the block is zeroed per launch
constexpr uint32_t GPOOL_CU_WORD = 16, GPOOL_CTL_BYTES = 4u * (GPOOL_CU_WORD + 1024u);
// the pool is on by default for fused launches (several env steps) and for launches whose update cap is at least
// this (pbn_abi.cpp env_launch): one env step at config 5's 4,096 cap lost more to the waiting workgroups'
// residency than the moved envs gave back (1.14 -> 1.18-1.20 ms per step)
constexpr uint32_t GPOOL_MIN_CAP = 16384;

constexpr uint32_t MT_ROW = 624;
constexpr uint32_t MT_TAIL_PAD = 64;  // words allocated past the last row (the twist's unconditional loads read up to 29)

// 1 / log2(1-p) from a geometric-gap table T_k = floor((1-p)^k 2^32) (host side): taken at the
// largest k whose T_k keeps >= 20 significant bits; 0 when every T_k is tiny (p ~ 1).
inline float gap_inv_log2(const uint32_t* T, int N) {
    for (int k = N; k >= 1; --k)
        if (T[k - 1] >= (1u << 20)) return (float)((double)k / __builtin_log2((double)T[k - 1] / 4294967296.0));
    return 0.0f;
}  // u32 words of one MT19937 state row

struct MTArgs {
    uint64_t* state;        // [B][W]
    const void* img;        // network image
    NetLayout L;
    uint64_t B;
    uint32_t T;             // transitions per launch (k_mt_step)
    int32_t n_nodes;
    int32_t init_state;     // k_mt_step: run genRandState / PBN.reset(None) (N init draws) instead of T updates
    const uint64_t* seeds;  // [B] (k_mt_seed)
    uint32_t* mt_py;        // [B][MT_ROW] CPython `random` state
    uint32_t* mt_np;        // [B][MT_ROW] numpy legacy RandomState (probability-table networks)
    uint32_t* pos_py;       // [B] next word index (624 = twist before next use: k_mt_step twists it, coalesced)
    uint32_t* pos_np;
    int32_t lane_walk;      // predictor-mix steps on k_mt_step instead of k_mt_staged (PBNSIM_MT_LANES=1, tests)
};

constexpr int SSD_DAG_KMAX = 6;
// waves per env in shared mode (k_ssd_wave): 4 measured faster than 8 (300 envs x 4,000: 0.19 vs
// 0.23 ms; 1,024 envs: 10.4 vs 8.8 G transitions/s; tools/ssd_shared_sweep.py)
constexpr int SSD_SHARED_WAVES = 4;  // truth-table nodes with more inputs: k_ssd_wave applies serially

struct SSDArgs {
    uint64_t* state;           // [B][W]
    const void* img;           // network image
    NetLayout L;
    uint64_t B, env_base, seed;
    uint64_t iter_base;        // SSD iteration counter of the first iteration (Philox c0/c1)
    uint32_t iters;
    int32_t n_targets;         // g <= 12 (2^g LDS bins)
    const int32_t* targets;    // [g] node indices, first = most significant bucket bit
    const uint32_t* gap_thr;   // [N] T_k = floor((1-p)^k 2^32), k = 1..N; null = no flips
    float gap_inv_log2;        // 1 / log2(1-p) estimated from the table (geo_gap's first guess)
    uint64_t* hist;            // [2^g] accumulated counts (device)
    uint32_t off_planes, off_gap, off_tbit, off_targets, off_hist, lds_bytes;
    int32_t wave;              // 1: one wave per env (k_ssd_wave), small batches
    int32_t dag;               // wave mode: resolve each 64-iteration chunk in parallel (predictor mix,
                               // or truth tables with <= SSD_DAG_KMAX inputs per node); the value is
                               // the waves per env (1, or 4: the workgroup shares one env)
    int32_t* error;            // set to 1 if a shared-mode wave gave up waiting for its turn (never expected)
};

struct SyncArgs {
    uint64_t* state;          // [B][W]
    const void* img;          // network image
    NetLayout L;
    uint64_t B, env_base, seed;
    uint64_t step_base;       // synchronous-step counter of the first step (Philox)
    uint32_t T;
    const uint32_t* gap_thr;  // [N] perturbation gap table (T_k = floor((1-p)^k 2^32)); null = off
    float gap_inv_log2;       // 1 / log2(1-p) estimated from the table
    uint32_t off_planes, off_gap, lds_bytes;
};

// Launchers (pbn_kernels.hip, pbn_mt.hip, pbn_ssd.hip, pbn_sync.hip). Return hipError_t as int.
int launch_bump(uint64_t* p, uint64_t k, void* stream);
int launch_step(int W, const StepArgs& a, int store_mode, int replay, int sb, int grid, void* stream);
uint32_t step_lds_bytes(int W, uint32_t image_bytes, int sb, int grp = 1);
int launch_init(int W, const InitArgs& a, int grid, void* stream);
int launch_flip(int W, const FlipArgs& a, int grid, void* stream);
int launch_unpack(const uint64_t* words, uint8_t* out, uint64_t B, uint32_t N, uint32_t W, int grid, void* stream);
int launch_env_multi(int W, const EnvArgs& a, int replay, int grid, void* stream);
int max_blocks_step(int W, int kind, uint32_t lds_bytes, int sb, int* blocks_per_cu, int rollout = 0, int grp = 1);

#ifndef PBN_ENV_CHUNK
#define PBN_ENV_CHUNK 32
#endif
constexpr uint32_t ENV_CHUNK = PBN_ENV_CHUNK;  // updates per lane between refill rounds
#ifndef PBN_ENV_UNROLL
#define PBN_ENV_UNROLL 8
#endif
constexpr uint32_t ENV_UNROLL = PBN_ENV_UNROLL;  // updates between the wave's "any lane active" tests
// k_env tail mode: live envs per wave at (or below) which a wave whose queue ran dry switches to
// resolving one env at a time across all 64 lanes (PBNSIM_ENV_TAIL overrides; measured: DESIGN.md §6)
constexpr uint32_t ENV_TAIL_DEFAULT = 16;
// Batches of up to this many envs per wave slot (n_cu x workgroups per CU x 4 waves: 3,072 for
// Bittner-200 on 256 CUs): one lane per wave takes envs (EnvArgs::lane_limit = 1), so every wave
// works in tail mode on one env at a time and takes the next from the queue. Measured against lane
// mode (profiles/r03_r6_lanes_sweep.json): faster or tied on every line up to 16,384 envs (5.3 per
// slot; e.g. 8,192 envs, cap 4,096: 0.19 vs 0.96 ms per step); at 32,768 the spec attractors' per-step
// line is 31 % slower (short env steps queue behind long ones in one wave), so 6 per slot
constexpr uint64_t ENV_ONE_LANE_ENVS_PER_SLOT = 6;
// Cooperative-draw kernels (EnvArgs::fast 2 / 4) take their chunk (updates per lane between draw
// rounds) per launch, EnvArgs::chunk: 48 by default -- fewer chunk prologues on the long per-lane
// chains of a per-step launch (131,072 envs, cap 4,096: 1.22 -> 1.17 ms per step) -- and 32 where the
// smaller draw buffers let one more workgroup onto a CU and the launch is throughput-bound (a fused
// multi-step launch over a queue of several envs per lane: 1M envs, T = 100, 3.46 vs 4.05 ms per env
// step); profiles/r04_r6_chunk_sweep.json
constexpr uint32_t ENV_CHUNK_SMALL = 32, ENV_CHUNK_LARGE = 48;
// a wave's draw buffer: the draw table [chunk][64] u16, 64 B (the hand-off flag in tail mode), the
// shared rounds' counter table [64] uint4 by rank (the hand-off box in tail mode)
constexpr uint32_t env_gen_wave_bytes(uint32_t chunk) { return chunk * 64u * 2u + 64u + 64u * 16u; }
int max_blocks_env(int W, int kind, int fast, int grp, uint32_t lds_bytes, int* blocks_per_cu, int n_nodes = 0,
                   uint32_t chunk = ENV_CHUNK_LARGE);
uint32_t env_lds_bytes(int W, uint32_t image_bytes, int fast, int grp, int n_nodes = 0, uint32_t chunk = ENV_CHUNK_LARGE);
inline int env_block(int fast) { return fast == 3 ? BLOCK : ENV_BLOCK; }  // threads per workgroup of the R6 kernel
int launch_mt_seed(int W, const MTArgs& a, int grid, void* stream);
int launch_mt_step(int W, const MTArgs& a, int n_cu, void* stream);  // grid from the kernel's occupancy
uint32_t ssd_block(const SSDArgs& a);
uint32_t ssd_layout(int W, uint32_t image_bytes, int n_nodes, int n_targets, SSDArgs* a);
int launch_ssd(int W, const SSDArgs& a, int grid, void* stream);
uint32_t sync_layout(int W, uint32_t image_bytes, int n_nodes, SyncArgs* a);
int launch_sync(int W, const SyncArgs& a, int grid, void* stream);

}  // namespace pbn
