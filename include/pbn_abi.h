/*
 * pbn_abi.h -- C ABI of libpbnsim.so, the MI355X (gfx950) vectorised PBN simulator.
 *
 * The reference (jakub-zarzycki2022/gym-PBN-stac) is pure Python; its hot path
 * sits behind plain method calls. Each entry point below names the reference
 * interface it replaces (file:line, relative to the reference root). A Python
 * ctypes binding lives in gym-pbn-stac_amd/gym_pbn_amd/_lib.py; INTEGRATION.md
 * shows the binding a gym-PBN maintainer would add.
 *
 * Conventions
 *  - Every function returns PBN_OK (0) or a negative PBN_E_* code and never
 *    aborts; pbn_last_error() returns a thread-local message for the last failure.
 *  - State is bit-packed: env e, node i lives in bit (i % 64) of word
 *    e*W + i/64, W = ceil(N/64). Host arrays are [B][W] uint64.
 *  - The library owns all device memory and copies network tables; callers own
 *    host arrays, which are read or written only during the call.
 *  - One batch = one device + one HIP stream. Calls on one batch must be
 *    serialised by the caller; different batches may be driven from different
 *    threads. Functions taking host outputs synchronise the batch stream; the
 *    rest are asynchronous until pbn_sync().
 *  - RNG modes: PHILOX (production; counter-based, keyed by
 *    (seed, global env id, update counter) so results do not depend on batch
 *    size or GPU count), REPLAY (caller supplies the reference's own draws), and
 *    MT (each env runs CPython's MT19937 -- and for probability-table networks
 *    numpy's legacy MT19937 too -- seeded like random.seed(s)/np.random.seed(s),
 *    reproducing the reference trajectory from the seed alone).
 */
#ifndef PBN_ABI_H
#define PBN_ABI_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PBN_ABI_VERSION 14

enum {
    PBN_OK = 0,
    PBN_E_INVALID = -1,     /* bad argument / descriptor */
    PBN_E_RANGE = -2,       /* node or action out of range (reference: ValueError, base.py:283-284) */
    PBN_E_HIP = -3,         /* HIP runtime failure */
    PBN_E_NOMEM = -4,       /* device allocation failed */
    PBN_E_UNSUPPORTED = -5, /* network outside kernel limits (N > 512, tables > LDS budget) */
    PBN_E_STATE = -6        /* wrong mode / uninitialised (reference: Exception, base.py:90-91) */
};

enum { PBN_KIND_PREDICTOR_MIX = 1, PBN_KIND_PROB_TABLE = 2 };

typedef struct pbn_net pbn_net;
typedef struct pbn_batch pbn_batch;
typedef struct pbn_envcfg pbn_envcfg;

/* Network tables (see gym_pbn_amd/network.py for how they are derived).
 * PREDICTOR_MIX replaces base.Node.predictors (base.py:30-45) + Predstep (:89-119):
 *   pred_offsets [N+1], pred_inputs [P][3] node indices, pred_tt [P] 16-entry truth
 *   table over (x0<<3|x1<<2|x2<<1|x_self), pred_thr [P] exact 53-bit selection
 *   thresholds (predictor j is selected for the first j with k53 < thr[j]).
 * PROB_TABLE replaces common/node.py Node (input_mask, function; :22-38):
 *   node_k [N], input_offsets [N+1], inputs [sum k] (ascending, first = MSB),
 *   thr_offsets [N+1], thr [sum 2^k] = ceil(p * 2^53). */
typedef struct {
    int32_t kind;
    int32_t n_nodes;
    int32_t n_preds;
    const int32_t *pred_offsets;
    const int32_t *pred_inputs;
    const uint16_t *pred_tt;
    const uint64_t *pred_thr;
    const int32_t *node_k;
    const int32_t *input_offsets;
    const int32_t *inputs;
    const int64_t *thr_offsets;
    const uint64_t *thr;
} pbn_net_desc;

typedef struct {
    int32_t n_nodes, n_words, kind, device;
    uint64_t n_envs, env_id_base, seed;
    uint64_t update_count; /* Philox updates applied so far (batch-wide counter) */
    uint32_t env_call_count, reset_count;
    int32_t mt_ready; /* 1 after pbn_mt_seed */
    int32_t env_lanes; /* last R6 env-step launch: 1 = one lane per env (k_env), 2/4/8 = lanes per env (k_env_grp) */
    int32_t roll_lanes; /* rollout kernel: 1 = one lane per env (k_rollout), 2/4/8 = lanes per env (k_rollout_grp) */
    int32_t env_grid;   /* last R6 env-step launch: workgroups (256 lanes each; lanes refill from a work counter) */
    int32_t env_kernel; /* last R6 env-step launch: 0 = cube matching, 1 = byte counters, 2 = byte counters +
                           wave-generated draws, 3 = group mode (k_env_grp), 4 = 2 with one counter word (<= 4 cubes) */
    int32_t env_lane_limit; /* last R6 env-step launch, env_kernel 4: lanes per wave taking envs from the work
                               queue (64 = every lane; 1 = one env per wave at a time, resolved 64 updates per block) */
    int32_t env_handoff;    /* last R6 env-step launch, env_kernel 4: 1 if a wave in tail mode could hand envs it had
                               not started on to idle waves of its workgroup (PBNSIM_ENV_STEAL=0 turns it off);
                               count: pbn_env_handoffs */
    int32_t env_chunk;      /* last R6 env-step launch, env_kernel 2/4: updates per lane between draw rounds (32 or 48;
                               PBNSIM_ENV_CHUNK overrides) */
} pbn_batch_info;

/* Attractor / goal description for the multi-flip env step (R6).
 * cubes: union of the attractor hypercubes (cabean output, '*' = don't care),
 *   care/value [n_cubes][W]: state s is attracting iff (s & care) == value for
 *   some cube -- the membership test of the expanded set built at
 *   pbn_target_multi.py:437-455 and queried at :489-492.
 * reset cubes: all_attractors[0] (reset draws one and fills '*' bits, :237-249).
 * target: all_attractors[-1][0] -- in_target() only ever tests target[0] (:190-199). */
typedef struct {
    int32_t n_cubes;
    const uint64_t *cube_care;
    const uint64_t *cube_value;
    int32_t n_reset_cubes;
    const uint64_t *reset_care;
    const uint64_t *reset_value;
    const uint64_t *target_care;  /* [W] */
    const uint64_t *target_value; /* [W] */
    int32_t horizon;              /* truncated = n_steps == horizon (:224) */
    int32_t reward_success;       /* +1000 (:218-219) */
    int32_t action_cost;          /* 1 per unique action value (:222) */
    /* 0: the first update's result is never tested -- the test after it is on the pre-update
     *    snapshot (PBNTargetMultiEnv, :133-134);
     * 1: the state after every update is tested (PBNTargetEnv.step(force=False), pbn_target.py:267-271). */
    int32_t first_update_tested;
} pbn_envcfg_desc;

/* flags returned per env by pbn_env_step_multi* */
enum { PBN_FLAG_TERMINATED = 1, PBN_FLAG_TRUNCATED = 2, PBN_FLAG_CAPPED = 4 };

/* ---- library ---- */
int pbn_abi_version(void);
const char *pbn_last_error(void);
int pbn_device_count(int *count);

/* ---- networks: replaces graph construction, bittner/utils.py:81-91 / pbn.py:78-87 ---- */
int pbn_net_create(const pbn_net_desc *desc, pbn_net **out);
void pbn_net_destroy(pbn_net *net);
/* Predictor-mix networks: the predictor record (in0 | in1<<16 | in2<<32 | tt<<48) that choice
 * word a selects for node `node`, read from the compact image the Philox kernels stage (u32
 * thresholds, saturated, overshoot slot) by the kernels' own rule -- host side, no device. For
 * tests: equals the record of predictor min(#{q : u32_k53(a) >= thr_q}, count - 1)
 * (Predstep's choice, base.py:94-97). */
int pbn_net_select_u32(const pbn_net *net, int32_t node, uint32_t a, uint64_t *record);

/* ---- batches of independent envs (the reference holds one Graph per env) ---- */
/* Tuning knobs, read from the environment once here (measurement and tests only):
 * PBNSIM_STORE_MODE, PBNSIM_ENVS_PER_THREAD, PBNSIM_STEP_BLOCK (step kernel);
 * PBNSIM_ENV_NO_GEN, PBNSIM_ENV_GROUP, PBNSIM_ENV_BPC, PBNSIM_ENV_CHUNK, PBNSIM_ENV_GRID, PBNSIM_ENV_TAIL,
 * PBNSIM_ENV_LANES, PBNSIM_ENV_STEAL, PBNSIM_ENV_HELPERS, PBNSIM_ENV_GRID_STEAL, PBNSIM_ENV_KERNEL_IMAGE (R6 env kernel);
 * every one is set by a `-m gpu` test; A/B-only knobs are compiled in by -DPBN_MEASURE_KNOBS (tools/build_exp.sh);
 * PBNSIM_SSD_WAVE, PBNSIM_SSD_SERIAL, PBNSIM_SSD_SHARED (SSD); PBNSIM_ROLL_GROUP (rollout lanes per env);
 * PBNSIM_STEP_GRAPH=0 (pbn_step without HIP graphs); PBNSIM_MT_LANES=1 (MT-mode steps of predictor-mix networks
 * on k_mt_step's per-lane loads instead of k_mt_staged's LDS windows). */
int pbn_batch_create(const pbn_net *net, int device, uint64_t n_envs, uint64_t env_id_base, uint64_t seed,
                     pbn_batch **out);
void pbn_batch_destroy(pbn_batch *b);
int pbn_batch_get_info(const pbn_batch *b, pbn_batch_info *info);
/* Run every later call of this batch on `stream` (a hipStream_t, e.g. torch's current stream, so
 * kernels order with the caller's own work without host syncs; NULL = the default stream), or on
 * the batch's own stream again (own != 0). Work queued on the previous stream is waited for first. */
int pbn_batch_set_stream(pbn_batch *b, int own, void *stream);
/* Waits for the batch stream. PBN_E_HIP if a device-path R6 launch since the last pbn_sync dropped an env in
 * the grid pool (see pbn_env_grid_stats; never expected). */
int pbn_sync(pbn_batch *b);

/* ---- state I/O: Graph.setState / getState (base.py:364-366, 320-324), PBN.reset(state) (pbn.py:96-119) ---- */
int pbn_set_state(pbn_batch *b, const uint64_t *words);          /* host [B][W] */
int pbn_get_state(pbn_batch *b, uint64_t *words);                /* host [B][W] */
int pbn_set_state_device(pbn_batch *b, const void *dev_words);   /* device [B][W], same device */
int pbn_get_state_device(pbn_batch *b, void *dev_words);
/* One byte per node, device [B][N] uint8, from device words [B][W] (NULL = the batch's state);
 * Graph.getState (base.py:320-324) for the whole batch without leaving the GPU. Asynchronous. */
int pbn_unpack_bits_device(pbn_batch *b, const void *d_words, void *d_bits);
/* Graph.genRandState (base.py:368-370) / PBN.reset(None) (pbn.py:105-118) in Philox mode */
int pbn_randomize_state(pbn_batch *b);

/* ---- intervention: Graph.flipNode (base.py:280-284), PBN.flip (pbn.py:121-127) ----
 * actions [B][A] host int32; value 0 = no action, value v flips node v - offset
 * (offset 1: gym-PBN target envs, pbn_target.py:266-267; offset 0: PBNEnv, pbn_env.py:141-142).
 * dedup 1: act on unique values per row (torch-tensor input, pbn_target_multi.py:120-121). */
int pbn_flip(pbn_batch *b, const int32_t *actions, int A, int offset, int dedup);
/* Same with the actions already on the device (d_actions [B][A] int32, e.g. a torch policy's
 * output), on the batch stream. A row holding an out-of-range value is left untouched (the other
 * rows are flipped) and noted in a device flag. check 1: wait for the kernel, return PBN_E_RANGE
 * if the flag is set (by this call or by earlier check-0 calls) and clear it; check 0: return
 * at once (asynchronous; a later check-1 call reports). */
int pbn_flip_device(pbn_batch *b, const int32_t *d_actions, int A, int offset, int dedup, int check);

/* ---- the hot path: Graph.step (base.py:306-312) / PBN.step (pbn.py:129-133) ---- */
/* Philox mode, n_updates launches of one update each (state round-trips HBM). For batches under
 * 2^20 state words (launch-bound kernels) calls of two or more launches replay captured HIP graphs
 * (not on the null stream, nor with per-launch timing): one graph of exactly n_updates (<= 64)
 * launches when one is cached (pbn_step_prepare, or a call with the same n_updates as the previous
 * call), otherwise graphs of 64, 32, ..., 2 launches by the binary digits of n_updates. Larger batches
 * launch plainly (PBNSIM_STEP_GRAPH=0/1 overrides). Results are identical either way. */
int pbn_step(pbn_batch *b, uint32_t n_updates);
/* Captures the graphs pbn_step(b, n_updates) will replay now (setup only: nothing runs, the state
 * is untouched): for n_updates <= 64 one graph of exactly that many launches (the batch keeps the
 * four most recently used lengths), above that the 64, 32, ..., 2-launch graphs. Batches that
 * launch plainly (see pbn_step): a no-op. n_updates < 2 is a no-op; above PBN_STEP_PREPARE_MAX,
 * PBN_E_INVALID. A failed capture is not an error (pbn_step then launches without it). */
#define PBN_STEP_PREPARE_MAX 4096
int pbn_step_prepare(pbn_batch *b, uint32_t n_updates);
/* Philox mode, one launch applying n_updates in registers; bit-identical to pbn_step. */
int pbn_rollout(pbn_batch *b, uint32_t n_updates);
/* Replay mode: node_idx [T][B] (randint result) and k53 [T][B] (random() * 2^53), host arrays. */
int pbn_step_replay(pbn_batch *b, const uint32_t *node_idx, const uint64_t *k53, uint32_t n_updates);
/* Forced node (replaces Graph.step(i=k), base.py:306-308: `i = randint(...) if i is None else i`):
 * node_idx [T][B] host array (PROB_TABLE: >= 1); update t of env e updates node node_idx[t][e] with
 * the choice word of the Philox step draw pbn_step would have used for that update (its node word
 * is discarded), and the batch's update counter advances by T like pbn_step's. Out-of-range
 * indices: PBN_E_RANGE, nothing launched. Synchronous. */
int pbn_step_forced(pbn_batch *b, const uint32_t *node_idx, uint32_t n_updates);
/* MT mode: seeds [B] (host). random.seed(seeds[e]) (and np.random.seed for PROB_TABLE).
 * init_state 1 also runs Graph.genRandState / PBN.reset(None) from that stream. */
int pbn_mt_seed(pbn_batch *b, const uint64_t *seeds, int init_state);
int pbn_mt_step(pbn_batch *b, uint32_t n_updates); /* asynchronous; seeds >= 2^32 rejected for PROB_TABLE */

/* ---- multi-flip until-attractor env step: PBNTargetMultiEnv.step (pbn_target_multi.py:119-154) ---- */
int pbn_envcfg_create(const pbn_net *net, const pbn_envcfg_desc *desc, pbn_envcfg **out);
void pbn_envcfg_destroy(pbn_envcfg *cfg);
/* PBNTargetMultiEnv.reset (:227-259), Philox mode: envs with mask[e] != 0 (mask NULL = all)
 * get a reset cube chosen uniformly, '*' bits drawn fair, n_steps = 0. */
int pbn_env_reset(pbn_batch *b, const pbn_envcfg *cfg, const uint8_t *mask);
/* Same on the device, asynchronous: d_mask device uint8 [B] (NULL = all envs). */
int pbn_env_reset_device(pbn_batch *b, const pbn_envcfg *cfg, const uint8_t *d_mask);
int pbn_set_n_steps(pbn_batch *b, const int64_t *n_steps);  /* host [B] */
int pbn_get_n_steps(pbn_batch *b, int64_t *n_steps);        /* host [B] */
/* Host arrays: actions [B][A]; outputs obs [B][W], reward [B], flags [B], n_updates [B] (any may be NULL). */
int pbn_env_step_multi(pbn_batch *b, const pbn_envcfg *cfg, const int32_t *actions, int A, int dedup, int offset,
                       uint32_t update_cap, uint64_t *obs, int32_t *reward, uint8_t *flags, uint32_t *n_updates);
/* Device arrays on the batch's device (e.g. torch tensors); asynchronous. */
int pbn_env_step_multi_device(pbn_batch *b, const pbn_envcfg *cfg, const int32_t *d_actions, int A, int dedup,
                              int offset, uint32_t update_cap, uint64_t *d_obs, int32_t *d_reward, uint8_t *d_flags,
                              uint32_t *d_n_updates);
/* n_steps consecutive env steps in one launch (open-loop trajectory collection): device arrays
 * d_actions [n_steps][B][A], outputs [n_steps][B][W] / [n_steps][B]; identical to n_steps calls of
 * pbn_env_step_multi_device with the actions' slices (same Philox draws, env_call_count += n_steps).
 * An env step with an out-of-range action is skipped for that env (error flag set, outputs left). */
int pbn_env_rollout_multi_device(pbn_batch *b, const pbn_envcfg *cfg, uint32_t n_steps, const int32_t *d_actions,
                                 int A, int dedup, int offset, uint32_t update_cap, uint64_t *d_obs, int32_t *d_reward,
                                 uint8_t *d_flags, uint32_t *d_n_updates);
/* Replay mode (parity): draw_offsets [B+1] (int64), draws_i / draws_k the reference's draws, host arrays. */
int pbn_env_step_multi_replay(pbn_batch *b, const pbn_envcfg *cfg, const int32_t *actions, int A, int dedup,
                              int offset, const int64_t *draw_offsets, const uint32_t *draws_i,
                              const uint64_t *draws_k, uint64_t *obs, int32_t *reward, uint8_t *flags,
                              uint32_t *n_updates);

/* ---- synchronous update: Graph.synch_step (base.py:286-303), Philox mode ----
 * every node from the pre-step snapshot, each with its own random(); perturb_gap_thr [N]
 * (T_k = floor((1-p)^k 2^32), NULL = perturbations off): if any node is perturbed, the
 * perturbed nodes flip and no update happens in that step (base.py:288-295). */
int pbn_synch_step(pbn_batch *b, uint32_t n_steps, const uint32_t *perturb_gap_thr);

/* ---- steady-state distribution: compute_ssd_hist / _ssd_run (gym_PBN/utils/eval.py:20-103) ----
 * Every env runs `iters` iterations of: count the bucket of target_nodes (first = MSB), flip each
 * node with probability p, one async transition (Philox). flip_gap_thr [N]: T_k = floor((1-p)^k 2^32),
 * k = 1..N (NULL: no flips). hist [2^n_targets] host counts, ACCUMULATED (+=). n_targets <= 12. */
int pbn_ssd_run(pbn_batch *b, const int32_t *target_nodes, int n_targets, const uint32_t *flip_gap_thr,
                uint32_t iters, uint64_t *hist);

/* ---- measurement: HIP events on the batch stream. mode 1: a pair around every kernel launch;
 *      mode 2: one region from before the first launch to after the last (launch gaps included) ---- */
int pbn_timing_enable(pbn_batch *b, int enable);
int pbn_timing_read(pbn_batch *b, double *kernel_ms, uint64_t *launches); /* syncs, then resets */
/* mode 1 only: each timed launch's kernel ms in launch order (up to cap; *launches = how many were timed);
 * syncs, then resets like pbn_timing_read. Lets a timed loop keep per-launch figures without host reads
 * inside it. */
int pbn_timing_read_each(pbn_batch *b, double *ms_each, uint64_t cap, uint64_t *launches);
/* Envs handed from a tail-mode wave to an idle one during the last R6 env-step launch (env_kernel 4;
 * 0 when the hand-off was off). Syncs the batch stream. Diagnostics: the reference has no counterpart
 * (its until-attractor loop, pbn_target_multi.py:135-146, runs one env in one process). */
int pbn_env_handoffs(pbn_batch *b, uint32_t *count);
/* Tail helpers recruited during the last R6 env-step launch (env_kernel 4): idle waves of a workgroup that
 * prepared a long tail session's blocks ahead of the session wave (draws, records, writer masks; the session
 * wave only resolves). Syncs the batch stream. Diagnostics; PBNSIM_ENV_HELPERS=0 turns them off. */
int pbn_env_tail_helpers(pbn_batch *b, uint32_t *count);
/* The last R6 launch's tail counters, stats[4]: envs handed off, helpers recruited, tail blocks the
 * sessions read from their helpers' rings, and of those the blocks not yet written when the session reached
 * them (the session waited). Syncs the batch stream. Diagnostics. */
int pbn_env_tail_stats(pbn_batch *b, uint32_t *stats);
/* The last R6 launch's grid-pool counters, stats[4] (env_kernel 4 with the hand-off on; on by default for fused
 * launches and update caps >= 16,384, PBNSIM_ENV_GRID_STEAL=0/1 forces it): envs a tail wave handed to a workgroup
 * that had run out of work (anywhere on the GPU), tickets those workgroups took, waits given up (0 unless a launch
 * failed with PBN_E_HIP), the live count at the launch's end (0). Syncs the batch stream. Diagnostics. A given-up
 * wait drops the env it waited for: host-path env calls return PBN_E_HIP at once, device-path launches
 * (pbn_env_step_multi_device, pbn_env_rollout_multi_device) at the next pbn_sync. */
int pbn_env_grid_stats(pbn_batch *b, uint32_t *stats);

#ifdef __cplusplus
}
#endif
#endif /* PBN_ABI_H */
