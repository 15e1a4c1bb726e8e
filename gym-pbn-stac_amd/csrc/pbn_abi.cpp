// pbn_abi.cpp -- host side of libpbnsim.so: the C ABI declared in include/pbn_abi.h.
//
// Owns device memory, validates descriptors, packs the network tables into the
// LDS image the kernels stage, and drives the kernels on one HIP stream per batch.
// There is no host compute path: every state transition runs on the GPU, and a
// missing/unsupported device is reported as an error, never silently emulated.
#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/pbn_abi.h"
#include "pbn_params.hpp"

using namespace pbn;

namespace {

thread_local std::string g_err;

int fail(int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}

#define HIP_TRY(expr)                                                                              \
    do {                                                                                           \
        hipError_t _e = (expr);                                                                    \
        if (_e != hipSuccess) return fail(PBN_E_HIP, "%s failed: %s", #expr, hipGetErrorString(_e)); \
    } while (0)

inline uint32_t align16(uint32_t x) { return (x + 15u) & ~15u; }

struct DevBuf {
    void* p = nullptr;
    size_t cap = 0;
    int ensure(size_t bytes) {
        if (bytes <= cap) return 0;
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
        hipError_t e = hipMalloc(&p, bytes);
        if (e != hipSuccess) return fail(PBN_E_NOMEM, "hipMalloc(%zu) failed: %s", bytes, hipGetErrorString(e));
        cap = bytes;
        return 0;
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
    }
};

// Pinned host staging for small transfers (single envs, small batches): pageable copies of a
// few bytes cost several microseconds each in the runtime's staging path.
struct PinBuf {
    static constexpr size_t CAP = 64 * 1024;
    uint8_t* p = nullptr;
    bool ready() {
        if (!p && hipHostMalloc((void**)&p, CAP, hipHostMallocDefault) != hipSuccess) p = nullptr;
        return p != nullptr;
    }
    void release() {
        if (p) (void)hipHostFree(p);
        p = nullptr;
    }
};

}  // namespace

struct pbn_net {
    int kind = 0, N = 0, W = 0;
    int kmax = 0;                // truth-table networks: most inputs of one node
    std::vector<uint8_t> image;  // host copy of the LDS image
    NetLayout L{};
    std::mutex mu;
    std::map<int, void*> dev_image;  // per device
    const void* image_on(int device) {
        std::lock_guard<std::mutex> g(mu);
        auto it = dev_image.find(device);
        if (it != dev_image.end()) return it->second;
        void* p = nullptr;
        if (hipMalloc(&p, image.size()) != hipSuccess) return nullptr;
        if (hipMemcpy(p, image.data(), image.size(), hipMemcpyHostToDevice) != hipSuccess) {
            (void)hipFree(p);
            return nullptr;
        }
        dev_image[device] = p;
        return p;
    }
};

struct pbn_envcfg {
    const pbn_net* net = nullptr;
    int W = 0, H = 0, H_reset = 0;
    std::vector<uint8_t> image;  // net image + cubes [H][2][W] + target [2][W]
    NetLayout L{};
    uint32_t off_cubes = 0, off_target = 0, off_ndelta = 0;
    int fast = 0;
    std::vector<uint64_t> reset_care, reset_value;
    int32_t horizon = 100, reward_success = 1000, action_cost = 1, first_tested = 0;
    std::mutex mu;
    struct Dev {
        void* image = nullptr;
        void* reset_care = nullptr;
        void* reset_value = nullptr;
        void* gen_image = nullptr;  // k_env modes 2/4: the LDS image as staged (env_gen_image), built once
    };
    std::vector<uint8_t> gen_image;  // host copy (erec_shift is fixed by the network and the cubes)
    std::map<int, Dev> dev;
    const Dev* on(int device) {
        std::lock_guard<std::mutex> g(mu);
        auto it = dev.find(device);
        if (it != dev.end()) return &it->second;
        Dev d;
        size_t rb = reset_care.size() * 8;
        if (hipMalloc(&d.image, image.size()) != hipSuccess) return nullptr;
        if (hipMemcpy(d.image, image.data(), image.size(), hipMemcpyHostToDevice) != hipSuccess) return nullptr;
        if (rb) {
            if (hipMalloc(&d.reset_care, rb) != hipSuccess || hipMalloc(&d.reset_value, rb) != hipSuccess)
                return nullptr;
            if (hipMemcpy(d.reset_care, reset_care.data(), rb, hipMemcpyHostToDevice) != hipSuccess ||
                hipMemcpy(d.reset_value, reset_value.data(), rb, hipMemcpyHostToDevice) != hipSuccess)
                return nullptr;
        }
        dev[device] = d;
        return &dev[device];
    }
};

constexpr uint32_t STEP_GRAPH_K = 64;  // longest captured run of step launches
constexpr int STEP_GRAPH_SIZES = 6;     // graphs of 64, 32, 16, 8, 4 and 2 launches
constexpr uint64_t STEP_GRAPH_MAX_WORDS = 1ull << 20;  // state words from which step mode launches plainly

struct pbn_batch {
    pbn_net* net = nullptr;
    int device = 0, W = 0, N = 0;
    hipStream_t stream = nullptr;      // the stream every call of this batch runs on
    hipStream_t own_stream = nullptr;  // created with the batch; `stream` unless pbn_batch_set_stream
    uint64_t B = 0, env_base = 0, seed = 0, update_count = 0;
    uint32_t env_calls = 0, reset_count = 0;
    int env_lanes = 0;  // lanes per env of the last R6 launch
    int env_grid_last = 0;  // workgroups of the last R6 launch
    int env_lane_limit_last = 0;  // lanes per wave taking envs in the last R6 launch
    int env_chunk_last = 0;       // draw-round chunk of the last R6 launch
    int env_kernel_last = -1;  // pbn_batch_info.env_kernel of the last R6 launch
    uint64_t* d_state = nullptr;
    int64_t* d_nsteps = nullptr;
    int32_t* d_error = nullptr;
    bool fault_check = false;  // a device-path env launch used the grid pool since the last pbn_sync
    const void* d_image = nullptr;
    int n_cu = 0, bpc_step = 1, bpc_env = 1, bpc_base = 1, bpc_roll = 1;
    int step_block = 1024;  // threads per workgroup of the Philox step kernel (256 or 1024)
    int store_mode = STORE_DIRTY;
    int envs_per_thread = 2;  // K: envs each thread walks per launch (pipelined)
    // R6 launch knobs (measurement / tests; read once at pbn_batch_create)
    bool env_no_gen = false;  // PBNSIM_ENV_NO_GEN: no cooperative draw generation
    int env_group = 0;        // PBNSIM_ENV_GROUP: lanes per env (1 = lane mode), 0 = by batch size
    int env_bpc = 0;          // PBNSIM_ENV_BPC: cap on resident workgroups per CU, 0 = none
    int env_chunk = 0;        // PBNSIM_ENV_CHUNK: draw-round chunk 32 / 48 of the cooperative-draw kernels, 0 = auto
    int env_grid_cap = 0;     // PBNSIM_ENV_GRID: the R6 kernel's workgroups (tests: lane refill, hand-offs), 0 = by size
    int env_tail = -1;        // PBNSIM_ENV_TAIL: the R6 kernel's tail-mode threshold (live envs per wave), -1 = default
    int env_lane_limit = 0;   // PBNSIM_ENV_LANES: lanes per wave taking envs in the tail-mode kernel, 0 = auto
    bool env_steal = true;    // PBNSIM_ENV_STEAL=0: no hand-off of tail envs between a workgroup's waves (k_env, mode 4)
    bool env_kernel_image = false;  // PBNSIM_ENV_KERNEL_IMAGE=1: k_env builds its LDS image (no host-built image)
    int env_helpers = 3;      // PBNSIM_ENV_HELPERS: at most this many tail helpers per session (0-3; 0 = off)
    // PBNSIM_ENV_GRID_STEAL: grid-wide hand-off of tail envs (k_env, mode 4): 1 on, 0 off, unset = fused launches
    // and update caps from GPOOL_MIN_CAP (below it one env step's loops are too short to repay the waiting
    // workgroups' residency)
    int env_grid_steal = -1;
    int env_pool_cu_idle = -1;    // PBNSIM_ENV_POOL_CU_IDLE: 1 only idle CUs take pool tickets, 0 any idle workgroup,
                                  // -1 = the default (1)
    int env_grid_slots = 0;      // PBNSIM_ENV_GRID_SLOTS: pool slots in use (measurement: 1 keeps the waiting workgroups
                                 // resident but moves at most one env), 0 = GPOOL_CAP
    int ssd_wave = -1;        // PBNSIM_SSD_WAVE: 1 = one wave per env, 0 = one lane per env, -1 = by size
    bool ssd_serial = false;  // PBNSIM_SSD_SERIAL=1: wave mode applies each chunk serially (no chunk DAG)
    int ssd_shared = -1;      // PBNSIM_SSD_SHARED: 0 = one wave per env, 4 / 8 = that many, 1 = the default
                              // count, -1 = by size
    int roll_group = 1;       // PBNSIM_ROLL_GROUP: lanes per env of the rollout kernel (default by size)
    bool mt_lane_walk = false;  // PBNSIM_MT_LANES=1: MT-mode steps of predictor-mix networks on k_mt_step
    // step mode without HIP graphs: by default for large batches (a graph replay's start on the
    // device costs more than host submission, which a long kernel hides: 1M Bittner-200 envs, 20
    // launches: 9.3 us per launch plain vs 9.9 us as one replay); PBNSIM_STEP_GRAPH=0/1 forces it
    bool step_graph_off = false;
    // step_graph[j]: (STEP_GRAPH_K >> j) step launches + k_bump, captured once (all sizes at the
    // first call of two or more steps)
    hipGraphExec_t step_graph[STEP_GRAPH_SIZES] = {};
    bool step_graph_built = false;
    bool step_graph_broken = false;       // capture or instantiation failed once: plain launches
    bool exact_broken = false;            // an exact-length capture failed once: no more of them
    // exact-length graphs: one replay for a whole call of n steps (pbn_step_prepare, or the second
    // call with the same n); each extra replay in a call costs a graph start on the device (~13 us)
    static constexpr int EXACT_GRAPHS = 4;
    uint32_t exact_n[EXACT_GRAPHS] = {};
    hipGraphExec_t exact_graph[EXACT_GRAPHS] = {};
    uint64_t exact_used[EXACT_GRAPHS] = {};  // LRU stamps
    uint64_t exact_clock = 0;
    uint32_t last_step_n = 0;
    DevBuf s_ubase;                       // device copy of update_count for graph replays
    DevBuf s_flip_err;                    // range-error flag of pbn_flip_device
    DevBuf s_act, s_obs, s_rew, s_flags, s_nup, s_replay_i, s_replay_k, s_off, s_mask;
    DevBuf mt_py, mt_np, mt_pos_py, mt_pos_np, mt_seeds;  // MT mode (allocated by pbn_mt_seed)
    DevBuf s_counter;                                     // env-step work-queue head
    DevBuf s_steal;                                       // k_env tail hand-off: count of envs handed off
    bool steal_last = false;                              // the last R6 launch had the hand-off on
    DevBuf s_gpool;                                       // k_env grid pool: control words, slot states, slots
    uint32_t gpool_epoch = 0;                             // the last R6 launch's pool epoch
    bool gpool_last = false;                              // the last R6 launch had the grid pool on
    PinBuf pin;                                           // staging for small host<->device copies
    DevBuf s_ssd_hist, s_ssd_tab;                         // SSD histogram + gap/target tables
    uint64_t ssd_iters = 0;                               // SSD iteration counter (Philox)
    DevBuf s_sync_tab;                                    // perturbation gap table
    uint64_t sync_steps = 0;                              // synchronous-step counter (Philox)
    // timing: mode 1 = an event pair around every launch; mode 2 = one region
    // (start before the first launch after enabling, stop after the latest launch)
    int timing = 0;
    std::vector<std::pair<hipEvent_t, hipEvent_t>> ev_pool;
    size_t ev_used = 0;
    uint64_t region_launches = 0;
    bool region_closed = false;
    hipEvent_t region_start = nullptr;  // ev_pool[0].first once the region's first launch is queued
    hipEvent_t region_end = nullptr;    // the closed region's stop event
    int mt_ready = 0;

    int grid_for(uint64_t items, int bpc, int block = BLOCK) const {
        uint64_t need = (items + block - 1) / block;
        uint64_t cap = (uint64_t)n_cu * (uint64_t)bpc;
        uint64_t g = std::min<uint64_t>(need, cap);
        return (int)std::max<uint64_t>(g, 1);
    }
    int grid_all(uint64_t items) const { return (int)std::max<uint64_t>((items + BLOCK - 1) / BLOCK, 1); }
    int ev_begin(hipEvent_t* stop) {
        *stop = nullptr;
        if (!timing) return 0;
        if (timing == 2) {
            if (ev_pool.empty()) {
                hipEvent_t a, b;
                HIP_TRY(hipEventCreate(&a));
                HIP_TRY(hipEventCreate(&b));
                ev_pool.emplace_back(a, b);
            }
            if (region_launches == 0) {
                HIP_TRY(hipEventRecord(ev_pool[0].first, stream));
                region_start = ev_pool[0].first;
            }
            region_launches++;
            ev_used = 1;
            return 0;  // the stop event is recorded once: pbn_timing_enable(0) or pbn_timing_read
        }
        if (ev_used == ev_pool.size()) {
            hipEvent_t a, b;
            HIP_TRY(hipEventCreate(&a));
            HIP_TRY(hipEventCreate(&b));
            ev_pool.emplace_back(a, b);
        }
        auto& pr = ev_pool[ev_used++];
        HIP_TRY(hipEventRecord(pr.first, stream));
        *stop = pr.second;
        return 0;
    }
    int ev_end(hipEvent_t stop) {
        if (stop) HIP_TRY(hipEventRecord(stop, stream));
        return 0;
    }
};

#define CHECK_NN(p, name) \
    if (!(p)) return fail(PBN_E_INVALID, "%s is NULL", name)
#define SET_DEV(b) HIP_TRY(hipSetDevice((b)->device))

static int build_predictor_image(const pbn_net_desc* d, pbn_net* n) {
    const int N = d->n_nodes, P = d->n_preds;
    CHECK_NN(d->pred_offsets, "pred_offsets");
    CHECK_NN(d->pred_inputs, "pred_inputs");
    CHECK_NN(d->pred_tt, "pred_tt");
    CHECK_NN(d->pred_thr, "pred_thr");
    if (P < 1 || P > 65535) return fail(PBN_E_UNSUPPORTED, "n_preds=%d outside [1, 65535]", P);
    if (d->pred_offsets[0] != 0 || d->pred_offsets[N] != P) return fail(PBN_E_INVALID, "pred_offsets must span [0, P]");
    for (int i = 0; i < N; i++) {
        int c = d->pred_offsets[i + 1] - d->pred_offsets[i];
        if (c < 1) return fail(PBN_E_INVALID, "node %d has no predictors (Predstep would fail, base.py:95-104)", i);
        for (int j = d->pred_offsets[i] + 1; j < d->pred_offsets[i + 1]; j++)
            if (d->pred_thr[j] < d->pred_thr[j - 1]) return fail(PBN_E_INVALID, "pred_thr not non-decreasing at node %d", i);
    }
    for (int j = 0; j < 3 * P; j++)
        if (d->pred_inputs[j] < 0 || d->pred_inputs[j] >= N)
            return fail(PBN_E_RANGE, "predictor input %d out of range [0, %d)", d->pred_inputs[j], N);
    uint32_t pmax = 1;
    for (int i = 0; i < N; i++) pmax = std::max(pmax, (uint32_t)(d->pred_offsets[i + 1] - d->pred_offsets[i]));
    NetLayout L{};
    L.tp = (pmax - 1 + 1) & ~1u;
    L.pmax = pmax;
    L.off_node = 0;
    L.off_thr = 0;
    L.off_rec = align16(8u * L.tp * (uint32_t)N);
    L.bytes = align16(L.off_rec + 8u * pmax * (uint32_t)N);
    {  // the Philox kernels' compact LDS image (thr32_layout, pbn_device.hpp): their planes follow it
        const uint32_t tp4 = (L.tp + 3u) & ~3u, rs = std::max(tp4 + 1u, pmax);
        L.plane_off = std::max(L.bytes, align16(align16(4u * tp4 * (uint32_t)N) + 8u * rs * (uint32_t)N));
    }
    L.kind = KIND_PREDICTOR_MIX;
    L.n_nodes = N;
    if (L.plane_off > MAX_IMAGE)
        return fail(PBN_E_UNSUPPORTED, "network tables (%u B) exceed the LDS budget", L.plane_off);
    n->image.assign(L.bytes, 0);
    uint8_t* im = n->image.data();
    for (int i = 0; i < N; i++) {
        const int o0 = d->pred_offsets[i], c = d->pred_offsets[i + 1] - d->pred_offsets[i];
        for (uint32_t q = 0; q < L.tp; q++) {
            // predictor j is skipped iff k53 >= thr[j]; thresholds past the last-but-one never are
            const uint64_t t = (int)q < c - 1 ? d->pred_thr[o0 + q] : ~0ull;
            memcpy(im + L.off_thr + 8 * ((size_t)i * L.tp + q), &t, 8);
        }
        for (int q = 0; q < c; q++) {
            const int j = o0 + q;
            uint64_t rec = (uint64_t)(uint32_t)d->pred_inputs[3 * j] |
                           ((uint64_t)(uint32_t)d->pred_inputs[3 * j + 1] << 16) |
                           ((uint64_t)(uint32_t)d->pred_inputs[3 * j + 2] << 32) | ((uint64_t)d->pred_tt[j] << 48);
            memcpy(im + L.off_rec + 8 * ((size_t)i * pmax + q), &rec, 8);
        }
    }
    // Compact image of the Philox kernels, appended after L.bytes (thr32_layout / stage_image_thr32
    // in pbn_device.hpp): u32 thresholds on the choice word, saturated; slot tp4 of a node's record
    // row holds the record a = 2^32 - 1 selects (its count of thresholds below 2^32), which is where
    // the saturated count lands.
    const uint32_t tp4 = (L.tp + 3u) & ~3u, rs = std::max(tp4 + 1u, pmax);
    const uint32_t rec_off = align16(4u * tp4 * (uint32_t)N);
    n->image.resize((size_t)L.bytes + align16(rec_off + 8u * rs * (uint32_t)N), 0);
    im = n->image.data();  // resize reallocates
    uint8_t* cm = im + L.bytes;
    auto k53 = [](uint64_t a) { return (a << 21) | (a >> 11); };
    for (int i = 0; i < N; i++) {
        uint32_t m = 0;
        for (uint32_t q = 0; q < tp4; q++) {
            uint64_t T = ~0ull;
            if (q < L.tp) memcpy(&T, im + L.off_thr + 8 * ((size_t)i * L.tp + q), 8);
            const uint64_t a0 = T >> 21;
            const uint64_t t = a0 >= (1ull << 32) ? (1ull << 32) : (k53(a0) >= T ? a0 : a0 + 1u);
            m += t >> 32 ? 0u : 1u;
            const uint32_t s = t >> 32 ? 0xFFFFFFFFu : (uint32_t)t;
            memcpy(cm + 4 * ((size_t)i * tp4 + q), &s, 4);
        }
        for (uint32_t q = 0; q < rs; q++) {
            const uint32_t src = q == tp4 ? m : q;
            if (src < pmax) memcpy(cm + rec_off + 8 * ((size_t)i * rs + q), im + L.off_rec + 8 * ((size_t)i * pmax + src), 8);
        }
    }
    n->L = L;
    return 0;
}

static int build_table_image(const pbn_net_desc* d, pbn_net* n) {
    const int N = d->n_nodes;
    CHECK_NN(d->node_k, "node_k");
    CHECK_NN(d->input_offsets, "input_offsets");
    CHECK_NN(d->thr_offsets, "thr_offsets");
    CHECK_NN(d->thr, "thr");
    if (N < 2) return fail(PBN_E_INVALID, "a PBN needs N >= 2 (node 0 is never updated, pbn.py:131)");
    int64_t sum_k = 0, sum_t = 0;
    for (int i = 0; i < N; i++)
        if (d->node_k[i] > 0 && !d->inputs) return fail(PBN_E_INVALID, "inputs is NULL");
    for (int i = 0; i < N; i++) {
        int k = d->node_k[i];
        if (k < 0 || k > 16) return fail(PBN_E_UNSUPPORTED, "node %d has %d inputs (max 16)", i, k);
        if (d->input_offsets[i] != sum_k) return fail(PBN_E_INVALID, "input_offsets inconsistent at node %d", i);
        if (d->thr_offsets[i] != sum_t) return fail(PBN_E_INVALID, "thr_offsets inconsistent at node %d", i);
        for (int q = 0; q < k; q++) {
            int in = d->inputs[sum_k + q];
            if (in < 0 || in >= N) return fail(PBN_E_RANGE, "input %d of node %d out of range", in, i);
        }
        sum_k += k;
        sum_t += (int64_t)1 << k;
        n->kmax = std::max(n->kmax, (int)k);
    }
    NetLayout L{};
    L.off_node = 0;
    L.off_rec = align16(8u * (uint32_t)N);
    uint64_t after_in = L.off_rec + 2u * (uint64_t)sum_k;
    if (after_in > MAX_IMAGE) return fail(PBN_E_UNSUPPORTED, "input lists exceed the LDS budget");
    L.off_thr = align16((uint32_t)after_in);
    uint64_t total = (uint64_t)L.off_thr + 8u * (uint64_t)sum_t;
    if (total > MAX_IMAGE) return fail(PBN_E_UNSUPPORTED, "probability tables (%llu B) exceed the LDS budget",
                                       (unsigned long long)total);
    L.bytes = align16((uint32_t)total);
    L.plane_off = L.bytes;
    L.kind = KIND_PROB_TABLE;
    L.n_nodes = N;
    n->image.assign(L.bytes, 0);
    uint8_t* im = n->image.data();
    for (int i = 0; i < N; i++) {
        uint64_t v = (uint64_t)(uint32_t)d->thr_offsets[i] | ((uint64_t)(uint32_t)d->input_offsets[i] << 32) |
                     ((uint64_t)(uint32_t)d->node_k[i] << 48);
        memcpy(im + L.off_node + 8 * i, &v, 8);
    }
    for (int64_t q = 0; q < sum_k; q++) {
        uint16_t v = (uint16_t)d->inputs[q];
        memcpy(im + L.off_rec + 2 * q, &v, 2);
    }
    memcpy(im + L.off_thr, d->thr, 8 * (size_t)sum_t);
    n->L = L;
    return 0;
}

extern "C" {

int pbn_abi_version(void) { return PBN_ABI_VERSION; }

const char* pbn_last_error(void) { return g_err.c_str(); }

int pbn_device_count(int* count) {
    CHECK_NN(count, "count");
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess) {
        *count = 0;
        return fail(PBN_E_HIP, "hipGetDeviceCount: %s", hipGetErrorString(e));
    }
    *count = n;
    return 0;
}

int pbn_net_create(const pbn_net_desc* d, pbn_net** out) {
    CHECK_NN(d, "desc");
    CHECK_NN(out, "out");
    *out = nullptr;
    if (d->n_nodes < 1 || d->n_nodes > 64 * MAX_WORDS)
        return fail(PBN_E_UNSUPPORTED, "n_nodes=%d outside [1, %d]", d->n_nodes, 64 * MAX_WORDS);
    pbn_net* n = new pbn_net;
    n->kind = d->kind;
    n->N = d->n_nodes;
    n->W = (d->n_nodes + 63) / 64;
    int rc;
    if (d->kind == PBN_KIND_PREDICTOR_MIX)
        rc = build_predictor_image(d, n);
    else if (d->kind == PBN_KIND_PROB_TABLE)
        rc = build_table_image(d, n);
    else
        rc = fail(PBN_E_INVALID, "unknown network kind %d", d->kind);
    if (rc) {
        delete n;
        return rc;
    }
    *out = n;
    return 0;
}

int pbn_net_select_u32(const pbn_net* n, int32_t node, uint32_t a, uint64_t* record) {
    CHECK_NN(n, "net");
    CHECK_NN(record, "record");
    if (n->L.kind != KIND_PREDICTOR_MIX) return fail(PBN_E_INVALID, "not a predictor-mix network");
    if (node < 0 || node >= n->L.n_nodes) return fail(PBN_E_RANGE, "node %d out of range", node);
    // thr32_layout / predictor_choice32 / predictor_record32 (pbn_device.hpp) on the host copy
    const uint32_t tp4 = (n->L.tp + 3u) & ~3u, rs = std::max(tp4 + 1u, n->L.pmax);
    const uint32_t rec_off = align16(4u * tp4 * (uint32_t)n->L.n_nodes);
    const uint8_t* cm = n->image.data() + n->L.bytes;
    uint32_t j = 0;
    for (uint32_t q = 0; q < tp4; q++) {
        uint32_t t;
        memcpy(&t, cm + 4 * ((size_t)node * tp4 + q), 4);
        j += a >= t ? 1u : 0u;
    }
    memcpy(record, cm + rec_off + 8 * ((size_t)node * rs + j), 8);
    return 0;
}

void pbn_net_destroy(pbn_net* n) {
    if (!n) return;
    for (auto& kv : n->dev_image) {
        (void)hipSetDevice(kv.first);
        (void)hipFree(kv.second);
    }
    delete n;
}

// k_rollout_grp: predictor mix, N <= 256 (byte-packed node lists of a group)
static bool roll_group_ok(const pbn_net* net) { return net->kind == PBN_KIND_PREDICTOR_MIX && net->N <= 256; }

// Lanes per env of the rollout kernel by batch size: the largest G with B x G <= 512 lanes per CU
// (8 waves per CU). Measured on MI355X (tools/rollout_group_sweep.py, node-updates/s): Bittner-28
// 65,536 envs 114 G (lane) -> 145 G (G = 2); 16,384 envs 31 -> 74 G (G = 8); Bittner-200
// 65,536 envs 164 -> 183 G (G = 2); from 131,072 envs on lane mode is as fast or faster (the
// group kernel spends ~1.1x (G = 2) to ~2x (G = 4, 8) the VALU work per update).
static int roll_group_size(const pbn_batch* b, const pbn_net* net) {
    if (!roll_group_ok(net)) return 1;
    const uint64_t lanes = (uint64_t)b->n_cu * 512u;
    for (int g = 8; g >= 2; g /= 2)
        if (b->B * (uint64_t)g <= lanes) return g;
    return 1;
}

int pbn_batch_create(const pbn_net* net_c, int device, uint64_t n_envs, uint64_t env_id_base, uint64_t seed,
                     pbn_batch** out) {
    CHECK_NN(net_c, "net");
    CHECK_NN(out, "out");
    *out = nullptr;
    pbn_net* net = const_cast<pbn_net*>(net_c);
    if (n_envs < 1) return fail(PBN_E_INVALID, "n_envs must be >= 1");
    if (env_id_base + n_envs > ((uint64_t)1 << 56)) return fail(PBN_E_RANGE, "global env ids must stay below 2^56");
    int ndev = 0;
    hipError_t e = hipGetDeviceCount(&ndev);
    if (e != hipSuccess || ndev < 1)
        return fail(PBN_E_HIP, "no HIP device available (hipGetDeviceCount: %s); libpbnsim has no CPU path",
                    hipGetErrorString(e));
    if (device < 0 || device >= ndev) return fail(PBN_E_RANGE, "device %d outside [0, %d)", device, ndev);
    HIP_TRY(hipSetDevice(device));
    pbn_batch* b = new pbn_batch;
    b->net = net;
    b->device = device;
    b->W = net->W;
    b->N = net->N;
    b->B = n_envs;
    b->env_base = env_id_base;
    b->seed = seed;
    if (const char* sm = getenv("PBNSIM_STORE_MODE")) b->store_mode = atoi(sm) ? STORE_DIRTY : STORE_FULL;
    if (const char* r = getenv("PBNSIM_ENVS_PER_THREAD")) b->envs_per_thread = std::max(1, std::min(64, atoi(r)));
    hipDeviceProp_t prop;
    int rc = 0;
    auto bail = [&](int code) {
        pbn_batch_destroy(b);
        return code;
    };
    if (hipGetDeviceProperties(&prop, device) != hipSuccess) return bail(fail(PBN_E_HIP, "hipGetDeviceProperties"));
    b->n_cu = prop.multiProcessorCount;
    if (const char* sbv = getenv("PBNSIM_STEP_BLOCK"))
        b->step_block = atoi(sbv) == 256 ? 256 : 1024;
    else  // 1024-thread groups stage the image 4x less often; small batches need more, smaller groups
        b->step_block = n_envs >= (uint64_t)b->n_cu * 1024u * (uint64_t)b->envs_per_thread ? 1024 : 256;
    b->env_no_gen = getenv("PBNSIM_ENV_NO_GEN") != nullptr;
    if (const char* v = getenv("PBNSIM_ENV_GROUP")) b->env_group = std::max(1, atoi(v));
    if (const char* v = getenv("PBNSIM_ENV_BPC")) b->env_bpc = std::max(1, atoi(v));
    if (const char* v = getenv("PBNSIM_ENV_CHUNK")) b->env_chunk = atoi(v);
    if (const char* v = getenv("PBNSIM_ENV_GRID")) b->env_grid_cap = std::max(1, atoi(v));
    if (const char* v = getenv("PBNSIM_ENV_TAIL")) b->env_tail = std::max(0, std::min(64, atoi(v)));
    if (const char* v = getenv("PBNSIM_ENV_LANES")) b->env_lane_limit = std::max(0, std::min(64, atoi(v)));
    if (const char* v = getenv("PBNSIM_ENV_STEAL")) b->env_steal = atoi(v) != 0;
    if (const char* v = getenv("PBNSIM_ENV_KERNEL_IMAGE")) b->env_kernel_image = atoi(v) != 0;
    if (const char* v = getenv("PBNSIM_ENV_HELPERS")) b->env_helpers = std::max(0, std::min(3, atoi(v)));
    if (const char* v = getenv("PBNSIM_ENV_GRID_STEAL")) b->env_grid_steal = atoi(v) != 0 ? 1 : 0;
#ifdef PBN_MEASURE_KNOBS  // A/B-only knobs: tools/build_exp.sh -DPBN_MEASURE_KNOBS
    if (const char* v = getenv("PBNSIM_ENV_POOL_CU_IDLE")) b->env_pool_cu_idle = atoi(v) != 0 ? 1 : 0;
    if (const char* v = getenv("PBNSIM_ENV_GRID_SLOTS")) b->env_grid_slots = std::max(1, std::min((int)GPOOL_CAP, atoi(v)));
#endif
    if (const char* v = getenv("PBNSIM_SSD_WAVE")) b->ssd_wave = atoi(v) ? 1 : 0;
    if (const char* v = getenv("PBNSIM_SSD_SERIAL")) b->ssd_serial = atoi(v) != 0;
    if (const char* v = getenv("PBNSIM_SSD_SHARED")) {
        const int w = atoi(v);
        b->ssd_shared = w == 0 ? 0 : (w == 4 || w == 8) ? w : 1;
    }
    b->step_graph_off = n_envs * (uint64_t)b->W >= STEP_GRAPH_MAX_WORDS;
    if (const char* v = getenv("PBNSIM_STEP_GRAPH")) b->step_graph_off = atoi(v) == 0;
    if (const char* v = getenv("PBNSIM_MT_LANES")) b->mt_lane_walk = atoi(v) != 0;
    // rollout lanes per env: 1 = k_rollout; 2/4/8 = k_rollout_grp (predictor mix, N <= 256)
    b->roll_group = roll_group_size(b, net);
    if (const char* v = getenv("PBNSIM_ROLL_GROUP")) {
        const int g = atoi(v);
        b->roll_group = (g == 2 || g == 4 || g == 8) && roll_group_ok(net) ? g : 1;
    }
    if (hipStreamCreateWithFlags(&b->stream, hipStreamNonBlocking) != hipSuccess)
        return bail(fail(PBN_E_HIP, "hipStreamCreate"));
    b->own_stream = b->stream;
    size_t sb = 8 * (size_t)b->W * n_envs;
    if (hipMalloc(&b->d_state, sb) != hipSuccess) return bail(fail(PBN_E_NOMEM, "state alloc (%zu B)", sb));
    if (hipMalloc(&b->d_nsteps, 8 * n_envs) != hipSuccess) return bail(fail(PBN_E_NOMEM, "n_steps alloc"));
    // [0] the launch's error flags (zeroed per launch), [1] sticky grid-pool faults of device-path env
    // launches, read and cleared by pbn_sync
    if (hipMalloc(&b->d_error, 8) != hipSuccess) return bail(fail(PBN_E_NOMEM, "error flag alloc"));
    if (hipMemsetAsync(b->d_error, 0, 8, b->stream) != hipSuccess || hipMemsetAsync(b->d_state, 0, sb, b->stream) != hipSuccess ||
        hipMemsetAsync(b->d_nsteps, 0, 8 * n_envs, b->stream) != hipSuccess)
        return bail(fail(PBN_E_HIP, "hipMemset"));
    b->d_image = net->image_on(device);
    if (!b->d_image) return bail(fail(PBN_E_NOMEM, "network image upload failed"));
    if ((rc = max_blocks_step(b->W, net->kind, net->L.bytes, BLOCK, &b->bpc_base)))
        return bail(fail(PBN_E_HIP, "occupancy query: %s", hipGetErrorString((hipError_t)rc)));
    if ((rc = max_blocks_step(b->W, net->kind, net->L.plane_off, b->step_block, &b->bpc_step)))
        return bail(fail(PBN_E_HIP, "occupancy query: %s", hipGetErrorString((hipError_t)rc)));
    if ((rc = max_blocks_step(b->W, net->kind, net->L.plane_off, BLOCK, &b->bpc_roll, 1, b->roll_group)))
        return bail(fail(PBN_E_HIP, "occupancy query: %s", hipGetErrorString((hipError_t)rc)));
    if (hipStreamSynchronize(b->stream) != hipSuccess) return bail(fail(PBN_E_HIP, "stream sync"));
    *out = b;
    return 0;
}

void pbn_batch_destroy(pbn_batch* b) {
    if (!b) return;
    (void)hipSetDevice(b->device);
    if (b->stream) (void)hipStreamSynchronize(b->stream);
    for (auto& pr : b->ev_pool) {
        (void)hipEventDestroy(pr.first);
        (void)hipEventDestroy(pr.second);
    }
    if (b->d_state) (void)hipFree(b->d_state);
    if (b->d_nsteps) (void)hipFree(b->d_nsteps);
    if (b->d_error) (void)hipFree(b->d_error);
    for (DevBuf* d : {&b->s_act, &b->s_obs, &b->s_rew, &b->s_flags, &b->s_nup, &b->s_replay_i, &b->s_replay_k,
                      &b->s_off, &b->s_mask, &b->mt_py, &b->mt_np, &b->mt_pos_py, &b->mt_pos_np, &b->mt_seeds,
                      &b->s_counter, &b->s_steal, &b->s_gpool, &b->s_ssd_hist, &b->s_ssd_tab, &b->s_sync_tab, &b->s_ubase, &b->s_flip_err})
        d->release();
    for (hipGraphExec_t& g : b->step_graph)
        if (g) (void)hipGraphExecDestroy(g);
    for (hipGraphExec_t& g : b->exact_graph)
        if (g) (void)hipGraphExecDestroy(g);
    b->pin.release();
    if (b->own_stream) {
        (void)hipStreamSynchronize(b->stream);
        (void)hipStreamDestroy(b->own_stream);
    }
    delete b;
}

int pbn_batch_set_stream(pbn_batch* b, int own, void* stream) {
    CHECK_NN(b, "batch");
    hipStream_t s = own ? b->own_stream : (hipStream_t)stream;  // NULL = the default stream
    if (s == b->stream) return 0;
    SET_DEV(b);
    HIP_TRY(hipStreamSynchronize(b->stream));  // work already queued on the old stream finishes first
    b->stream = s;
    return 0;
}

int pbn_batch_get_info(const pbn_batch* b, pbn_batch_info* info) {
    CHECK_NN(b, "batch");
    CHECK_NN(info, "info");
    info->n_nodes = b->N;
    info->n_words = b->W;
    info->kind = b->net->kind;
    info->device = b->device;
    info->n_envs = b->B;
    info->env_id_base = b->env_base;
    info->seed = b->seed;
    info->update_count = b->update_count;
    info->env_call_count = b->env_calls;
    info->reset_count = b->reset_count;
    info->mt_ready = b->mt_ready;
    info->env_lanes = b->env_lanes;
    info->roll_lanes = b->roll_group;
    info->env_grid = b->env_grid_last;
    info->env_kernel = b->env_kernel_last;
    info->env_lane_limit = b->env_lane_limit_last;
    info->env_handoff = b->steal_last ? 1 : 0;
    info->env_chunk = b->env_chunk_last;
    return 0;
}

int pbn_sync(pbn_batch* b) {
    CHECK_NN(b, "batch");
    SET_DEV(b);
    HIP_TRY(hipStreamSynchronize(b->stream));
    if (b->fault_check) {
        // a device-path env launch ran with the grid pool: its outputs reach the caller without a host
        // read, so a dropped env (a claimed slot whose words never arrived) is reported here
        b->fault_check = false;
        int32_t f = 0;
        HIP_TRY(hipMemcpy(&f, b->d_error + 1, 4, hipMemcpyDeviceToHost));
        if (f) {
            HIP_TRY(hipMemset(b->d_error + 1, 0, 4));
            return fail(PBN_E_HIP, "k_env grid pool: a wait timed out in a device-path launch (an env's outputs "
                                   "were not written)");
        }
    }
    return 0;
}

static int check_state_words(const pbn_batch* b, const uint64_t* w) {
    const int r = b->N & 63;
    if (!r) return 0;
    const uint64_t bad = ~(((uint64_t)1 << r) - 1);
    for (uint64_t e = 0; e < b->B; e++)
        if (w[e * b->W + b->W - 1] & bad) return fail(PBN_E_RANGE, "env %llu has bits set beyond node %d",
                                                       (unsigned long long)e, b->N - 1);
    return 0;
}

// host -> device through the pinned staging buffer when small (the caller syncs before reuse)
static int h2d(pbn_batch* b, void* dst, const void* src, size_t bytes) {
    if (bytes <= PinBuf::CAP && b->pin.ready()) {
        HIP_TRY(hipStreamSynchronize(b->stream));  // the staging buffer may still feed an earlier copy
        memcpy(b->pin.p, src, bytes);
        HIP_TRY(hipMemcpyAsync(dst, b->pin.p, bytes, hipMemcpyHostToDevice, b->stream));
    } else {
        HIP_TRY(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, b->stream));
    }
    return 0;
}

int pbn_set_state(pbn_batch* b, const uint64_t* words) {
    CHECK_NN(b, "batch");
    CHECK_NN(words, "words");
    if (int rc = check_state_words(b, words)) return rc;
    SET_DEV(b);
    if (int rc = h2d(b, b->d_state, words, 8 * (size_t)b->W * b->B)) return rc;
    HIP_TRY(hipStreamSynchronize(b->stream));
    return 0;
}

int pbn_get_state(pbn_batch* b, uint64_t* words) {
    CHECK_NN(b, "batch");
    CHECK_NN(words, "words");
    SET_DEV(b);
    const size_t bytes = 8 * (size_t)b->W * b->B;
    if (bytes <= PinBuf::CAP && b->pin.ready()) {
        HIP_TRY(hipMemcpyAsync(b->pin.p, b->d_state, bytes, hipMemcpyDeviceToHost, b->stream));
        HIP_TRY(hipStreamSynchronize(b->stream));
        memcpy(words, b->pin.p, bytes);
        return 0;
    }
    HIP_TRY(hipMemcpyAsync(words, b->d_state, bytes, hipMemcpyDeviceToHost, b->stream));
    HIP_TRY(hipStreamSynchronize(b->stream));
    return 0;
}

int pbn_set_state_device(pbn_batch* b, const void* dev_words) {
    CHECK_NN(b, "batch");
    CHECK_NN(dev_words, "dev_words");
    SET_DEV(b);
    HIP_TRY(hipMemcpyAsync(b->d_state, dev_words, 8 * (size_t)b->W * b->B, hipMemcpyDeviceToDevice, b->stream));
    return 0;
}

int pbn_get_state_device(pbn_batch* b, void* dev_words) {
    CHECK_NN(b, "batch");
    CHECK_NN(dev_words, "dev_words");
    SET_DEV(b);
    HIP_TRY(hipMemcpyAsync(dev_words, b->d_state, 8 * (size_t)b->W * b->B, hipMemcpyDeviceToDevice, b->stream));
    return 0;
}

int pbn_unpack_bits_device(pbn_batch* b, const void* d_words, void* d_bits) {
    CHECK_NN(b, "batch");
    CHECK_NN(d_bits, "d_bits");
    SET_DEV(b);
    const uint64_t total = b->B * (uint64_t)b->N;
    const int grid = (int)std::min<uint64_t>((total + BLOCK - 1) / BLOCK, (uint64_t)b->n_cu * 32u);
    int e = launch_unpack(d_words ? (const uint64_t*)d_words : b->d_state, (uint8_t*)d_bits, b->B, (uint32_t)b->N,
                          (uint32_t)b->W, std::max(grid, 1), b->stream);
    if (e) return fail(PBN_E_HIP, "k_unpack launch: %s", hipGetErrorString((hipError_t)e));
    return 0;
}

static int run_init(pbn_batch* b, const pbn_envcfg* cfg, const void* d_mask, const void* care, const void* value) {
    InitArgs a{};
    a.state = b->d_state;
    a.B = b->B;
    a.env_base = b->env_base;
    a.seed = b->seed;
    a.reset_count = b->reset_count;
    a.n_nodes = b->N;
    a.kind = b->net->kind;
    a.cube_care = (const uint64_t*)care;
    a.cube_value = (const uint64_t*)value;
    a.n_cubes = cfg ? cfg->H_reset : 0;
    a.mask = (const uint8_t*)d_mask;
    a.n_steps = cfg ? b->d_nsteps : nullptr;
    hipEvent_t stop;
    if (int rc = b->ev_begin(&stop)) return rc;
    int e = launch_init(b->W, a, b->grid_all(b->B), b->stream);
    if (e) return fail(PBN_E_HIP, "k_init launch: %s", hipGetErrorString((hipError_t)e));
    if (int rc = b->ev_end(stop)) return rc;
    b->reset_count++;
    return 0;
}

int pbn_randomize_state(pbn_batch* b) {
    CHECK_NN(b, "batch");
    SET_DEV(b);
    return run_init(b, nullptr, nullptr, nullptr, nullptr);
}

static int validate_actions(const pbn_batch* b, const int32_t* actions, int A, int offset) {
    if (A < 1 || A > 4096) return fail(PBN_E_INVALID, "A=%d outside [1, 4096]", A);
    if (offset != 0 && offset != 1) return fail(PBN_E_INVALID, "offset must be 0 or 1");
    const uint64_t n = b->B * (uint64_t)A;
    for (uint64_t k = 0; k < n; k++) {
        int32_t v = actions[k];
        if (v == 0) continue;
        int32_t idx = v - offset;
        if (idx >= b->N || idx < -b->N)
            return fail(PBN_E_RANGE, "Invalid action, no node at index %d (env %llu)", idx,
                        (unsigned long long)(k / A));  // base.py:283-284
    }
    return 0;
}

int pbn_flip(pbn_batch* b, const int32_t* actions, int A, int offset, int dedup) {
    CHECK_NN(b, "batch");
    CHECK_NN(actions, "actions");
    if (int rc = validate_actions(b, actions, A, offset)) return rc;
    SET_DEV(b);
    size_t bytes = 4 * (size_t)A * b->B;
    if (int rc = b->s_act.ensure(bytes)) return rc;
    HIP_TRY(hipMemcpyAsync(b->s_act.p, actions, bytes, hipMemcpyHostToDevice, b->stream));
    HIP_TRY(hipMemsetAsync(b->d_error, 0, 4, b->stream));
    FlipArgs a{b->d_state, (const int32_t*)b->s_act.p, b->B, A, offset, dedup ? 1 : 0, b->N, b->d_error};
    int e = launch_flip(b->W, a, b->grid_all(b->B), b->stream);
    if (e) return fail(PBN_E_HIP, "k_flip launch: %s", hipGetErrorString((hipError_t)e));
    HIP_TRY(hipStreamSynchronize(b->stream));
    return 0;
}

int pbn_flip_device(pbn_batch* b, const int32_t* d_actions, int A, int offset, int dedup, int check) {
    CHECK_NN(b, "batch");
    CHECK_NN(d_actions, "d_actions");
    if (A < 1 || A > 4096) return fail(PBN_E_INVALID, "A=%d outside [1, 4096]", A);
    if (offset != 0 && offset != 1) return fail(PBN_E_INVALID, "offset must be 0 or 1");
    SET_DEV(b);
    int32_t* flag = (int32_t*)b->s_flip_err.p;  // zeroed at allocation and after every check
    if (!flag) {
        if (int rc = b->s_flip_err.ensure(4)) return rc;
        flag = (int32_t*)b->s_flip_err.p;
        HIP_TRY(hipMemsetAsync(flag, 0, 4, b->stream));
    }
    FlipArgs a{b->d_state, d_actions, b->B, A, offset, dedup ? 1 : 0, b->N, flag};
    int e = launch_flip(b->W, a, b->grid_all(b->B), b->stream);
    if (e) return fail(PBN_E_HIP, "k_flip launch: %s", hipGetErrorString((hipError_t)e));
    if (!check) return 0;
    if (!b->pin.ready()) return fail(PBN_E_NOMEM, "pinned staging buffer");
    HIP_TRY(hipMemcpyAsync(b->pin.p, flag, 4, hipMemcpyDeviceToHost, b->stream));
    HIP_TRY(hipMemsetAsync(flag, 0, 4, b->stream));
    HIP_TRY(hipStreamSynchronize(b->stream));
    int32_t err;
    memcpy(&err, b->pin.p, 4);
    if (err) return fail(PBN_E_RANGE, "Invalid action: a value names no node (rows holding one were left untouched)");
    return 0;
}

static int step_launch(pbn_batch* b, uint32_t T, uint64_t update_base, int replay, const void* d_i, const void* d_k,
                       const uint64_t* ubase_dev = nullptr, bool timed = true) {
    StepArgs a{};
    a.ubase_dev = ubase_dev;
    a.state = b->d_state;
    a.img = b->d_image;
    a.L = b->net->L;
    a.B = b->B;
    a.env_base = b->env_base;
    a.seed = b->seed;
    a.update_base = update_base;
    a.T = T;
    a.replay_node = (const uint32_t*)d_i;
    a.replay_k53 = (const uint64_t*)d_k;
    hipEvent_t stop = nullptr;
    if (timed)
        if (int rc = b->ev_begin(&stop)) return rc;
    int store = (T == 1 && !replay) ? b->store_mode : STORE_FULL;
    // step mode: K envs per thread (their loads overlap); rollout: one env per lane up to the
    // resident grid -- its T updates are the work, and more lanes hide more LDS latency
    // (Bittner-28 @65,536 envs, T = 256: 115 vs 62 G updates/s with K = 2)
    const bool rollout = T > 1 && !replay;  // k_rollout (or k_rollout_grp), 256-thread groups
    a.grp = rollout ? b->roll_group : 1;
    const uint64_t K = rollout ? 1u : (uint64_t)b->envs_per_thread;
    const uint64_t lanes = rollout ? b->B * (uint64_t)a.grp : (b->B + K - 1) / K;
    const int sb = (replay || rollout) ? BLOCK : b->step_block;
    const int grid = replay    ? b->grid_for(lanes, b->bpc_base)
                     : rollout ? b->grid_for(lanes, b->bpc_roll, sb)
                               : b->grid_for(lanes, b->bpc_step, sb);
    int e = launch_step(b->W, a, store, replay, sb, grid, b->stream);
    if (e) return fail(PBN_E_HIP, "k_step launch: %s", hipGetErrorString((hipError_t)e));
    return timed ? b->ev_end(stop) : 0;
}

// Step mode is launch-bound between kernels (one HBM pass each): runs of step launches go out
// as captured HIP graphs -- the same kernels with the same arguments, except that the update
// counter comes from device memory (*ubase + k for launch k; k_bump adds the graph's length at
// its end), so one instantiated graph per length serves every replay. Lengths 64, 32, ..., 2 are
// all captured at the first call of two or more steps; a call of n steps replays 64-graphs, then
// the binary digits of the rest (n = 20: the 16- and the 4-graph), then one plain launch if n is odd.
static bool step_graph_ready(pbn_batch* b) {
    if (b->step_graph_built) return true;
    if (b->step_graph_broken || b->step_graph_off || !b->stream) return false;  // the null stream cannot capture
    if (b->s_ubase.ensure(64)) return false;
    bool ok = true;
    for (int j = 0; ok && j < STEP_GRAPH_SIZES; ++j) {
        const uint32_t K = STEP_GRAPH_K >> j;
        hipGraph_t g = nullptr;
        ok = hipStreamBeginCapture(b->stream, hipStreamCaptureModeThreadLocal) == hipSuccess;
        bool launched = ok;
        for (uint32_t k = 0; launched && k < K; ++k)
            launched = step_launch(b, 1, k, 0, nullptr, nullptr, (const uint64_t*)b->s_ubase.p, false) == 0;
        if (launched) launched = launch_bump((uint64_t*)b->s_ubase.p, K, b->stream) == 0;
        if (ok) ok = hipStreamEndCapture(b->stream, &g) == hipSuccess && launched && g;
        if (ok) ok = hipGraphInstantiate(&b->step_graph[j], g, nullptr, nullptr, 0) == hipSuccess;
        if (g) (void)hipGraphDestroy(g);
    }
    if (!ok) {
        for (hipGraphExec_t& g : b->step_graph) {
            if (g) (void)hipGraphExecDestroy(g);
            g = nullptr;
        }
        b->step_graph_broken = true;
        (void)hipGetLastError();  // the failed capture is not the caller's error
        g_err.clear();
        return false;
    }
    b->step_graph_built = true;
    return true;
}

// Captures n step launches as one graph in a free (or the least recently used) exact-length slot.
// Returns the slot, or -1 (plain launches / power-of-two graphs then).
static int exact_graph_build(pbn_batch* b, uint32_t n) {
    if (n < 2 || n > STEP_GRAPH_K || b->step_graph_broken || b->step_graph_off || b->exact_broken || !b->stream)
        return -1;
    if (b->s_ubase.ensure(64)) return -1;
    // capture and instantiate into a fresh exec first: a failed capture leaves the cached graphs
    // as they were and marks the batch, so later calls do not re-capture n launches to fail again
    // no k_bump: pbn_step writes the device counter before every replay of an exact graph
    hipGraph_t g = nullptr;
    hipGraphExec_t x = nullptr;
    bool ok = hipStreamBeginCapture(b->stream, hipStreamCaptureModeThreadLocal) == hipSuccess;
    bool launched = ok;
    for (uint32_t k = 0; launched && k < n; ++k)
        launched = step_launch(b, 1, k, 0, nullptr, nullptr, (const uint64_t*)b->s_ubase.p, false) == 0;
    if (ok) ok = hipStreamEndCapture(b->stream, &g) == hipSuccess && launched && g;
    if (ok) ok = hipGraphInstantiate(&x, g, nullptr, nullptr, 0) == hipSuccess;
    // upload now, so the first replay (e.g. a timed one) does not pay for it
    if (ok) ok = hipGraphUpload(x, b->stream) == hipSuccess;
    if (g) (void)hipGraphDestroy(g);
    if (!ok) {
        if (x) (void)hipGraphExecDestroy(x);
        b->exact_broken = true;
        (void)hipGetLastError();
        g_err.clear();
        return -1;
    }
    int slot = 0;
    for (int j = 1; j < pbn_batch::EXACT_GRAPHS; ++j)
        if (b->exact_used[j] < b->exact_used[slot]) slot = j;
    if (b->exact_graph[slot]) {
        // the evicted exec may still be queued or running from an earlier asynchronous pbn_step on
        // this stream (HIP documents no deferred free): drain the stream first. Eviction happens
        // only at capture time, never in a steady replay loop.
        if (hipStreamSynchronize(b->stream) != hipSuccess) {
            (void)hipGraphExecDestroy(x);
            (void)fail(PBN_E_HIP, "stream sync before graph eviction failed");
            return -1;
        }
        (void)hipGraphExecDestroy(b->exact_graph[slot]);
    }
    b->exact_graph[slot] = x;
    b->exact_n[slot] = n;
    b->exact_used[slot] = ++b->exact_clock;
    return slot;
}

static int exact_graph_find(pbn_batch* b, uint32_t n) {
    for (int j = 0; j < pbn_batch::EXACT_GRAPHS; ++j)
        if (b->exact_graph[j] && b->exact_n[j] == n) return j;
    return -1;
}

static bool stream_capturing(pbn_batch* b) {
    hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
    if (b->stream && hipStreamIsCapturing(b->stream, &cap) != hipSuccess) return true;
    return cap != hipStreamCaptureStatusNone;
}

int pbn_step_prepare(pbn_batch* b, uint32_t n_updates) {
    CHECK_NN(b, "batch");
    if (n_updates > PBN_STEP_PREPARE_MAX)
        return fail(PBN_E_INVALID, "n_updates=%u above PBN_STEP_PREPARE_MAX", n_updates);
    SET_DEV(b);
    if (n_updates < 2 || b->step_graph_off || stream_capturing(b)) return 0;
    // on failure pbn_step falls back to plain launches; runs longer than STEP_GRAPH_K replay the
    // power-of-two graphs (one graph of thousands of launches replayed slower: 3.43 vs 3.16 us per
    // launch at 65,536 Bittner-28 envs)
    if (n_updates > STEP_GRAPH_K) (void)step_graph_ready(b);
    else if (exact_graph_find(b, n_updates) < 0) (void)exact_graph_build(b, n_updates);
    return 0;
}

int pbn_step(pbn_batch* b, uint32_t n_updates) {
    CHECK_NN(b, "batch");
    SET_DEV(b);
    uint32_t t = 0;
    // not while the caller is capturing the stream into a graph of its own: plain launches then
    const bool cap = stream_capturing(b);
    const uint32_t smallest = STEP_GRAPH_K >> (STEP_GRAPH_SIZES - 1);
    int exact = -1;
    if (!cap && b->timing != 1 && n_updates >= 2 && !b->step_graph_off) {
        exact = exact_graph_find(b, n_updates);
        // a length seen twice in a row gets its own graph (an RL loop's fixed step count)
        if (exact < 0 && n_updates == b->last_step_n && n_updates <= STEP_GRAPH_K)
            exact = exact_graph_build(b, n_updates);
    }
    b->last_step_n = n_updates;
    if (exact >= 0) {
        uint32_t* c = (uint32_t*)b->s_ubase.p;
        HIP_TRY(hipMemsetD32Async((hipDeviceptr_t)c, (int)(uint32_t)b->update_count, 1, b->stream));
        HIP_TRY(hipMemsetD32Async((hipDeviceptr_t)(c + 1), (int)(uint32_t)(b->update_count >> 32), 1, b->stream));
        hipEvent_t stop;
        if (int rc = b->ev_begin(&stop)) return rc;
        if (b->timing == 2) b->region_launches += n_updates - 1;  // ev_begin counted one
        HIP_TRY(hipGraphLaunch(b->exact_graph[exact], b->stream));
        if (int rc = b->ev_end(stop)) return rc;
        b->exact_used[exact] = ++b->exact_clock;
        b->update_count += n_updates;
        return 0;
    }
    if (n_updates >= smallest && b->timing != 1 && !cap && step_graph_ready(b)) {
        // device counter <- update_count (two 32-bit memsets: stream-ordered, no host buffer)
        uint32_t* c = (uint32_t*)b->s_ubase.p;
        HIP_TRY(hipMemsetD32Async((hipDeviceptr_t)c, (int)(uint32_t)b->update_count, 1, b->stream));
        HIP_TRY(hipMemsetD32Async((hipDeviceptr_t)(c + 1), (int)(uint32_t)(b->update_count >> 32), 1, b->stream));
        for (int j = 0; j < STEP_GRAPH_SIZES; ++j) {
            const uint32_t K = STEP_GRAPH_K >> j;
            while (n_updates - t >= K && (j == 0 || n_updates - t < 2 * K)) {
                hipEvent_t stop;
                if (int rc = b->ev_begin(&stop)) return rc;
                if (b->timing == 2) b->region_launches += K - 1;  // ev_begin counted one
                HIP_TRY(hipGraphLaunch(b->step_graph[j], b->stream));
                if (int rc = b->ev_end(stop)) return rc;
                b->update_count += K;
                t += K;
            }
        }
    }
    for (; t < n_updates; t++) {
        if (int rc = step_launch(b, 1, b->update_count, 0, nullptr, nullptr)) return rc;
        b->update_count++;
    }
    return 0;
}

int pbn_rollout(pbn_batch* b, uint32_t n_updates) {
    CHECK_NN(b, "batch");
    if (!n_updates) return 0;
    SET_DEV(b);
    if (int rc = step_launch(b, n_updates, b->update_count, 0, nullptr, nullptr)) return rc;
    b->update_count += n_updates;
    return 0;
}

int pbn_step_replay(pbn_batch* b, const uint32_t* node_idx, const uint64_t* k53, uint32_t n_updates) {
    CHECK_NN(b, "batch");
    if (!n_updates) return 0;
    CHECK_NN(node_idx, "node_idx");
    CHECK_NN(k53, "k53");
    const uint64_t n = (uint64_t)n_updates * b->B;
    const uint32_t lo = (uint32_t)b->net->kind == PBN_KIND_PROB_TABLE ? 1u : 0u;
    for (uint64_t q = 0; q < n; q++) {
        if (node_idx[q] >= (uint32_t)b->N || node_idx[q] < lo)
            return fail(PBN_E_RANGE, "replay node index %u outside [%u, %d)", node_idx[q], lo, b->N);
        if (k53[q] >> 53) return fail(PBN_E_RANGE, "replay k53 must be < 2^53");
    }
    SET_DEV(b);
    if (int rc = b->s_replay_i.ensure(4 * n)) return rc;
    if (int rc = b->s_replay_k.ensure(8 * n)) return rc;
    HIP_TRY(hipMemcpyAsync(b->s_replay_i.p, node_idx, 4 * n, hipMemcpyHostToDevice, b->stream));
    HIP_TRY(hipMemcpyAsync(b->s_replay_k.p, k53, 8 * n, hipMemcpyHostToDevice, b->stream));
    if (int rc = step_launch(b, n_updates, 0, 1, b->s_replay_i.p, b->s_replay_k.p)) return rc;
    HIP_TRY(hipStreamSynchronize(b->stream));
    return 0;
}

int pbn_step_forced(pbn_batch* b, const uint32_t* node_idx, uint32_t n_updates) {
    CHECK_NN(b, "batch");
    if (!n_updates) return 0;
    CHECK_NN(node_idx, "node_idx");
    const uint64_t n = (uint64_t)n_updates * b->B;
    const uint32_t lo = (uint32_t)b->net->kind == PBN_KIND_PROB_TABLE ? 1u : 0u;
    for (uint64_t q = 0; q < n; q++)
        if (node_idx[q] >= (uint32_t)b->N || node_idx[q] < lo)
            return fail(PBN_E_RANGE, "forced node index %u outside [%u, %d)", node_idx[q], lo, b->N);
    SET_DEV(b);
    if (int rc = b->s_replay_i.ensure(4 * n)) return rc;
    HIP_TRY(hipMemcpyAsync(b->s_replay_i.p, node_idx, 4 * n, hipMemcpyHostToDevice, b->stream));
    // replay-mode kernel with no k53 array: update t takes the choice word of Philox step update
    // update_count + t (the draw pbn_step would use), so the stream stays in step with pbn_step
    if (int rc = step_launch(b, n_updates, b->update_count, 1, b->s_replay_i.p, nullptr)) return rc;
    b->update_count += n_updates;
    HIP_TRY(hipStreamSynchronize(b->stream));  // the staging buffer is reused by the next call
    return 0;
}

static MTArgs mt_args(pbn_batch* b) {
    MTArgs a{};
    a.state = b->d_state;
    a.img = b->d_image;
    a.L = b->net->L;
    a.B = b->B;
    a.n_nodes = b->N;
    a.mt_py = (uint32_t*)b->mt_py.p;
    a.mt_np = (uint32_t*)b->mt_np.p;
    a.pos_py = (uint32_t*)b->mt_pos_py.p;
    a.pos_np = (uint32_t*)b->mt_pos_np.p;
    a.lane_walk = b->mt_lane_walk ? 1 : 0;
    return a;
}

int pbn_mt_seed(pbn_batch* b, const uint64_t* seeds, int init_state) {
    CHECK_NN(b, "batch");
    CHECK_NN(seeds, "seeds");
    const bool table = b->net->kind == PBN_KIND_PROB_TABLE;
    if (table)  // np.random.seed(s) accepts 0 <= s < 2^32 only
        for (uint64_t e = 0; e < b->B; e++)
            if (seeds[e] >> 32) return fail(PBN_E_RANGE, "Seed must be between 0 and 2**32 - 1 (env %llu)",
                                            (unsigned long long)e);
    SET_DEV(b);
    const size_t row = 4 * ((size_t)MT_ROW * b->B + MT_TAIL_PAD);
    if (int rc = b->mt_py.ensure(row)) return rc;
    if (int rc = b->mt_pos_py.ensure(4 * b->B)) return rc;
    if (table) {
        if (int rc = b->mt_np.ensure(row)) return rc;
        if (int rc = b->mt_pos_np.ensure(4 * b->B)) return rc;
    }
    if (int rc = b->mt_seeds.ensure(8 * b->B)) return rc;
    HIP_TRY(hipMemcpyAsync(b->mt_seeds.p, seeds, 8 * b->B, hipMemcpyHostToDevice, b->stream));
    MTArgs a = mt_args(b);
    a.seeds = (const uint64_t*)b->mt_seeds.p;
    hipEvent_t stop;
    if (int rc = b->ev_begin(&stop)) return rc;
    int e = launch_mt_seed(b->W, a, b->grid_all(b->B), b->stream);
    if (e) return fail(PBN_E_HIP, "k_mt_seed launch: %s", hipGetErrorString((hipError_t)e));
    if (int rc = b->ev_end(stop)) return rc;
    if (init_state) {  // genRandState / PBN.reset(None): the step kernel's init draws
        a.init_state = 1;
        if (int rc = b->ev_begin(&stop)) return rc;
        e = launch_mt_step(b->W, a, b->n_cu, b->stream);
        if (e) return fail(PBN_E_HIP, "k_mt_step (init) launch: %s", hipGetErrorString((hipError_t)e));
        if (int rc = b->ev_end(stop)) return rc;
    }
    HIP_TRY(hipStreamSynchronize(b->stream));
    b->mt_ready = 1;
    return 0;
}

int pbn_mt_step(pbn_batch* b, uint32_t n_updates) {
    CHECK_NN(b, "batch");
    if (!b->mt_ready) return fail(PBN_E_STATE, "pbn_mt_seed has not been called");
    if (!n_updates) return 0;
    SET_DEV(b);
    MTArgs a = mt_args(b);
    a.T = n_updates;
    hipEvent_t stop;
    if (int rc = b->ev_begin(&stop)) return rc;
    int e = launch_mt_step(b->W, a, b->n_cu, b->stream);
    if (e) return fail(PBN_E_HIP, "k_mt_step launch: %s", hipGetErrorString((hipError_t)e));
    return b->ev_end(stop);
}

// ------------------------------------------------------------------ synchronous update
int pbn_synch_step(pbn_batch* b, uint32_t n_steps, const uint32_t* perturb_gap_thr) {
    CHECK_NN(b, "batch");
    if (!n_steps) return 0;
    if (perturb_gap_thr)
        for (int k = 1; k < b->N; k++)
            if (perturb_gap_thr[k] > perturb_gap_thr[k - 1])
                return fail(PBN_E_INVALID, "perturb_gap_thr must be non-increasing");
    SET_DEV(b);
    SyncArgs a{};
    a.state = b->d_state;
    a.img = b->d_image;
    a.L = b->net->L;
    a.B = b->B;
    a.env_base = b->env_base;
    a.seed = b->seed;
    a.step_base = b->sync_steps;
    a.T = n_steps;
    if (perturb_gap_thr) {
        if (int rc = b->s_sync_tab.ensure(4 * (size_t)b->N)) return rc;
        HIP_TRY(hipMemcpyAsync(b->s_sync_tab.p, perturb_gap_thr, 4 * (size_t)b->N, hipMemcpyHostToDevice,
                               b->stream));
        a.gap_thr = (const uint32_t*)b->s_sync_tab.p;
        a.gap_inv_log2 = gap_inv_log2(perturb_gap_thr, b->N);
    }
    a.lds_bytes = sync_layout(b->W, b->net->L.bytes, b->N, &a);
    if (a.lds_bytes > 160u * 1024u) return fail(PBN_E_UNSUPPORTED, "sync LDS footprint %u B too large", a.lds_bytes);
    hipEvent_t stop;
    if (int rc = b->ev_begin(&stop)) return rc;
    int e = launch_sync(b->W, a, b->grid_for(b->B, b->bpc_base), b->stream);
    if (e) return fail(PBN_E_HIP, "k_sync launch: %s", hipGetErrorString((hipError_t)e));
    if (int rc = b->ev_end(stop)) return rc;
    b->sync_steps += n_steps;
    if (perturb_gap_thr) HIP_TRY(hipStreamSynchronize(b->stream));  // table buffer is reused by later calls
    return 0;
}

// ------------------------------------------------------------------ SSD histogram
int pbn_ssd_run(pbn_batch* b, const int32_t* target_nodes, int n_targets, const uint32_t* flip_gap_thr,
                uint32_t iters, uint64_t* hist) {
    CHECK_NN(b, "batch");
    CHECK_NN(target_nodes, "target_nodes");
    CHECK_NN(hist, "hist");
    if (n_targets < 1 || n_targets > 12) return fail(PBN_E_UNSUPPORTED, "n_targets=%d outside [1, 12]", n_targets);
    for (int j = 0; j < n_targets; j++) {
        if (target_nodes[j] < 0 || target_nodes[j] >= b->N)
            return fail(PBN_E_RANGE, "target node %d out of range [0, %d)", target_nodes[j], b->N);
        for (int q = 0; q < j; q++)
            if (target_nodes[q] == target_nodes[j]) return fail(PBN_E_INVALID, "duplicate target node %d", target_nodes[j]);
    }
    if (flip_gap_thr)
        for (int k = 1; k < b->N; k++)
            if (flip_gap_thr[k] > flip_gap_thr[k - 1]) return fail(PBN_E_INVALID, "flip_gap_thr must be non-increasing");
    SET_DEV(b);
    const size_t nb = (size_t)1 << n_targets;
    if (int rc = b->s_ssd_hist.ensure(8 * nb)) return rc;
    if (int rc = b->s_ssd_tab.ensure(4 * (size_t)b->N + 4 * (size_t)n_targets)) return rc;
    uint32_t* d_gap = (uint32_t*)b->s_ssd_tab.p;
    int32_t* d_tgt = (int32_t*)(d_gap + b->N);
    if (flip_gap_thr) HIP_TRY(hipMemcpyAsync(d_gap, flip_gap_thr, 4 * (size_t)b->N, hipMemcpyHostToDevice, b->stream));
    HIP_TRY(hipMemcpyAsync(d_tgt, target_nodes, 4 * (size_t)n_targets, hipMemcpyHostToDevice, b->stream));
    HIP_TRY(hipMemsetAsync(b->s_ssd_hist.p, 0, 8 * nb, b->stream));
    SSDArgs a{};
    a.state = b->d_state;
    a.img = b->d_image;
    a.L = b->net->L;
    a.B = b->B;
    a.env_base = b->env_base;
    a.seed = b->seed;
    a.iter_base = b->ssd_iters;
    a.iters = iters;
    a.n_targets = n_targets;
    a.targets = d_tgt;
    a.gap_thr = flip_gap_thr ? d_gap : nullptr;
    a.gap_inv_log2 = flip_gap_thr ? gap_inv_log2(flip_gap_thr, b->N) : 0.0f;
    a.hist = (uint64_t*)b->s_ssd_hist.p;
    a.error = b->d_error;
    HIP_TRY(hipMemsetAsync(b->d_error, 0, 4, b->stream));
    // one wave per env while the batch is small against the chip (the reference's 300 resets).
    // Crossovers measured on MI355X (tools/ssd_mode_sweep.py, Bittner-200, p = 0.01, G transitions/s):
    // 4,096 envs shared 19.4 / wave 16.4 / lane 0.9; 16,384: 18.4 / 19.8 / 3.8; 65,536: - / 20.1 / 14.7;
    // 262,144: - / 19.8 / 39.4
    a.wave = b->ssd_wave >= 0 ? b->ssd_wave : (b->B <= (uint64_t)b->n_cu * 256u ? 1 : 0);
    a.dag = a.wave && !b->ssd_serial && (b->net->kind == PBN_KIND_PREDICTOR_MIX || b->net->kmax <= SSD_DAG_KMAX) ? 1 : 0;
    // chunk resolution with the workgroup's 4 waves on one env while even that leaves SIMDs free
    if (a.dag && (b->ssd_shared >= 0 ? b->ssd_shared > 0 : b->B <= (uint64_t)b->n_cu * 8u))
        a.dag = b->ssd_shared > 1 ? b->ssd_shared : SSD_SHARED_WAVES;
    a.lds_bytes = ssd_layout(b->W, b->net->L.bytes, b->N, n_targets, &a);
    if (a.lds_bytes > 160u * 1024u) return fail(PBN_E_UNSUPPORTED, "SSD LDS footprint %u B too large", a.lds_bytes);
    hipEvent_t stop;
    if (int rc = b->ev_begin(&stop)) return rc;
    const uint64_t envs_per_block = a.dag > 1 ? 1u : BLOCK / 64;
    const int grid = a.wave ? (int)std::min<uint64_t>((b->B + envs_per_block - 1) / envs_per_block, (uint64_t)b->n_cu * 8u)
                            : b->grid_for(b->B, b->bpc_base);
    int e = launch_ssd(b->W, a, grid, b->stream);
    if (e) return fail(PBN_E_HIP, "k_ssd launch: %s", hipGetErrorString((hipError_t)e));
    if (int rc = b->ev_end(stop)) return rc;
    std::vector<uint64_t> h(nb);
    int32_t err = 0;
    HIP_TRY(hipMemcpyAsync(h.data(), b->s_ssd_hist.p, 8 * nb, hipMemcpyDeviceToHost, b->stream));
    HIP_TRY(hipMemcpyAsync(&err, b->d_error, 4, hipMemcpyDeviceToHost, b->stream));
    HIP_TRY(hipStreamSynchronize(b->stream));
    if (err) return fail(PBN_E_HIP, "k_ssd_wave: a wave timed out waiting for its turn (internal error)");
    for (size_t k = 0; k < nb; k++) hist[k] += h[k];
    b->ssd_iters += iters;
    return 0;
}

// ------------------------------------------------------------------ R6 env
int pbn_envcfg_create(const pbn_net* net, const pbn_envcfg_desc* d, pbn_envcfg** out) {
    CHECK_NN(net, "net");
    CHECK_NN(d, "desc");
    CHECK_NN(out, "out");
    *out = nullptr;
    const int W = net->W;
    if (d->n_cubes < 0 || d->n_cubes > 4096) return fail(PBN_E_INVALID, "n_cubes=%d outside [0, 4096]", d->n_cubes);
    if (d->n_cubes && (!d->cube_care || !d->cube_value)) return fail(PBN_E_INVALID, "cube arrays are NULL");
    if (d->n_reset_cubes < 0 || (d->n_reset_cubes && (!d->reset_care || !d->reset_value)))
        return fail(PBN_E_INVALID, "bad reset cubes");
    CHECK_NN(d->target_care, "target_care");
    CHECK_NN(d->target_value, "target_value");
    pbn_envcfg* c = new pbn_envcfg;
    c->net = net;
    c->W = W;
    c->H = d->n_cubes;
    c->H_reset = d->n_reset_cubes;
    c->L = net->L;
    c->off_cubes = net->L.bytes;
    c->off_target = align16(c->off_cubes + 16u * (uint32_t)W * (uint32_t)c->H);
    c->off_ndelta = align16(c->off_target + 16u * (uint32_t)W);
    uint32_t bytes = align16(c->off_ndelta + 8u * (uint32_t)net->N);
    if (bytes > MAX_IMAGE) {
        delete c;
        return fail(PBN_E_UNSUPPORTED, "network + %d attractor cubes exceed the LDS budget", d->n_cubes);
    }
    c->image.assign(bytes, 0);
    memcpy(c->image.data(), net->image.data(), net->L.bytes);  // not the compact image appended after it
    uint64_t* cubes = reinterpret_cast<uint64_t*>(c->image.data() + c->off_cubes);
    for (int h = 0; h < c->H; h++)
        for (int k = 0; k < W; k++) {
            uint64_t care = d->cube_care[(size_t)h * W + k];
            cubes[(size_t)h * 2 * W + k] = care;
            cubes[(size_t)h * 2 * W + W + k] = d->cube_value[(size_t)h * W + k] & care;
        }
    uint64_t* tgt = reinterpret_cast<uint64_t*>(c->image.data() + c->off_target);
    for (int k = 0; k < W; k++) {
        tgt[k] = d->target_care[k];
        tgt[W + k] = d->target_value[k] & d->target_care[k];
    }
    // Fast attractor test: one byte counter per cube (<= 8 cubes) holding the number of cared
    // bits where the state differs from the cube. Node i going 0 -> 1 adds +1 to the cubes
    // that want it 0 and -1 to those that want it 1; per node that is one packed delta
    // d = plus - minus per 32-bit half (bytes 0-3 = cubes 0-3, 4-7 = cubes 4-7). The
    // counters never leave [0, 255], so M += d (or M -= d for 1 -> 0) is exact word arithmetic.
    int max_care = 0;
    for (int h = 0; h < c->H; h++) {
        int pc = 0;
        for (int k = 0; k < W; k++) pc += __builtin_popcountll(d->cube_care[(size_t)h * W + k]);
        max_care = std::max(max_care, pc);
    }
    c->fast = (c->H <= 8 && max_care <= 255) ? 1 : 0;
    uint32_t* nd = reinterpret_cast<uint32_t*>(c->image.data() + c->off_ndelta);
    for (int i = 0; i < net->N; i++) {
        uint32_t plus[2] = {0, 0}, minus[2] = {0, 0};
        for (int h = 0; h < c->H && h < 8; h++) {
            const uint64_t cw = d->cube_care[(size_t)h * W + i / 64], vw = d->cube_value[(size_t)h * W + i / 64];
            if (!((cw >> (i % 64)) & 1u)) continue;
            const uint32_t byte = 1u << (8 * (h & 3));
            if ((vw >> (i % 64)) & 1u)
                minus[h >> 2] |= byte;
            else
                plus[h >> 2] |= byte;
        }
        nd[2 * i] = plus[0] - minus[0];
        nd[2 * i + 1] = plus[1] - minus[1];
    }
    c->L.bytes = bytes;
    c->L.plane_off = bytes;
    c->reset_care.assign(d->reset_care, d->reset_care + (size_t)c->H_reset * W);
    c->reset_value.assign(d->reset_value, d->reset_value + (size_t)c->H_reset * W);
    c->horizon = d->horizon;
    c->reward_success = d->reward_success;
    c->action_cost = d->action_cost;
    c->first_tested = d->first_update_tested ? 1 : 0;
    *out = c;
    return 0;
}

void pbn_envcfg_destroy(pbn_envcfg* c) {
    if (!c) return;
    for (auto& kv : c->dev) {
        (void)hipSetDevice(kv.first);
        if (kv.second.image) (void)hipFree(kv.second.image);
        if (kv.second.gen_image) (void)hipFree(kv.second.gen_image);
        if (kv.second.reset_care) (void)hipFree(kv.second.reset_care);
        if (kv.second.reset_value) (void)hipFree(kv.second.reset_value);
    }
    delete c;
}

int pbn_env_reset(pbn_batch* b, const pbn_envcfg* cfg_c, const uint8_t* mask) {
    CHECK_NN(b, "batch");
    CHECK_NN(cfg_c, "cfg");
    pbn_envcfg* cfg = const_cast<pbn_envcfg*>(cfg_c);
    if (cfg->net != b->net) return fail(PBN_E_INVALID, "envcfg belongs to another network");
    if (cfg->H_reset < 1) return fail(PBN_E_STATE, "envcfg has no reset cubes (all_attractors[0])");
    SET_DEV(b);
    const pbn_envcfg::Dev* dv = cfg->on(b->device);
    if (!dv) return fail(PBN_E_NOMEM, "envcfg upload failed");
    const void* d_mask = nullptr;
    if (mask) {
        if (int rc = b->s_mask.ensure(b->B)) return rc;
        HIP_TRY(hipMemcpyAsync(b->s_mask.p, mask, b->B, hipMemcpyHostToDevice, b->stream));
        d_mask = b->s_mask.p;
    }
    if (int rc = run_init(b, cfg, d_mask, dv->reset_care, dv->reset_value)) return rc;
    HIP_TRY(hipStreamSynchronize(b->stream));
    return 0;
}

int pbn_env_reset_device(pbn_batch* b, const pbn_envcfg* cfg_c, const uint8_t* d_mask) {
    CHECK_NN(b, "batch");
    CHECK_NN(cfg_c, "cfg");
    pbn_envcfg* cfg = const_cast<pbn_envcfg*>(cfg_c);
    if (cfg->net != b->net) return fail(PBN_E_INVALID, "envcfg belongs to another network");
    if (cfg->H_reset < 1) return fail(PBN_E_STATE, "envcfg has no reset cubes (all_attractors[0])");
    SET_DEV(b);
    const pbn_envcfg::Dev* dv = cfg->on(b->device);
    if (!dv) return fail(PBN_E_NOMEM, "envcfg upload failed");
    return run_init(b, cfg, d_mask, dv->reset_care, dv->reset_value);
}

int pbn_set_n_steps(pbn_batch* b, const int64_t* n_steps) {
    CHECK_NN(b, "batch");
    CHECK_NN(n_steps, "n_steps");
    SET_DEV(b);
    HIP_TRY(hipMemcpyAsync(b->d_nsteps, n_steps, 8 * b->B, hipMemcpyHostToDevice, b->stream));
    HIP_TRY(hipStreamSynchronize(b->stream));
    return 0;
}

int pbn_get_n_steps(pbn_batch* b, int64_t* n_steps) {
    CHECK_NN(b, "batch");
    CHECK_NN(n_steps, "n_steps");
    SET_DEV(b);
    HIP_TRY(hipMemcpyAsync(n_steps, b->d_nsteps, 8 * b->B, hipMemcpyDeviceToHost, b->stream));
    HIP_TRY(hipStreamSynchronize(b->stream));
    return 0;
}

// Lanes per env for the R6 kernel: 1 (lane mode, k_env) while the batch fills the chip
// several times over; group mode where it does not and the until-attractor tail would
// leave lanes idle (measured: DESIGN.md section 6).
// Per-step call, Bittner-200, 1 MI355X (256 CUs): G = 8 beats lane mode up to 32k envs (0.21 vs
// 0.33 ms at B = 1, 0.88 vs 1.99 ms at 8k, 1.85 vs 2.04 ms at 32k) and loses from 64k on (2.31 vs
// 2.07 ms; 131k: 3.28 vs 2.60 ms) -- the crossover sits near 48k envs.
// The LDS image of k_env's cooperative-draw modes (2 / 4), built on the host once per env config: the
// thresholds re-expressed on the draw word (u32, rows of tp4, saturated), the cubes / target / counter
// deltas moved up by erec_shift, and the 16-B env records (pbn_device.hpp env_record) in rows of rs,
// slot tp4 holding the record a = 2^32 - 1 selects. The kernel used to build these itself from the u64
// image in its prologue (dependent global reads in every workgroup: ~8 us of a 63 us lone-env launch);
// now it stages them with plain 16-B copies. Same bytes as the kernel's construction (every R6 test).
static std::vector<uint8_t> env_gen_image(const pbn_envcfg* cfg, uint32_t erec_shift) {
    const NetLayout& L = cfg->L;
    const uint32_t N = (uint32_t)L.n_nodes, tp = L.tp, tp4 = (tp + 3u) & ~3u, rs = std::max(tp4 + 1u, L.pmax);
    std::vector<uint8_t> g((size_t)L.bytes + erec_shift, 0);
    const uint8_t* im = cfg->image.data();
    auto thr = [&](uint32_t i, uint32_t q) -> uint64_t {  // u32_threshold of u64 threshold q of node i (2^32: never)
        uint64_t T;
        memcpy(&T, im + L.off_thr + 8 * ((size_t)i * tp + q), 8);
        const uint64_t a0 = T >> 21;
        if (a0 >= (1ull << 32)) return 1ull << 32;
        return ((a0 << 21) | (a0 >> 11)) >= T ? a0 : a0 + 1u;
    };
    for (uint32_t i = 0; i < N; i++)
        for (uint32_t q = 0; q < tp4; q++) {
            const uint64_t t = q < tp ? thr(i, q) : (1ull << 32);
            const uint32_t v = t >> 32 ? 0xFFFFFFFFu : (uint32_t)t;
            memcpy(g.data() + 4 * ((size_t)i * tp4 + q), &v, 4);
        }
    memcpy(g.data() + cfg->off_cubes + erec_shift, im + cfg->off_cubes, L.bytes - cfg->off_cubes);
    const uint32_t nd_off = cfg->off_ndelta + erec_shift, ROW = ENV_BLOCK * 4u;
    auto off = [&](uint32_t x) { return (x >> 5) * ROW; };
    for (uint32_t i = 0; i < N; i++)
        for (uint32_t q = 0; q < rs; q++) {
            uint32_t src = q;
            if (q == tp4) {  // the node's thresholds below 2^32 on a
                src = 0;
                for (uint32_t p = 0; p < tp; p++) src += (thr(i, p) >> 32) ? 0u : 1u;
            }
            uint64_t rec = 0;
            if (src < L.pmax) memcpy(&rec, im + L.off_rec + 8 * ((size_t)i * L.pmax + src), 8);
            const uint32_t x0 = (uint32_t)rec & 0xFFFFu, x1 = (uint32_t)(rec >> 16) & 0xFFFFu,
                           x2 = (uint32_t)(rec >> 32) & 0xFFFFu;
            const uint32_t w[4] = {off(x0) | (off(x1) << 16), off(x2) | (off(i) << 16),
                                   (x0 & 31u) | ((x1 & 31u) << 8) | ((x2 & 31u) << 16) | ((i & 31u) << 24),
                                   (uint32_t)(rec >> 48) | ((nd_off + 8u * i) << 16)};
            memcpy(g.data() + L.off_rec + 16 * ((size_t)i * rs + q), w, 16);
        }
    return g;
}

// Group mode (G = 8 lanes per env) for small batches -- except where the tail kernel (k_env mode 4:
// <= 4 cubes and its 16-B env records fit) applies: its tail mode with one env per wave
// (env_lane_limit) is faster at every batch size measured (profiles/r03_r6_lanes_sweep.json)
static int env_group_size(const pbn_batch* b, bool tail_kernel) {
    if (tail_kernel) return 1;
    return b->B * 8 <= (uint64_t)b->n_cu * 1536 ? 8 : 1;
}

static int env_launch(pbn_batch* b, pbn_envcfg* cfg, const int32_t* d_act, int A, int dedup, int offset,
                      uint32_t cap, uint64_t* d_obs, int32_t* d_rew, uint8_t* d_flags, uint32_t* d_nup, int replay,
                      const void* d_off, const void* d_di, const void* d_dk, uint32_t n_calls = 1) {
    const pbn_envcfg::Dev* dv = cfg->on(b->device);
    if (!dv) return fail(PBN_E_NOMEM, "envcfg upload failed");
    // cooperative draw generation: predictor mix, Philox, record index fits the u16 entry
    int mode = (cfg->fast && !replay && b->net->kind == KIND_PREDICTOR_MIX && cfg->L.pmax <= 16 &&
                b->net->N <= 512 && !b->env_no_gen)
                   ? 2
                   : cfg->fast;
    // cooperative-draw mode keeps 16-B env records in LDS where the 8-B predictor records were
    // (pbn_device.hpp env_record): the tables after them move up by erec_shift. Whether they fit is
    // decided first, so that the group-size rule below knows whether the tail kernel (mode 4) applies
    uint32_t erec_shift = 0;
    bool erec_fits = false;
    if (mode == 2) {
        // rows of rs records (thr32_layout: tp4 + 1 slots at least, for the saturated choice)
        const uint32_t tp4 = (cfg->L.tp + 3u) & ~3u;
        const uint32_t nrec = (uint32_t)b->net->N * std::max(tp4 + 1u, cfg->L.pmax);
        erec_shift = cfg->L.off_rec + 16u * nrec - cfg->off_cubes;
        erec_fits = nrec <= 65535u &&
                    env_lds_bytes(b->W, cfg->L.bytes + erec_shift, 2, 1, 0, ENV_CHUNK_SMALL) <= ENV_LDS_MAX;
    }
    // group mode (k_env_grp: G lanes per env, G updates per round trip; its rows need no env records)
    int grp = 1;
    if (mode == 2 && b->net->N <= 256) {
        grp = b->env_group ? b->env_group : env_group_size(b, erec_fits && cfg->H <= 4);
        if (grp != 2 && grp != 4 && grp != 8) grp = 1;
        if (grp > 1) mode = 3;
    }
    if (mode == 2) {
        if (!erec_fits)
            mode = cfg->fast;  // too large for the u16 record index / one workgroup's LDS
        else if (cfg->H <= 4)
            mode = 4;  // the same kernel with one packed counter word (<= 4 cubes)
        // mode 4 adds the workgroup hand-off control words: re-check the fit with the final mode
        if (mode == 4 && env_lds_bytes(b->W, cfg->L.bytes + erec_shift, 4, 1, 0, ENV_CHUNK_SMALL) > ENV_LDS_MAX)
            mode = cfg->fast;
    }
    if (mode != 2 && mode != 4) erec_shift = 0;
    const void* gen_img = nullptr;
    // PBNSIM_ENV_KERNEL_IMAGE=1: the kernel builds its LDS image itself (tests keep that path covered)
    if ((mode == 2 || mode == 4) && (cfg->L.bytes + erec_shift) % 16u == 0u && !b->env_kernel_image) {
        std::lock_guard<std::mutex> g(cfg->mu);
        if (cfg->gen_image.empty()) cfg->gen_image = env_gen_image(cfg, erec_shift);
        auto& d = cfg->dev[b->device];  // on() above created it
        if (!d.gen_image) {
            HIP_TRY(hipMalloc(&d.gen_image, cfg->gen_image.size()));
            HIP_TRY(hipMemcpy(d.gen_image, cfg->gen_image.data(), cfg->gen_image.size(), hipMemcpyHostToDevice));
        }
        gen_img = d.gen_image;
    }
    int bpc = 1;
    uint32_t chunk = ENV_CHUNK_SMALL;
    if (mode == 2 || mode == 4) {
        // the draw-round chunk (pbn_params.hpp ENV_CHUNK_SMALL / _LARGE): the large one unless the small
        // one's draw buffers let more workgroups onto a CU and the launch is a throughput-bound fused run
        // (>= 16 env steps per env over a queue of >= 4 envs per lane of the large one's grid), or the large
        // one does not fit one workgroup's 64 KiB; PBNSIM_ENV_CHUNK=32 / 48 overrides
        int bpc_s = 1, bpc_l = 1;
        const uint32_t img = cfg->L.bytes + erec_shift;
        if (int e = max_blocks_env(b->W, b->net->kind, mode, grp, img, &bpc_s, b->net->N, ENV_CHUNK_SMALL))
            return fail(PBN_E_HIP, "occupancy query: %s", hipGetErrorString((hipError_t)e));
        const bool large_fits = env_lds_bytes(b->W, img, mode, 1, 0, ENV_CHUNK_LARGE) <= ENV_LDS_MAX;
        if (large_fits)
            if (int e = max_blocks_env(b->W, b->net->kind, mode, grp, img, &bpc_l, b->net->N, ENV_CHUNK_LARGE))
                return fail(PBN_E_HIP, "occupancy query: %s", hipGetErrorString((hipError_t)e));
        const uint64_t lanes_l = (uint64_t)b->n_cu * (uint64_t)bpc_l * ENV_BLOCK;
        const bool throughput = n_calls >= 16u && b->B >= 4u * lanes_l && bpc_s > bpc_l;
        chunk = large_fits && !throughput ? ENV_CHUNK_LARGE : ENV_CHUNK_SMALL;
        if (b->env_chunk == (int)ENV_CHUNK_SMALL || (b->env_chunk == (int)ENV_CHUNK_LARGE && large_fits))
            chunk = (uint32_t)b->env_chunk;
        bpc = chunk == ENV_CHUNK_LARGE ? bpc_l : bpc_s;
    } else if (int e = max_blocks_env(b->W, b->net->kind, mode, grp, cfg->L.bytes + erec_shift, &bpc, b->net->N)) {
        return fail(PBN_E_HIP, "occupancy query: %s", hipGetErrorString((hipError_t)e));
    }
    if (b->env_bpc) bpc = std::min(bpc, b->env_bpc);
    EnvArgs a{};
    a.state = b->d_state;
    a.n_steps = b->d_nsteps;
    a.actions = d_act;
    a.obs = d_obs;
    a.reward = d_rew;
    a.flags = d_flags;
    a.n_updates = d_nup;
    a.error = b->d_error;
    a.img = dv->image;
    a.gen_img = gen_img;
    a.L = cfg->L;
    a.off_cubes = cfg->off_cubes + erec_shift;
    a.off_target = cfg->off_target + erec_shift;
    a.off_ndelta = cfg->off_ndelta + erec_shift;
    a.erec_shift = erec_shift;
    a.tail_max = b->env_tail >= 0 ? (uint32_t)b->env_tail : ENV_TAIL_DEFAULT;
    // tail-mode kernel: small batches (ENV_ONE_LANE_ENVS_PER_SLOT envs per wave slot) take one env per
    // wave at a time -- every wave resolves its env 64 updates per block and takes the next from the
    // queue when it is done (PBNSIM_ENV_LANES overrides; 64 = lane mode, the tail at the end)
    a.lane_limit = 64u;
    if (mode == 4) {
        const uint64_t slots = (uint64_t)b->n_cu * (uint64_t)bpc * (ENV_BLOCK / 64);
        if (b->env_lane_limit > 0)
            a.lane_limit = (uint32_t)b->env_lane_limit;
        else if (a.tail_max >= 1 && b->B <= ENV_ONE_LANE_ENVS_PER_SLOT * slots)
            a.lane_limit = 1u;
    }
    a.fast = mode;
    a.grp = grp;
    a.chunk = chunk;
    a.off_gen = mode == 3 ? cfg->L.bytes : cfg->L.bytes + erec_shift + 8u * (uint32_t)b->W * ENV_BLOCK;
    if (int rc = b->s_counter.ensure(8)) return rc;
    a.counter = (unsigned long long*)b->s_counter.p;
    a.n_cubes = cfg->H;
    a.B = b->B;
    a.env_base = b->env_base;
    a.seed = b->seed;
    a.call_idx = b->env_calls;
    a.update_cap = cap;
    a.A = A;
    a.offset = offset;
    a.dedup = dedup ? 1 : 0;
    a.horizon = cfg->horizon;
    a.reward_success = cfg->reward_success;
    a.action_cost = cfg->action_cost;
    a.first_tested = cfg->first_tested;
    a.n_calls = n_calls;
    a.draw_off = (const int64_t*)d_off;
    a.draws_i = (const uint32_t*)d_di;
    a.draws_k = (const uint64_t*)d_dk;
    HIP_TRY(hipMemsetAsync(b->d_error, 0, 4, b->stream));
    HIP_TRY(hipMemsetAsync(b->s_counter.p, 0, 8, b->stream));
    // lanes per env (group mode) or, with a lane limit, 64 / limit lane slots per env
    int grid = b->grid_for(a.lane_limit < 64u ? (b->B * 64u + a.lane_limit - 1u) / a.lane_limit : b->B * (uint64_t)grp, bpc,
                           env_block(mode));
    // PBNSIM_ENV_GRID: exactly that many workgroups (at most the resident count; persistent waves: any grid
    // drains the counter, and surplus workgroups find the queue empty)
    if (b->env_grid_cap) grid = std::min(b->env_grid_cap, b->n_cu * bpc);
    // tail hand-off (k_env mode 4): a wave holding several envs in tail mode passes envs it has not
    // started on to idle waves of its workgroup (LDS). One lane per wave taking envs (small batches)
    // never holds two: off there
    b->steal_last = false;
    if (mode == 4 && b->env_steal && a.tail_max >= 1u && a.lane_limit >= 2u) {
        if (int rc = b->s_steal.ensure(16)) return rc;
        HIP_TRY(hipMemsetAsync(b->s_steal.p, 0, 16, b->stream));
        a.steal_local = 1;
        // [0] envs handed off, [1] tail helpers recruited, [2] tail blocks read from helper rings, [3] of those,
        // the ones whose helper had not written them when the session reached them
        a.steal_count = (uint32_t*)b->s_steal.p;
        a.tail_helpers = b->env_helpers;
        b->steal_last = true;
        // grid pool: control words (GPOOL_CTL_BYTES, zeroed per launch), then the slots' state words, then the slots
        b->gpool_last = false;
        if (b->env_grid_steal > 0 || (b->env_grid_steal < 0 && (cap >= GPOOL_MIN_CAP || n_calls > 1u))) {
            const size_t st_bytes = 4 * (size_t)GPOOL_CAP, sl_bytes = 8 * (size_t)GPOOL_GRANULES * GPOOL_CAP;
            if (int rc = b->s_gpool.ensure(GPOOL_CTL_BYTES + st_bytes + sl_bytes)) return rc;
            HIP_TRY(hipMemsetAsync(b->s_gpool.p, 0, GPOOL_CTL_BYTES, b->stream));
            uint8_t* base = static_cast<uint8_t*>(b->s_gpool.p);
            // epochs 1 .. 2^30 - 1: slot words of earlier launches never match; the whole pool is zeroed at its
            // first use and when the epoch wraps
            if (b->gpool_epoch == 0u || b->gpool_epoch >= 0x3FFFFFFEu)
                HIP_TRY(hipMemsetAsync(base, 0, GPOOL_CTL_BYTES + st_bytes + sl_bytes, b->stream));
            b->gpool_epoch = b->gpool_epoch % 0x3FFFFFFEu + 1u;
            a.gpool_ctl = reinterpret_cast<uint32_t*>(base);
            a.gpool_state = reinterpret_cast<uint32_t*>(base + GPOOL_CTL_BYTES);
            a.gpool = reinterpret_cast<uint64_t*>(base + GPOOL_CTL_BYTES + st_bytes);
            a.gpool_cap = b->env_grid_slots > 0 ? (uint32_t)b->env_grid_slots : GPOOL_CAP;
            a.gpool_epoch = b->gpool_epoch;
            a.gpool_cu_idle = b->env_pool_cu_idle != 0 ? 1u : 0u;
            b->gpool_last = true;
            if (d_obs != b->s_obs.p) b->fault_check = true;  // device path: pbn_sync reads the sticky fault word
        }
    }
    hipEvent_t stop;
    if (int rc = b->ev_begin(&stop)) return rc;
    int e = launch_env_multi(b->W, a, replay, grid, b->stream);
    if (e) return fail(PBN_E_HIP, "k_env launch: %s", hipGetErrorString((hipError_t)e));
    if (int rc = b->ev_end(stop)) return rc;
    if (!replay) b->env_calls += n_calls;
    b->env_lanes = grp;
    b->env_grid_last = grid;
    b->env_lane_limit_last = (int)a.lane_limit;
    b->env_chunk_last = (a.fast == 2 || a.fast == 4) ? (int)a.chunk : 0;
    b->env_kernel_last = replay ? std::min(mode, 1) : mode;
    return 0;
}

static int env_host_common(pbn_batch* b, pbn_envcfg* cfg, const int32_t* actions, int A, int offset) {
    if (cfg->net != b->net) return fail(PBN_E_INVALID, "envcfg belongs to another network");
    if (int rc = validate_actions(b, actions, A, offset)) return rc;
    size_t ab = 4 * (size_t)A * b->B;
    if (int rc = b->s_act.ensure(ab)) return rc;
    if (int rc = b->s_obs.ensure(8 * (size_t)b->W * b->B)) return rc;
    if (int rc = b->s_rew.ensure(4 * b->B)) return rc;
    if (int rc = b->s_flags.ensure(b->B)) return rc;
    if (int rc = b->s_nup.ensure(4 * b->B)) return rc;
    return h2d(b, b->s_act.p, actions, ab);
}

static int env_host_out(pbn_batch* b, uint64_t* obs, int32_t* reward, uint8_t* flags, uint32_t* n_updates) {
    const size_t so = 8 * (size_t)b->W * b->B, sr = 4 * b->B, sf = b->B, sn = 4 * b->B;
    const size_t oo = 0, orr = oo + so, of = orr + sr, on = of + sf, oe = (on + sn + 3) & ~(size_t)3;
    if (oe + 4 <= PinBuf::CAP && b->pin.ready()) {  // one pinned block, one sync
        uint8_t* q = b->pin.p;
        HIP_TRY(hipMemcpyAsync(q + oo, b->s_obs.p, so, hipMemcpyDeviceToHost, b->stream));
        HIP_TRY(hipMemcpyAsync(q + orr, b->s_rew.p, sr, hipMemcpyDeviceToHost, b->stream));
        HIP_TRY(hipMemcpyAsync(q + of, b->s_flags.p, sf, hipMemcpyDeviceToHost, b->stream));
        HIP_TRY(hipMemcpyAsync(q + on, b->s_nup.p, sn, hipMemcpyDeviceToHost, b->stream));
        HIP_TRY(hipMemcpyAsync(q + oe, b->d_error, 4, hipMemcpyDeviceToHost, b->stream));
        HIP_TRY(hipStreamSynchronize(b->stream));
        if (obs) memcpy(obs, q + oo, so);
        if (reward) memcpy(reward, q + orr, sr);
        if (flags) memcpy(flags, q + of, sf);
        if (n_updates) memcpy(n_updates, q + on, sn);
        int32_t err;
        memcpy(&err, q + oe, 4);
        if (err & 2) return fail(PBN_E_HIP, "k_env grid pool: a wait timed out");
        if (err) return fail(PBN_E_RANGE, "an action was out of range");
        return 0;
    }
    if (obs) HIP_TRY(hipMemcpyAsync(obs, b->s_obs.p, 8 * (size_t)b->W * b->B, hipMemcpyDeviceToHost, b->stream));
    if (reward) HIP_TRY(hipMemcpyAsync(reward, b->s_rew.p, 4 * b->B, hipMemcpyDeviceToHost, b->stream));
    if (flags) HIP_TRY(hipMemcpyAsync(flags, b->s_flags.p, b->B, hipMemcpyDeviceToHost, b->stream));
    if (n_updates) HIP_TRY(hipMemcpyAsync(n_updates, b->s_nup.p, 4 * b->B, hipMemcpyDeviceToHost, b->stream));
    int32_t err = 0;
    HIP_TRY(hipMemcpyAsync(&err, b->d_error, 4, hipMemcpyDeviceToHost, b->stream));
    HIP_TRY(hipStreamSynchronize(b->stream));
    if (err & 2) return fail(PBN_E_HIP, "k_env grid pool: a wait timed out");
    if (err) return fail(PBN_E_RANGE, "an action was out of range");
    return 0;
}

int pbn_env_step_multi(pbn_batch* b, const pbn_envcfg* cfg_c, const int32_t* actions, int A, int dedup, int offset,
                       uint32_t update_cap, uint64_t* obs, int32_t* reward, uint8_t* flags, uint32_t* n_updates) {
    CHECK_NN(b, "batch");
    CHECK_NN(cfg_c, "cfg");
    CHECK_NN(actions, "actions");
    pbn_envcfg* cfg = const_cast<pbn_envcfg*>(cfg_c);
    SET_DEV(b);
    if (int rc = env_host_common(b, cfg, actions, A, offset)) return rc;
    if (int rc = env_launch(b, cfg, (const int32_t*)b->s_act.p, A, dedup, offset, update_cap, (uint64_t*)b->s_obs.p,
                            (int32_t*)b->s_rew.p, (uint8_t*)b->s_flags.p, (uint32_t*)b->s_nup.p, 0, nullptr, nullptr,
                            nullptr))
        return rc;
    return env_host_out(b, obs, reward, flags, n_updates);
}

int pbn_env_step_multi_device(pbn_batch* b, const pbn_envcfg* cfg_c, const int32_t* d_actions, int A, int dedup,
                              int offset, uint32_t update_cap, uint64_t* d_obs, int32_t* d_reward, uint8_t* d_flags,
                              uint32_t* d_n_updates) {
    CHECK_NN(b, "batch");
    CHECK_NN(cfg_c, "cfg");
    CHECK_NN(d_actions, "d_actions");
    CHECK_NN(d_obs, "d_obs");
    CHECK_NN(d_reward, "d_reward");
    CHECK_NN(d_flags, "d_flags");
    CHECK_NN(d_n_updates, "d_n_updates");
    pbn_envcfg* cfg = const_cast<pbn_envcfg*>(cfg_c);
    if (cfg->net != b->net) return fail(PBN_E_INVALID, "envcfg belongs to another network");
    if (A < 1 || A > 4096) return fail(PBN_E_INVALID, "A=%d outside [1, 4096]", A);
    if (offset != 0 && offset != 1) return fail(PBN_E_INVALID, "offset must be 0 or 1");
    SET_DEV(b);
    return env_launch(b, cfg, d_actions, A, dedup, offset, update_cap, d_obs, d_reward, d_flags, d_n_updates, 0,
                      nullptr, nullptr, nullptr);
}

int pbn_env_rollout_multi_device(pbn_batch* b, const pbn_envcfg* cfg_c, uint32_t n_steps, const int32_t* d_actions,
                                 int A, int dedup, int offset, uint32_t update_cap, uint64_t* d_obs, int32_t* d_reward,
                                 uint8_t* d_flags, uint32_t* d_n_updates) {
    CHECK_NN(b, "batch");
    CHECK_NN(cfg_c, "cfg");
    CHECK_NN(d_actions, "d_actions");
    CHECK_NN(d_obs, "d_obs");
    CHECK_NN(d_reward, "d_reward");
    CHECK_NN(d_flags, "d_flags");
    CHECK_NN(d_n_updates, "d_n_updates");
    pbn_envcfg* cfg = const_cast<pbn_envcfg*>(cfg_c);
    if (cfg->net != b->net) return fail(PBN_E_INVALID, "envcfg belongs to another network");
    if (A < 1 || A > 4096) return fail(PBN_E_INVALID, "A=%d outside [1, 4096]", A);
    if (offset != 0 && offset != 1) return fail(PBN_E_INVALID, "offset must be 0 or 1");
    if (n_steps < 1 || n_steps > (1u << 20)) return fail(PBN_E_INVALID, "n_steps=%u outside [1, 2^20]", n_steps);
    SET_DEV(b);
    return env_launch(b, cfg, d_actions, A, dedup, offset, update_cap, d_obs, d_reward, d_flags, d_n_updates, 0,
                      nullptr, nullptr, nullptr, n_steps);
}

int pbn_env_step_multi_replay(pbn_batch* b, const pbn_envcfg* cfg_c, const int32_t* actions, int A, int dedup,
                              int offset, const int64_t* draw_offsets, const uint32_t* draws_i,
                              const uint64_t* draws_k, uint64_t* obs, int32_t* reward, uint8_t* flags,
                              uint32_t* n_updates) {
    CHECK_NN(b, "batch");
    CHECK_NN(cfg_c, "cfg");
    CHECK_NN(actions, "actions");
    CHECK_NN(draw_offsets, "draw_offsets");
    pbn_envcfg* cfg = const_cast<pbn_envcfg*>(cfg_c);
    const int64_t nd = draw_offsets[b->B];
    if (draw_offsets[0] != 0 || nd < 0) return fail(PBN_E_INVALID, "draw_offsets must start at 0");
    for (uint64_t e = 0; e < b->B; e++)
        if (draw_offsets[e + 1] < draw_offsets[e]) return fail(PBN_E_INVALID, "draw_offsets not non-decreasing");
    const uint32_t lo = b->net->kind == PBN_KIND_PROB_TABLE ? 1u : 0u;
    for (int64_t q = 0; q < nd; q++)
        if (draws_i[q] >= (uint32_t)b->N || draws_i[q] < lo || (draws_k[q] >> 53))
            return fail(PBN_E_RANGE, "replay draw %lld out of range", (long long)q);
    SET_DEV(b);
    if (int rc = env_host_common(b, cfg, actions, A, offset)) return rc;
    if (int rc = b->s_off.ensure(8 * (b->B + 1))) return rc;
    if (int rc = b->s_replay_i.ensure(4 * (size_t)std::max<int64_t>(nd, 1))) return rc;
    if (int rc = b->s_replay_k.ensure(8 * (size_t)std::max<int64_t>(nd, 1))) return rc;
    HIP_TRY(hipMemcpyAsync(b->s_off.p, draw_offsets, 8 * (b->B + 1), hipMemcpyHostToDevice, b->stream));
    if (nd) {
        HIP_TRY(hipMemcpyAsync(b->s_replay_i.p, draws_i, 4 * (size_t)nd, hipMemcpyHostToDevice, b->stream));
        HIP_TRY(hipMemcpyAsync(b->s_replay_k.p, draws_k, 8 * (size_t)nd, hipMemcpyHostToDevice, b->stream));
    }
    if (int rc = env_launch(b, cfg, (const int32_t*)b->s_act.p, A, dedup, offset, 0xFFFFFFFFu, (uint64_t*)b->s_obs.p,
                            (int32_t*)b->s_rew.p, (uint8_t*)b->s_flags.p, (uint32_t*)b->s_nup.p, 1, b->s_off.p,
                            b->s_replay_i.p, b->s_replay_k.p))
        return rc;
    return env_host_out(b, obs, reward, flags, n_updates);
}

// ------------------------------------------------------------------ timing
// Region timing: the stop event is recorded on the stream now, right behind the last launch.
static int close_region(pbn_batch* b) {
    b->region_end = nullptr;
    if (!b->region_launches) return 0;
    if (b->ev_pool.empty()) return fail(PBN_E_HIP, "timing region without events");
    HIP_TRY(hipEventRecord(b->ev_pool[0].second, b->stream));
    b->region_end = b->ev_pool[0].second;
    return 0;
}

int pbn_timing_enable(pbn_batch* b, int enable) {
    CHECK_NN(b, "batch");
    if (enable < 0 || enable > 2) return fail(PBN_E_INVALID, "timing mode must be 0, 1 or 2");
    if (b->timing == 2 && enable != 2) {
        // close the open region right behind the last launch; pbn_timing_read reports it
        if (int rc = close_region(b)) return rc;
        b->region_closed = true;
        b->timing = enable;
        return 0;
    }
    if (enable == 2 && b->ev_pool.empty()) {
        // create the region's event pair now, not at its first launch (inside a timed window)
        SET_DEV(b);
        hipEvent_t e0, e1;
        HIP_TRY(hipEventCreate(&e0));
        HIP_TRY(hipEventCreate(&e1));
        b->ev_pool.emplace_back(e0, e1);
    }
    b->timing = enable;
    b->ev_used = 0;
    b->region_launches = 0;
    b->region_closed = false;
    b->region_start = b->region_end = nullptr;
    return 0;
}

int pbn_env_handoffs(pbn_batch* b, uint32_t* count) {
    CHECK_NN(b, "batch");
    CHECK_NN(count, "count");
    SET_DEV(b);
    *count = 0;
    if (!b->steal_last) return 0;
    HIP_TRY(hipStreamSynchronize(b->stream));
    HIP_TRY(hipMemcpy(count, b->s_steal.p, 4, hipMemcpyDeviceToHost));
    return 0;
}

int pbn_env_tail_stats(pbn_batch* b, uint32_t* stats) {
    CHECK_NN(b, "batch");
    CHECK_NN(stats, "stats");
    SET_DEV(b);
    for (int k = 0; k < 4; k++) stats[k] = 0;
    if (!b->steal_last) return 0;
    HIP_TRY(hipStreamSynchronize(b->stream));
    HIP_TRY(hipMemcpy(stats, b->s_steal.p, 16, hipMemcpyDeviceToHost));
    return 0;
}

int pbn_env_grid_stats(pbn_batch* b, uint32_t* stats) {
    CHECK_NN(b, "batch");
    CHECK_NN(stats, "stats");
    SET_DEV(b);
    for (int k = 0; k < 4; k++) stats[k] = 0;
    if (!b->gpool_last) return 0;
    HIP_TRY(hipStreamSynchronize(b->stream));
    uint32_t ctl[6];
    HIP_TRY(hipMemcpy(ctl, b->s_gpool.p, sizeof ctl, hipMemcpyDeviceToHost));
    stats[0] = ctl[3];  // envs pushed
    stats[1] = ctl[1];  // tickets taken
    stats[2] = ctl[4];  // waits given up
    stats[3] = ctl[2];  // live count at the end (0 after a complete launch)
    return 0;
}

int pbn_env_tail_helpers(pbn_batch* b, uint32_t* count) {
    CHECK_NN(b, "batch");
    CHECK_NN(count, "count");
    SET_DEV(b);
    *count = 0;
    if (!b->steal_last) return 0;
    HIP_TRY(hipStreamSynchronize(b->stream));
    HIP_TRY(hipMemcpy(count, (const uint32_t*)b->s_steal.p + 1, 4, hipMemcpyDeviceToHost));
    return 0;
}

int pbn_timing_read_each(pbn_batch* b, double* ms_each, uint64_t cap, uint64_t* launches) {
    CHECK_NN(b, "batch");
    if (b->timing == 2 || b->region_closed) return fail(PBN_E_INVALID, "per-launch times need timing mode 1");
    SET_DEV(b);
    HIP_TRY(hipStreamSynchronize(b->stream));
    for (size_t k = 0; k < b->ev_used && k < cap; k++) {
        float ms = 0;
        HIP_TRY(hipEventElapsedTime(&ms, b->ev_pool[k].first, b->ev_pool[k].second));
        if (ms_each) ms_each[k] = ms;
    }
    if (launches) *launches = b->ev_used;
    b->ev_used = 0;
    return 0;
}

int pbn_timing_read(pbn_batch* b, double* kernel_ms, uint64_t* launches) {
    CHECK_NN(b, "batch");
    SET_DEV(b);
    const bool region = b->timing == 2 || b->region_closed;
    if (b->timing == 2)
        if (int rc = close_region(b)) return rc;
    HIP_TRY(hipStreamSynchronize(b->stream));
    double tot = 0;
    if (region) {
        float ms = 0;
        if (b->region_launches) HIP_TRY(hipEventElapsedTime(&ms, b->region_start, b->region_end));
        tot = ms;
    } else {
        for (size_t k = 0; k < b->ev_used; k++) {
            float ms = 0;
            HIP_TRY(hipEventElapsedTime(&ms, b->ev_pool[k].first, b->ev_pool[k].second));
            tot += ms;
        }
    }
    if (kernel_ms) *kernel_ms = tot;
    if (launches) *launches = region ? b->region_launches : b->ev_used;
    b->ev_used = 0;
    b->region_launches = 0;
    b->region_closed = false;
    b->region_start = b->region_end = nullptr;
    return 0;
}

}  // extern "C"
