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
// row's read position. A lane's successive words share cache lines; the twist is run
// by the lane itself when its position reaches 624 (sequential in-place MT19937).
#include <hip/hip_runtime.h>

#include "pbn_device.hpp"
#include "pbn_params.hpp"

namespace pbn {

constexpr uint32_t MT_N = 624, MT_M = 397;

__device__ __forceinline__ uint32_t mt_temper(uint32_t y) {
    y ^= (y >> 11);
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= (y >> 18);
    return y;
}

__device__ void mt_twist(uint32_t* __restrict__ mt) {
    uint32_t cur = mt[0];
    for (uint32_t kk = 0; kk < MT_N; ++kk) {
        const uint32_t nxt = mt[kk + 1 < MT_N ? kk + 1 : 0];  // mt[0] is already new when kk == 623
        const uint32_t y = (cur & 0x80000000u) | (nxt & 0x7fffffffu);
        const uint32_t src = mt[kk + MT_M < MT_N ? kk + MT_M : kk + MT_M - MT_N];
        mt[kk] = src ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
        cur = nxt;
    }
}

struct MTStream {
    uint32_t* row;
    uint32_t pos;
    __device__ __forceinline__ uint32_t next() {
        if (pos >= MT_N) {
            mt_twist(row);
            pos = 0;
        }
        return mt_temper(row[pos++]);
    }
    // random.Random._randbelow_with_getrandbits(n), 1 <= n < 2^32 (CPython 3.10)
    __device__ __forceinline__ uint32_t randbelow(uint32_t n, uint32_t kshift) {
        uint32_t r = next() >> kshift;
        while (r >= n) r = next() >> kshift;
        return r;
    }
    __device__ __forceinline__ uint64_t k53() {
        const uint32_t a = next(), b = next();
        return k53_of(a, b);
    }
};

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

// Seed every env's generators; optionally run Graph.genRandState (base.py:368-370:
// N x randint(0, 1)) or PBN.reset(None) (pbn.py:105-118: np.random.rand(N) > 0.5; state[0] = 0).
template <int W, int KIND>
__global__ __launch_bounds__(BLOCK) void k_mt_seed(MTArgs a) {
    const uint64_t e = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
    if (e >= a.B) return;
    const uint64_t s = a.seeds[e];
    uint32_t* py = a.mt_py + e * MT_ROW;
    mt_seed_python(py, s);
    a.pos_py[e] = MT_N;
    uint32_t* np_row = nullptr;
    if constexpr (KIND == KIND_PROB_TABLE) {
        np_row = a.mt_np + e * MT_ROW;
        mt_init_genrand(np_row, (uint32_t)s);
        a.pos_np[e] = MT_N;
    }
    if (!a.init_state) return;
    uint64_t st[W];
#pragma unroll
    for (int k = 0; k < W; ++k) st[k] = 0;
    const uint32_t N = (uint32_t)a.n_nodes;
    if constexpr (KIND == KIND_PREDICTOR_MIX) {
        MTStream r{py, MT_N};
        for (uint32_t i = 0; i < N; ++i) setbit<W>(st, i, r.randbelow(2u, kshift_of(2u)));
        a.pos_py[e] = r.pos;
    } else {
        MTStream r{np_row, MT_N};
        for (uint32_t i = 0; i < N; ++i) setbit<W>(st, i, r.k53() > (1ull << 52) ? 1u : 0u);
        setbit<W>(st, 0u, 0u);
        a.pos_np[e] = r.pos;
    }
    store_state<W>(a.state + e * W, st);
}

// T reference transitions per env from its own generators:
//   Bittner Graph.step (base.py:306-312): i = randint(0, N-1); r = random() * CODsum
//   PBN.step (pbn.py:129-133): i = randint(1, N-1) [stdlib]; u = np.random.uniform() [numpy]
template <int W, int KIND>
__global__ __launch_bounds__(BLOCK) void k_mt_step(MTArgs a) {
    extern __shared__ __align__(16) uint8_t lds[];
    stage_image(reinterpret_cast<const uint4*>(a.img), a.L.bytes / 16, reinterpret_cast<uint4*>(lds));
    __syncthreads();
    const Plane P{reinterpret_cast<uint32_t*>(lds + a.L.bytes) + threadIdx.x};
    const uint32_t N = (uint32_t)a.L.n_nodes;
    const uint64_t stride = (uint64_t)gridDim.x * BLOCK;
    for (uint64_t e = (uint64_t)blockIdx.x * BLOCK + threadIdx.x; e < a.B; e += stride) {
        uint64_t st[W];
        load_state<W>(a.state + e * W, st);
        to_plane<W>(P, st);
        MTStream py{a.mt_py + e * MT_ROW, a.pos_py[e]};
        if constexpr (KIND == KIND_PREDICTOR_MIX) {
            const uint32_t ks = kshift_of(N);
            for (uint32_t t = 0; t < a.T; ++t) {
                const uint32_t i = py.randbelow(N, ks);
                const uint64_t k53 = py.k53();
                predictor_update_lds(P, i, k53, lds, a.L);
            }
        } else {
            MTStream np_{a.mt_np + e * MT_ROW, a.pos_np[e]};
            const uint32_t ks = kshift_of(N - 1);
            for (uint32_t t = 0; t < a.T; ++t) {
                const uint32_t i = 1u + py.randbelow(N - 1, ks);
                const uint64_t k53 = np_.k53();
                table_update_lds(P, i, k53, lds, a.L);
            }
            a.pos_np[e] = np_.pos;
        }
        a.pos_py[e] = py.pos;
        from_plane<W>(P, st);
        store_state<W>(a.state + e * W, st);
    }
}

template <int KIND>
static void* mt_seed_fn(int W) {
    switch (W) {
        case 1: return (void*)k_mt_seed<1, KIND>;
        case 2: return (void*)k_mt_seed<2, KIND>;
        case 3: return (void*)k_mt_seed<3, KIND>;
        case 4: return (void*)k_mt_seed<4, KIND>;
        case 5: return (void*)k_mt_seed<5, KIND>;
        case 6: return (void*)k_mt_seed<6, KIND>;
        case 7: return (void*)k_mt_seed<7, KIND>;
        case 8: return (void*)k_mt_seed<8, KIND>;
    }
    return nullptr;
}

template <int KIND>
static void* mt_step_fn(int W) {
    switch (W) {
        case 1: return (void*)k_mt_step<1, KIND>;
        case 2: return (void*)k_mt_step<2, KIND>;
        case 3: return (void*)k_mt_step<3, KIND>;
        case 4: return (void*)k_mt_step<4, KIND>;
        case 5: return (void*)k_mt_step<5, KIND>;
        case 6: return (void*)k_mt_step<6, KIND>;
        case 7: return (void*)k_mt_step<7, KIND>;
        case 8: return (void*)k_mt_step<8, KIND>;
    }
    return nullptr;
}

int launch_mt_seed(int W, const MTArgs& a, int grid, void* stream) {
    void* fn = a.L.kind == KIND_PREDICTOR_MIX ? mt_seed_fn<KIND_PREDICTOR_MIX>(W) : mt_seed_fn<KIND_PROB_TABLE>(W);
    if (!fn) return (int)hipErrorInvalidValue;
    MTArgs c = a;
    void* kargs[] = {&c};
    return (int)hipLaunchKernel(fn, dim3((unsigned)grid), dim3(BLOCK), kargs, 0, (hipStream_t)stream);
}

int launch_mt_step(int W, const MTArgs& a, int grid, void* stream) {
    void* fn = a.L.kind == KIND_PREDICTOR_MIX ? mt_step_fn<KIND_PREDICTOR_MIX>(W) : mt_step_fn<KIND_PROB_TABLE>(W);
    if (!fn) return (int)hipErrorInvalidValue;
    MTArgs c = a;
    void* kargs[] = {&c};
    return (int)hipLaunchKernel(fn, dim3((unsigned)grid), dim3(BLOCK), kargs, step_lds_bytes(W, a.L.bytes, BLOCK),
                                (hipStream_t)stream);
}

}  // namespace pbn
