// mall_probe.hip -- memory ceiling of the step-mode access pattern (measurement only, not product).
//
// The bench kernel (k_step, Bittner-200 at 1M envs) reads every env's 32-B state and writes
// it back; at 1M envs the 32 MiB state stays in the 256 MiB Infinity Cache (MALL) between
// launches, so its ceiling is the MALL's, for which MI355X_MICROARCH.md gives no streaming
// figure. This probe measures it on the box: the same envs (32 B each, two 16-B loads per
// env, pairs (e, e + stride) per thread, 1024-thread groups, 2 groups per CU), no compute,
// P passes inside ONE launch so the launch-to-launch gap is not charged. Pass p works on
// envs rotated by p * 1024 so a workgroup's envs of pass p were another XCD's in pass p - 1
// (its own L2 does not hold them: the rate is the MALL's, not the L2's).
//
// Built by __graft_entry__.build() into tools/libmallprobe.so; bench.py loads it via ctypes.
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace {

__global__ __launch_bounds__(1024) void k_probe(uint64_t* __restrict__ s, uint64_t B, uint32_t write_pct,
                                                uint32_t passes, uint64_t* __restrict__ sink, uint32_t salt,
                                                uint32_t glog, uint32_t wbytes) {
    const uint64_t stride = (uint64_t)gridDim.x * 1024u;
    uint64_t acc = 0;
    for (uint32_t p = 0; p < passes; ++p) {
        const uint64_t rot = ((uint64_t)p * 1024u) % B;
        for (uint64_t e0 = (uint64_t)blockIdx.x * 1024u + threadIdx.x; e0 < B; e0 += 2 * stride) {
            uint64_t ea = e0 + rot, eb = e0 + stride + rot;
            ea -= ea >= B ? B : 0;
            eb -= eb >= B ? B : 0;
            const bool hb = e0 + stride < B;
            ulonglong2* qa = reinterpret_cast<ulonglong2*>(s + 4 * ea);
            ulonglong2* qb = reinterpret_cast<ulonglong2*>(s + 4 * eb);
            ulonglong2 a0 = qa[0], a1 = qa[1], b0, b1;
            if (hb) {
                b0 = qb[0];
                b1 = qb[1];
            }
            acc ^= a0.x ^ a1.y;
            // a fixed subset of envs is written (write_pct %), as the dirty-store kernel writes
            // the envs whose updated bit changed
            // wbytes: 32 = the whole env (the kernel's store), 16 = the half holding the changed word,
            // 8 = only the changed word (word index from the env id, as the updated node's word varies)
            auto wr = [&](ulonglong2* q, uint64_t e, const ulonglong2& v0, const ulonglong2& v1) {
                if (wbytes >= 32u) {  // the kernel's store (the default, what bench.py's floor uses)
                    q[0] = v0;
                    q[1] = v1;
                    return;
                }
                const uint32_t wsel = (uint32_t)(e * 0x9E3779B9u) >> 30;
                if (wbytes == 16u) {
                    if (wsel >> 1)
                        q[1] = v1;
                    else
                        q[0] = v0;
                } else {
                    uint64_t* w = reinterpret_cast<uint64_t*>(q) + wsel;
                    *w = v0.x ^ v1.y;
                }
            };
            if ((uint32_t)((((ea >> glog) ^ salt) * 2654435761u) >> 7) % 100u < write_pct) {
                a0.x += 1;
                wr(qa, ea, a0, a1);
            }
            if (hb) {
                acc ^= b0.x ^ b1.y;
                if ((uint32_t)((((eb >> glog) ^ salt) * 2654435761u) >> 7) % 100u < write_pct) {
                    b0.x += 1;
                    wr(qb, eb, b0, b1);
                }
            }
        }
    }
    if (acc == 0x9E3779B97F4A7C15ull) sink[0] = acc;  // keeps the loads live
}

}  // namespace

// Average time per PASS over the state (microseconds) for n_envs 32-B envs, the given write
// fraction, `passes` passes per launch and `launches` timed launches (after 3 untimed ones).
// Returns 0 on success, a HIP error code otherwise.
static int probe_impl(uint64_t n_envs, int write_pct, int passes, int launches, int vary, int glog,
                      double* us_per_pass, int wbytes = 32) {
    if (!us_per_pass || n_envs < 2048 || passes < 1 || launches < 1) return -1;
    int dev = 0, n_cu = 0;
    if (hipGetDevice(&dev) != hipSuccess) return -2;
    if (hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return -2;
    uint64_t* s = nullptr;
    uint64_t* sink = nullptr;
    hipError_t e = hipMalloc(&s, 32 * n_envs);
    if (e == hipSuccess) e = hipMalloc(&sink, 64);
    if (e == hipSuccess) e = hipMemset(s, 0, 32 * n_envs);
    hipEvent_t t0 = nullptr, t1 = nullptr;
    if (e == hipSuccess) e = hipEventCreate(&t0);
    if (e == hipSuccess) e = hipEventCreate(&t1);
    const uint64_t pairs = (n_envs + 1) / 2;
    const uint64_t want = (pairs + 1023) / 1024;
    const int grid = (int)(want < (uint64_t)n_cu * 2u ? want : (uint64_t)n_cu * 2u);
    if (e == hipSuccess) {
        for (int w = 0; w < 3; ++w) hipLaunchKernelGGL(k_probe, dim3(grid), dim3(1024), 0, 0, s, n_envs,
                                                       (uint32_t)write_pct, (uint32_t)passes, sink,
                                                       vary ? (uint32_t)(w * 0x9E3779B1u) : 0u, (uint32_t)glog,
                                                       (uint32_t)wbytes);
        e = hipEventRecord(t0, 0);
    }
    if (e == hipSuccess) {
        for (int k = 0; k < launches; ++k)
            hipLaunchKernelGGL(k_probe, dim3(grid), dim3(1024), 0, 0, s, n_envs, (uint32_t)write_pct,
                               (uint32_t)passes, sink, vary ? (uint32_t)((k + 3) * 0x9E3779B1u) : 0u,
                               (uint32_t)glog, (uint32_t)wbytes);
        e = hipGetLastError();
    }
    if (e == hipSuccess) e = hipEventRecord(t1, 0);
    if (e == hipSuccess) e = hipEventSynchronize(t1);
    float ms = 0.f;
    if (e == hipSuccess) e = hipEventElapsedTime(&ms, t0, t1);
    if (e == hipSuccess) *us_per_pass = (double)ms * 1e3 / ((double)launches * passes);
    if (t0) (void)hipEventDestroy(t0);
    if (t1) (void)hipEventDestroy(t1);
    if (s) (void)hipFree(s);
    if (sink) (void)hipFree(sink);
    return e == hipSuccess ? 0 : (int)e;
}

extern "C" int mall_probe(uint64_t n_envs, int write_pct, int passes, int launches, double* us_per_pass) {
    return probe_impl(n_envs, write_pct, passes, launches, 0, 0, us_per_pass);
}

// The same with the written subset drawn afresh every launch (as the step kernel's changed envs are).
extern "C" int mall_probe_vary(uint64_t n_envs, int write_pct, int passes, int launches, double* us_per_pass) {
    return probe_impl(n_envs, write_pct, passes, launches, 1, 0, us_per_pass);
}

// Written envs decided per aligned group of 2^glog envs (all or none), drawn afresh per launch.
extern "C" int mall_probe_group(uint64_t n_envs, int write_pct, int glog, int launches, double* us_per_pass) {
    return probe_impl(n_envs, write_pct, 1, launches, 1, glog, us_per_pass);
}

// The vary pattern with only wbytes (8, 16 or 32) of each written env stored.
extern "C" int mall_probe_wbytes(uint64_t n_envs, int write_pct, int wbytes, int launches, double* us_per_pass) {
    if (wbytes != 8 && wbytes != 16 && wbytes != 32) return -1;
    return probe_impl(n_envs, write_pct, 1, launches, 1, 0, us_per_pass, wbytes);
}
