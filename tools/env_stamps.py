"""Phase timeline of the R6 env kernel (k_env, cooperative-draw path) in one per-step launch.

Measurement build only: tools/build_exp.sh stamps -DPBN_STAMPS, run with
PBNSIM_LIB=build_exp/stamps/libpbnsim.so. Workload = bench.py's config-5 supplement, one launch per
env step: Bittner-200, B envs (default 131,072), the r6_bittner199 fixture's attractor cubes, A = 4
action slots (0 w.p. 0.75), update cap 4,096 (argv[2]). A few env steps run first (untimed), then
one launch with the stamps cleared. Per wave (s_memrealtime, 100 MHz, written by k_env): start,
first chunk with < 40 active lanes (shared draw tables), first chunk after a lane found the work queue
empty, first chunk with
<= 32 / 16 / 8 / 2 active lanes, end; chunk counts and active-lane sums (whole wave and tail).

Prints JSON: percentiles (us from the first wave's start) of every phase, the launch span, and the
per-chunk time of the tail (queue empty) from waves' chunk counts. Output of
`python tools/env_stamps.py 131072 4096` -> profiles/r03_r6_env_stamps_131k.json.
"""
import ctypes as C
import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "gym-pbn-stac_amd"))
sys.path.insert(0, str(ROOT / "tests"))
from gym_pbn_amd import _lib  # noqa: E402
from gym_pbn_amd.batch import EnvConfig, Net, PBNBatch, attractors_from_cubes  # noqa: E402
from gym_pbn_amd.network import load_network  # noqa: E402

NS = 40
PHASES = {0: "start", 1: "below_40_active", 2: "queue_empty", 3: "le32_active", 4: "le16_active",
          5: "le8_active", 6: "le2_active", 7: "end"}


def main():
    import torch

    B = int(sys.argv[1]) if len(sys.argv) > 1 else 131072
    CAP = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    lib = _lib.lib
    lib.pbn_exp_env_stamps.argtypes = [C.c_void_p, C.c_size_t]
    z = np.load(ROOT / "tests" / "golden" / "r6_bittner199.npz", allow_pickle=False)
    net = Net(load_network("bittner199"))
    cfg = EnvConfig(net, attractors_from_cubes(z["cube_care"], z["cube_value"], z["cube_attractor"], net.n_nodes),
                    horizon=100)
    dev = torch.device("cuda", 0)
    A, W = 4, net.n_words
    g = torch.Generator(device=dev)
    g.manual_seed(0xAC7)
    T = 4 + reps
    v = torch.randint(1, net.n_nodes + 1, (T, B, A), device=dev, generator=g, dtype=torch.int32)
    acts = (v * (torch.rand((T, B, A), device=dev, generator=g) >= 0.75)).to(torch.int32).contiguous()
    obs = torch.empty((B, W), dtype=torch.int64, device=dev)
    rew = torch.empty(B, dtype=torch.int32, device=dev)
    flg = torch.empty(B, dtype=torch.uint8, device=dev)
    nup = torch.empty(B, dtype=torch.int32, device=dev)
    b = PBNBatch(net, B, seed=0xAC7)
    b.env_reset(cfg)

    def step(t):
        b.env_step_multi_device(cfg, acts[t].data_ptr(), A, obs.data_ptr(), rew.data_ptr(), flg.data_ptr(),
                                nup.data_ptr(), update_cap=CAP)

    for t in range(4):
        step(t)
    b.sync()
    out = {"B": B, "update_cap": CAP, "env_kernel": b.info().get("env_kernel"), "reps": []}
    for r in range(reps):
        assert lib.pbn_exp_stamps_clear() == 0
        b.timing(1)
        step(4 + r)
        b.sync()
        ms, _ = b.timing_read()
        b.timing(0)
        st = np.zeros(16384 * NS, dtype=np.uint64)
        assert lib.pbn_exp_env_stamps(st.ctypes.data, st.nbytes) == 0
        st = st.reshape(-1, NS)
        st = st[st[:, 0] != 0].astype(np.int64)
        t0 = st[:, 0].min()
        res = {"kernel_ms_events": ms, "waves": int(len(st))}
        for k, name in PHASES.items():
            col = st[:, k]
            seen = col != 0
            vv = (col[seen] - t0) / 100.0  # 100 MHz ticks -> us
            res[name] = {"waves_reaching": int(seen.sum())}
            if seen.any():
                res[name].update({f"p{q}": round(float(np.percentile(vv, q)), 1) for q in (0, 10, 50, 90, 100)})
        n_up = nup.cpu().numpy()
        res["n_updates"] = {"mean": float(n_up.mean()), "max": int(n_up.max()),
                            "capped_frac": float((n_up >= CAP).mean())}
        tail = st[:, 10] > 0
        span = (st[:, 7] - st[:, 2]) / 100.0
        res["tail"] = {"waves_with_tail": int(tail.sum()),
                       "chunks_p50": float(np.median(st[tail, 10])) if tail.any() else None,
                       "mean_active_lanes_p50": float(np.median(st[tail, 11] / st[tail, 10])) if tail.any() else None,
                       "us_per_chunk_p50": float(np.median(span[tail] / st[tail, 10])) if tail.any() else None}
        # the launch ends with its slowest waves: their end time against the capped env steps they held
        ncap = st[:, 14]
        endt = (st[:, 7] - t0) / 100.0
        res["end_us_by_capped_envs"] = {int(k): round(float(np.median(endt[ncap == k])), 1)
                                        for k in np.unique(ncap) if (ncap == k).sum() >= 8}
        res["capped_envs_per_wave"] = {q: float(np.percentile(ncap, q)) for q in (10, 50, 90, 100)}
        # tail hand-off between a workgroup's waves (k_env mode 4, EnvArgs::steal_local): per wave envs
        # received / handed off, time spent idle waiting for one, first time idle
        pct = lambda v: {f"p{q}": round(float(np.percentile(v, q)), 1) for q in (0, 10, 50, 90, 100)}
        res["handoff"] = {"envs_received": pct(st[:, 15]), "envs_pushed": pct(st[:, 16] & 0xFFFF),
                          "total_received": int(st[:, 15].sum()), "total_pushed": int((st[:, 16] & 0xFFFF).sum()),
                          "idle_wait_us": pct(st[:, 17] / 100.0),
                          "first_idle_us": pct((st[st[:, 18] > 0, 18] - t0) / 100.0) if (st[:, 18] > 0).any() else None}
        lt = st[:, 35] > 0  # the wave's last tail block's end (realtime)
        res["last_tail_block_end_us"] = pct((st[lt, 35] - t0) / 100.0) if lt.any() else None
        res["envs_from_grid_pool"] = int((st[:, 16] >> 16).sum())
        # the critical path: the waves whose last tail block ends last, and their longest session
        order = np.argsort(-st[:, 35])[:5]
        res["last_waves"] = [{"last_block_end_us": round(float((st[w, 35] - t0) / 100.0), 1),
                              "lane_phase_le16_us": round(float((st[w, 4] - t0) / 100.0), 1) if st[w, 4] else None,
                              "longest_session_start_us": round(float((st[w, 36] - t0) / 100.0), 1) if st[w, 36] else None,
                              "longest_session_blocks": int(st[w, 37]),
                              "longest_session_end_us": round(float((st[w, 38] - t0) / 100.0), 1) if st[w, 38] else None,
                              "updates_before_session": int(st[w, 39]),
                              "tail_blocks": int(st[w, 19]), "envs_received": int(st[w, 15]),
                              "from_pool": int(st[w, 16] >> 16), "pushed_local": int(st[w, 16] & 0xFFFF)}
                             for w in order]
        res["tail_blocks"] = int(st[:, 19].sum())
        res["tail_block_us_mean"] = round(float(st[:, 32].sum() / max(st[:, 19].sum(), 1) / 100.0), 4)
        res["tail_block_rounds_mean"] = round(float(st[:, 21].sum() / max(st[:, 19].sum(), 1)), 3)
        # shader clock while in tail blocks: s_memtime cycles (est 20) per s_memrealtime 10-ns tick (est 32)
        res["tail_clock_GHz"] = round(float(st[:, 20].sum() / max(st[:, 32].sum(), 1) / 10.0), 4)
        res["chunks_per_wave_p50"] = float(np.median(st[:, 8]))
        res["mean_active_lanes_per_chunk_p50"] = float(np.median(st[:, 9] / np.maximum(st[:, 8], 1)))
        out["reps"].append(res)
    b.close()
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
