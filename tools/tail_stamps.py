#!/usr/bin/env python3
"""Cost of k_env's tail-mode block (64 updates of one env resolved by the whole wave), from the
PBN_STAMPS measurement build (tools/build_exp.sh stamps -DPBN_STAMPS; PBNSIM_LIB=...): per wave,
tail blocks, shader cycles per block (s_memtime, top of one block to the top of the next), the
cycles from the block's top to the next block's draws prepared (plane reads issued + prepare), the
fixed-point resolution's cycles and rounds, and the blocks per round count.

Workloads (argv[1]): "lone" = 64 envs, one per wave (the small-batch path: every wave in tail mode),
fixture attractors, cap 4,096, one launch per env step -- the tail block alone on its SIMD;
"highcap" = 131,072 envs per step at cap 2^20 (config 5's high_cap figure); "ring" = one env alone in one
workgroup (two lanes per wave take envs, so the tail helpers of its idle waves prepare its blocks), cap 2^20,
24 env steps (PBNSIM_ENV_HELPERS=0 for the same without helpers). Prints JSON.
"""
import ctypes as C
import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "gym-pbn-stac_amd"))
from gym_pbn_amd import _lib  # noqa: E402
from gym_pbn_amd.batch import EnvConfig, Net, PBNBatch, attractors_from_cubes  # noqa: E402
from gym_pbn_amd.network import load_network  # noqa: E402

NS = 40


def main():
    import torch

    mode = sys.argv[1] if len(sys.argv) > 1 else "lone"
    B, CAP = {"lone": (64, 4096), "highcap": (131072, 1 << 20), "ring": (1, 1 << 20)}[mode]
    if mode == "ring":  # one env, one workgroup, two lanes per wave: the tail helpers' ring (PBNSIM_ENV_HELPERS)
        import os
        os.environ.setdefault("PBNSIM_ENV_GRID", "1")
        os.environ.setdefault("PBNSIM_ENV_LANES", "2")
    lib = _lib.lib
    lib.pbn_exp_env_stamps.argtypes = [C.c_void_p, C.c_size_t]
    z = np.load(ROOT / "tests" / "golden" / "r6_bittner199.npz", allow_pickle=False)
    net = Net(load_network("bittner199"))
    cfg = EnvConfig(net, attractors_from_cubes(z["cube_care"], z["cube_value"], z["cube_attractor"], net.n_nodes),
                    horizon=100)
    dev = torch.device("cuda", 0)
    A, W, T = 4, net.n_words, (24 if mode == "ring" else 8)
    g = torch.Generator(device=dev)
    g.manual_seed(0xAC7)
    v = torch.randint(1, net.n_nodes + 1, (T, B, A), device=dev, generator=g, dtype=torch.int32)
    acts = (v * (torch.rand((T, B, A), device=dev, generator=g) >= 0.75)).to(torch.int32).contiguous()
    obs = torch.empty((B, W), dtype=torch.int64, device=dev)
    rew = torch.empty(B, dtype=torch.int32, device=dev)
    flg = torch.empty(B, dtype=torch.uint8, device=dev)
    nup = torch.empty(B, dtype=torch.int32, device=dev)
    b = PBNBatch(net, B, seed=0xAC7)
    b.env_reset(cfg)
    acc = np.zeros(NS, dtype=np.float64)
    per_step = []
    for t in range(T):
        assert lib.pbn_exp_stamps_clear() == 0
        b.timing(1)
        b.env_step_multi_device(cfg, acts[t].data_ptr(), A, obs.data_ptr(), rew.data_ptr(), flg.data_ptr(),
                                nup.data_ptr(), update_cap=CAP)
        b.sync()
        ms, _ = b.timing_read()
        b.timing(0)
        st = np.zeros(16384 * NS, dtype=np.uint64)
        assert lib.pbn_exp_env_stamps(st.ctypes.data, st.nbytes) == 0
        st = st.reshape(-1, NS).astype(np.float64)
        if t >= 1:  # the first launch warms up
            acc += st[st[:, 19] > 0].sum(axis=0)
            live = st[st[:, 0] > 0]
            t0 = live[:, 33].min()
            tl = live[live[:, 19] > 0]
            per_step.append({"kernel_ms": ms, "max_updates": int(nup.max().item()),
                             # realtime (10 ns ticks) from the first wave's entry, us
                             "staged_us_max": float((live[:, 0] - t0).max() / 100),
                             "first_tail_block_us_p50": float(np.median(tl[:, 34] - t0) / 100) if len(tl) else None,
                             "last_wave_end_us": float((live[:, 7] - t0).max() / 100),
                             "most_tail_blocks_in_a_wave": int(tl[:, 19].max()) if len(tl) else 0,
                             "that_wave_tail_us": float(tl[np.argmax(tl[:, 19]), 32] / 100) if len(tl) else None,
                             # timelines (us from the first entry): entry, staged, first tail block, last tail
                             # block end, wave end -- of the wave with the most blocks and of the last wave to end
                             "longest_wave": [round(float((tl[np.argmax(tl[:, 19]), k] - t0) / 100), 2)
                                              for k in (33, 0, 34, 35, 7)] if len(tl) else None,
                             "last_wave": [round(float((live[np.argmax(live[:, 7]), k] - t0) / 100), 2) if
                                           live[np.argmax(live[:, 7]), k] else None for k in (33, 0, 34, 35, 7)],
                             "last_wave_blocks": int(live[np.argmax(live[:, 7]), 19]),
                             # the longest tail session of the launch (one env step of one env): start / end us,
                             # blocks, updates the env had made before it (lane mode or earlier sessions)
                             "longest_session": (lambda w: {"start_us": round(float((w[36] - t0) / 100), 1),
                                                            "end_us": round(float((w[38] - t0) / 100), 1),
                                                            "blocks": int(w[37]), "updates_before": int(w[39]),
                                                            "wave_end_us": round(float((w[7] - t0) / 100), 1)})(
                                 live[np.argmax(live[:, 37])]),
                             "last_wave_received_envs": int(live[np.argmax(live[:, 7]), 15])})
    blocks = acc[19]
    out = {"mode": mode, "B": B, "update_cap": CAP, "env_kernel": b.info().get("env_kernel"),
           "tail_blocks": int(blocks), "steps": per_step}
    if blocks:
        out.update({
            "cycles_per_block": acc[20] / blocks,
            "us_per_block_realtime": acc[32] / blocks / 100,
            "memtime_ticks_per_us": acc[20] / (acc[32] / 100),
            "cycles_top_to_next_prepared": acc[23] / blocks,
            "cycles_fixed_point": acc[22] / blocks,
            "cycles_rest": (acc[20] - acc[22] - acc[23]) / blocks,
            "rounds_per_block": acc[21] / blocks,
            "blocks_by_rounds": {str(k) if k < 7 else "7+": int(acc[24 + k]) for k in range(8)},
            "note": "s_memtime shader cycles; the stamps themselves add waits (measurement build)",
        })
    b.close()
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
