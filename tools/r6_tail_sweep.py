"""R6 env kernel's tail mode (k_env<.., 4>: a wave whose work queue ran dry resolves its remaining
envs one at a time, 64 updates per block) against its threshold PBNSIM_ENV_TAIL (live envs per
wave; 0 = off). Bittner-200, bench.py's config-5 settings (A = 4, 0 w.p. 0.75, horizon 100), lane
mode (PBNSIM_ENV_GROUP=1), both attractor specs and both caps; per batch size B: T env steps as
one fused launch and as T per-step launches, ms per env step (best of 2). Measurement only.

Usage: python tools/r6_tail_sweep.py B[,B...] TAIL[:LANES[:STEAL]][,...] [T] [spec:cap,...]
(LANES: PBNSIM_ENV_LANES, lanes per wave that take envs; 0 or absent = the library default.
STEAL: PBNSIM_ENV_STEAL, hand-off of tail envs between waves, 1 = on (default) / 0 = off.)
Output of `python tools/r6_tail_sweep.py 1,64,131072 0,2,8,64 10` -> profiles/r03_r6_tail_sweep.json."""
import json
import os
import subprocess
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]


def child(B, T, spec, cap):
    sys.path.insert(0, str(ROOT / "gym-pbn-stac_amd"))
    sys.path.insert(0, str(ROOT))
    import torch

    from bench import r6_attractors
    from gym_pbn_amd.batch import EnvConfig, Net, PBNBatch
    from gym_pbn_amd.network import load_network

    net = Net(load_network("bittner199"))
    atts, _ = r6_attractors(spec, net.n_nodes)
    cfg = EnvConfig(net, atts, horizon=100)
    dev = torch.device("cuda", 0)
    A, W = 4, net.n_words
    g = torch.Generator(device=dev)
    g.manual_seed(0xAC7)
    v = torch.randint(1, net.n_nodes + 1, (T, B, A), device=dev, generator=g, dtype=torch.int32)
    acts = (v * (torch.rand((T, B, A), device=dev, generator=g) >= 0.75)).to(torch.int32).contiguous()
    outs = [torch.empty((T, B, W), dtype=torch.int64, device=dev), torch.empty((T, B), dtype=torch.int32, device=dev),
            torch.empty((T, B), dtype=torch.uint8, device=dev), torch.empty((T, B), dtype=torch.int32, device=dev)]
    res = {}
    for fused in (True, False):
        b = PBNBatch(net, B, seed=0xAC7)
        best = None
        for _ in range(2):
            b.env_reset(cfg)
            b.sync()
            t0 = time.perf_counter()
            if fused:
                b.env_rollout_multi_device(cfg, T, acts.data_ptr(), A, *[x.data_ptr() for x in outs], update_cap=cap)
            else:
                for t in range(T):
                    b.env_step_multi_device(cfg, acts[t].data_ptr(), A, *[x[t].data_ptr() for x in outs],
                                            update_cap=cap)
            b.sync()
            dt = time.perf_counter() - t0
            best = dt if best is None else min(best, dt)
        inf = b.info()
        handoffs = b.env_handoffs()
        helpers = b.env_tail_helpers() if hasattr(b, "env_tail_helpers") else None
        pool = b.env_grid_stats() if hasattr(b, "env_grid_stats") else None
        b.close()
        n = outs[3].to(torch.int64)
        res["fused" if fused else "per_step"] = {"ms_per_env_step": best * 1e3 / T, "env_steps_per_s": B * T / best,
                                                 "max_updates": int(n.max()), "mean_updates": float(n.float().mean()),
                                                "env_grid": inf["env_grid"], "env_lane_limit": inf["env_lane_limit"], "env_chunk": inf.get("env_chunk"),
                                                "handoffs_last_launch": handoffs, "helpers_last_launch": helpers,
                                                 "pool_last_launch": pool}
    print(json.dumps(res))


def main():
    if sys.argv[1] == "--child":
        child(int(sys.argv[2]), int(sys.argv[3]), sys.argv[4], int(sys.argv[5]))
        return
    Bs = [int(x) for x in sys.argv[1].split(",")]
    tails = [tuple(int(v) for v in (x.split(":") + ["0", "1"][len(x.split(":")) - 1:])[:3])
             for x in sys.argv[2].split(",")]
    T = int(sys.argv[3]) if len(sys.argv) > 3 else 10
    specs = [(s.split(":")[0], int(s.split(":")[1])) for s in sys.argv[4].split(",")] if len(sys.argv) > 4 \
        else [("fixture", 4096), ("fixture", 1 << 20), ("spec", 1 << 20)]
    out = []
    for spec, cap in specs:
        for B in Bs:
            for tail, lanes, steal in tails:
                env = dict(os.environ, PBNSIM_ENV_GROUP="1", PBNSIM_ENV_TAIL=str(tail), PBNSIM_ENV_LANES=str(lanes),
                           PBNSIM_ENV_STEAL=str(steal))
                p = subprocess.run([sys.executable, __file__, "--child", str(B), str(T), spec, str(cap)], env=env,
                                   capture_output=True, text=True, timeout=300)
                if p.returncode:
                    print(p.stderr[-2000:], file=sys.stderr)
                    sys.exit(p.returncode)
                row = {"attractors": spec, "update_cap": cap, "B": B, "tail_max": tail, "lanes": lanes or "auto",
                       "steal": steal, "T": T,
                       **json.loads(p.stdout.strip().splitlines()[-1])}
                print(json.dumps(row), flush=True)
                out.append(row)
    print(json.dumps({"sweep": out, "source": "python tools/r6_tail_sweep.py " + " ".join(sys.argv[1:])}))


if __name__ == "__main__":
    main()
