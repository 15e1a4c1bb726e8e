#!/usr/bin/env python3
"""A/B of MT-mode builds (measurement only): each library (PBNSIM_LIB) in its own process runs bench.py's MT
workload (Bittner-199, 1,048,576 envs seeded 12345 + id, genRandState, T = 256 updates per pbn_mt_step launch:
one warm-up launch, then `reps` timed with HIP events) and a 65,536-env case, alternated `alts` times on one box;
every variant must leave the same state digest (bit-exact).
Usage: python tools/mt_ab.py alts lib1.so lib2.so ..."""
import json
import os
import subprocess
import sys
import zlib
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]


def child():
    sys.path.insert(0, str(ROOT / "gym-pbn-stac_amd"))
    import numpy as np

    from gym_pbn_amd.batch import PBNBatch
    from gym_pbn_amd.network import load_network

    net = load_network("bittner199")
    out = {}
    for B, T, reps in ((1 << 20, 256, 3), (65536, 512, 3)):
        b = PBNBatch(net, B, seed=1)
        b.mt_seed(np.arange(B, dtype=np.uint64) + 12345, init_state=True)
        b.mt_step(T)
        b.sync()
        b.timing(2)
        for _ in range(reps):
            b.mt_step(T)
        b.timing(0)
        ms, n = b.timing_read()
        s = ms / 1e3 / reps
        out[f"{B}x{T}"] = {"ms_per_launch": s * 1e3, "node_updates_per_s": B * T / s,
                           "digest": zlib.crc32(b.get_state().tobytes())}
        b.close()
    print(json.dumps(out))


def main():
    if sys.argv[1] == "--child":
        return child()
    alts, libs = int(sys.argv[1]), sys.argv[2:]
    rows = []
    for rep in range(alts):
        for lib in libs:
            env = dict(os.environ, PBNSIM_LIB=str(Path(lib).resolve()))
            r = subprocess.run([sys.executable, __file__, "--child"], capture_output=True, text=True, env=env, timeout=300)
            if r.returncode:
                print(r.stderr[-2000:], file=sys.stderr)
                sys.exit(1)
            d = json.loads(r.stdout.strip().splitlines()[-1])
            row = {"rep": rep, "lib": lib, **{k: {"G_updates_per_s": round(v["node_updates_per_s"] / 1e9, 2),
                                                  "ms": round(v["ms_per_launch"], 3), "digest": v["digest"]}
                                              for k, v in d.items()}}
            rows.append(row)
            print(json.dumps(row), flush=True)
    digests = {(k, r[k]["digest"]) for r in rows for k in r if "x" in k}
    print(json.dumps({"rows": rows, "bit_exact_across_variants": len(digests) == 2}))


if __name__ == "__main__":
    main()
