#!/usr/bin/env python3
"""A/B of R6 kernel settings given as environment assignments (e.g. PBNSIM_ENV_HELPERS=0 vs =1), each
run as its own process (tools/r6_tail_sweep.py --child: config 5's shard, T env steps fused and per step,
best of 2), alternated `reps` times on one box. Measurement only.
Usage: python tools/r6_env_ab.py B T reps 'spec:cap,...' 'A=1 B=2' 'A=0' ..."""
import json
import os
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
B, T, reps = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
specs = [(s.split(":")[0], int(s.split(":")[1])) for s in sys.argv[4].split(",")]
variants = sys.argv[5:]
out = []
for rep in range(reps):
    for spec, cap in specs:
        for v in variants:
            env = dict(os.environ)
            for kv in v.split():
                k, val = kv.split("=", 1)
                env[k] = val
            r = subprocess.run([sys.executable, str(ROOT / "tools" / "r6_tail_sweep.py"), "--child", str(B), str(T), spec,
                                str(cap)], capture_output=True, text=True, env=env, timeout=300)
            if r.returncode != 0:
                print(r.stderr[-2000:], file=sys.stderr)
                sys.exit(1)
            d = json.loads(r.stdout.strip().splitlines()[-1])
            row = {"rep": rep, "spec": spec, "cap": cap, "variant": v,
                   "per_step_ms": round(d["per_step"]["ms_per_env_step"], 4), "fused_ms": round(d["fused"]["ms_per_env_step"], 4),
                   "per_step_M": round(d["per_step"]["env_steps_per_s"] / 1e6, 1),
                   "fused_M": round(d["fused"]["env_steps_per_s"] / 1e6, 1),
                   "helpers": [d["per_step"].get("helpers_last_launch"), d["fused"].get("helpers_last_launch")],
                   "handoffs": [d["per_step"].get("handoffs_last_launch"), d["fused"].get("handoffs_last_launch")],
                   "pool": [d["per_step"].get("pool_last_launch"), d["fused"].get("pool_last_launch")]}
            out.append(row)
            print(json.dumps(row), flush=True)
print(json.dumps({"B": B, "T": T, "rows": out}))
