#!/usr/bin/env python3
"""R6 tail hand-off threshold (PBNSIM_ENV_PARK: a wave with at most that many active lanes, once the
work queue is empty, parks its env steps for a second, dense launch): ms per env step, fused
T = 100 chunk and one launch per env step, lane mode (measurement only)."""
import json
import os
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
B = sys.argv[1] if len(sys.argv) > 1 else "131072"
res = {}
for park in (sys.argv[2] if len(sys.argv) > 2 else "0,8,16,32,64").split(","):
    env = dict(os.environ, PBNSIM_ENV_PARK=park)
    out = subprocess.run([sys.executable, str(ROOT / "tools" / "r6_group_sweep.py"), B, "1"], env=env,
                         capture_output=True, text=True, check=True).stdout
    res[park] = json.loads(out.strip().splitlines()[-1])
print(json.dumps(res))
