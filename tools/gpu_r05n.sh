#!/bin/bash
# Round 5: what the grid pool's cost at cap 4,096 per step is made of -- pool on, pool on with one slot (waiting
# workgroups resident, at most one env moved), pool off
set -o pipefail
O=gpurun_out/r05n; mkdir -p $O
timeout -k 10 600 python tools/r6_env_ab.py 131072 10 2 fixture:4096,fixture:1048576 'PBNSIM_ENV_GRID_STEAL=1' 'PBNSIM_ENV_GRID_SLOTS=1' 'PBNSIM_ENV_GRID_STEAL=0' > $O/ab.jsonl 2> $O/ab.err || { echo AB FAILED; tail $O/ab.err; exit 1; }
python - <<'PY'
import json
for l in open('gpurun_out/r05n/ab.jsonl'):
    d=json.loads(l)
    if 'rows' in d: continue
    print(d['rep'], d['spec'], d['cap'], d['variant'], 'per_step', d['per_step_ms'], 'fused', d['fused_ms'], d['helpers'], d['handoffs'])
PY
echo ALL OK
