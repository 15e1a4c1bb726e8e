#!/bin/bash
# Round 6: keep the grid pool / session migration only if config 5's numbers show them.
# Shipped tree, three alternations: default vs PBNSIM_ENV_GRID_STEAL=0 vs PBNSIM_ENV_MIGRATE_BLOCKS=0,
# config 5's shard (131,072 envs, rank-3 style), T = 100 per step and fused, both caps and both specs.
set -o pipefail
O=gpurun_out/r06a; mkdir -p $O
timeout -k 10 1000 python tools/r6_env_ab.py 131072 100 3 fixture:1048576,spec:1048576,fixture:4096 'PBNSIM_ENV_HELPERS=3' 'PBNSIM_ENV_GRID_STEAL=0' 'PBNSIM_ENV_MIGRATE_BLOCKS=0' > $O/ab.jsonl 2> $O/ab.err || { echo AB FAILED; tail $O/ab.err; exit 1; }
python - <<'PY'
import json
for l in open('gpurun_out/r06a/ab.jsonl'):
    d=json.loads(l)
    if 'rows' in d: continue
    print(d['rep'], d['spec'], d['cap'], d['variant'][-28:], 'per_step', d['per_step_ms'], 'fused', d['fused_ms'])
PY
echo ALL OK
