#!/bin/bash
# Round 5: pool tickets from idle CUs only vs any idle workgroup (and the migration threshold with either)
set -o pipefail
O=gpurun_out/r05r; mkdir -p $O
timeout -k 10 1000 python tools/r6_env_ab.py 131072 10 2 fixture:4096,fixture:1048576,spec:1048576 'PBNSIM_ENV_GRID_STEAL=1' 'PBNSIM_ENV_GRID_STEAL=1 PBNSIM_ENV_POOL_CU_IDLE=0' 'PBNSIM_ENV_GRID_STEAL=1 PBNSIM_ENV_POOL_CU_IDLE=0 PBNSIM_ENV_MIGRATE_BLOCKS=32' 'PBNSIM_ENV_GRID_STEAL=0' > $O/ab.jsonl 2> $O/ab.err || { echo AB FAILED; tail $O/ab.err; exit 1; }
python - <<'PY'
import json
for l in open('gpurun_out/r05r/ab.jsonl'):
    d=json.loads(l)
    if 'rows' in d: continue
    print(d['rep'], d['spec'], d['cap'], d['variant'][21:], 'per_step', d['per_step_ms'], 'fused', d['fused_ms'])
PY
echo ALL OK
