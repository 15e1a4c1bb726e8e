#!/bin/bash
# Round 5: launch-shape / tail-threshold sweep with helpers on (grid cap, lane limit, tail threshold), config 5's shard
set -o pipefail
O=gpurun_out/r05k; mkdir -p $O
timeout -k 10 900 python tools/r6_env_ab.py 131072 10 1 fixture:4096,fixture:1048576,spec:1048576 \
  'PBNSIM_ENV_HELPERS=3' 'PBNSIM_ENV_GRID=256' 'PBNSIM_ENV_GRID=384' 'PBNSIM_ENV_TAIL=24' 'PBNSIM_ENV_TAIL=32' \
  'PBNSIM_ENV_LANES=32' 'PBNSIM_ENV_LANES=48' 'PBNSIM_ENV_TAIL=8' > $O/shape_ab.jsonl 2> $O/shape_ab.err || { echo AB FAILED; tail $O/shape_ab.err; exit 1; }
python - <<'PY'
import json
for l in open('gpurun_out/r05k/shape_ab.jsonl'):
    d=json.loads(l)
    if 'rows' in d: continue
    print(d['spec'], d['cap'], d['variant'], 'per_step', d['per_step_ms'], 'fused', d['fused_ms'], d['helpers'], d['handoffs'])
PY
echo ALL OK
