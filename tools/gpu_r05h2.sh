#!/bin/bash
# Round 5: tail helpers per session, 3 (default) vs 2 vs 1, at config 5's shard
set -o pipefail
O=gpurun_out/r05h2; mkdir -p $O
timeout -k 10 900 python tools/r6_env_ab.py 131072 10 2 fixture:1048576,spec:1048576,fixture:4096 'PBNSIM_ENV_HELPERS=3' 'PBNSIM_ENV_HELPERS=2' 'PBNSIM_ENV_HELPERS=1' > $O/ab.jsonl 2> $O/ab.err || { echo AB FAILED; tail $O/ab.err; exit 1; }
python - <<'PY'
import json
for l in open('gpurun_out/r05h2/ab.jsonl'):
    d=json.loads(l)
    if 'rows' in d: continue
    print(d['rep'], d['spec'], d['cap'], d['variant'], 'per_step', d['per_step_ms'], 'fused', d['fused_ms'])
PY
echo ALL OK
