#!/bin/bash
# Round 5: session migration threshold (blocks a lone session runs before it moves itself to a waiting workgroup)
set -o pipefail
O=gpurun_out/r05q; mkdir -p $O
B=$PWD/build_exp
timeout -k 10 900 python tools/r6_env_ab.py 131072 10 2 fixture:1048576,spec:1048576 'PBNSIM_ENV_GRID_STEAL=1' "PBNSIM_LIB=$B/mig16/libpbnsim.so" "PBNSIM_LIB=$B/mig256/libpbnsim.so" "PBNSIM_LIB=$B/mig100000/libpbnsim.so" > $O/ab.jsonl 2> $O/ab.err || { echo AB FAILED; tail $O/ab.err; exit 1; }
python - <<'PY'
import json
for l in open('gpurun_out/r05q/ab.jsonl'):
    d=json.loads(l)
    if 'rows' in d: continue
    print(d['rep'], d['spec'], d['cap'], d['variant'][-30:], 'per_step', d['per_step_ms'], 'fused', d['fused_ms'], d['helpers'], d['handoffs'])
PY
echo ALL OK
