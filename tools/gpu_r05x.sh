#!/bin/bash
# Round 5: config 5's A/B, k_env with 512-thread workgroups (build_exp/eb512) vs the shipped 256
set -o pipefail
O=gpurun_out/r05x; mkdir -p $O
E=$PWD/build_exp/eb512/libpbnsim.so
timeout -k 10 900 python tools/r6_env_ab.py 131072 10 2 fixture:1048576,spec:1048576,fixture:4096 'PBNSIM_ENV_HELPERS=3' "PBNSIM_LIB=$E" > $O/ab.jsonl 2> $O/ab.err || { echo AB FAILED; tail $O/ab.err; exit 1; }
python - <<'PY'
import json
for l in open('gpurun_out/r05x/ab.jsonl'):
    d=json.loads(l)
    if 'rows' in d: continue
    print(d['rep'], d['spec'], d['cap'], d['variant'][-24:], 'per_step', d['per_step_ms'], 'fused', d['fused_ms'], d['helpers'], d['handoffs'])
PY
echo ALL OK
