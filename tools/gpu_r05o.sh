#!/bin/bash
# Round 5: the grid pool's residency cost -- one waiting workgroup per CU vs all
set -o pipefail
O=gpurun_out/r05o; mkdir -p $O
S=$PWD/build_exp/onepercu/libpbnsim.so
timeout -k 10 700 python tools/r6_env_ab.py 131072 10 2 fixture:4096,fixture:1048576,spec:1048576 'PBNSIM_ENV_GRID_STEAL=1' "PBNSIM_LIB=$S" 'PBNSIM_ENV_GRID_STEAL=0' > $O/ab2.jsonl 2> $O/ab.err || { echo AB FAILED; tail $O/ab.err; exit 1; }
python - <<'PY'
import json
for l in open('gpurun_out/r05o/ab2.jsonl'):
    d=json.loads(l)
    if 'rows' in d: continue
    print(d['rep'], d['spec'], d['cap'], d['variant'][-40:], 'per_step', d['per_step_ms'], 'fused', d['fused_ms'], d['helpers'], d['handoffs'])
PY
echo ALL OK
