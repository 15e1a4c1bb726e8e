#!/bin/bash
# Round 5: grid pool (k_env tail envs handed to workgroups that ran out of work anywhere on the GPU) --
# the R6 tests, then config 5's A/B (pool on / off)
set -o pipefail
O=gpurun_out/r05l; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_r6_regimes.py -x -v --timeout 240 --timeout-method thread > $O/r6_tests.log 2>&1 || { echo R6 TESTS FAILED; grep -E "PASS|FAIL|Error|error" $O/r6_tests.log | tail -30; tail -30 $O/r6_tests.log; exit 1; }
tail -2 $O/r6_tests.log
timeout -k 10 600 python tools/r6_env_ab.py 131072 10 2 fixture:4096,fixture:1048576,spec:1048576 'PBNSIM_ENV_GRID_STEAL=1' 'PBNSIM_ENV_GRID_STEAL=0' > $O/grid_ab.jsonl 2> $O/grid_ab.err || { echo AB FAILED; tail $O/grid_ab.err; exit 1; }
python - <<'PY'
import json
for l in open('gpurun_out/r05l/grid_ab.jsonl'):
    d=json.loads(l)
    if 'rows' in d: continue
    print(d['rep'], d['spec'], d['cap'], d['variant'], 'per_step', d['per_step_ms'], 'fused', d['fused_ms'], d['helpers'], d['handoffs'])
PY
echo ALL OK
