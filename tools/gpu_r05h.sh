#!/bin/bash
# Round 5: 128-update ring blocks -- R6 tests, lone block cost (helpers 3 / 2 / 0), helpers A/B at config 5
set -o pipefail
O=gpurun_out/r05h; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_r6_regimes.py -x -q --timeout 240 --timeout-method thread > $O/r6_tests.log 2>&1 || { echo R6 TESTS FAILED; tail -40 $O/r6_tests.log; exit 1; }
tail -2 $O/r6_tests.log
for h in 3 2 0; do
  PBNSIM_ENV_HELPERS=$h timeout -k 10 120 python tools/r6_lone_fit.py 80 >> $O/lone_fit.jsonl 2>> $O/lone_fit.err || { echo LONE FAILED; tail $O/lone_fit.err; exit 1; }
done
python - <<'PY'
import json
for l in open('gpurun_out/r05h/lone_fit.jsonl'):
    d=json.loads(l); print(d['env'], 'us/block', round(d['us_per_block'],4), 'fixed', round(d['fixed_us'],2), 'helpers', d['helpers_per_launch_median'], 'ring blocks', d['ring_blocks'], 'waits', d['ring_waits'])
PY
timeout -k 10 400 python tools/r6_env_ab.py 131072 10 2 fixture:4096,fixture:1048576,spec:1048576 'PBNSIM_ENV_HELPERS=3' 'PBNSIM_ENV_HELPERS=0' > $O/helpers_ab.jsonl 2> $O/helpers_ab.err || { echo AB FAILED; tail $O/helpers_ab.err; exit 1; }
python - <<'PY'
import json
for l in open('gpurun_out/r05h/helpers_ab.jsonl'):
    d=json.loads(l)
    if 'rows' in d: continue
    print(d['rep'], d['spec'], d['cap'], d['variant'], 'per_step', d['per_step_ms'], 'fused', d['fused_ms'])
PY
echo ALL OK
