#!/bin/bash
# Round 5: tail session order -- farthest-from-the-attractors first (build_exp/taildist) vs longest-run first;
# R6 tests on that build, then config 5's A/B
set -o pipefail
O=gpurun_out/r05y; mkdir -p $O
E=$PWD/build_exp/taildist/libpbnsim.so
PBNSIM_LIB=$E timeout -k 10 500 python -u -m pytest tests/test_r6_regimes.py -x -q --timeout 240 --timeout-method thread > $O/r6_tests.log 2>&1 || { echo R6 TESTS FAILED; tail -30 $O/r6_tests.log; exit 1; }
tail -1 $O/r6_tests.log
timeout -k 10 900 python tools/r6_env_ab.py 131072 10 2 fixture:1048576,spec:1048576,fixture:4096 'PBNSIM_ENV_HELPERS=3' "PBNSIM_LIB=$E" > $O/ab.jsonl 2> $O/ab.err || { echo AB FAILED; tail $O/ab.err; exit 1; }
python - <<'PY'
import json
for l in open('gpurun_out/r05y/ab.jsonl'):
    d=json.loads(l)
    if 'rows' in d: continue
    print(d['rep'], d['spec'], d['cap'], d['variant'][-24:], 'per_step', d['per_step_ms'], 'fused', d['fused_ms'])
PY
echo ALL OK
