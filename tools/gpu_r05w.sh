#!/bin/bash
# Round 5: k_env with 512-thread workgroups (8 waves: a larger hand-off / helper domain) -- R6 tests on that build,
# then config 5's A/B against the shipped 256
set -o pipefail
O=gpurun_out/r05w; mkdir -p $O
E=$PWD/build_exp/eb512/libpbnsim.so
PBNSIM_LIB=$E timeout -k 10 500 python -u -m pytest tests/test_r6_regimes.py -x -q --timeout 240 --timeout-method thread > $O/r6_tests.log 2>&1 || { echo R6 TESTS FAILED; tail -30 $O/r6_tests.log; exit 1; }
tail -1 $O/r6_tests.log
timeout -k 10 500 python -u -m pytest tests/test_r6_regimes.py -x -q --timeout 240 --timeout-method thread > $O/r6_tests_256.log 2>&1 || { echo R6 TESTS 256 FAILED; tail -30 $O/r6_tests_256.log; exit 1; }
tail -1 $O/r6_tests_256.log
timeout -k 10 900 python tools/r6_env_ab.py 131072 10 2 fixture:1048576,spec:1048576,fixture:4096 'PBNSIM_ENV_HELPERS=3' "PBNSIM_LIB=$E" > $O/ab.jsonl 2> $O/ab.err || { echo AB FAILED; tail $O/ab.err; exit 1; }
python - <<'PY'
import json
for l in open('gpurun_out/r05w/ab.jsonl'):
    d=json.loads(l)
    if 'rows' in d: continue
    print(d['rep'], d['spec'], d['cap'], d['variant'][-24:], 'per_step', d['per_step_ms'], 'fused', d['fused_ms'], d['helpers'], d['handoffs'])
PY
echo ALL OK
