#!/bin/bash
# Round 5: waiting workgroups leave quietly after 20 ms -- the R6 tests, then the pool A/B (shipped build vs the
# previous one, build_exp/prevpool) at config 5's shard incl. a long fused launch (T = 100)
set -o pipefail
O=gpurun_out/r05z; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_r6_regimes.py -x -q --timeout 240 --timeout-method thread > $O/r6_tests.log 2>&1 || { echo R6 TESTS FAILED; tail -30 $O/r6_tests.log; exit 1; }
tail -1 $O/r6_tests.log
P=$PWD/build_exp/prevpool/libpbnsim.so
timeout -k 10 900 python tools/r6_env_ab.py 131072 100 1 fixture:1048576,spec:1048576,fixture:4096 'PBNSIM_ENV_HELPERS=3' "PBNSIM_LIB=$P" > $O/ab.jsonl 2> $O/ab.err || { echo AB FAILED; tail $O/ab.err; exit 1; }
python - <<'PY'
import json
for l in open('gpurun_out/r05z/ab.jsonl'):
    d=json.loads(l)
    if 'rows' in d: continue
    print(d['rep'], d['spec'], d['cap'], d['variant'][-24:], 'per_step', d['per_step_ms'], 'fused', d['fused_ms'])
PY
echo ALL OK
