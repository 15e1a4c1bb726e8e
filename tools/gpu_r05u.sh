#!/bin/bash
# Round 5: ring blocks resolved in exactly their dependency depth's rounds (helpers measure it) -- R6 tests, the lone
# block cost, config-5 A/B against the previous build (build_exp/headenv)
set -o pipefail
O=gpurun_out/r05u; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_r6_regimes.py -x -q --timeout 240 --timeout-method thread > $O/r6_tests.log 2>&1 || { echo R6 TESTS FAILED; tail -30 $O/r6_tests.log; exit 1; }
tail -1 $O/r6_tests.log
for L in $PWD/gym-pbn-stac_amd/gym_pbn_amd/libpbnsim.so $PWD/build_exp/headenv/libpbnsim.so; do
  PBNSIM_LIB=$L timeout -k 10 120 python tools/r6_lone_fit.py 80 >> $O/lone_fit.jsonl 2>> $O/lone.err || { echo LONE FAILED; tail $O/lone.err; exit 1; }
done
python -c "
import json
for l in open('$O/lone_fit.jsonl'): d=json.loads(l); print('lone us/64', round(d['us_per_block'],4), 'ring blocks', d['ring_blocks'])"
H=$PWD/build_exp/headenv/libpbnsim.so
timeout -k 10 800 python tools/r6_env_ab.py 131072 10 2 fixture:1048576,spec:1048576,fixture:4096 'PBNSIM_ENV_HELPERS=3' "PBNSIM_LIB=$H" > $O/ab.jsonl 2> $O/ab.err || { echo AB FAILED; tail $O/ab.err; exit 1; }
python - <<'PY'
import json
for l in open('gpurun_out/r05u/ab.jsonl'):
    d=json.loads(l)
    if 'rows' in d: continue
    print(d['rep'], d['spec'], d['cap'], d['variant'][-28:], 'per_step', d['per_step_ms'], 'fused', d['fused_ms'])
PY
echo ALL OK
