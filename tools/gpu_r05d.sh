#!/bin/bash
# Round 5: two-ahead ring prefetch -- R6 tests, lone-env block cost, helpers A/B; then the 8-B store A/B
set -o pipefail
O=gpurun_out/r05d; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_r6_regimes.py -x -q --timeout 240 --timeout-method thread > $O/r6_tests.log 2>&1 || { echo R6 TESTS FAILED; tail -40 $O/r6_tests.log; exit 1; }
tail -2 $O/r6_tests.log
for h in 1 0; do
  PBNSIM_ENV_HELPERS=$h timeout -k 10 120 python tools/r6_lone_fit.py 80 >> $O/lone_fit.jsonl 2>> $O/lone_fit.err || { echo LONE FAILED; tail $O/lone_fit.err; exit 1; }
done
python - <<'PY'
import json
for l in open('gpurun_out/r05d/lone_fit.jsonl'):
    d=json.loads(l); print(d['env'], 'us/block', d['us_per_block'], 'fixed', d['fixed_us'], 'fit', d['fit_steps'], 'helpers', d['helpers_per_launch_median'])
PY
timeout -k 10 400 python tools/r6_env_ab.py 131072 10 2 fixture:4096,fixture:1048576,spec:1048576 'PBNSIM_ENV_HELPERS=1' 'PBNSIM_ENV_HELPERS=0' > $O/helpers_ab.jsonl 2> $O/helpers_ab.err || { echo AB FAILED; tail $O/helpers_ab.err; exit 1; }
python - <<'PY'
import json
for l in open('gpurun_out/r05d/helpers_ab.jsonl'):
    d=json.loads(l)
    if 'rows' in d: continue
    print(d['rep'], d['spec'], d['cap'], d['variant'], 'per_step', d['per_step_ms'], 'fused', d['fused_ms'])
PY
for rep in 1 2; do
  for L in gym-pbn-stac_amd/gym_pbn_amd/libpbnsim.so build_exp/store8/libpbnsim.so; do
    r=$(PBNSIM_LIB=$PWD/$L timeout -k 10 120 python tools/step_time.py 7) || { echo STEP_TIME FAILED; exit 1; }
    echo "$L $r" >> $O/store8_ab.txt
  done
done
cat $O/store8_ab.txt
echo ALL OK
