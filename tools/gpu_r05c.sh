#!/bin/bash
# Round 5: lone-env tail block cost with and without helpers, then the bench line and the probes
set -o pipefail
O=gpurun_out/r05c; mkdir -p $O
for h in 1 0 1 0; do
  PBNSIM_ENV_HELPERS=$h timeout -k 10 120 python tools/r6_lone_fit.py 80 >> $O/lone_fit.jsonl 2>> $O/lone_fit.err || { echo LONE FAILED; tail $O/lone_fit.err; exit 1; }
done
python - <<'PY'
import json
for l in open('gpurun_out/r05c/lone_fit.jsonl'):
    d=json.loads(l); print(d['env'], 'us/block', d['us_per_block'], 'fixed', d['fixed_us'], 'fit', d['fit_steps'], 'helpers', d['helpers_per_launch_median'])
PY
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS FAILED; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { echo BENCH FAILED; tail $O/bench.err; exit 1; }
timeout -k 10 200 python tools/write_width.py > $O/write_width.json || exit 1
for rep in 1 2; do
  for L in gym-pbn-stac_amd/gym_pbn_amd/libpbnsim.so build_exp/store8/libpbnsim.so; do
    echo "$L $(PBNSIM_LIB=$PWD/$L timeout -k 10 120 python tools/step_time.py 7)" >> $O/store8_ab.txt || exit 1
  done
done
echo ALL OK
