#!/bin/bash
# Round 5: tail helpers -- how many helpers the lone ring session needs (1/2/3), with ring-wait counts
set -o pipefail
O=gpurun_out/r05e; mkdir -p $O
for h in 3 2 1 0; do
  PBNSIM_ENV_HELPERS=$h timeout -k 10 120 python tools/r6_lone_fit.py 80 >> $O/lone_fit.jsonl 2>> $O/lone_fit.err || { echo LONE FAILED; tail $O/lone_fit.err; exit 1; }
done
python - <<'PY'
import json
for l in open('gpurun_out/r05e/lone_fit.jsonl'):
    d=json.loads(l); print(d['env'], 'us/block', round(d['us_per_block'],4), 'fixed', round(d['fixed_us'],2), 'helpers', d['helpers_per_launch_median'], 'ring blocks', d['ring_blocks'], 'waits', d['ring_waits'])
PY
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "mt_mode" -x -q --timeout 120 --timeout-method thread > $O/mt_tests.log 2>&1 || { echo MT TESTS FAILED; tail -40 $O/mt_tests.log; exit 1; }
tail -2 $O/mt_tests.log
timeout -k 10 200 python tools/mt_bench.py > $O/mt.json 2>&1 || { echo MT BENCH FAILED; tail $O/mt.json; exit 1; }
tail -1 $O/mt.json
timeout -k 10 120 python tools/write_width.py > $O/write_width.json || exit 1
cat $O/write_width.json
echo ALL OK
