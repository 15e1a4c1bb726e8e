#!/bin/bash
# Round 5: ring128 without scratch reloads on its chain -- R6 tests, lone block cost, stamps, helpers A/B
set -o pipefail
O=gpurun_out/r05j; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_r6_regimes.py -x -q --timeout 240 --timeout-method thread > $O/r6_tests.log 2>&1 || { echo R6 TESTS FAILED; tail -40 $O/r6_tests.log; exit 1; }
tail -2 $O/r6_tests.log
for h in 3 0; do
  PBNSIM_ENV_HELPERS=$h timeout -k 10 120 python tools/r6_lone_fit.py 80 >> $O/lone_fit.jsonl 2>> $O/lone_fit.err || { echo LONE FAILED; tail $O/lone_fit.err; exit 1; }
done
python - <<'PY'
import json
for l in open('gpurun_out/r05j/lone_fit.jsonl'):
    d=json.loads(l); print(d['env'], 'us/64', round(d['us_per_block'],4), 'fixed', round(d['fixed_us'],2), 'ring blocks', d['ring_blocks'], 'waits', d['ring_waits'])
PY
PBNSIM_LIB=$PWD/build_exp/stamps/libpbnsim.so timeout -k 10 120 python tools/tail_stamps.py ring > $O/stamps_ring.json 2> $O/err1 || { echo STAMPS FAILED; tail $O/err1; exit 1; }
python -c "
import json; d=json.load(open('$O/stamps_ring.json')); print({k:d.get(k) for k in ('tail_blocks','cycles_per_block','cycles_top_to_next_prepared','cycles_fixed_point','cycles_rest','rounds_per_block')})"
timeout -k 10 400 python tools/r6_env_ab.py 131072 10 2 fixture:4096,fixture:1048576,spec:1048576 'PBNSIM_ENV_HELPERS=3' 'PBNSIM_ENV_HELPERS=0' > $O/helpers_ab.jsonl 2> $O/helpers_ab.err || { echo AB FAILED; tail $O/helpers_ab.err; exit 1; }
python - <<'PY'
import json
for l in open('gpurun_out/r05j/helpers_ab.jsonl'):
    d=json.loads(l)
    if 'rows' in d: continue
    print(d['rep'], d['spec'], d['cap'], d['variant'], 'per_step', d['per_step_ms'], 'fused', d['fused_ms'])
PY
echo ALL OK
