#!/bin/bash
# Round 5: MT mode change vs the round's MT kernel (build_exp/mthead) on one box -- MT tests, then the rates
set -o pipefail
O=gpurun_out/r05t; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -k "mt" -x -q --timeout 240 --timeout-method thread > $O/mt_tests.log 2>&1 || { echo MT TESTS FAILED; tail -30 $O/mt_tests.log; exit 1; }
tail -2 $O/mt_tests.log
rm -f $O/mt_ab.txt
for rep in 1 2; do
  for v in new head; do
    if [ $v = new ]; then L=$PWD/gym-pbn-stac_amd/gym_pbn_amd/libpbnsim.so; else L=$PWD/build_exp/mthead/libpbnsim.so; fi
    echo "== $v" >> $O/mt_ab.txt
    PBNSIM_LIB=$L timeout -k 10 300 python tools/mt_bench.py 2>> $O/err | tail -1 >> $O/mt_ab.txt || { echo MT FAILED; tail $O/err; exit 1; }
  done
done
python - <<'PY'
import json
v=None
for l in open('gpurun_out/r05t/mt_ab.txt'):
    if l.startswith('=='): v=l.split()[1]; continue
    d=json.loads(l); print(v, [(r['B'], r['T'], round(r['node_updates_per_s']/1e9,1)) for r in d['mt_mode']])
PY
echo ALL OK
