#!/bin/bash
# Round 5: MT mode -- window prefetch depth 1 / 2 / 3 and the twist's share (no-twist build, timing only)
set -o pipefail
O=gpurun_out/r05s; mkdir -p $O
B=$PWD/build_exp
for rep in 1 2; do
  for v in product mtahead2 mtahead3 mtnotwist; do
    if [ $v = product ]; then L=$PWD/gym-pbn-stac_amd/gym_pbn_amd/libpbnsim.so; else L=$B/$v/libpbnsim.so; fi
    echo "== $v" >> $O/mt.txt
    PBNSIM_LIB=$L timeout -k 10 300 python tools/mt_bench.py 2>> $O/err | tail -1 >> $O/mt.txt || { echo MT FAILED; tail $O/err; exit 1; }
  done
done
python - <<'PY'
import json
v=None
for l in open('gpurun_out/r05s/mt.txt'):
    if l.startswith('=='): v=l.split()[1]; continue
    d=json.loads(l)
    print(v, [(r['B'], r['T'], round(r['node_updates_per_s']/1e9,1)) for r in d['mt_mode']])
PY
echo ALL OK
