#!/bin/bash
# Round 5: the critical path of one per-step launch at cap 2^20 (phase stamps, pool on / off)
set -o pipefail
O=gpurun_out/r05p; mkdir -p $O
for g in 1 0; do
  PBNSIM_ENV_GRID_STEAL=$g PBNSIM_LIB=$PWD/build_exp/stamps/libpbnsim.so timeout -k 10 200 python tools/env_stamps.py 131072 1048576 2 > $O/stamps_grid$g.json 2> $O/err$g || { echo STAMPS FAILED; tail $O/err$g; exit 1; }
done
python - <<'PY'
import json
for g in (1,0):
    d=json.load(open(f'gpurun_out/r05p/stamps_grid{g}.json'))
    for r in d['reps']:
        print('grid',g,'ms',round(r['kernel_ms_events'],3),'end p50/p100',r['end'].get('p50'),r['end'].get('p100'),'le16 p50',r['le16_active'].get('p50'),'pool',r['envs_from_grid_pool'],'us/block',r['tail_block_us_mean'])
        for w in r['last_waves'][:3]: print('   ',w)
PY
echo ALL OK
