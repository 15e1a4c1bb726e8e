#!/bin/bash
# Round 5: phase stamps of one per-step launch at cap 4,096 with the grid pool on / off
set -o pipefail
O=gpurun_out/r05m; mkdir -p $O
for g in 1 0; do
  PBNSIM_ENV_GRID_STEAL=$g PBNSIM_LIB=$PWD/build_exp/stamps/libpbnsim.so timeout -k 10 200 python tools/env_stamps.py 131072 4096 2 > $O/stamps_grid$g.json 2> $O/err$g || { echo STAMPS FAILED; tail $O/err$g; exit 1; }
done
python - <<'PY'
import json
for g in (1,0):
    d=json.load(open(f'gpurun_out/r05m/stamps_grid{g}.json'))
    for r in d['reps']:
        print('grid',g,'ms',round(r['kernel_ms_events'],3),'end',r['end'],'last_block_end',r['last_tail_block_end_us'],'le16',r['le16_active'].get('p50'),'first_idle',r['handoff']['first_idle_us'],'from_pool',r['envs_from_grid_pool'],'blocks',r['tail_blocks'],'us/block',r['tail_block_us_mean'])
PY
echo ALL OK
