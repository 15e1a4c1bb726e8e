#!/bin/bash
# Round 5: is the waiting workgroups' residency cost a clock effect? Shader clock in tail blocks (stamps build),
# cap 4,096 per step: pool on, pool with one slot (resident, nothing moved), pool off
set -o pipefail
O=gpurun_out/r05v; mkdir -p $O
S=$PWD/build_exp/stamps/libpbnsim.so
for v in "PBNSIM_ENV_GRID_STEAL=1" "PBNSIM_ENV_GRID_STEAL=1 PBNSIM_ENV_GRID_SLOTS=1" "PBNSIM_ENV_GRID_STEAL=0"; do
  env $v PBNSIM_LIB=$S timeout -k 10 200 python tools/env_stamps.py 131072 4096 3 > $O/tmp.json 2>> $O/err || { echo STAMPS FAILED; tail $O/err; exit 1; }
  python -c "
import json; d=json.load(open('$O/tmp.json'))
print('$v', [(round(r['kernel_ms_events'],3), r['tail_clock_GHz'], r['tail_block_us_mean']) for r in d['reps']])" | tee -a $O/clock.txt
done
echo ALL OK
