#!/bin/bash
# A/B of R6 env-kernel builds (measurement only): per-step and fused chunk throughput.
# Usage: tools/env_ab.sh lib1.so lib2.so ...   (PBNSIM_ENV_* knobs pass through)
for L in "$@"; do
  for B in 131072 1048576; do
    echo -n "$L B=$B step: "
    PBNSIM_LIB=$PWD/$L timeout -k 5 60 python tools/bench_env.py $B 5 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['s_per_call']*1e3,3),'ms',round(d['node_updates_per_s']/1e9,1),'G/s')" || exit 1
    echo -n "$L B=$B fused: "
    PBNSIM_LIB=$PWD/$L timeout -k 5 90 python tools/bench_r6.py --batch $B --chunks 2 --warmup 1 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['value']/1e6,1),'M env-steps/s',round(d['node_updates_per_s']/1e9,1),'G/s')" || exit 1
  done
done
