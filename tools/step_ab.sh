#!/bin/bash
# A/B of step/rollout kernel builds (measurement only), alternating builds twice: the bench line
# (the driver's command: --steps 20 --warmup 5, headline value + kernel us) and the rollout
# sweep (tools/rollout_sweep.py, first repetition).  Usage: tools/step_ab.sh lib1.so lib2.so ...
for rep in 1 2; do
  for L in "$@"; do
    echo -n "$L bench: "
    PBNSIM_LIB=$PWD/$L timeout -k 5 200 python bench.py --steps 20 --warmup 5 2>/dev/null | tail -1 \
      | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print(round(d['value']/1e9,2), 'G', round(d['ms_per_step']*1e3,2), 'us', 'frac', round(r['frac'],3), 'q', r.get('changed_env_frac'), 'kern_us', round(r['avg_kernel_us'],2), 'hbm8m_us', round((r.get('hbm_8m') or {}).get('avg_kernel_us') or 0,1))" || exit 1
    echo "$L rollout: $(PBNSIM_LIB=$PWD/$L timeout -k 5 120 python tools/rollout_sweep.py 2>/dev/null | head -4 | tr '\n' ' ')" || exit 1
  done
done
