#!/bin/bash
# A/B of R6 env-kernel builds (measurement only), alternating the builds twice: config-5 chunk
# (131,072 envs, lane mode) fused and per step (tools/r6_group_sweep.py), 1M envs fused and per
# step, and one capped chain alone on a SIMD (tools/r6_lone_wave.py, lane mode).
# Usage: tools/r6_ab.sh lib1.so lib2.so ...
for rep in 1 2; do
  for L in "$@"; do
    echo "$L 131k: $(PBNSIM_LIB=$PWD/$L timeout -k 5 100 python tools/r6_group_sweep.py 131072 1 2>/dev/null)" || exit 1
    echo "$L 1M: $(PBNSIM_LIB=$PWD/$L timeout -k 5 100 python tools/r6_group_sweep.py 1048576 1 2>/dev/null)" || exit 1
    echo "$L lone: $(PBNSIM_ENV_GROUP=1 PBNSIM_LIB=$PWD/$L timeout -k 5 60 python tools/r6_lone_wave.py 2>/dev/null)" || exit 1
  done
done
