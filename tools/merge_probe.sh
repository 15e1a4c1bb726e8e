#!/bin/bash
# Tail-merge probe (measurement only): config-5 per-step and fused at 131,072 envs with the env
# grid capped (PBNSIM_ENV_GRID) at 256 / 512 workgroups, for the given builds.
for g in 256 512; do
  for L in "$@"; do
    echo "$L grid=$g: $(PBNSIM_ENV_GRID=$g PBNSIM_LIB=$PWD/$L timeout -k 5 100 python tools/r6_group_sweep.py 131072 1 2>/dev/null)" || exit 1
  done
done
