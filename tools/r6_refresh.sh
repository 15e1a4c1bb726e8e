#!/bin/bash
# Refresh the R6 measurements in profiles/ for the current kernels (GPU box): lane-mode timings at
# 131,072 and 1M envs, one capped chain alone, and the VALU PMC pass the bench line reads.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
export TMPDIR=/tmp
O=gpurun_out/final
mkdir -p $O
run() {
  local label=$1 tmo=$2; shift 2
  echo "=== [$label] $(date +%T)"
  timeout -k 10 "$tmo" "$@" > $O/$label.out 2> $O/$label.err
  local rc=$?
  echo "=== [$label] rc=$rc"; tail -n 2 $O/$label.out
  [ $rc -eq 0 ] || exit $rc
}
run r6_lane_131k 200 python tools/r6_group_sweep.py 131072 1
run r6_lane_1m 200 python tools/r6_group_sweep.py 1048576 1
run r6_lone_lane 100 env PBNSIM_ENV_GROUP=1 python tools/r6_lone_wave.py
run valu_pmc 600 python tools/valu_pmc.py
