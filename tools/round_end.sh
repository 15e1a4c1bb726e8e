#!/bin/bash
# Round-end measurement set (GPU box): the bench line (the driver's command) and its rocprofv3
# kernel stats + run split, config-5 R6 kernel timings (lane mode, 131,072 and 1M envs), one
# capped chain alone, VALU and HBM-traffic PMC passes. Outputs under gpurun_out/final/; the judged
# summaries are copied into profiles/ afterwards. Stops at the first failing step.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
export TMPDIR=/tmp
O=gpurun_out/final
mkdir -p $O
run() {
  local label=$1 tmo=$2; shift 2
  echo "=== [$label] $(date +%T) $*"
  timeout -k 10 "$tmo" "$@" > $O/$label.out 2> $O/$label.err
  local rc=$?
  echo "=== [$label] rc=$rc"; tail -n 3 $O/$label.out
  [ $rc -eq 0 ] || exit $rc
}
run bench 300 python bench.py --steps 20 --warmup 5
run bench_prof 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_bench -o bench -- python3 bench.py --steps 20 --warmup 5
run trace_split 60 python tools/trace_split.py $(ls $O/prof_bench/*/bench_kernel_trace.csv $O/prof_bench/bench_kernel_trace.csv 2>/dev/null | head -n 1)
run r6_lane_131k 200 python tools/r6_group_sweep.py 131072 1
run r6_lane_1m 200 python tools/r6_group_sweep.py 1048576 1
run r6_lone_lane 100 env PBNSIM_ENV_GROUP=1 PBNSIM_ENV_LANES=64 python tools/r6_lone_wave.py
run r6_lone_tail 100 env PBNSIM_ENV_GROUP=1 python tools/r6_lone_wave.py
run valu_pmc 600 python tools/valu_pmc.py
run pmc_traffic 600 python tools/pmc_traffic.py
