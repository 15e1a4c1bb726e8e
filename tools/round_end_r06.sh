#!/bin/bash
# Round-6 measurement set (GPU box): the HBM-traffic PMC passes at 1M and 8M envs over the launches bench.py
# times (separate FETCH_SIZE / WRITE_SIZE runs, tagged with the profiled tree), then the bench line (the driver's
# command) reading them, its rocprofv3 kernel stats and run split, and the VALU PMC pass.
# Usage: PMC_TREE=<commit> bash tools/round_end_r06.sh
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
export TMPDIR=/tmp
O=gpurun_out/final6
mkdir -p $O
rm -f gpurun_out/pmc_traffic.json
run() {
  local label=$1 tmo=$2; shift 2
  echo "=== [$label] $(date +%T) $*"
  timeout -k 10 "$tmo" "$@" > $O/$label.out 2> $O/$label.err
  local rc=$?
  echo "=== [$label] rc=$rc"; tail -n 3 $O/$label.out | cut -c1-300
  [ $rc -eq 0 ] || exit $rc
}
run pmc_traffic_1m 300 python tools/pmc_traffic.py bittner199 1048576
run pmc_traffic_8m 300 python tools/pmc_traffic.py bittner199 8388608
cp gpurun_out/pmc_traffic.json profiles/pmc_traffic.json
run bench 300 python bench.py --steps 20 --warmup 5
run bench_prof 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_bench -o bench -- python3 bench.py --steps 20 --warmup 5
run trace_split 60 python tools/trace_split.py $(ls $O/prof_bench/*/bench_kernel_trace.csv $O/prof_bench/bench_kernel_trace.csv 2>/dev/null | head -n 1)
run valu_pmc 400 python tools/valu_pmc.py
