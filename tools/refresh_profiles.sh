#!/bin/bash
# Round-end measurement set (GPU box): bench line, rocprofv3 kernel stats, PMC traffic, env/R6 benches.
# Outputs under gpurun_out/; the judged summaries are copied into profiles/ afterwards.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
set -o pipefail
step() { echo "=== $1 ($(date +%T))"; shift; "$@"; rc=$?; echo "=== rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
echo bench; timeout -k 10 300 python bench.py > gpurun_out/bench_full.json 2> gpurun_out/bench_full.err || exit $?
echo stats; timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_bench -o bench -- python3 bench.py > gpurun_out/bench_prof.json 2> gpurun_out/bench_prof.err || exit $?
step pmc timeout -k 10 600 python tools/pmc_traffic.py
echo beyond; timeout -k 10 200 python bench.py --steps 200 --warmup 50 --beyond-mall --no-config2 --r6-chunks 0 --no-cpu-baseline --rollout 0 > gpurun_out/beyond_mall.json || exit $?
step envstats timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_env -o env -- python3 tools/bench_env.py 1048576 3
step r6_131k timeout -k 10 300 python tools/bench_r6.py --batch 131072 --chunks 4 --warmup 2 > gpurun_out/r6_131k.json
step r6_1m timeout -k 10 300 python tools/bench_r6.py --batch 1048576 --chunks 2 --warmup 1 > gpurun_out/r6_1m.json
step aux timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_aux -o aux -- python3 tools/bench_aux.py
echo auxjson; timeout -k 10 300 python tools/bench_aux.py > gpurun_out/aux.json || exit $?
echo torchenv; timeout -k 10 200 python tools/bench_torch_env.py 1048576 10 > gpurun_out/torch_env.json || exit $?
echo single; timeout -k 10 200 python tools/bench_single_env.py > gpurun_out/single_env.json || exit $?
echo rgsweep; timeout -k 10 200 python tools/rollout_group_sweep.py > gpurun_out/rollout_group_sweep.txt || exit $?
echo ssdtime; timeout -k 10 200 python tools/ssd_time.py > gpurun_out/ssd_time.txt || exit $?
