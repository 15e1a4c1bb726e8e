#!/bin/bash
# SQ counters (one rocprofv3 --pmc pass, kernel trace only) for the env kernel and the step kernel.
# Usage (GPU box): bash tools/sqpmc.sh <tag>   -> gpurun_out/sqpmc_<tag>_{env,step}/
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
tag=${1:-x}
C="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU"
timeout -k 10 300 rocprofv3 --pmc $C --kernel-trace --output-format csv -d gpurun_out/sqpmc_${tag}_env -o run -- python3 tools/bench_env.py ${SQ_B:-1048576} 2 > gpurun_out/sqpmc_${tag}_env.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc $C --kernel-trace --output-format csv -d gpurun_out/sqpmc_${tag}_step -o run -- python3 bench.py --kernel-only --steps 50 --warmup 0 > gpurun_out/sqpmc_${tag}_step.log 2>&1 || exit $?
