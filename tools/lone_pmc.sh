#!/bin/bash
# SQ counters over the lone-chain R6 run (tools/r6_lone_wave.py, lane mode): where a lone wave's
# cycles go (measurement only). Two rocprofv3 --pmc passes, kernel trace only.
# Usage (GPU box): bash tools/lone_pmc.sh  -> gpurun_out/lone_pmc_{1,2}/
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
export PBNSIM_ENV_GROUP=1
C1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU"
C2="SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM SQ_WAVES SQ_INSTS_VMEM"
timeout -s KILL 120 rocprofv3 --pmc $C1 --kernel-trace --output-format csv -d gpurun_out/lone_pmc_1 -o run -- python3 tools/r6_lone_wave.py > gpurun_out/lone_pmc_1.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc $C2 --kernel-trace --output-format csv -d gpurun_out/lone_pmc_2 -o run -- python3 tools/r6_lone_wave.py > gpurun_out/lone_pmc_2.log 2>&1 || exit $?
