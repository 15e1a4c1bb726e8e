#!/bin/bash
# Round 6 final tree: the whole GPU suite, then the round-end measurement set (tools/round_end_r06.sh)
set -o pipefail
mkdir -p gpurun_out/final6  # usage: bash tools/gpu_r06q.sh <tree commit>
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/final6/gpu_tests.log 2>&1 || { tail -20 gpurun_out/final6/gpu_tests.log; exit 1; }
tail -2 gpurun_out/final6/gpu_tests.log
PMC_TREE=$1 bash tools/round_end_r06.sh
