#!/bin/bash
# Round 6: the whole GPU suite on the current tree (one process, per-test time limit)
set -o pipefail
O=gpurun_out/r06j; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?
tail -5 $O/gpu_tests.log
exit $rc
