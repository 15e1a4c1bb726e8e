#!/bin/bash
# Round 6: the whole GPU suite on the tree with the forced-node step, the pool fixes (acquire CAS, sticky fault
# word, slot-less tickets leave), migration removed, and the full-size oracle parity tests (config 5's shard
# every env at cap 4,096 and 2^20, MT mode on every env incl. bench's 1M workload)
set -o pipefail
O=gpurun_out/${OUT:-r06b}; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread --durations=25 > $O/gpu_tests.log 2>&1 || { echo GPU TESTS FAILED; tail -40 $O/gpu_tests.log; exit 1; }
tail -32 $O/gpu_tests.log
echo ALL OK
