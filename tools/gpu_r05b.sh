#!/bin/bash
# Round 5: R6 tests with the tail helpers, then their A/B at config 5's shard.
set -o pipefail
O=gpurun_out/r05b; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_r6_regimes.py -x -q --timeout 240 --timeout-method thread > $O/r6_tests.log 2>&1 || { echo R6 TESTS FAILED; tail -40 $O/r6_tests.log; exit 1; }
tail -3 $O/r6_tests.log
timeout -k 10 600 python tools/r6_env_ab.py 131072 10 2 fixture:4096,fixture:1048576,spec:1048576 'PBNSIM_ENV_HELPERS=1' 'PBNSIM_ENV_HELPERS=0' > $O/helpers_ab.jsonl 2> $O/helpers_ab.err || { echo AB FAILED; tail $O/helpers_ab.err; exit 1; }
echo ALL OK
