#!/bin/bash
# Round 5: R6 + MT tests with the tail helpers and the new MT kernel, the helpers' A/B at config 5's shard
# (with tail thresholds 16 / 32), MT-mode throughput.
set -o pipefail
O=gpurun_out/r05b; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "mt_mode" -x -q --timeout 120 --timeout-method thread > $O/mt_tests.log 2>&1 || { echo MT TESTS FAILED; tail -40 $O/mt_tests.log; exit 1; }
tail -2 $O/mt_tests.log
timeout -k 10 200 python tools/mt_bench.py > $O/mt.json 2>&1 || { echo MT BENCH FAILED; tail $O/mt.json; exit 1; }
tail -1 $O/mt.json
timeout -k 10 400 python -u -m pytest tests/test_r6_regimes.py -x -q --timeout 240 --timeout-method thread > $O/r6_tests.log 2>&1 || { echo R6 TESTS FAILED; tail -40 $O/r6_tests.log; exit 1; }
tail -2 $O/r6_tests.log
timeout -k 10 500 python tools/r6_env_ab.py 131072 10 2 fixture:4096,fixture:1048576,spec:1048576 'PBNSIM_ENV_HELPERS=1' 'PBNSIM_ENV_HELPERS=0' 'PBNSIM_ENV_HELPERS=1 PBNSIM_ENV_TAIL=32' > $O/helpers_ab.jsonl 2> $O/helpers_ab.err || { echo AB FAILED; tail $O/helpers_ab.err; exit 1; }
echo ALL OK
