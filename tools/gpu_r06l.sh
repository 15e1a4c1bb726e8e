#!/bin/bash
# Round 6: MT walk with fewer VALU per iteration (window word address from pos in three ops, k53 halves by alignbit,
# the loop test as the AND of two compares' lane masks) -- MT parity on the new build, then the A/B vs HEAD's walk
set -o pipefail
O=gpurun_out/${TAG:-r06l}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -k "mt_mode" -x -v --timeout 300 --timeout-method thread > $O/mt_tests.log 2>&1 || { tail -30 $O/mt_tests.log; exit 1; }
tail -3 $O/mt_tests.log
timeout -k 10 500 python -u tools/mt_ab.py 3 build_exp/base/libpbnsim.so build_exp/prev/libpbnsim.so build_exp/new/libpbnsim.so > $O/ab.jsonl 2> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
tail -1 $O/ab.jsonl | head -c 300
