#!/bin/bash
# Round 6: MT walk A/B of experiment builds against the current library (tools/mt_ab.py, 3 alternations) after the
# MT parity tests on the first experiment build; usage: TAG=... bash tools/gpu_r06o.sh build_exp/X ...
set -o pipefail
O=gpurun_out/${TAG:-r06o}; mkdir -p $O
PBNSIM_LIB=$PWD/$1/libpbnsim.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -k "mt_mode" -x -v --timeout 300 --timeout-method thread > $O/mt_tests.log 2>&1 || { tail -30 $O/mt_tests.log; exit 1; }
tail -3 $O/mt_tests.log
libs="gym-pbn-stac_amd/gym_pbn_amd/libpbnsim.so"; for d in "$@"; do libs="$libs $d/libpbnsim.so"; done
timeout -k 10 500 python -u tools/mt_ab.py 3 $libs > $O/ab.jsonl 2> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
tail -1 $O/ab.jsonl | head -c 200
