#!/bin/bash
# Round 6: MT staged walk -- thresholds as u32 high parts (LDS image 14.0 -> 10.9 KiB) to fit a 4th workgroup per CU;
# MT parity on the t32w12 build, then the A/B (tools/mt_ab.py, 2 alternations)
set -o pipefail
O=gpurun_out/r06k; mkdir -p $O
PBNSIM_LIB=$PWD/build_exp/t32w12/libpbnsim.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -k "mt_mode" -x -v --timeout 300 --timeout-method thread > $O/mt_tests.log 2>&1 || { tail -30 $O/mt_tests.log; exit 1; }
tail -3 $O/mt_tests.log
timeout -k 10 500 python -u tools/mt_ab.py 2 build_exp/base/libpbnsim.so build_exp/t32w16/libpbnsim.so build_exp/t32w12/libpbnsim.so build_exp/t32r8a4/libpbnsim.so build_exp/t32r8a8/libpbnsim.so build_exp/basew12/libpbnsim.so > $O/ab.jsonl 2> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
tail -1 $O/ab.jsonl | head -c 300
