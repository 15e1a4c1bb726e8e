#!/bin/bash
# Round 6: MT walk with asm LDS-DMA and prefetched circular windows -- parity (both walks) on the default build,
# then the A/B of the window variants on bench.py's MT workload (tools/mt_ab.py, 2 alternations)
set -o pipefail
O=gpurun_out/r06i; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -k "mt_mode" -x -v --timeout 300 --timeout-method thread > $O/mt_tests.log 2>&1 || { tail -30 $O/mt_tests.log; exit 1; }
tail -3 $O/mt_tests.log
timeout -k 10 500 python -u tools/mt_ab.py 2 build_exp/pf0/libpbnsim.so build_exp/pf1/libpbnsim.so build_exp/pf2a2/libpbnsim.so build_exp/pf2a4/libpbnsim.so build_exp/pf2a8/libpbnsim.so build_exp/pf2w32a8/libpbnsim.so build_exp/pf2w32a16/libpbnsim.so > $O/ab.jsonl 2> $O/ab.err || { cat $O/ab.err | tail -20; exit 1; }
tail -1 $O/ab.jsonl | head -c 300
