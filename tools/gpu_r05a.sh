#!/bin/bash
# Round-5 first GPU pass: the GPU tests, the bench line, the write-width probe, the 8-B store A/B, MT mode.
set -o pipefail
O=gpurun_out/r05a; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS FAILED; tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { echo BENCH FAILED; tail $O/bench.err; exit 1; }
timeout -k 10 200 python tools/write_width.py > $O/write_width.json || exit 1
for rep in 1 2; do
  for L in gym-pbn-stac_amd/gym_pbn_amd/libpbnsim.so build_exp/store8/libpbnsim.so; do
    echo "$L $(PBNSIM_LIB=$PWD/$L timeout -k 10 120 python tools/step_time.py 7)" >> $O/store8_ab.txt || exit 1
  done
done
timeout -k 10 300 python tools/mt_bench.py > $O/mt.json || exit 1
echo ALL OK
