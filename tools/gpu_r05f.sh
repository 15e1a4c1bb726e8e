#!/bin/bash
# Round 5: full GPU tests, the bench line, and the R6 issue-vs-latency PMC passes
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05f; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS FAILED; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { echo BENCH FAILED; tail $O/bench.err; exit 1; }
timeout -k 10 400 python tools/valu_pmc.py stall > $O/pmc_stall.out 2> $O/pmc_stall.err || { echo PMC STALL FAILED; tail $O/pmc_stall.err; exit 1; }
tail -c 1500 $O/pmc_stall.out
timeout -k 10 400 python tools/valu_pmc.py insts > $O/pmc_insts.out 2> $O/pmc_insts.err || { echo PMC INSTS FAILED; tail $O/pmc_insts.err; exit 1; }
tail -c 1500 $O/pmc_insts.out
echo ALL OK
