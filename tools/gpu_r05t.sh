#!/bin/bash
# Round 5: MT mode with double-buffered rows (next generation twisted ahead of use) -- MT tests, then the rates
set -o pipefail
O=gpurun_out/r05t; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -k "mt" -x -q --timeout 240 --timeout-method thread > $O/mt_tests.log 2>&1 || { echo MT TESTS FAILED; tail -30 $O/mt_tests.log; exit 1; }
tail -2 $O/mt_tests.log
timeout -k 10 300 python tools/mt_bench.py > $O/mt.json 2> $O/err || { echo MT FAILED; tail $O/err; exit 1; }
python -c "
import json; d=json.loads(open('$O/mt.json').read().splitlines()[-1]); print([(r['B'], r['T'], round(r['node_updates_per_s']/1e9,1), round(r['frac_of_8TBs'],3)) for r in d['mt_mode']])"
echo ALL OK
