#!/bin/bash
# Round 6: the cooperative MT walk (k_mt_coop) -- MT tests (reference fixtures + oracle on every env, both walks),
# then the A/B against round 5's kernel and the u16-draw per-lane walk
set -o pipefail
O=gpurun_out/r06f; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "mt_mode" -x -v --timeout 120 --timeout-method thread > $O/mt_tests.log 2>&1 || { echo MT TESTS FAILED; tail -40 $O/mt_tests.log; exit 1; }
tail -3 $O/mt_tests.log
timeout -k 10 600 python tools/mt_ab.py 2 build_exp/mtbase/libpbnsim.so build_exp/mtreload/libpbnsim.so gym-pbn-stac_amd/gym_pbn_amd/libpbnsim.so ${EXTRA_LIBS} > $O/mt_ab.jsonl 2> $O/mt_ab.err || { echo AB FAILED; tail $O/mt_ab.err; exit 1; }
python - <<'PY'
import json
for l in open('gpurun_out/r06f/mt_ab.jsonl'):
    d=json.loads(l)
    if 'rows' in d: print('bit_exact', d['bit_exact_across_variants']); continue
    print(d['rep'], d['lib'], d['1048576x256']['G_updates_per_s'], d['65536x512']['G_updates_per_s'])
PY
