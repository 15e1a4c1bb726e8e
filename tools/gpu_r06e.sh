#!/bin/bash
# Round 6: MT-mode A/B -- u16 draws + reload (mtreload) vs the same with an LDS-DMA touch of the line 2 / 4 lines
# ahead when a lane enters a new 128-B line of its row (mtT2, mtT4), and mtT2 at 6-draw chunks (6 workgroups/CU)
set -o pipefail
O=gpurun_out/r06e; mkdir -p $O
timeout -k 10 600 python tools/mt_ab.py 2 build_exp/mtreload/libpbnsim.so build_exp/mtT2/libpbnsim.so build_exp/mtT2c6/libpbnsim.so build_exp/mtT4/libpbnsim.so > $O/mt_ab.jsonl 2> $O/mt_ab.err || { echo AB FAILED; tail $O/mt_ab.err; exit 1; }
python - <<'PY'
import json
for l in open('gpurun_out/r06e/mt_ab.jsonl'):
    d=json.loads(l)
    if 'rows' in d: print('bit_exact', d['bit_exact_across_variants']); continue
    print(d['rep'], d['lib'].split('/')[1], d['1048576x256']['G_updates_per_s'], d['65536x512']['G_updates_per_s'])
PY
