#!/bin/bash
# Round 5: where the ring session's block goes (stamps build), helpers on / off
set -o pipefail
O=gpurun_out/r05g; mkdir -p $O
PBNSIM_LIB=$PWD/build_exp/stamps/libpbnsim.so timeout -k 10 120 python tools/tail_stamps.py ring > $O/stamps_ring.json 2> $O/err1 || { echo STAMPS FAILED; tail $O/err1; exit 1; }
PBNSIM_ENV_HELPERS=0 PBNSIM_LIB=$PWD/build_exp/stamps/libpbnsim.so timeout -k 10 120 python tools/tail_stamps.py ring > $O/stamps_ring_off.json 2> $O/err2 || { echo STAMPS2 FAILED; tail $O/err2; exit 1; }
for f in $O/stamps_ring.json $O/stamps_ring_off.json; do python -c "
import json,sys; d=json.load(open('$f')); print('$f', {k:d.get(k) for k in ('tail_blocks','cycles_per_block','us_per_block_realtime','cycles_top_to_next_prepared','cycles_fixed_point','cycles_rest','rounds_per_block','blocks_by_rounds')})"; done
echo ALL OK
