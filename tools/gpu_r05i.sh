#!/bin/bash
# Round 5: tail helpers' poll sleep A/B (1 / 4 / 8 x 64 cycles): lone block cost and the stamps split
set -o pipefail
O=gpurun_out/r05i; mkdir -p $O
for rep in 1 2; do
for L in gym-pbn-stac_amd/gym_pbn_amd/libpbnsim.so build_exp/hs4/libpbnsim.so build_exp/hs8/libpbnsim.so; do
  r=$(PBNSIM_LIB=$PWD/$L timeout -k 10 120 python tools/r6_lone_fit.py 80) || { echo LONE FAILED; exit 1; }
  echo "$r" | python -c "import json,sys; d=json.load(sys.stdin); print('$L', 'us/64', round(d['us_per_block'],4), 'fixed', round(d['fixed_us'],2), 'waits', d['ring_waits'], 'of', d['ring_blocks'])" | tee -a $O/sleep_ab.txt
done
done
PBNSIM_LIB=$PWD/build_exp/stamps_hs4/libpbnsim.so timeout -k 10 120 python tools/tail_stamps.py ring > $O/stamps_ring_hs4.json 2> $O/err1 || { echo STAMPS FAILED; tail $O/err1; exit 1; }
python -c "
import json; d=json.load(open('$O/stamps_ring_hs4.json')); print({k:d.get(k) for k in ('tail_blocks','cycles_per_block','cycles_top_to_next_prepared','cycles_fixed_point','cycles_rest','rounds_per_block')})"
echo ALL OK
