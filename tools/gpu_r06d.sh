#!/bin/bash
# Round 6: MT-mode A/B -- round-5 kernel vs u16 draw entries (choice resolved in the generation pass, 6 workgroups
# per CU) with the twisted row's window reloaded / taken from registers (scratch 32 B) / from registers at <= 5 waves
set -o pipefail
O=gpurun_out/r06d; mkdir -p $O
timeout -k 10 600 python tools/mt_ab.py 2 build_exp/mtbase/libpbnsim.so build_exp/mtreload/libpbnsim.so build_exp/mtregwin/libpbnsim.so build_exp/mtregwin5/libpbnsim.so > $O/mt_ab.jsonl 2> $O/mt_ab.err || { echo AB FAILED; tail $O/mt_ab.err; exit 1; }
cat $O/mt_ab.jsonl
