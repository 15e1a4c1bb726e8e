#!/bin/bash
# Round 6: SQ counters of the MT kernels (one --pmc pass each, kernel trace only): k_mt_coop vs k_mt_step (u16)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06g; mkdir -p $O
C="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS"
timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $O/coop -o run -- python3 tools/mt_pmc_child.py > $O/coop.log 2>&1 || exit 1
PBNSIM_MT_LANES=1 timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $O/lanes -o run -- python3 tools/mt_pmc_child.py > $O/lanes.log 2>&1 || exit 1
python3 - <<'PY'
import csv, collections
for tag in ("coop", "lanes"):
    rows = list(csv.DictReader(open(f"gpurun_out/r06g/{tag}/run_counter_collection.csv")))
    agg = collections.defaultdict(float); n = collections.Counter()
    for r in rows:
        if "k_mt" in r["Kernel_Name"] and "seed" not in r["Kernel_Name"]:
            agg[(r["Kernel_Name"][:40], r["Counter_Name"])] += float(r["Counter_Value"]); n[(r["Kernel_Name"][:40], r["Counter_Name"])] += 1
    for k, v in sorted(agg.items()): print(tag, k, v, n[k])
PY
