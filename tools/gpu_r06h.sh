#!/bin/bash
# Round 6: counters of the staged MT walk (k_mt_staged) on bench.py's MT workload: SQ issue/wait, HBM bytes
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06h${TAG}; mkdir -p $O
C="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS"
timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $O/sq -o run -- python3 tools/mt_pmc_child.py > $O/sq.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/fetch -o run -- python3 tools/mt_pmc_child.py > $O/fetch.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/write -o run -- python3 tools/mt_pmc_child.py > $O/write.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES SQ_INSTS_SMEM SQ_INST_CYCLES_VMEM_RD SQ_INSTS_BRANCH --kernel-trace --output-format csv -d $O/vm -o run -- python3 tools/mt_pmc_child.py > $O/vm.log 2>&1 || exit 1
TAG=${TAG} python3 - <<'PY'
import csv, collections
for tag in ("sq", "fetch", "write", "vm"):
    rows = list(csv.DictReader(open(f"gpurun_out/r06h{__import__('os').environ.get('TAG','')}/{tag}/run_counter_collection.csv")))
    agg = collections.defaultdict(float); n = collections.Counter()
    for r in rows:
        if "k_mt" in r["Kernel_Name"] and "seed" not in r["Kernel_Name"]:
            agg[(r["Kernel_Name"][:40], r["Counter_Name"])] += float(r["Counter_Value"]); n[(r["Kernel_Name"][:40], r["Counter_Name"])] += 1
    for k, v in sorted(agg.items()): print(tag, k, v, n[k])
PY
