#!/usr/bin/env python3
"""Summarise tools/sqpmc.sh output: per-kernel mean of each counter (+ VALU busy fraction)."""
import collections
import csv
import sys
from pathlib import Path

for d in sys.argv[1:]:
    rows = list(csv.DictReader(open(Path(d) / "run_counter_collection.csv")))
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in rows:
        k = r["Kernel_Name"]
        if "k_env" in k or "k_step" in k:
            agg[k.split("(")[0]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, c in agg.items():
        m = {n: sum(v) / len(v) for n, v in c.items()}
        print(d, k, {n: f"{v:.3g}" for n, v in m.items()},
              "valu_frac_of_wave_cycles=%.2f" % (m.get("SQ_ACTIVE_INST_VALU", 0) / max(m.get("SQ_WAVE_CYCLES", 1), 1)))
