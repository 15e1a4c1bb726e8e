"""Measurement tooling that the profiles/ figures are reproduced with (CPU, synthetic inputs)."""

import csv
import json
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]


def test_trace_split_separates_runs(tmp_path):
    """tools/trace_split.py: back-to-back launches of the step kernel form one run; an idle gap
    longer than --gap starts the next; other kernels and runs shorter than --min-launches are left out."""
    cols = ["Kind", "Dispatch_Id", "Kernel_Name", "Start_Timestamp", "End_Timestamp"]
    rows, t, d = [], 1_000_000, 0

    def launch(name, dur_ns, gap_ns=0):
        nonlocal t, d
        t += gap_ns
        d += 1
        rows.append({"Kind": "KERNEL_DISPATCH", "Dispatch_Id": d, "Kernel_Name": name, "Start_Timestamp": t,
                     "End_Timestamp": t + dur_ns})
        t += dur_ns

    step = "void pbn::k_step<4, 1, 1, 0, 1024>(pbn::StepArgs)"
    for _ in range(5):
        launch(step, 10_000)
    launch("void pbn::k_init<4>(pbn::InitArgs)", 3_000, 200_000)
    for k in range(20):
        launch(step, 9_000 + 100 * (k % 3), 200_000 if k == 0 else 500)
    launch(step, 12_000, 5_000_000)  # a lone launch: dropped
    p = tmp_path / "trace.csv"
    with open(p, "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=cols)
        w.writeheader()
        w.writerows(rows)
    out = subprocess.run([sys.executable, str(ROOT / "tools" / "trace_split.py"), str(p)], capture_output=True,
                         text=True, check=True).stdout
    runs = json.loads(out)["runs"]
    assert [r["launches"] for r in runs] == [5, 20]
    assert abs(runs[1]["mean_us"] - sum(9.0 + 0.1 * (k % 3) for k in range(20)) / 20) < 1e-9
    assert runs[1]["first_dispatch"] == 7
