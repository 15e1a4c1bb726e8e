#!/usr/bin/env python3
"""HBM traffic of the step kernel from rocprofv3 PMC counters -> profiles/pmc_traffic.json.

Per MI355X_MICROARCH.md §HBM / cdna_hip_programming.md §7: FETCH_SIZE and WRITE_SIZE
are collected in SEPARATE passes (they do not fit one TCC pass), with --kernel-trace
only (no sys/runtime trace). Units are KiB. gfx950 correction: FETCH_SIZE reports
exactly half of the bytes of a wide coalesced streaming read, so it is doubled;
WRITE_SIZE is exact for 16-B-per-lane streaming stores.

Runs rocprofv3 as a CHILD process (this script never touches the GPU itself).
"""

from __future__ import annotations

import csv
import json
import statistics
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]


def run_pass(counter: str, outdir: Path, network: str, batch: int, steps: int) -> list:
    cmd = ["rocprofv3", "--pmc", counter, "--kernel-trace", "--output-format", "csv", "-d", str(outdir), "-o", "run",
           "--", sys.executable, str(ROOT / "bench.py"), "--kernel-only", "--steps", str(steps), "--warmup", "0",
           "--network", network, "--batch", str(batch)]
    subprocess.run(cmd, check=True, cwd=str(ROOT))
    rows = list(csv.DictReader(open(outdir / "run_counter_collection.csv")))
    rows = [r for r in rows if "k_step" in r["Kernel_Name"] and r["Counter_Name"] == counter]
    rows.sort(key=lambda r: int(r.get("Dispatch_Id", 0)))  # launch order: the window is a range of launches
    return [float(r["Counter_Value"]) for r in rows]


# the launches bench.py's figures are timed over (and its changed fraction q measured over): the headline's
# --warmup 5 --steps 20 at 1M envs, beyond_mall_supplement's 50 + 200 at 8M -- so traffic and alg bytes share q
WINDOWS = {1 << 20: (5, 20), 1 << 23: (50, 200)}


def main():
    network = sys.argv[1] if len(sys.argv) > 1 else "bittner199"
    batch = int(sys.argv[2]) if len(sys.argv) > 2 else 1 << 20
    w0, wn = WINDOWS.get(batch, (0, 40))
    base = ROOT / "gpurun_out" / "pmc"
    fetch = run_pass("FETCH_SIZE", base / "fetch", network, batch, w0 + wn)[w0:w0 + wn]
    write = run_pass("WRITE_SIZE", base / "write", network, batch, w0 + wn)[w0:w0 + wn]
    f_kib, w_kib = statistics.median(fetch), statistics.median(write)
    per_launch = f_kib * 1024 * 2 + w_kib * 1024
    out_path = ROOT / "gpurun_out" / "pmc_traffic.json"  # copied into profiles/ after review
    prev = out_path if out_path.exists() else ROOT / "profiles" / "pmc_traffic.json"  # several sizes, one file
    doc = json.loads(prev.read_text()) if prev.exists() else {}
    doc.setdefault("per_launch_bytes", {})[f"{network}:{batch}"] = per_launch
    doc.setdefault("detail", {})[f"{network}:{batch}"] = {
        "FETCH_SIZE_KiB_median": f_kib, "WRITE_SIZE_KiB_median": w_kib, "dispatches": [len(fetch), len(write)],
        "window": [w0, w0 + wn], "FETCH_SIZE_KiB_mean": statistics.fmean(fetch),
        "WRITE_SIZE_KiB_mean": statistics.fmean(write),
        "read_bytes_corrected": f_kib * 1024 * 2, "write_bytes": w_kib * 1024,
        "alg_bytes": 16 * ((json.loads((ROOT / "gym-pbn-stac_amd/gym_pbn_amd/data/networks.json").read_text())
                            ["networks"].get(network, {}).get("n_nodes", 199) + 63) // 64) * batch,
    }
    import os
    tree = os.environ.get("PMC_TREE", "unknown tree")  # the commit the caller profiled (no .git on the GPU box)
    doc["detail"][f"{network}:{batch}"]["tree"] = tree
    doc["source"] = ("rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes) on bench.py --kernel-only; "
                     "per-launch median over the launches bench.py times (1M: 5..25, 8M: 50..250); FETCH_SIZE x2 (gfx950 wide-read correction), WRITE_SIZE as is; "
                     f"profiled tree {tree}")
    out_path.write_text(json.dumps(doc, indent=1) + "\n")
    print(json.dumps(doc["detail"][f"{network}:{batch}"]))


if __name__ == "__main__":
    main()
