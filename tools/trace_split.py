#!/usr/bin/env python3
"""Split a rocprofv3 kernel trace into runs of back-to-back launches of one kernel.

bench.py launches the same step kernel (k_step<4,1,1,0,1024>, same grid) for the 8M-env
supplement, the headline's warm-up + timed launches and the twin batch that measures the changed
fraction, so the --stats average mixes sizes. A run = consecutive dispatches of the kernel whose
start follows the previous end by less than --gap microseconds. Prints one JSON object: every
run's launch count, mean / min / max duration (us) and first dispatch id; the headline's K timed
launches are the run of length K right after its W warm-up launches (the host syncs between the
two leave the GPU idle for tens of microseconds, so they are separate runs at the default gap).

Usage: trace_split.py <kernel_trace.csv> [--kernel SUBSTR] [--gap US] [--min-launches N]
"""
import argparse
import csv
import json


def main():
    p = argparse.ArgumentParser()
    p.add_argument("trace")
    p.add_argument("--kernel", default="k_step<4, 1, 1, 0, 1024>")
    p.add_argument("--gap", type=float, default=10.0)
    p.add_argument("--min-launches", type=int, default=2, help="runs shorter than this are left out")
    a = p.parse_args()
    rows = [r for r in csv.DictReader(open(a.trace)) if a.kernel in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    runs, cur, prev_end = [], [], None
    for r in rows:
        st, en = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if cur and (st - prev_end) / 1e3 > a.gap:
            runs.append(cur)
            cur = []
        cur.append((int(r["Dispatch_Id"]), (en - st) / 1e3))
        prev_end = en
    if cur:
        runs.append(cur)
    out = [{"first_dispatch": run[0][0], "launches": len(run), "mean_us": sum(d for _, d in run) / len(run),
            "min_us": min(d for _, d in run), "max_us": max(d for _, d in run)}
           for run in runs if len(run) >= a.min_launches]
    print(json.dumps({"kernel": a.kernel, "gap_us": a.gap, "runs": out}, indent=1))


if __name__ == "__main__":
    main()
