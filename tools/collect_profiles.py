#!/usr/bin/env python3
"""Copy the judged measurement summaries of tools/refresh_profiles.sh from gpurun_out/ into profiles/.

Also writes r01_bench_trace_check.json: the rocprofv3 kernel-trace average of the step kernel over
the timed launches only (the first --warmup launches excluded), next to bench.py's HIP-event average.
"""
import csv
import json
import shutil
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
G, P = ROOT / "gpurun_out", ROOT / "profiles"
tag = sys.argv[1] if len(sys.argv) > 1 else "r01"

lines = [l for l in (G / "bench_full.json").read_text().splitlines() if l.startswith("{")]
bench = json.loads(lines[-1])
(P / f"{tag}_bench.json").write_text(json.dumps(bench) + "\n")
shutil.copy(G / "prof_bench" / "bench_kernel_stats.csv", P / f"{tag}_bench_kernel_stats.csv")
rows = [r for r in csv.DictReader(open(G / "prof_bench" / "bench_kernel_trace.csv"))
        if "k_step<4, 1, 1, 0, 1024>" in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
d = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rows]
w, n = bench["warmup"], bench["steps"]
check = {"kernel": "pbn::k_step<4, 1, 1, 0, 1024>", "launches": len(d), "warmup_excluded": w,
         "rocprof_avg_us_timed": sum(d[w:w + n]) / len(d[w:w + n]) / 1e3, "rocprof_avg_us_all": sum(d) / len(d) / 1e3,
         "bench_hip_event_avg_us": bench["roofline"]["avg_kernel_us"],
         "command": "rocprofv3 --kernel-trace --stats -- python3 bench.py (same defaults as the bench line)"}
prof_line = G / "bench_prof.json"
if prof_line.exists():  # bench.py's own HIP-event average in the profiled process (same launches)
    pl = [l for l in prof_line.read_text().splitlines() if l.startswith("{")]
    if pl:
        check["profiled_run_hip_event_avg_us"] = json.loads(pl[-1])["roofline"]["avg_kernel_us"]
        check["note"] = ("rocprof_avg_us_timed and profiled_run_hip_event_avg_us come from the same profiled "
                         "process; bench_hip_event_avg_us is the unprofiled bench line (kernel tracing adds a "
                         "completion signal per dispatch)")
(P / f"{tag}_bench_trace_check.json").write_text(json.dumps(check, indent=1) + "\n")
shutil.copy(G / "pmc_traffic.json", P / "pmc_traffic.json")
for k in ("fetch", "write"):
    src = G / "pmc" / k / "run_counter_collection.csv"
    if src.exists():
        shutil.copy(src, P / f"{tag}_pmc_{k}_size.csv")
shutil.copy(G / "prof_env" / "env_kernel_stats.csv", P / f"{tag}_env_kernel_stats.csv")
bm = G / "beyond_mall.json"
if bm.exists():
    ls = [l for l in bm.read_text().splitlines() if l.startswith("{")]
    (P / f"{tag}_beyond_mall_8m.json").write_text(json.dumps(json.loads(ls[-1])["beyond_mall_8m"], indent=1) + "\n")
if (G / "prof_aux" / "aux_kernel_stats.csv").exists():
    shutil.copy(G / "prof_aux" / "aux_kernel_stats.csv", P / f"{tag}_aux_kernel_stats.csv")
for src, dst in (("aux.json", "aux_kernels.json"), ("torch_env.json", "torch_env.json"),
                 ("single_env.json", "single_env.json")):
    if (G / src).exists():
        ls = [l for l in (G / src).read_text().splitlines() if l.startswith("{")]
        (P / f"{tag}_{dst}").write_text(ls[-1] + "\n")
for src in ("rollout_group_sweep.txt", "ssd_time.txt"):  # text tables of the measurement helpers
    if (G / src).exists():
        ls = [l for l in (G / src).read_text().splitlines() if "=" in l and not l.startswith("/opt")]
        (P / f"{tag}_{src}").write_text("\n".join(ls) + "\n")
for n in ("r6_131k", "r6_1m"):
    ls = [l for l in (G / f"{n}.json").read_text().splitlines() if l.startswith("{")]
    (P / f"{tag}_config5_{n[3:]}.json").write_text(ls[-1] + "\n")
print(json.dumps(check))
