#!/usr/bin/env python3
"""VALU roofline inputs for the compute-bound kernels -> gpurun_out/r06_valu_pmc.json (copied to
profiles/ after review; bench.py reads it for the rollout and config-5 rooflines).

One rocprofv3 --pmc pass (kernel trace only; 5 SQ counters + 1 GRBM counter, within one pass's
limits) over tools/valu_pmc_child.py, which runs the bench line's rollout (1M envs, T = 64) and
config-5 R6 chunks (131,072 envs, T = 100; fused and one launch per env step) with the bench's
seeds and logs every launch's node updates. Per kernel configuration:
  valu_wave_insts_per_update = sum SQ_INSTS_VALU / sum node updates (wave64 instructions)
  valu_busy_frac             = SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES (both quad-cycles; the share of
                               wave time spent issuing VALU)
  active_lane_frac           = SQ_THREAD_CYCLES_VALU / (SQ_ACTIVE_INST_VALU x 64): the mean share of a
                               wave's 64 lanes enabled in its VALU instructions (rocprofv3's derived
                               VALUUtilization / 100); lane-ops x this = useful lane-ops
  effective_clock_GHz        = GRBM_GUI_ACTIVE / 8 XCDs / kernel wall time (MI355X_MICROARCH.md
                               'DVFS give-back'; reads high on dispatches under ~0.3 ms)
The first launch of each configuration is dropped (warm-up). Runs rocprofv3 as a CHILD process.

`valu_pmc.py lds`: the same launches with LDS counters -> gpurun_out/r04_lds_pmc.json:
  lds_insts_per_update       = SQ_INSTS_LDS / node updates (wave instructions)
  bank_conflict_frac         = SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE (extra cycles over all LDS-array
                               cycles, MI355X_MICROARCH.md LDS)
  lds_cycles_per_update      = SQ_LDS_IDX_ACTIVE / node updates
  lds_issue_stall_frac       = SQ_WAIT_INST_LDS / SQ_WAVE_CYCLES
"""
import collections
import csv
import json
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
SETS = {"valu": ["SQ_INSTS_VALU", "SQ_ACTIVE_INST_VALU", "SQ_THREAD_CYCLES_VALU", "SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES",
                 "GRBM_GUI_ACTIVE"],
        "lds": ["SQ_INSTS_LDS", "SQ_ACTIVE_INST_LDS", "SQ_WAIT_INST_LDS", "SQ_LDS_BANK_CONFLICT", "SQ_LDS_IDX_ACTIVE",
                "SQ_WAVE_CYCLES", "SQ_INSTS_VALU", "GRBM_GUI_ACTIVE"],
        # issue vs dependency-latency breakdown of the R6 kernels
        "stall": ["SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_SCA", "SQ_ACTIVE_INST_LDS",
                  "SQ_ACTIVE_INST_MISC", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_WAVE_CYCLES", "GRBM_GUI_ACTIVE"],
        "insts": ["SQ_INSTS_SALU", "SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_SMEM", "SQ_INSTS_BRANCH", "SQ_WAVES",
                  "SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES", "GRBM_GUI_ACTIVE"]}
SET = sys.argv[1] if len(sys.argv) > 1 else "valu"
COUNTERS = SETS[SET]


def main():
    outdir = ROOT / "gpurun_out" / f"{SET}_pmc"
    cmd = ["rocprofv3", "--pmc", *COUNTERS, "--kernel-trace", "--output-format", "csv", "-d", str(outdir), "-o",
           "run", "--", sys.executable, str(ROOT / "tools" / "valu_pmc_child.py")]
    subprocess.run(cmd, check=True, cwd=str(ROOT))
    log = json.loads((ROOT / "gpurun_out" / "valu_child.json").read_text())
    files = list(outdir.rglob("*counter_collection.csv"))
    rows = list(csv.DictReader(open(files[0])))
    disp = collections.OrderedDict()
    for r in rows:
        name = r["Kernel_Name"]
        if not ("k_env" in name or "k_rollout" in name):
            continue
        d = disp.setdefault(int(r["Dispatch_Id"]), {"name": name, "t": 0.0})
        d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        if "Start_Timestamp" in r and r.get("End_Timestamp"):
            d["t"] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    seq = [disp[k] for k in sorted(disp)]
    if len(seq) != len(log):
        raise SystemExit(f"{len(seq)} profiled dispatches vs {len(log)} logged launches")
    groups = collections.OrderedDict()
    for d, (kind, key, ups) in zip(seq, log):
        assert kind in d["name"], (kind, d["name"])
        groups.setdefault(key, []).append((d, ups))
    res = {}
    for key, items in groups.items():
        items = items[1:] if len(items) > 1 else items  # drop the warm-up launch
        ups = sum(u for _, u in items)
        tot = {c: sum(d.get(c, 0.0) for d, _ in items) for c in COUNTERS}
        wall = sum(d["t"] for d, _ in items)
        if SET in ("stall", "insts"):
            wc = max(tot["SQ_WAVE_CYCLES"], 1)
            gui = tot["GRBM_GUI_ACTIVE"]
            r = {"kernel": items[0][0]["name"], "launches": len(items), "node_updates": ups, "profiled_kernel_s": wall,
                 # SQ_WAVE_CYCLES counts quad-cycles summed over waves (MI355X_MICROARCH.md): x 4 / (1,024 SIMDs x
                 # the kernel's cycles, GRBM_GUI_ACTIVE / 8 XCDs) = mean resident waves per SIMD
                 "resident_waves_per_simd": (4 * wc) / (1024 * gui / 8) if gui else None,
                 "counters": tot, "source": "rocprofv3 --pmc " + " ".join(COUNTERS) + " --kernel-trace on "
                                            "tools/valu_pmc_child.py"}
            if SET == "stall":  # shares of wave time (all quad-cycle counters)
                for c in ("SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_SCA", "SQ_ACTIVE_INST_LDS",
                          "SQ_ACTIVE_INST_MISC", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY"):
                    r[c.lower().replace("sq_", "") + "_frac"] = tot[c] / wc
            else:  # instructions per node update
                for c in ("SQ_INSTS_SALU", "SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_SMEM", "SQ_INSTS_BRANCH"):
                    r[c.lower().replace("sq_insts_", "") + "_insts_per_update"] = tot[c] / ups
                r["busy_frac"] = tot["SQ_BUSY_CYCLES"] / max(gui / 8, 1)
            res[key] = r
            continue
        if SET == "lds":
            res[key] = {"kernel": items[0][0]["name"], "launches": len(items), "node_updates": ups,
                        "lds_insts_per_update": tot["SQ_INSTS_LDS"] / ups,
                        "valu_wave_insts_per_update": tot["SQ_INSTS_VALU"] / ups,
                        "bank_conflict_frac": tot["SQ_LDS_BANK_CONFLICT"] / max(tot["SQ_LDS_IDX_ACTIVE"], 1),
                        "lds_cycles_per_update": tot["SQ_LDS_IDX_ACTIVE"] / ups,
                        "lds_issue_stall_frac": tot["SQ_WAIT_INST_LDS"] / max(tot["SQ_WAVE_CYCLES"], 1),
                        "profiled_kernel_s": sum(d["t"] for d, _ in items), "counters": tot,
                        "source": "rocprofv3 --pmc " + " ".join(COUNTERS) + " --kernel-trace on tools/valu_pmc_child.py"}
            continue
        res[key] = {"kernel": items[0][0]["name"], "launches": len(items), "node_updates": ups,
                    "valu_wave_insts_per_update": tot["SQ_INSTS_VALU"] / ups,
                    "valu_busy_frac": tot["SQ_ACTIVE_INST_VALU"] / max(tot["SQ_WAVE_CYCLES"], 1),
                    "active_lane_frac": tot["SQ_THREAD_CYCLES_VALU"] / max(tot["SQ_ACTIVE_INST_VALU"] * 64, 1),
                    "effective_clock_GHz": (tot["GRBM_GUI_ACTIVE"] / 8 / wall / 1e9) if wall else None,
                    "profiled_kernel_s": wall, "counters": tot,
                    "source": "rocprofv3 --pmc " + " ".join(COUNTERS) + " --kernel-trace on tools/valu_pmc_child.py"}
    doc = {"kernels": res, "valu_peak": "256 CUs x 4 SIMD32 x 32 lanes/clk x 2.4 GHz = 78.6 T lane-ops/s "
                                        "(MI355X_MICROARCH.md: chip parameters, wave scheduling)"}
    (ROOT / "gpurun_out" / f"r06_{SET}_pmc.json").write_text(json.dumps(doc, indent=1) + "\n")
    print(json.dumps({k: {kk: v for kk, v in r.items() if kk not in ("counters", "source", "kernel")}
                      for k, r in res.items()}))


if __name__ == "__main__":
    main()
