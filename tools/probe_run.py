#!/usr/bin/env python3
"""Print the MALL / HBM ceilings of the step-mode access pattern (tools/mall_probe.hip)."""
import ctypes
import json
import sys
from pathlib import Path

lib = ctypes.CDLL(str(Path(__file__).resolve().parent / "libmallprobe.so"))
lib.mall_probe.argtypes = [ctypes.c_uint64, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_double)]
out = []
for B in (1 << 20, 1 << 22, 1 << 23):
    for pct in (0, 45, 100):
        for passes in (1, 16):
            us = ctypes.c_double()
            rc = lib.mall_probe(B, pct, passes, 200 if passes == 1 else 20, ctypes.byref(us))
            alg = 64 * B
            mv = 32 * B * (1 + pct / 100)
            out.append({"B": B, "write_pct": pct, "passes": passes, "rc": rc, "us_per_pass": us.value,
                        "moved_GBs": mv / us.value / 1e3, "alg64_GBs": alg / us.value / 1e3})
            print(json.dumps(out[-1]), flush=True)
