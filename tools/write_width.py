#!/usr/bin/env python3
"""the step pattern's no-compute floor (tools/mall_probe.hip, 1024-thread groups,
env pairs, 32 B read per env) with the changed envs written back whole (32 B), as their 16-B half, or
only the 8-B word holding the updated node; 1M (MALL-resident) and 8M envs (past the MALL), several
changed fractions. Measurement only: python tools/write_width.py"""
import ctypes
import json
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
lib = ctypes.CDLL(str(ROOT / "tools" / "libmallprobe.so"))
lib.mall_probe_wbytes.argtypes = [ctypes.c_uint64, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                  ctypes.POINTER(ctypes.c_double)]
out = {}
for rep in range(2):
    for n in (1 << 20, 1 << 23):
        for pct in (9, 30, 44, 100):
            for wb in (32, 16, 8):
                us = ctypes.c_double()
                rc = lib.mall_probe_wbytes(n, pct, wb, 200 if n == 1 << 20 else 50, ctypes.byref(us))
                assert rc == 0, rc
                out.setdefault(f"{n}:{pct}:{wb}B", []).append(round(us.value, 2))
print(json.dumps(out))
