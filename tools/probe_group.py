#!/usr/bin/env python3
"""Memory-floor probe: does writing changed envs in aligned groups (pairs / 128-B lines) cost less
than writing single 32-B envs, at the equivalent dirty fractions? (measurement only)"""
import ctypes
import json
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
lib = ctypes.CDLL(str(ROOT / "tools" / "libmallprobe.so"))
lib.mall_probe_group.argtypes = [ctypes.c_uint64, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                 ctypes.POINTER(ctypes.c_double)]
res = {}
for n in (1 << 20, 1 << 23):
    for q in (0.43, 0.10):  # per-env dirty probability: fresh states / late trajectory
        for g in (0, 1, 2):
            pct = round(100 * (1 - (1 - q) ** (1 << g)))
            us = ctypes.c_double()
            assert lib.mall_probe_group(n, pct, g, 200, ctypes.byref(us)) == 0
            res[f"{n}:q{q}:g{g}:pct{pct}"] = round(us.value, 2)
print(json.dumps(res))
