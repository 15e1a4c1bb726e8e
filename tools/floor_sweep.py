#!/usr/bin/env python3
"""Memory floor of the step-mode access pattern vs the step kernel (measurement only).

tools/libmallprobe.so: read every env's 32 B, write back write_pct % of them, no compute; the
written subset fixed across launches (mall_probe) or drawn afresh per launch (mall_probe_vary,
as the kernel's changed envs are). Beside it the step kernel on a fresh batch, per 20-launch
window, with the window's changed-env fraction, in dirty-store mode and in full-store mode."""
import ctypes
import json
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "gym-pbn-stac_amd"))
import numpy as np  # noqa: E402

from gym_pbn_amd.batch import PBNBatch  # noqa: E402
from gym_pbn_amd.network import load_network  # noqa: E402

lib = ctypes.CDLL(str(ROOT / "tools" / "libmallprobe.so"))
for f in (lib.mall_probe, lib.mall_probe_vary):
    f.argtypes = [ctypes.c_uint64, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_double)]


def probe(fn, n, pct, launches=200):
    us = ctypes.c_double()
    assert fn(n, pct, 1, launches, ctypes.byref(us)) == 0
    return round(us.value, 2)


net = load_network("bittner199")
res = {"floor": {}, "kernel": {}}
for n in (1 << 20, 1 << 23):
    for pct in (0, 20, 45, 100):
        res["floor"][f"{n}:{pct}:fixed"] = probe(lib.mall_probe, n, pct)
        res["floor"][f"{n}:{pct}:vary"] = probe(lib.mall_probe_vary, n, pct)


def windows(B, k, store_full=False, n=20):
    if store_full:
        os.environ["PBNSIM_STORE_MODE"] = "0"
    b = PBNBatch(net, B, seed=0x5EED)
    os.environ.pop("PBNSIM_STORE_MODE", None)
    b.randomize()
    b.step(5)
    out = []
    for w in range(k):
        b.timing(2)
        b.step(n)
        b.timing(0)
        ms, L = b.timing_read()
        a = b.get_state()
        b.step(1)  # the per-launch changed fraction at this point of the trajectory
        c = b.get_state()
        out.append([round(ms * 1e3 / L, 2), round(float(np.any(a != c, axis=1).mean()), 3)])
        if w % 5 == 4:
            b.step(500)  # jump ahead
    b.close()
    return out


res["kernel"]["1M_dirty"] = windows(1 << 20, 15)
res["kernel"]["1M_full"] = windows(1 << 20, 5, store_full=True)
res["kernel"]["8M_dirty"] = windows(1 << 23, 10)
print(json.dumps(res))
