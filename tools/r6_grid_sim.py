#!/usr/bin/env python3
"""Grid-wide R6 schedules for one per-step launch at config 5's size (131,072 envs), driven by the real
loop lengths (tools/r6_nupdates.py), in a coarse model calibrated on round 4's measurements
(profiles/r04_r6_sched_sim.txt, r04_r6_lone_caps.txt): a lane-mode update costs c_lane[ws] us per wave
and a 64-update tail block c_blk[ws] us, ws = the waves sharing the SIMD. Policies:

* ``budget``: VERDICT r04's -- lane mode until every env has run K updates or ended (launch 1), the live
  envs parked to a device list, then a tail launch whose waves each pull the next parked env from a
  global counter (launch 2), P2 waves per SIMD, parked envs taken longest-first when ``order='used'``.
* ``levels``: lane launches with refill from a compacted list of live envs, budgets K0, K1, ...; once
  the live count drops to <= tail_at envs, a tail launch as above.

Measurement tooling only (no product code reads it). Usage: python tools/r6_grid_sim.py nup_*.npy"""
import heapq
import math
import sys

import numpy as np

SIMDS = 1024
LANES = 64
CH = 48
C_LANE = {1: 0.167, 2: 0.25, 3: 0.34, 4: 0.43}
C_BLK = {1: 0.67, 2: 0.85, 3: 1.15, 4: 1.5}
C_LAUNCH = 15.0  # fixed cost per launch (image staging, first refill; r04_r6_lone_caps: 18 us lone)
C_SESS = 2.0


def lane_phase(rem, K, n_waves, ws):
    """Lane mode over envs `rem` (remaining updates) with refill from the list: every wave keeps 64 lanes
    busy while the list has envs; an env leaves after min(rem, K) updates (K rounded up to the chunk).
    Returns (end time, remaining after the phase)."""
    Kc = int(math.ceil(K / CH) * CH)
    take = np.minimum(rem, Kc)
    # chunks per env (an env occupies its lane for ceil(take / CH) chunks)
    ch = np.ceil(take / CH).astype(np.int64)
    c_chunk = CH * C_LANE[ws] * 1.25  # + draw generation
    # lanes: n_waves * 64 slots, envs dealt in list order to the first free lane (greedy)
    slots = n_waves * LANES
    if len(ch) <= slots:
        # one env per lane: a wave lasts its longest lane
        pad = np.zeros(int(math.ceil(len(ch) / LANES)) * LANES, np.int64)
        pad[:len(ch)] = ch
        w = pad.reshape(-1, LANES).max(axis=1)
        t = float(w.max()) * c_chunk
    else:
        # refill: lanes free up at chunk granularity; per wave the chunk loop runs while any lane is busy
        h = [0] * slots
        for c in ch:
            heapq.heapreplace(h, h[0] + int(c))
        lanes = np.array(h).reshape(n_waves, LANES)
        t = float(lanes.max()) * c_chunk
    return t + C_LAUNCH, rem - take


def tail_phase(rem, n_waves, ws, order):
    r = rem[rem > 0]
    if order == 'used':
        r = np.sort(r)[::-1]  # stand-in for longest-used-first (exact knowledge: an upper bound)
    cost = np.ceil(r / 64) * C_BLK[ws] + C_SESS
    h = [0.0] * n_waves
    for c in cost:
        heapq.heapreplace(h, h[0] + float(c))
    return max(h) + C_LAUNCH if len(r) else 0.0


def budget(nup, K, ws1=2, ws2=2, order='list'):
    n_waves = len(nup) // LANES
    t1, rem = lane_phase(nup.astype(np.int64), K, n_waves, ws1)
    return t1 + tail_phase(rem, SIMDS * ws2, ws2, order)


def levels(nup, Ks, tail_at, ws=2, ws2=2, order='list'):
    rem = nup.astype(np.int64)
    t = 0.0
    for K in Ks:
        live = rem[rem > 0]
        if len(live) <= tail_at:
            break
        n_waves = min(SIMDS * ws, int(math.ceil(len(live) / LANES)))
        wsl = max(1, min(ws, int(math.ceil(n_waves / SIMDS))))
        dt, rem2 = lane_phase(live, K, n_waves, wsl)
        t += dt
        rem = rem2
    return t + tail_phase(rem, SIMDS * ws2, ws2, order)


if __name__ == '__main__':
    D = {f.split('/')[-1]: np.load(f) for f in sys.argv[1:]}

    def run(label, fn):
        print(f'{label:44s}', {k: round(float(np.mean([fn(v[t]) for t in range(min(2, v.shape[0]))])) / 1e3, 3)
                               for k, v in D.items()}, flush=True)
    for K in (128, 512, 1024, 2048):
        for o in ('list', 'used'):
            run(f'budget K={K} order={o}', lambda n, K=K, o=o: budget(n, K, order=o))
    run('budget K=1024 tail 4/SIMD', lambda n: budget(n, 1024, ws2=4))
    for Ks in ((128, 256, 512, 1024, 2048, 4096), (256, 1024, 4096), (512, 2048, 8192)):
        for ta in (2048, 4096, 8192):
            run(f'levels {Ks} tail<={ta}', lambda n, Ks=Ks, ta=ta: levels(n, Ks, ta))
