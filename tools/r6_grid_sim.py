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
* ``global_handoff``: the ideal of an in-launch grid-wide hand-off (any idle wave takes any wave's unstarted
  tail env at no cost) -- the bound on what moving envs between workgroups could give.

Finding (profiles/r05_r6_grid_sim.txt): without knowing which envs will run long, the budget policy gains
nothing (parked envs all have used = K, so "longest-used first" is a random order: 2.12 vs 2.15 ms at cap 2^20;
with the exact remaining lengths as an oracle order, 1.55); even the ideal grid-wide hand-off gives 1.82 at the
measured block cost (0.7 us) -- the lever is the tail block's cost: at 0.35 us the same schedules give
1.1-1.7 ms. Hence round 5's tail helpers.

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


def global_handoff(nup, c_blk=0.7, tail_max=16, lanes=64, c_chunk=48 * 0.25, c_draw=0.25, c_sess=2.0,
                   c_push=1.0):
    """The ideal of an in-launch GRID-wide hand-off (no cost to reach any idle wave): per wave lane mode until
    <= tail_max live envs, then tail sessions, longest-used first; a wave's unstarted envs go to a grid-wide
    pool (sorted by used) that ANY idle wave pulls from. Same constants as tools/r6_sched_sim.py."""
    B = len(nup)
    waves = []
    for w in range(B // lanes):
        E = [[int(x), 0] for x in nup[w * lanes:(w + 1) * lanes]]
        t = 20.0
        E = [e for e in E if e[0] > 0]
        while len(E) > tail_max:
            n = len(E)
            t += c_chunk + c_draw * (math.ceil(n * 16 / 64) if n < 40 else 8) * 1.5
            for e in E:
                p = min(48, e[0])
                e[0] -= p
                e[1] += p
            E = [e for e in E if e[0] > 0]
        waves.append([t, E])
    pool, cnt, idle, tend = [], 0, [], 0.0
    ev = [(t, i) for i, (t, _) in enumerate(waves)]
    heapq.heapify(ev)
    while ev:
        t, i = heapq.heappop(ev)
        E = waves[i][1]
        if not E:
            if pool:
                _, _, env = heapq.heappop(pool)
                E = [env]
                t += c_push
            else:
                idle.append((t, i))
                tend = max(tend, t)
                continue
        k = max(range(len(E)), key=lambda j: E[j][1]) if any(e[1] >= 1024 for e in E) else 0
        env, others = E[k], [e for j, e in enumerate(E) if j != k]
        for e in others:
            cnt += 1
            heapq.heappush(pool, (-e[1], cnt, e))
        while idle and pool:
            ti, j = idle.pop()
            _, _, e = heapq.heappop(pool)
            waves[j][1] = [e]
            heapq.heappush(ev, (max(ti, t) + c_push, j))
        t += c_sess + math.ceil(env[0] / 64) * c_blk
        env[1] += env[0]
        env[0] = 0
        waves[i][1] = []
        heapq.heappush(ev, (t, i))
        tend = max(tend, t)
    return tend


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
    for cb in (0.7, 0.35):
        for tm in (16, 32):
            run(f'ideal grid-wide hand-off c_blk {cb} tail {tm}', lambda n, cb=cb, tm=tm: global_handoff(n, cb, tm))
