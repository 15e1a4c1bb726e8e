"""R6 (``PBNTargetMultiEnv.step``, pbn_target_multi.py:119-154) in the regimes the bench numbers
come from, checked against the oracle (``oracle.env_step_multi``, the CPU restatement).

* Lane refill: ``k_env`` is persistent -- a lane that finishes its env takes the next one from
  a global work counter. At the bench sizes (131,072 and 1,048,576 envs) every lane handles
  several envs, mixing envs at different update counts inside one wave's shared draw tables.
  ``PBNSIM_ENV_GRID`` caps the grid so a few thousand envs put every lane through >= 3 envs:
  waves start full (>= 40 active lanes: each lane draws its own entries) and end in the tail
  (< 40: the rank / counter tables of the shared path). All envs are compared.
* Config 5 per GPU: 131,072 Bittner-199 envs, one T = 100 chunk in one fused launch, equal in
  full to 100 per-step launches and, on every env, field and step, to the oracle; the same shard at
  the reference-faithful cap 2^20 for both attractor specs (per step and fused, library defaults:
  grid pool, tail helpers, hand-off), every env against the oracle.

Production settings: the r6_bittner199 fixture's attractor cubes, A = 4 (0 w.p. 0.75),
update cap 4,096 (about a fifth of the env steps run into it).
"""

import numpy as np
import pytest

from conftest import cubes_to_attractors, golden, r6_config
from gym_pbn_amd.network import load_network

pytestmark = pytest.mark.gpu

CAP = 4096


def _actions(rng, shape, N):
    a = rng.integers(1, N + 1, size=shape).astype(np.int32)
    a[rng.random(shape) < 0.75] = 0
    return a


def _setup(G, B, seed, env_base):
    z = golden("r6_bittner199.npz")
    net = load_network("bittner199")
    gnet = G.Net(net)
    cfg = G.EnvConfig(gnet, cubes_to_attractors(z, net.n_nodes), horizon=100)
    cfgd = r6_config(z)
    cfgd["horizon"] = 100
    b = G.PBNBatch(gnet, B, seed=seed, env_id_base=env_base)
    b.env_reset(cfg)
    return net, cfg, cfgd, b


@pytest.fixture(scope="module")
def G():
    from gym_pbn_amd import _lib, batch

    assert _lib.device_count() >= 1, "gpu tests need a HIP device"
    return batch


@pytest.mark.parametrize("mode", ["per_step", "fused", "grp8_per_step", "one_lane_per_step", "one_lane_fused",
                                  "per_step_chunk32", "fused_chunk32", "per_step_kernel_image", "fused_bpc1"])
def test_lane_refill_matches_oracle(G, oracle_mod, monkeypatch, mode):
    """... and with either draw-round chunk (EnvArgs::chunk: 48 for these launches, 32 forced by
    PBNSIM_ENV_CHUNK -- the chunk the host picks for long fused launches over large batches); and with
    the kernel building its LDS image itself (PBNSIM_ENV_KERNEL_IMAGE=1) instead of staging the
    host-built one (pbn_abi.cpp env_gen_image), so both constructions stay exact; and with the workgroups per CU
    capped at one (PBNSIM_ENV_BPC=1)."""
    import torch

    if mode.endswith("kernel_image"):
        monkeypatch.setenv("PBNSIM_ENV_KERNEL_IMAGE", "1")
    if mode.endswith("bpc1"):
        monkeypatch.setenv("PBNSIM_ENV_BPC", "1")  # one workgroup per CU (the occupancy the host sizes against)

    grp = "8" if mode.startswith("grp8") else "1"
    chunk32 = mode.endswith("chunk32")
    if chunk32:
        monkeypatch.setenv("PBNSIM_ENV_CHUNK", "32")
    monkeypatch.setenv("PBNSIM_ENV_GROUP", grp)
    # every lane takes envs (lane mode proper), or one lane per wave (tail mode from the first env,
    # each wave taking its next env from the queue when one ends)
    monkeypatch.setenv("PBNSIM_ENV_LANES", "1" if mode.startswith("one_lane") else "64")
    grid = 4 if grp == "1" else 2
    monkeypatch.setenv("PBNSIM_ENV_GRID", str(grid))
    B = 6144 if grp == "1" else 1024
    lanes = grid * 256 // int(grp)  # env slots in flight
    assert B >= 3 * lanes  # every lane (group) takes >= 3 envs from the work counter
    seed, base, T, A = 0xAC7, 5000, 3, 4
    net, cfg, cfgd, b = _setup(G, B, seed, base)
    o = oracle_mod.Oracle(net)
    st, ns = o.env_reset_philox(np.zeros((B, net.n_words), np.uint64), np.ones(B, np.int64), cfgd["reset_care"],
                                cfgd["reset_value"], seed=seed, env_base=base, reset_count=0)
    assert np.array_equal(b.get_state(), st)
    acts = _actions(np.random.default_rng(17), (T, B, A), net.n_nodes)
    if "fused" in mode:
        dev = torch.device("cuda", 0)
        d_a = torch.from_numpy(acts).to(dev)
        o_ = torch.empty((T, B, net.n_words), dtype=torch.int64, device=dev)
        r_ = torch.empty((T, B), dtype=torch.int32, device=dev)
        f_ = torch.empty((T, B), dtype=torch.uint8, device=dev)
        n_ = torch.empty((T, B), dtype=torch.int32, device=dev)
        b.env_rollout_multi_device(cfg, T, d_a.data_ptr(), A, o_.data_ptr(), r_.data_ptr(), f_.data_ptr(),
                                   n_.data_ptr(), update_cap=CAP)
        b.sync()
        got = [(o_[t].cpu().numpy().view(np.uint64), r_[t].cpu().numpy(), f_[t].cpu().numpy(),
                n_[t].cpu().numpy().view(np.uint32)) for t in range(T)]
    else:
        got = [b.env_step_multi(cfg, acts[t], update_cap=CAP) for t in range(T)]
    info = b.info()
    assert info["env_grid"] == grid and info["env_lanes"] == int(grp)
    if grp == "1":
        assert info["env_kernel"] == 4 and info["env_lane_limit"] == (1 if mode.startswith("one_lane") else 64)
        assert info["env_chunk"] == (32 if chunk32 else 48)
    capped = 0
    for t in range(T):
        ref = o.env_step_multi(cfgd, st, ns, acts[t], seed=seed, env_base=base, call_idx=t, update_cap=CAP)
        obs, rew, flags, nup = got[t]
        assert np.array_equal(nup, ref["n_updates"]), t
        assert np.array_equal(obs, ref["obs"]) and np.array_equal(rew, ref["reward"]), t
        assert np.array_equal(flags, ref["flags"]), t
        st, ns = ref["state"], ref["n_steps"]
        capped += int(((flags & 4) != 0).sum())
    assert np.array_equal(b.get_state(), st) and np.array_equal(b.get_n_steps(), ns)
    assert 0 < capped < T * B  # both regimes: envs that hit the cap and envs that reached an attractor


_C5 = {}  # config 5's shard per bench figure, computed once: device outputs, then the oracle's progress through them
_C5_PARTS = 4
# bench.py's three config-5 figures (r6_supplement): the headline (fixture cubes, cap 4,096), high_cap and
# spec_attractors (cap 2^20, R6_HIGH_CAP)
_C5_FIGURES = [("fixture", CAP), ("fixture", 1 << 20), ("spec", 1 << 20)]


def _config5_device(G, spec, cap):
    """Config 5's shard as bench.py runs it (r6_figure): 131,072 envs of rank 3 of the 8-GPU run (global ids
    3 * 131,072 ...), actions from ``actions.env_actions`` (Philox 0xAC7 keyed by global env id), T = 100,
    library defaults. One fused T = 100 launch (grid pool on) and 100 per-step launches of a second batch
    (pool on from cap 16,384), which must agree on every env and field; host copies of the fused outputs are
    kept for the oracle parts."""
    key = (spec, cap)
    if key in _C5:
        return _C5[key]
    import sys
    from pathlib import Path

    import torch

    sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
    import bench
    from gym_pbn_amd.actions import env_actions

    _C5.clear()  # one figure's host copies at a time
    B, T, A, seed, base = 131072, 100, 4, 0xAC7, 3 * 131072
    dev = torch.device("cuda", 0)
    net = load_network("bittner199")
    gnet = G.Net(net)
    atts, _ = bench.r6_attractors(spec, net.n_nodes)
    cfg = G.EnvConfig(gnet, atts, horizon=T)
    cfgd = dict(care=cfg.cube_care, value=cfg.cube_value, target_care=cfg.target_care, target_value=cfg.target_value,
                horizon=T)
    d_a = env_actions(T, base, B, A, net.n_nodes, seed=0xAC7, device=dev)
    b1 = G.PBNBatch(gnet, B, seed=seed, env_id_base=base)
    b1.env_reset(cfg)
    init = b1.get_state()
    ns0 = b1.get_n_steps()

    def outs():
        return (torch.empty((T, B, net.n_words), dtype=torch.int64, device=dev),
                torch.empty((T, B), dtype=torch.int32, device=dev),
                torch.empty((T, B), dtype=torch.uint8, device=dev),
                torch.empty((T, B), dtype=torch.int32, device=dev))

    fo = outs()
    b1.env_rollout_multi_device(cfg, T, d_a.data_ptr(), A, *[x.data_ptr() for x in fo], update_cap=cap)
    b1.sync()  # raises if the pool dropped an env
    pools = [b1.env_grid_stats()]
    b2 = G.PBNBatch(gnet, B, seed=seed, env_id_base=base)
    b2.env_reset(cfg)
    po = outs()
    for t in range(T):
        b2.env_step_multi_device(cfg, d_a[t].data_ptr(), A, *[x[t].data_ptr() for x in po], update_cap=cap)
        if t % 10 == 9:
            pools.append(b2.env_grid_stats())
    b2.sync()
    for x, y in zip(fo, po):
        assert torch.equal(x, y)
    assert np.array_equal(b1.get_state(), b2.get_state()) and np.array_equal(b1.get_n_steps(), b2.get_n_steps())
    c = dict(net=net, cfgd=cfgd, B=B, T=T, seed=seed, base=base, cap=cap, acts=d_a.cpu().numpy(), pools=pools,
             obs=fo[0].cpu().numpy().view(np.uint64), rew=fo[1].cpu().numpy(), flags=fo[2].cpu().numpy(),
             nup=fo[3].cpu().numpy().view(np.uint32), final=b1.get_state(), final_ns=b1.get_n_steps(),
             orc_t=0, orc_st=init, orc_ns=ns0)
    b1.close()
    b2.close()
    _C5[key] = c
    return c


@pytest.mark.parametrize("spec,cap", _C5_FIGURES)
def test_config5_chunk_131k_fused_equals_per_step(G, spec, cap):
    """BASELINE config 5's per-GPU shard (131,072 envs, rank 3's global ids, T = 100 env steps, the bench's
    actions) for each of bench.py's three figures: the fused chunk (one launch, grid pool on) equals 100
    per-step launches on every env and field; the pool moved envs and dropped none."""
    c = _config5_device(G, spec, cap)
    assert (c["flags"][-1] & 2).all()  # truncated at the horizon
    if cap == CAP:
        assert 0.05 < ((c["flags"] & 4) != 0).mean() < 0.5 and c["nup"].max() == CAP  # the capped regime
    else:
        assert not (c["flags"] & 4).any()  # the reference's unbounded loop is never cut
    assert all(p["gave_up"] == 0 and p["live_at_end"] == 0 for p in c["pools"]), c["pools"]
    assert c["pools"][0]["pushed"] > 0, c["pools"]  # the fused launch moved envs between workgroups
    if cap >= 16384:
        assert sum(p["pushed"] for p in c["pools"][1:]) > 0, c["pools"]  # ... and so did per-step launches


@pytest.mark.parametrize("part", range(_C5_PARTS))
@pytest.mark.parametrize("spec,cap", _C5_FIGURES)
def test_config5_chunk_131k_every_env_vs_oracle(G, oracle_mod, spec, cap, part):
    """... and EVERY env of it equals the oracle (OpenMP over the envs) on every field of every env step:
    steps [25 part, 25 part + 25) here (a part run alone first advances the oracle through the earlier steps;
    the whole figure takes ~40 s of the box's 16 threads)."""
    c = _config5_device(G, spec, cap)
    o = oracle_mod.Oracle(c["net"])
    per = c["T"] // _C5_PARTS
    t0, t1 = part * per, (part + 1) * per
    while c["orc_t"] < t1:
        t = c["orc_t"]
        ref = o.env_step_multi(c["cfgd"], c["orc_st"], c["orc_ns"], c["acts"][t], seed=c["seed"], env_base=c["base"],
                               call_idx=t, update_cap=cap)
        if t >= t0:
            assert np.array_equal(c["nup"][t], ref["n_updates"]), t
            assert np.array_equal(c["obs"][t], ref["obs"]), t
            assert np.array_equal(c["rew"][t], ref["reward"]), t
            assert np.array_equal(c["flags"][t], ref["flags"]), t
        c["orc_st"], c["orc_ns"], c["orc_t"] = ref["state"], ref["n_steps"], t + 1
    if t1 == c["T"]:
        assert np.array_equal(c["final"], c["orc_st"]) and np.array_equal(c["final_ns"], c["orc_ns"])


def test_collector_does_not_reuse_a_buffer_still_being_gathered(G):
    """rollout.TrajectoryCollector double-buffers chunks; with RCCL, ``Work.wait()`` only orders
    torch's current stream, not the batch stream the env kernel runs on. A stand-in process group
    whose all-gather reads the chunk late (on a side stream, behind a ~50 ms device sleep) and whose
    ``wait()`` has RCCL's semantics shows that the gathered copy of chunk 0 is still chunk 0 after
    chunk 2 has been written into the same buffer."""
    import torch

    from gym_pbn_amd.rollout import TrajectoryCollector

    dev = torch.device("cuda", 0)

    class _Work:
        def __init__(self, ev):
            self.ev = ev

        def wait(self):  # like RCCL: the current stream waits, the host does not
            torch.cuda.current_stream(dev).wait_event(self.ev)

    class _LateGather:
        def __init__(self):
            self.side = torch.cuda.Stream(dev)
            self.snaps = []

        def is_initialized(self):
            return True

        def get_world_size(self):
            return 2

        def all_gather_into_tensor(self, dst, src, async_op=False):
            self.side.wait_stream(torch.cuda.current_stream(dev))
            with torch.cuda.stream(self.side):
                torch.cuda._sleep(100_000_000)
                snap = src.clone()
                ev = torch.cuda.Event()
                ev.record(self.side)
            self.snaps.append(snap)
            return _Work(ev)

    z = golden("r6_bittner28.npz")
    net = G.Net(load_network("bittner28"))
    cfg = G.EnvConfig(net, cubes_to_attractors(z, 28), horizon=5)
    B, T, A = 2048, 5, 2
    acts = torch.from_numpy(_actions(np.random.default_rng(3), (T, B, A), 28)).to(dev)
    fake = _LateGather()
    col = TrajectoryCollector(G.PBNBatch(net, B, seed=11), cfg, T, A, dev, update_cap=4096, dist=fake)
    ref = TrajectoryCollector(G.PBNBatch(net, B, seed=11), cfg, T, A, dev, update_cap=4096)
    expect = []
    for _ in range(3):
        col.step_chunk(acts)
        buf, _ = ref.step_chunk(acts)
        torch.cuda.synchronize()
        expect.append(buf["obs"].clone())
    col.finish()
    torch.cuda.synchronize()
    obs_snaps = fake.snaps[0::4]  # one gather per field, obs first
    assert not torch.equal(expect[0], expect[2])
    for k in range(3):
        assert torch.equal(obs_snaps[k].view(expect[k].shape), expect[k]), k


@pytest.mark.parametrize("spec", ["fixture", "spec"])
def test_high_cap_full_shard_matches_oracle(G, oracle_mod, spec):
    """The loop the reference runs unbounded (pbn_target_multi.py:135-146) at the cap bench.py reports it at
    (R6_HIGH_CAP, 2^20; the longest loop measured at config 5 ran 78,057 updates, profiles/r03_r6_cap_sweep.json),
    for both attractor specs the bench line carries -- the fixture's cubes and SURVEY §8(d)'s 4 cubes over the 7
    target genes -- on config 5's whole shard (131,072 envs, rank 3's global ids) at the library defaults (tail
    helpers, the workgroup hand-off and the grid pool all on): 3 per-step launches and, on a second batch, one
    fused T = 3 launch; every env and field of both against the oracle, no env capped, and the grid pool moved
    envs between workgroups in the launches (pushed > 0, nothing given up, live count 0 at the end)."""
    import sys
    from pathlib import Path

    import torch

    sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
    import bench

    net = load_network("bittner199")
    gnet = G.Net(net)
    atts, _ = bench.r6_attractors(spec, net.n_nodes)
    cfg = G.EnvConfig(gnet, atts, horizon=100)
    cfgd = dict(care=cfg.cube_care, value=cfg.cube_value, target_care=cfg.target_care, target_value=cfg.target_value,
                horizon=100)
    B, seed, base, T, A = 131072, 0xAC7, 3 * 131072, 3, 4
    cap = bench.R6_HIGH_CAP
    acts = _actions(np.random.default_rng(123), (T, B, A), net.n_nodes)
    b = G.PBNBatch(gnet, B, seed=seed, env_id_base=base)
    b.env_reset(cfg)
    o = oracle_mod.Oracle(net)
    st, ns = o.env_reset_philox(np.zeros((B, net.n_words), np.uint64), np.ones(B, np.int64), cfg.reset_care,
                                cfg.reset_value, seed=seed, env_base=base, reset_count=0)
    assert np.array_equal(b.get_state(), st)
    got, pools = [], []
    for t in range(T):
        got.append(b.env_step_multi(cfg, acts[t], update_cap=cap))
        pools.append(b.env_grid_stats())
    final_step = (b.get_state(), b.get_n_steps())
    b.close()
    dev = torch.device("cuda", 0)
    bf = G.PBNBatch(gnet, B, seed=seed, env_id_base=base)
    bf.env_reset(cfg)
    d_a = torch.from_numpy(acts).to(dev)
    fo = (torch.empty((T, B, net.n_words), dtype=torch.int64, device=dev), torch.empty((T, B), dtype=torch.int32, device=dev),
          torch.empty((T, B), dtype=torch.uint8, device=dev), torch.empty((T, B), dtype=torch.int32, device=dev))
    bf.env_rollout_multi_device(cfg, T, d_a.data_ptr(), A, *[x.data_ptr() for x in fo], update_cap=cap)
    bf.sync()  # raises if the pool dropped an env (sticky fault word)
    pools.append(bf.env_grid_stats())
    fused = [(fo[0][t].cpu().numpy().view(np.uint64), fo[1][t].cpu().numpy(), fo[2][t].cpu().numpy(),
              fo[3][t].cpu().numpy().view(np.uint32)) for t in range(T)]
    final_fused = (bf.get_state(), bf.get_n_steps())
    bf.close()
    assert all(p["gave_up"] == 0 and p["live_at_end"] == 0 for p in pools), pools
    assert sum(p["pushed"] for p in pools[:T]) > 0 and pools[T]["pushed"] > 0, pools
    for t in range(T):
        ref = o.env_step_multi(cfgd, st, ns, acts[t], seed=seed, env_base=base, call_idx=t, update_cap=cap)
        for name, g in (("per_step", got[t]), ("fused", fused[t])):
            obs, rew, flags, nup = g
            assert np.array_equal(nup, ref["n_updates"]), (name, t)
            assert np.array_equal(obs, ref["obs"]) and np.array_equal(rew, ref["reward"]), (name, t)
            assert np.array_equal(flags, ref["flags"]), (name, t)
            assert not (flags & 4).any()  # nothing reached the cap
        st, ns = ref["state"], ref["n_steps"]
    for fs in (final_step, final_fused):
        assert np.array_equal(fs[0], st) and np.array_equal(fs[1], ns)


@pytest.mark.parametrize("steal", ["1", "0"])
@pytest.mark.parametrize("mode", ["per_step", "fused"])
def test_tail_handoff_between_waves_matches_oracle(G, oracle_mod, monkeypatch, mode, steal):
    """Tail envs handed from wave to wave (k_env mode 4, ``EnvArgs::steal_local``): at the reference's
    unbounded-loop cap (2^20) a wave's long until-attractor loops would run one after another in its
    tail while sibling waves whose envs all ended sit idle, so a tail wave passes envs it has not
    started on (registers + plane column, through the idle wave's LDS draw buffer) to idle waves of its
    workgroup, which resume them in lane 0. 32 workgroups (128 waves) hold one env per lane; with the
    hand-off on (the default) the launches normally hand envs off (a warning if, by the waves' timing,
    none did), with PBNSIM_ENV_STEAL=0 none; either way every env of every step equals the oracle (obs, reward, flags, update counts, final state and
    step counters)."""
    import torch

    monkeypatch.setenv("PBNSIM_ENV_LANES", "64")
    monkeypatch.setenv("PBNSIM_ENV_GRID", "32")
    monkeypatch.setenv("PBNSIM_ENV_STEAL", steal)
    import sys
    from pathlib import Path

    sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
    import bench

    net = load_network("bittner199")
    gnet = G.Net(net)
    atts, _ = bench.r6_attractors("fixture", net.n_nodes)
    cfg = G.EnvConfig(gnet, atts, horizon=100)
    cfgd = dict(care=cfg.cube_care, value=cfg.cube_value, target_care=cfg.target_care, target_value=cfg.target_value,
                horizon=100)
    B, seed, base, T, A = 8192, 0x5EED, 70001, 3, 4
    cap = bench.R6_HIGH_CAP
    b = G.PBNBatch(gnet, B, seed=seed, env_id_base=base)
    b.env_reset(cfg)
    o = oracle_mod.Oracle(net)
    st, ns = o.env_reset_philox(np.zeros((B, net.n_words), np.uint64), np.ones(B, np.int64), cfg.reset_care,
                                cfg.reset_value, seed=seed, env_base=base, reset_count=0)
    acts = _actions(np.random.default_rng(321), (T, B, A), net.n_nodes)
    handed, helpers = [], []
    if mode == "fused":
        dev = torch.device("cuda", 0)
        d_a = torch.from_numpy(acts).to(dev)
        o_ = torch.empty((T, B, net.n_words), dtype=torch.int64, device=dev)
        r_ = torch.empty((T, B), dtype=torch.int32, device=dev)
        f_ = torch.empty((T, B), dtype=torch.uint8, device=dev)
        n_ = torch.empty((T, B), dtype=torch.int32, device=dev)
        b.env_rollout_multi_device(cfg, T, d_a.data_ptr(), A, o_.data_ptr(), r_.data_ptr(), f_.data_ptr(),
                                   n_.data_ptr(), update_cap=cap)
        b.sync()  # the launch is asynchronous on the batch's stream (env_handoffs syncs only with the hand-off on)
        handed.append(b.env_handoffs())
        got = [(o_[t].cpu().numpy().view(np.uint64), r_[t].cpu().numpy(), f_[t].cpu().numpy(),
                n_[t].cpu().numpy().view(np.uint32)) for t in range(T)]
    else:
        got = []
        for t in range(T):
            got.append(b.env_step_multi(cfg, acts[t], update_cap=cap))
            handed.append(b.env_handoffs())
    info = b.info()
    assert info["env_kernel"] == 4 and info["env_lane_limit"] == 64 and info["env_grid"] == 32
    assert info["env_handoff"] == int(steal)
    if steal == "0":
        assert sum(handed) == 0, handed  # hand-off off: nothing passed between waves
    elif sum(handed) == 0:  # whether a wave goes idle while a sibling holds unstarted envs depends on
        import warnings    # wave scheduling: a diagnostic, not a correctness condition

        warnings.warn(f"no tail hand-off happened in this run ({handed}); exactness still checked below")
    for t in range(T):
        ref = o.env_step_multi(cfgd, st, ns, acts[t], seed=seed, env_base=base, call_idx=t, update_cap=cap)
        obs, rew, flags, nup = got[t]
        assert np.array_equal(nup, ref["n_updates"]), t
        assert np.array_equal(obs, ref["obs"]) and np.array_equal(rew, ref["reward"]), t
        assert np.array_equal(flags, ref["flags"]), t
        st, ns = ref["state"], ref["n_steps"]
    assert np.array_equal(b.get_state(), st) and np.array_equal(b.get_n_steps(), ns)
    b.close()


@pytest.mark.parametrize("case", ["handoff", "helpers", "helpers_off", "grid", "grid_off"])
@pytest.mark.parametrize("mode", ["per_step", "fused"])
def test_tail_handoff_forced_happens_and_matches_oracle(G, oracle_mod, monkeypatch, mode, case):
    """A case in which the workgroup hand-off must happen: one workgroup (4 waves), two
    lanes per wave taking envs, 6 envs -- three waves hold two envs each, the fourth none and goes idle
    at once. Every env's first env step is long (its action row is chosen with the oracle so that
    each runs >= 2,048 updates: per env, action rows are tried on the oracle until one does), so a wave resolving its first env reaches its 16-block re-check
    (tail_session: every 16 blocks) with its second env unstarted while the idle wave waits: the
    hand-off happens (asserted), and every output equals the oracle.

    ``helpers``: 2 envs, both taken by one wave (two lanes); at its 16-block re-check it hands its
    unstarted env to an idle wave and recruits the other idle waves as tail helpers, which prepare its
    blocks (draws, records, writer masks) into its LDS ring while it resolves them (asserted: helpers
    recruited; exact against the oracle). ``helpers_off``: the same with PBNSIM_ENV_HELPERS=0 (none).

    ``grid``: the grid pool (k_env, EnvArgs::gpool) -- two workgroups, 16 lanes per wave taking envs, 16
    envs: the first wave to reach the work queue takes all of them, every other wave of both workgroups
    goes idle, so the other workgroup waits on a ticket while the loaded wave, after handing three envs
    to its idle siblings, still holds unstarted ones: it pushes envs into the pool (asserted) and the
    waiting workgroup resumes them; every output equals the oracle. ``grid_off``: PBNSIM_ENV_GRID_STEAL=0
    (nothing pushed). (Round 5's ``migrate`` case -- a running session moving itself into the pool -- went with
    the feature: config 5's A/B showed no gain, profiles/r06_r6_pool_migrate_ab.json.)"""
    import torch

    grid_case = case.startswith("grid")
    monkeypatch.setenv("PBNSIM_ENV_LANES", "16" if grid_case else "2")
    monkeypatch.setenv("PBNSIM_ENV_GRID", "2" if grid_case else "1")
    if case == "helpers_off":
        monkeypatch.setenv("PBNSIM_ENV_HELPERS", "0")
    if case == "grid_off":
        monkeypatch.setenv("PBNSIM_ENV_GRID_STEAL", "0")
    import sys
    from pathlib import Path

    sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
    import bench

    net = load_network("bittner199")
    gnet = G.Net(net)
    atts, _ = bench.r6_attractors("fixture", net.n_nodes)
    cfg = G.EnvConfig(gnet, atts, horizon=100)
    cfgd = dict(care=cfg.cube_care, value=cfg.cube_value, target_care=cfg.target_care, target_value=cfg.target_value,
                horizon=100)
    o = oracle_mod.Oracle(net)
    B = {"handoff": 6, "grid": 16, "grid_off": 16}.get(case, 2)
    seed, base, T, A, cap = 0xAC7, 90001, 2, 4, bench.R6_HIGH_CAP
    st, ns = o.env_reset_philox(np.zeros((B, net.n_words), np.uint64), np.ones(B, np.int64), cfg.reset_care,
                                cfg.reset_value, seed=seed, env_base=base, reset_count=0)
    # per env, the first candidate action row (oracle) whose first env step runs >= 2,048 updates
    acts = _actions(np.random.default_rng(77), (T, B, A), net.n_nodes)
    rng = np.random.default_rng(78)
    need = np.ones(B, bool)
    for _ in range(400):
        cand = _actions(rng, (B, A), net.n_nodes)
        r = o.env_step_multi(cfgd, st, ns, cand, seed=seed, env_base=base, call_idx=0, update_cap=cap)
        ok = need & (r["n_updates"] >= 2048)
        acts[0][ok] = cand[ok]
        need &= ~ok
        if not need.any():
            break
    assert not need.any()
    b = G.PBNBatch(gnet, B, seed=seed, env_id_base=base)
    b.env_reset(cfg)
    st, ns = o.env_reset_philox(np.zeros((B, net.n_words), np.uint64), np.ones(B, np.int64), cfg.reset_care,
                                cfg.reset_value, seed=seed, env_base=base, reset_count=0)
    assert np.array_equal(b.get_state(), st)
    handed, helpers, pool = [], [], []
    if mode == "fused":
        dev = torch.device("cuda", 0)
        d_a = torch.from_numpy(acts).to(dev)
        o_ = torch.empty((T, B, net.n_words), dtype=torch.int64, device=dev)
        r_ = torch.empty((T, B), dtype=torch.int32, device=dev)
        f_ = torch.empty((T, B), dtype=torch.uint8, device=dev)
        n_ = torch.empty((T, B), dtype=torch.int32, device=dev)
        b.env_rollout_multi_device(cfg, T, d_a.data_ptr(), A, o_.data_ptr(), r_.data_ptr(), f_.data_ptr(),
                                   n_.data_ptr(), update_cap=cap)
        b.sync()
        handed.append(b.env_handoffs())
        helpers.append(b.env_tail_helpers())
        pool.append(b.env_grid_stats())
        got = [(o_[t].cpu().numpy().view(np.uint64), r_[t].cpu().numpy(), f_[t].cpu().numpy(),
                n_[t].cpu().numpy().view(np.uint32)) for t in range(T)]
    else:
        got = []
        for t in range(T):
            got.append(b.env_step_multi(cfg, acts[t], update_cap=cap))
            handed.append(b.env_handoffs())
            helpers.append(b.env_tail_helpers())
            pool.append(b.env_grid_stats())
    info = b.info()
    assert info["env_kernel"] == 4 and info["env_lane_limit"] == (16 if grid_case else 2)
    assert info["env_grid"] == (2 if grid_case else 1)
    assert info["env_handoff"] == 1
    assert handed[0] > 0, handed  # the first launch (every env long) must hand off
    assert all(p["gave_up"] == 0 and p["live_at_end"] == 0 for p in pool), pool
    if case == "grid":
        assert pool[0]["pushed"] > 0, pool  # ... and push envs to the waiting workgroup
    if case == "grid_off":
        assert sum(p["pushed"] + p["tickets"] for p in pool) == 0, pool
    if case == "helpers":
        assert helpers[0] > 0, helpers  # ... and recruit the remaining idle waves as helpers
    if case == "helpers_off":
        assert sum(helpers) == 0, helpers
    for t in range(T):
        ref = o.env_step_multi(cfgd, st, ns, acts[t], seed=seed, env_base=base, call_idx=t, update_cap=cap)
        obs, rew, flags, nup = got[t]
        assert np.array_equal(nup, ref["n_updates"]), t
        assert np.array_equal(obs, ref["obs"]) and np.array_equal(rew, ref["reward"]), t
        assert np.array_equal(flags, ref["flags"]), t
        st, ns = ref["state"], ref["n_steps"]
    assert np.array_equal(b.get_state(), st) and np.array_equal(b.get_n_steps(), ns)
    b.close()
