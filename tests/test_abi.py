"""The C-ABI library loads and exports every entry point include/pbn_abi.h declares (CPU only).

No compute call is made here; without a GPU the library must refuse loudly
(there is no CPU path to fall back to).
"""

import re
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]


def declared_functions():
    text = (ROOT / "include" / "pbn_abi.h").read_text()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    names = re.findall(r"\b(pbn_[a-z0-9_]+)\s*\(", text)
    return sorted(set(names))


def test_header_declares_the_boundary():
    names = declared_functions()
    for must in ("pbn_net_create", "pbn_batch_create", "pbn_step", "pbn_rollout", "pbn_step_replay",
                 "pbn_env_step_multi", "pbn_flip", "pbn_get_state", "pbn_set_state", "pbn_last_error",
                 "pbn_mt_seed", "pbn_mt_step"):
        assert must in names


def test_library_exports_every_declared_symbol():
    from gym_pbn_amd import _lib

    for name in declared_functions():
        assert hasattr(_lib.lib, name), name
        assert name in _lib.SIGNATURES, f"{name} missing from the ctypes signature table"
    want = int(re.search(r"#define PBN_ABI_VERSION (\d+)", (ROOT / "include" / "pbn_abi.h").read_text()).group(1))
    assert _lib.lib.pbn_abi_version() == want


def test_net_create_validates_on_host():
    import ctypes as C

    import numpy as np

    from gym_pbn_amd import _lib
    from gym_pbn_amd.batch import Net
    from gym_pbn_amd.network import load_network

    net = Net(load_network("bittner199"))  # host-side validation + LDS image packing
    assert net.handle.value
    d = _lib.NetDesc()
    d.kind, d.n_nodes = 1, 4
    h = C.c_void_p()
    assert _lib.lib.pbn_net_create(C.byref(d), C.byref(h)) == _lib.PBN_E_INVALID
    assert "NULL" in _lib.last_error()
    d.kind, d.n_nodes = 7, 4
    assert _lib.lib.pbn_net_create(C.byref(d), C.byref(h)) == _lib.PBN_E_INVALID
    d.n_nodes = 100000
    assert _lib.lib.pbn_net_create(C.byref(d), C.byref(h)) == _lib.PBN_E_UNSUPPORTED
    bad = load_network("bittner28")
    bad.pred_inputs = bad.pred_inputs.copy()
    bad.pred_inputs[0, 0] = 99
    with pytest.raises(ValueError):
        Net(bad)
    del np


def test_no_silent_cpu_fallback_without_gpu():
    from gym_pbn_amd import _lib
    from gym_pbn_amd.batch import PBNBatch

    if _lib.device_count() > 0:
        pytest.skip("a GPU is present; covered by the gpu tests")
    with pytest.raises(_lib.PbnError) as ei:
        PBNBatch("bittner28", 16)
    assert "no HIP device" in str(ei.value) or "HIP" in str(ei.value)


def test_batch_create_validates_sizes_on_host():
    """Empty batches and global env ids past the Philox counter field are refused before any
    device call (so the same on a CPU-only host and on a GPU box)."""
    import ctypes as C

    from gym_pbn_amd import _lib
    from gym_pbn_amd.batch import Net
    from gym_pbn_amd.network import load_network

    net = Net(load_network("bittner28"))
    h = C.c_void_p()
    assert _lib.lib.pbn_batch_create(net.handle, 0, 0, 0, 1, C.byref(h)) == _lib.PBN_E_INVALID
    assert "n_envs" in _lib.last_error()
    assert _lib.lib.pbn_batch_create(net.handle, 0, 16, (1 << 56) - 8, 1, C.byref(h)) == _lib.PBN_E_RANGE
    assert _lib.lib.pbn_batch_create(None, 0, 16, 0, 1, C.byref(h)) == _lib.PBN_E_INVALID


def _u32_threshold(T):
    a0 = T >> 21
    if a0 >= 1 << 32:
        return 1 << 32
    return a0 if ((a0 << 21) | (a0 >> 11)) >= T else a0 + 1


@pytest.mark.parametrize("name", ["bittner28", "bittner199", "bittner70", "edges"])
def test_compact_image_choice_matches_predstep(name):
    """The compact image the Philox kernels stage (u32 thresholds on the choice word, saturated at
    2^32 - 1, an overshoot record slot per node) selects Predstep's predictor (base.py:94-97) for
    every choice word, including a = 0 and 2^32 - 1, the words either side of every threshold, zero
    thresholds (leading predictors with COD 0) and never-reached ones. Host side: the same bytes
    and rule as the device (pbn_net_select_u32 mirrors predictor_choice32)."""
    import ctypes as C

    import numpy as np

    from gym_pbn_amd import _lib
    from gym_pbn_amd.batch import Net
    from gym_pbn_amd.network import load_network

    net = load_network("bittner28" if name == "edges" else name)
    if name == "edges":  # rewrite some nodes' thresholds to the edge cases (non-decreasing per node)
        net.pred_thr = net.pred_thr.copy()
        o = net.pred_offsets
        two53 = 1 << 53
        edge_rows = [[0, 0, 5], [two53, two53], [two53 - 1, two53], [0, (1 << 21) - 1, 1 << 21, (1 << 21) + 1],
                     [two53 - (1 << 21), two53 - (1 << 21) + 1, two53 - 1]]
        k = 0
        for i in range(net.n_nodes):
            c = int(o[i + 1] - o[i])
            if c < 2:
                continue
            row = edge_rows[k % len(edge_rows)]
            k += 1
            t = sorted((row * c)[: c - 1])
            net.pred_thr[o[i]:o[i] + c - 1] = np.asarray(t, dtype=np.uint64)
    h = Net(net)
    o = net.pred_offsets
    rng = np.random.default_rng(7)
    out = C.c_uint64()
    for i in range(net.n_nodes):
        c = int(o[i + 1] - o[i])
        T = [int(x) for x in net.pred_thr[o[i]:o[i] + c - 1]]
        words = {0, 1, 0xFFFFFFFE, 0xFFFFFFFF, *map(int, rng.integers(0, 1 << 32, 64))}
        for t in map(_u32_threshold, T):
            words |= {w for w in (t - 1, t, t + 1) if 0 <= w < 1 << 32}
        for a in sorted(words):
            k53 = (a << 21) | (a >> 11)
            j = min(sum(1 for x in T if k53 >= x), c - 1)
            q = o[i] + j
            want = (int(net.pred_inputs[q, 0]) | int(net.pred_inputs[q, 1]) << 16 | int(net.pred_inputs[q, 2]) << 32
                    | int(net.pred_tt[q]) << 48)
            assert _lib.lib.pbn_net_select_u32(h.handle, i, a, C.byref(out)) == 0
            assert out.value == want, (name, i, a, j)
