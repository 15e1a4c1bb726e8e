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
