"""ctypes binding of libpbnsim.so (the C ABI in include/pbn_abi.h).

The library is the only compute path: if it is missing, importing this module
raises, and there is no Python/NumPy fallback for any transition.

``torch`` is imported first when available so that libpbnsim binds to the same
HIP runtime (soname libamdhip64.so.7) torch already loaded; two runtimes in one
process would not share streams or device pointers.
"""

from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

try:  # share torch's HIP runtime if torch is present (see module docstring)
    import torch  # noqa: F401
except Exception:  # pragma: no cover - torch is plumbing, not required
    torch = None

PKG_DIR = Path(__file__).resolve().parent
LIB_PATH = Path(os.environ.get("PBNSIM_LIB", PKG_DIR / "libpbnsim.so"))

PBN_OK = 0
PBN_E_INVALID = -1
PBN_E_RANGE = -2
PBN_E_HIP = -3
PBN_E_NOMEM = -4
PBN_E_UNSUPPORTED = -5
PBN_E_STATE = -6

FLAG_TERMINATED = 1
FLAG_TRUNCATED = 2
FLAG_CAPPED = 4

_u64p = C.POINTER(C.c_uint64)
_i64p = C.POINTER(C.c_int64)
_u32p = C.POINTER(C.c_uint32)
_i32p = C.POINTER(C.c_int32)
_u16p = C.POINTER(C.c_uint16)
_u8p = C.POINTER(C.c_uint8)
_vp = C.c_void_p


class PbnError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"[{code}] {msg}")
        self.code = code


class NetDesc(C.Structure):
    _fields_ = [
        ("kind", C.c_int32), ("n_nodes", C.c_int32), ("n_preds", C.c_int32),
        ("pred_offsets", _i32p), ("pred_inputs", _i32p), ("pred_tt", _u16p), ("pred_thr", _u64p),
        ("node_k", _i32p), ("input_offsets", _i32p), ("inputs", _i32p), ("thr_offsets", _i64p), ("thr", _u64p),
    ]


class BatchInfo(C.Structure):
    _fields_ = [
        ("n_nodes", C.c_int32), ("n_words", C.c_int32), ("kind", C.c_int32), ("device", C.c_int32),
        ("n_envs", C.c_uint64), ("env_id_base", C.c_uint64), ("seed", C.c_uint64), ("update_count", C.c_uint64),
        ("env_call_count", C.c_uint32), ("reset_count", C.c_uint32), ("mt_ready", C.c_int32),
        ("env_lanes", C.c_int32), ("roll_lanes", C.c_int32), ("env_grid", C.c_int32), ("env_kernel", C.c_int32),
        ("env_lane_limit", C.c_int32), ("env_handoff", C.c_int32), ("env_chunk", C.c_int32),
    ]


class EnvCfgDesc(C.Structure):
    _fields_ = [
        ("n_cubes", C.c_int32), ("cube_care", _u64p), ("cube_value", _u64p),
        ("n_reset_cubes", C.c_int32), ("reset_care", _u64p), ("reset_value", _u64p),
        ("target_care", _u64p), ("target_value", _u64p),
        ("horizon", C.c_int32), ("reward_success", C.c_int32), ("action_cost", C.c_int32),
        ("first_update_tested", C.c_int32),
    ]


_PP = C.POINTER(_vp)

# name -> (restype, argtypes); mirrors include/pbn_abi.h one to one
SIGNATURES = {
    "pbn_abi_version": (C.c_int, []),
    "pbn_last_error": (C.c_char_p, []),
    "pbn_device_count": (C.c_int, [C.POINTER(C.c_int)]),
    "pbn_net_create": (C.c_int, [C.POINTER(NetDesc), _PP]),
    "pbn_net_destroy": (None, [_vp]),
    "pbn_net_select_u32": (C.c_int, [_vp, C.c_int32, C.c_uint32, _u64p]),
    "pbn_batch_create": (C.c_int, [_vp, C.c_int, C.c_uint64, C.c_uint64, C.c_uint64, _PP]),
    "pbn_batch_destroy": (None, [_vp]),
    "pbn_batch_get_info": (C.c_int, [_vp, C.POINTER(BatchInfo)]),
    "pbn_sync": (C.c_int, [_vp]),
    "pbn_set_state": (C.c_int, [_vp, _u64p]),
    "pbn_get_state": (C.c_int, [_vp, _u64p]),
    "pbn_set_state_device": (C.c_int, [_vp, _vp]),
    "pbn_get_state_device": (C.c_int, [_vp, _vp]),
    "pbn_randomize_state": (C.c_int, [_vp]),
    "pbn_flip": (C.c_int, [_vp, _i32p, C.c_int, C.c_int, C.c_int]),
    "pbn_flip_device": (C.c_int, [_vp, _vp, C.c_int, C.c_int, C.c_int, C.c_int]),
    "pbn_step": (C.c_int, [_vp, C.c_uint32]),
    "pbn_step_prepare": (C.c_int, [_vp, C.c_uint32]),
    "pbn_rollout": (C.c_int, [_vp, C.c_uint32]),
    "pbn_step_replay": (C.c_int, [_vp, _u32p, _u64p, C.c_uint32]),
    "pbn_step_forced": (C.c_int, [_vp, _u32p, C.c_uint32]),
    "pbn_mt_seed": (C.c_int, [_vp, _u64p, C.c_int]),
    "pbn_mt_step": (C.c_int, [_vp, C.c_uint32]),
    "pbn_envcfg_create": (C.c_int, [_vp, C.POINTER(EnvCfgDesc), _PP]),
    "pbn_envcfg_destroy": (None, [_vp]),
    "pbn_env_reset": (C.c_int, [_vp, _vp, _u8p]),
    "pbn_env_reset_device": (C.c_int, [_vp, _vp, _vp]),
    "pbn_batch_set_stream": (C.c_int, [_vp, C.c_int, _vp]),
    "pbn_unpack_bits_device": (C.c_int, [_vp, _vp, _vp]),
    "pbn_set_n_steps": (C.c_int, [_vp, _i64p]),
    "pbn_get_n_steps": (C.c_int, [_vp, _i64p]),
    "pbn_env_step_multi": (C.c_int, [_vp, _vp, _i32p, C.c_int, C.c_int, C.c_int, C.c_uint32, _u64p, _i32p, _u8p,
                                     _u32p]),
    "pbn_env_step_multi_device": (C.c_int, [_vp, _vp, _vp, C.c_int, C.c_int, C.c_int, C.c_uint32, _vp, _vp, _vp,
                                            _vp]),
    "pbn_env_rollout_multi_device": (C.c_int, [_vp, _vp, C.c_uint32, _vp, C.c_int, C.c_int, C.c_int, C.c_uint32,
                                               _vp, _vp, _vp, _vp]),
    "pbn_env_step_multi_replay": (C.c_int, [_vp, _vp, _i32p, C.c_int, C.c_int, C.c_int, _i64p, _u32p, _u64p, _u64p,
                                            _i32p, _u8p, _u32p]),
    "pbn_ssd_run": (C.c_int, [_vp, _i32p, C.c_int, _u32p, C.c_uint32, _u64p]),
    "pbn_synch_step": (C.c_int, [_vp, C.c_uint32, _u32p]),
    "pbn_timing_enable": (C.c_int, [_vp, C.c_int]),
    "pbn_timing_read": (C.c_int, [_vp, C.POINTER(C.c_double), C.POINTER(C.c_uint64)]),
    "pbn_timing_read_each": (C.c_int, [_vp, C.POINTER(C.c_double), C.c_uint64, C.POINTER(C.c_uint64)]),
    "pbn_env_handoffs": (C.c_int, [_vp, _u32p]),
    "pbn_env_tail_helpers": (C.c_int, [_vp, _u32p]),
    "pbn_env_tail_stats": (C.c_int, [_vp, _u32p]),
    "pbn_env_grid_stats": (C.c_int, [_vp, _u32p]),
}


def _load():
    if not LIB_PATH.exists():
        raise ImportError(
            f"{LIB_PATH} not found: build it with `make -C gym-pbn-stac_amd` (or __graft_entry__.build()). "
            "gym_pbn_amd has no CPU fallback."
        )
    lib = C.CDLL(str(LIB_PATH))
    for name, (res, args) in SIGNATURES.items():
        f = getattr(lib, name)
        f.restype = res
        f.argtypes = args
    return lib


lib = _load()


def last_error() -> str:
    m = lib.pbn_last_error()
    return m.decode() if m else ""


def check(rc: int) -> None:
    if rc == PBN_OK:
        return
    msg = last_error()
    if rc in (PBN_E_RANGE, PBN_E_INVALID):
        raise ValueError(msg)
    raise PbnError(rc, msg)


def device_count() -> int:
    n = C.c_int(0)
    rc = lib.pbn_device_count(C.byref(n))
    return n.value if rc == PBN_OK else 0


def ptr(a, t):
    return a.ctypes.data_as(t) if a is not None else None
