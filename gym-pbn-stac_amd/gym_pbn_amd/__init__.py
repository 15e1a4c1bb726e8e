"""gym_pbn_amd -- MI355X-native vectorised Probabilistic Boolean Network simulator.

Drop-in for the async-update hot path of gym-PBN (``gym_PBN/envs``): bit-packed
env states in HBM, hand-written gfx950 HIP kernels (libpbnsim.so, C ABI in
``include/pbn_abi.h``), reached through ctypes.

Importing the network/descriptor helpers needs no GPU; anything that steps
envs loads libpbnsim and fails loudly if it is missing.
"""

from .network import (  # noqa: F401
    KIND_PREDICTOR_MIX,
    KIND_PROB_TABLE,
    PredictorNetwork,
    TruthTableNetwork,
    load_network,
    synthetic_truth_table_pbn,
)

__version__ = "0.1.0"


def __getattr__(name):
    # lazy: loading libpbnsim (and torch) only when a device object is needed
    if name in ("Net", "EnvConfig", "PBNBatch", "pack_bits", "unpack_bits"):
        from . import batch

        return getattr(batch, name)
    if name in ("Graph", "PBN", "PBNTargetEnv", "PBNTargetMultiEnv", "VecPBNTargetMultiEnv", "PBNEnv", "state_to_idx"):
        from . import envs

        return getattr(envs, name)
    if name == "make":
        from .registry import make

        return make
    raise AttributeError(name)
