#!/usr/bin/env python3
"""The README's Python example, run as written (docs check)."""
import sys; sys.path.insert(0, "gym-pbn-stac_amd")  # noqa: E702
from gym_pbn_amd.batch import PBNBatch  # noqa: E402
b = PBNBatch("bittner199", 1 << 20, seed=7)   # 1,048,576 envs of the 199-node Bittner network
b.randomize()                                  # Graph.genRandState for every env
b.step(100)                                    # 100 async updates per env (Graph.step x100)
bits = b.get_bits()                            # [B][N] uint8
print(bits.shape, bits.dtype, int(bits.sum()))
