#!/usr/bin/env python3
"""Host-side timing of each call inside TorchVecPBNTargetMultiEnv.step (measurement only)."""
import sys
import time

sys.path.insert(0, "gym-pbn-stac_amd")
sys.path.insert(0, "tests")
import numpy as np  # noqa: E402
import torch  # noqa: E402

from conftest import cubes_to_attractors  # noqa: E402
from gym_pbn_amd import _lib as L  # noqa: E402
from gym_pbn_amd.torch_env import TorchVecPBNTargetMultiEnv  # noqa: E402

B = 1 << 20
side = len(sys.argv) > 1 and sys.argv[1] == "side"
if side:  # a dedicated (non-default) torch stream for the env and its tensor ops
    torch.cuda.set_stream(torch.cuda.Stream())
z = np.load("tests/golden/r6_bittner199.npz")
env = TorchVecPBNTargetMultiEnv("bittner199", cubes_to_attractors(z, 199), B, horizon=100, update_cap=4096,
                                auto_reset=True, seed=7)
g = torch.Generator(device="cuda")
g.manual_seed(7)
a = (torch.randint(1, 200, (B, 4), device="cuda", generator=g, dtype=torch.int32)
     * (torch.rand((B, 4), device="cuda", generator=g) >= 0.75))
env.reset()
torch.cuda.synchronize()
T = {}


def tick(name, t0):
    t = time.perf_counter()
    T[name] = T.get(name, 0.0) + (t - t0)
    return t


for it in range(8):
    if it == 3:  # the first iterations load torch's kernels lazily
        torch.cuda.synchronize()
        T.clear()
    t = time.perf_counter()
    env._use_stream()
    t = tick("use_stream", t)
    words = torch.empty((B, env.W), dtype=torch.int64, device="cuda")
    t = tick("empty", t)
    env.batch.env_step_multi_device(env.cfg, a.data_ptr(), 4, words.data_ptr(), env._reward.data_ptr(),
                                    env._flags.data_ptr(), env._nup.data_ptr(), update_cap=4096)
    t = tick("env_step", t)
    term = (env._flags & L.FLAG_TERMINATED) != 0
    trunc = (env._flags & L.FLAG_TRUNCATED) != 0
    t = tick("flags", t)
    obs = env._bits(words)
    t = tick("unpack", t)
    r = env._reward.clone()
    t = tick("clone", t)
    done = (term | trunc).to(torch.uint8).contiguous()
    t = tick("done", t)
    env.batch.env_reset_device(env.cfg, done.data_ptr())
    t = tick("reset", t)
torch.cuda.synchronize()
for k, v in T.items():
    print(f"{k:12s} {v / 5 * 1e3:8.3f} ms/step", flush=True)
t0 = time.perf_counter()
for _ in range(5):
    obs, r, te, tr, info = env.step(a)
torch.cuda.synchronize()
print("env.step total", round((time.perf_counter() - t0) / 5 * 1e3, 3), "ms/step")
