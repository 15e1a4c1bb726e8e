"""Wall-clock window of the bench headline (20 timed launches at 1M envs) under variants of the
host-side bracket: the idle sleep before it, the batch-stream sync before torch's device sync,
the HIP event region. Measurement only; prints one JSON line per variant (median of reps)."""
import json
import statistics
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "gym-pbn-stac_amd"))
import torch  # noqa: E402

from gym_pbn_amd.batch import PBNBatch  # noqa: E402
from gym_pbn_amd.network import load_network  # noqa: E402


def window(net, B, sleep, batch_sync, events, steps=20, warmup=5):
    b = PBNBatch(net, B, device=0, env_id_base=0, seed=12345)
    b.randomize()
    b.step(warmup)
    b.prepare_steps(steps)
    b.sync()
    if sleep == 1:
        time.sleep(0.005)
    elif sleep == 2:  # busy wait (bench.py's gap)
        t = time.perf_counter()
        while time.perf_counter() - t < 2e-4:
            pass
    torch.cuda.synchronize()
    if events:
        b.timing(2)
    t0 = time.perf_counter()
    b.step(steps)
    if events:
        b.timing(0)
    if batch_sync:
        b.sync()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    ev = b.timing_read()[0] / steps * 1e3 if events else None
    b.close()
    return (t1 - t0) / steps * 1e6, ev


def main():
    net = load_network("bittner199")
    B = 1 << 20
    torch.zeros(1, device="cuda")
    variants = {"bench": (1, 1, 1), "no_sleep": (0, 1, 1), "torch_sync_only": (1, 0, 1),
                "no_events": (1, 1, 0), "no_sleep_torch_sync_only": (0, 0, 1), "bare": (0, 0, 0),
                "spin_torch_sync_only (bench.py now)": (2, 0, 1)}
    res = {k: [] for k in variants}
    for _ in range(int(sys.argv[1]) if len(sys.argv) > 1 else 7):
        for k, v in variants.items():
            res[k].append(window(net, B, *v))
    for k, r in res.items():
        w = [x[0] for x in r]
        e = [x[1] for x in r if x[1] is not None]
        print(json.dumps({"variant": k, "wall_us_per_step_median": round(statistics.median(w), 3),
                          "wall_us_all": [round(x, 2) for x in w],
                          "event_us_median": round(statistics.median(e), 3) if e else None}))


if __name__ == "__main__":
    main()
