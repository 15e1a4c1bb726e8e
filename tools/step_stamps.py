"""Phase stamps of the step kernel (measurement build: tools/build_exp.sh stamps -DPBN_STAMPS, run
with PBNSIM_LIB=build_exp/stamps/libpbnsim.so). One 1M-env Bittner-200 launch in the bench's window
(after 5 warm-up launches from fair-bit states); per wave s_memrealtime (100 MHz) at: entry, draws
done, barrier passed (image staged; the staging wait also covers the state loads), records read and
state landed, first pair's stores issued, all stores done. Prints percentiles (us from the first
wave's entry) per phase and the kernel span."""
import ctypes as C
import json
import os
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "gym-pbn-stac_amd"))
from gym_pbn_amd import _lib  # noqa: E402
from gym_pbn_amd.batch import PBNBatch  # noqa: E402

PHASES = ["entry", "draws_done", "barrier_passed", "landed_records_read", "stores_issued", "stores_done"]


def main():
    lib = _lib.lib
    lib.pbn_exp_stamps.argtypes = [C.c_void_p, C.c_size_t]
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
    out = {}
    for rep in range(3):
        b = PBNBatch("bittner199", B, seed=12345)
        b.randomize()
        b.step(5)
        b.sync()
        lib.pbn_exp_stamps_clear()
        b.step(1)
        b.sync()
        st = np.zeros(16384 * 8, dtype=np.uint64)
        assert lib.pbn_exp_stamps(st.ctypes.data, st.nbytes) == 0
        st = st.reshape(-1, 8)
        st = st[st[:, 0] != 0].astype(np.int64)
        t0 = st[:, 0].min()
        res = {"waves": int(len(st))}
        for k, name in enumerate(PHASES):
            v = (st[:, k] - t0) / 100.0  # 100 MHz ticks -> us
            res[name] = {q: round(float(np.percentile(v, q)), 2) for q in (0, 10, 50, 90, 100)}
        # per wave durations
        res["landed_minus_barrier_p50"] = round(float(np.median(st[:, 3] - st[:, 2])) / 100, 2)
        res["stores_done_minus_issued_p50"] = round(float(np.median(st[:, 5] - st[:, 4])) / 100, 2)
        res["issued_minus_landed_p50"] = round(float(np.median(st[:, 4] - st[:, 3])) / 100, 2)
        out[f"rep{rep}"] = res
        b.close()
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
