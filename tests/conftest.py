import sys
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parents[1]
for p in (ROOT, ROOT / "gym-pbn-stac_amd", ROOT / "oracle"):
    if str(p) not in sys.path:
        sys.path.insert(0, str(p))

GOLDEN = ROOT / "tests" / "golden"


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs through libpbnsim on the device)")


@pytest.fixture(scope="session")
def oracle_mod():
    import oracle

    oracle.build()
    return oracle


def golden(name):
    return np.load(GOLDEN / name, allow_pickle=False)


def r6_config(z):
    """EnvConfig pieces of an r6 fixture: cubes, reset cubes (attractor 0), target (last attractor, cube 0)."""
    attr = z["cube_attractor"]
    last = int(np.nonzero(attr == attr.max())[0][0])
    first = np.nonzero(attr == 0)[0]
    return dict(care=z["cube_care"], value=z["cube_value"], target_care=z["cube_care"][last],
                target_value=z["cube_value"][last], reset_care=z["cube_care"][first],
                reset_value=z["cube_value"][first], horizon=int(z["horizon"]))


def cubes_to_attractors(z, n_nodes):
    """Rebuild all_attractors (lists of '*'/int tuples) from an r6 fixture's care/value arrays."""
    from gym_pbn_amd.batch import attractors_from_cubes

    return attractors_from_cubes(z["cube_care"], z["cube_value"], z["cube_attractor"], n_nodes)
