"""Load the reference's hot-path modules from /root/reference by file path.

Fixture tooling only: used by ``make_golden.py`` in the build container, never
by tests, ``smoke()`` or ``bench.py`` (the GPU box has no /root/reference).

``gym_PBN/__init__.py`` registers gymnasium envs and is skipped: the hot-path
modules (``bittner/base.py``, ``common/node.py``, ``common/pbn.py`` and their
``gym_PBN.types`` / ``gym_PBN.utils`` imports) load without any stand-in.
The env module ``pbn_target_multi.py`` (R6) additionally imports gymnasium,
numba (unused, ``predictor_sets.py:10``) and colomoto (``get_attractors_from_cabean.py:4``),
none of which is installed; for that module only, inert import stand-ins are
registered (an empty ``gymnasium.Env`` base class, space classes that just
record their arguments, a pass-through ``njit``, dict subclasses for the
colomoto types). None of them is on the computed path of ``step()``.
The macro-action env modules (``pbn_env.py``, ``pbcn_env.py``, ``sampled_data.py``,
``self_triggering.py``) use the same stand-ins; their spaces' ``contains`` accepts
everything (only valid actions are fed), so action validation is not pinned.
"""

from __future__ import annotations

import importlib.util
import sys
import types
from pathlib import Path

REF = Path("/root/reference")
PKG = REF / "gym_PBN"


def _load(modname: str, path: Path, package: str | None = None):
    if modname in sys.modules:
        return sys.modules[modname]
    is_pkg = path.name == "__init__.py"
    spec = importlib.util.spec_from_file_location(
        modname, path, submodule_search_locations=[str(path.parent)] if is_pkg else None
    )
    mod = importlib.util.module_from_spec(spec)
    if package is not None:
        mod.__package__ = package
    sys.modules[modname] = mod
    spec.loader.exec_module(mod)
    return mod


def _shell(modname: str, path: Path):
    """A namespace entry for a package whose __init__ must not run."""
    if modname not in sys.modules:
        m = types.ModuleType(modname)
        m.__path__ = [str(path)]
        m.__package__ = modname
        sys.modules[modname] = m
    return sys.modules[modname]


def load_hot_path():
    """Return (base, node, pbn) reference modules."""
    _shell("gym_PBN", PKG)
    _load("gym_PBN.types", PKG / "types.py")
    _load("gym_PBN.utils", PKG / "utils" / "__init__.py")
    _load("gym_PBN.utils.logic", PKG / "utils" / "logic" / "__init__.py")
    _load("gym_PBN.utils.logic.eval", PKG / "utils" / "logic" / "eval.py")
    _load("gym_PBN.utils.converters", PKG / "utils" / "converters.py")
    _shell("gym_PBN.envs", PKG / "envs")
    _shell("gym_PBN.envs.bittner", PKG / "envs" / "bittner")
    base = _load("gym_PBN.envs.bittner.base", PKG / "envs" / "bittner" / "base.py")
    _shell("gym_PBN.envs.common", PKG / "envs" / "common")
    node = _load("gym_PBN.envs.common.node", PKG / "envs" / "common" / "node.py")
    pbn = _load("gym_PBN.envs.common.pbn", PKG / "envs" / "common" / "pbn.py")
    return base, node, pbn


def _install_env_import_standins():
    if "gymnasium" not in sys.modules:
        gym = types.ModuleType("gymnasium")

        class Env:  # inert base class
            pass

        gym.Env = Env
        gym.register = lambda *a, **k: None
        spaces = types.ModuleType("gymnasium.spaces")

        class _Space:
            """Records its arguments; ``n`` is the first one. ``contains`` accepts everything:
            fixtures only ever feed valid actions, so action validation is not pinned by them."""

            def __init__(self, *a, **k):
                self.args = a
                self.n = a[0] if a else None
                self.start = k.get("start", 0)

            def contains(self, x):
                return True

        for n in ("Discrete", "MultiBinary", "MultiDiscrete", "Box", "Tuple"):
            setattr(spaces, n, type(n, (_Space,), {}))
        gym.spaces = spaces
        sys.modules["gymnasium"] = gym
        sys.modules["gymnasium.spaces"] = spaces
    if "numba" not in sys.modules:
        nb = types.ModuleType("numba")
        nb.njit = lambda *a, **k: (a[0] if a and callable(a[0]) else (lambda f: f))
        sys.modules["numba"] = nb
    if "colomoto" not in sys.modules:
        c = types.ModuleType("colomoto")
        ct = types.ModuleType("colomoto.types")
        ct.PartialState = type("PartialState", (dict,), {})
        ct.Hypercube = type("Hypercube", (dict,), {})
        c.types = ct
        sys.modules["colomoto"] = c
        sys.modules["colomoto.types"] = ct


def load_multi_env():
    """Return the reference ``pbn_target_multi`` module (R6)."""
    load_hot_path()
    _install_env_import_standins()
    bt = PKG / "envs" / "bittner"
    _load("gym_PBN.envs.bittner.gen.binarise", bt / "gen" / "binarise.py")
    _load("gym_PBN.envs.bittner.gen.predictor_sets", bt / "gen" / "predictor_sets.py")
    _load("gym_PBN.envs.bittner.gen", bt / "gen" / "__init__.py")
    _load("gym_PBN.envs.bittner.utils", bt / "utils.py")
    sys.modules["gym_PBN.envs.bittner"].base = sys.modules["gym_PBN.envs.bittner.base"]
    sys.modules["gym_PBN.envs.bittner"].utils = sys.modules["gym_PBN.envs.bittner.utils"]
    _shell("gym_PBN.utils", PKG / "utils")
    _load("gym_PBN.utils.get_cabean_model", PKG / "utils" / "get_cabean_model.py")
    _load("gym_PBN.utils.get_attractors_from_cabean", PKG / "utils" / "get_attractors_from_cabean.py")
    return _load("gym_PBN.envs.pbn_target_multi", PKG / "envs" / "pbn_target_multi.py",
                 package="gym_PBN.envs")


def load_target_env():
    """Return the reference ``pbn_target`` module (R5; its ``step`` raises at HEAD, ``reset`` runs)."""
    load_multi_env()
    return _load("gym_PBN.envs.pbn_target", PKG / "envs" / "pbn_target.py", package="gym_PBN.envs")


def load_mdp_envs():
    """Return the reference modules (pbn_env, pbcn_env, sampled_data, self_triggering, pbcn)."""
    load_hot_path()
    _install_env_import_standins()
    common = PKG / "envs" / "common"
    pbcn = _load("gym_PBN.envs.common.pbcn", common / "pbcn.py")
    envs = PKG / "envs"
    pbn_env = _load("gym_PBN.envs.pbn_env", envs / "pbn_env.py", package="gym_PBN.envs")
    pbcn_env = _load("gym_PBN.envs.pbcn_env", envs / "pbcn_env.py", package="gym_PBN.envs")
    sampled = _load("gym_PBN.envs.sampled_data", envs / "sampled_data.py", package="gym_PBN.envs")
    selftrig = _load("gym_PBN.envs.self_triggering", envs / "self_triggering.py", package="gym_PBN.envs")
    return pbn_env, pbcn_env, sampled, selftrig, pbcn


def build_graph(base, predictor_sets, node_ids):
    """A reference ``base.Graph`` with ``base.Node(i, i, name, ID).add_predictors(ps[i])``
    (as ``bittner/utils.py:81-91`` builds it)."""
    g = base.Graph(2)
    nodes = []
    for i, (ps, nid) in enumerate(zip(predictor_sets, node_ids)):
        n = base.Node(i, i, f"gene{nid}", int(nid))
        n.add_predictors(ps)
        nodes.append(n)
    g.nodes = nodes
    return g


class DrawRecorder:
    """Proxy for a module-level RNG that logs each draw it forwards."""

    def __init__(self, rng):
        self._rng = rng
        self.log = []

    def randint(self, a, b):
        v = self._rng.randint(a, b)
        self.log.append(("i", v))
        return v

    def random(self):
        v = self._rng.random()
        self.log.append(("u", v))
        return v

    def uniform(self, a, b):
        v = self._rng.uniform(a, b)
        self.log.append(("u", v))
        return v

    def __getattr__(self, n):
        return getattr(self._rng, n)
