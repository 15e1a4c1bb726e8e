"""Attractor input format: CABEAN hypercube output -> ``all_attractors``.

Restates ``parse_state`` / ``parse_attractors``
(``gym_PBN/utils/get_attractors_from_cabean.py:9-36``): each attractor block
``=== find attractor #k : n states ===`` is followed by hypercube lines whose
first token lists one character per node at even positions, ``'-'`` meaning
"don't care" (``'*'`` in gym-PBN). The result feeds :class:`gym_pbn_amd.EnvConfig`.
Running cabean itself (``get_cabean_model.py:95``) is outside this package.
"""

from __future__ import annotations

from typing import Dict, List, Tuple


def parse_state(spec: str) -> Tuple:
    spec = spec[0:len(spec):2]
    return tuple(int(v) if v != "-" else "*" for v in spec)


def parse_attractors(cabean_out: str) -> Dict[int, List[Tuple]]:
    attractors: Dict[int, List[Tuple]] = {}
    num = None
    for line in cabean_out.split("\n"):
        if line.startswith("=") and "=== find attractor #" in line:
            parts = line.split()
            num = int(parts[3][1:]) - 1
        elif num is not None:
            if line.startswith(":"):
                continue
            if not line:
                num = None
                continue
            attractors.setdefault(num, []).append(parse_state(line.split()[0]))
    return attractors


def attractors_list(cabean_out: str) -> List[List[Tuple]]:
    """``list(parse_attractors(out).values())`` as ``get_attractors`` returns it (:50)."""
    return list(parse_attractors(cabean_out).values())
