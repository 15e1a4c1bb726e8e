"""Attractors of small truth-table PBNs, as ``PBNEnv`` computes them at construction.

``PBNEnv.__init__`` always derives ``all_attractors`` from the full asynchronous
state transition graph (``pbn_env.py:54``, ``compute_attractors`` ``:233-240``):
``PBN.print_STG`` (``common/pbn.py:129-158``) adds one node per state,
``str(state.astype(int))`` with node 0 as the most significant bit of the state
index (``utils/__init__.py:4-12``), and an edge to every single-bit neighbour the
node can move to (``_compute_next_states`` async branch, ``pbn.py:178-191``):
node i set from 0 when ``P(x_i'=1) > 0``, cleared from 1 when ``P < 1``. The
attractors are networkx's attracting components, in networkx's order.

This is construction-time host work, exponential in N (the reference's too);
it is meant for the small networks ``PBNEnv`` is used with. Edge lists are built
vectorised over all 2^N states; the graph is handed to networkx in the same
node / edge insertion order as the reference so the attractor order matches.
"""

from __future__ import annotations

from typing import List, Set, Tuple

import numpy as np

from .network import TruthTableNetwork

MAX_STG_NODES = 22


def _state_bits(n: int) -> np.ndarray:
    idx = np.arange(1 << n, dtype=np.int64)
    return ((idx[:, None] >> (n - 1 - np.arange(n))) & 1).astype(np.int64)  # [2^n][n], node 0 = MSB


def prob_true_all(net: TruthTableNetwork, bits: np.ndarray) -> np.ndarray:
    """``P(x_i' = 1)`` for every state and node: ``function.item(tuple(state[input_mask]))``."""
    S, N = bits.shape
    out = np.empty((S, N), dtype=np.float64)
    for i in range(N):
        k = int(net.node_k[i])
        ins = net.inputs[net.input_offsets[i]:net.input_offsets[i + 1]]
        code = np.zeros(S, dtype=np.int64)
        for j in ins:  # first (lowest-index) input is the most significant axis
            code = (code << 1) | bits[:, j]
        base = int(net.thr_offsets[i])
        out[:, i] = net.probs[base:base + (1 << k)][code]
    return out


def async_stg_edges(net: TruthTableNetwork):
    """Per state, the (neighbour, probability) pairs in the reference's node order."""
    N = net.n_nodes
    if N > MAX_STG_NODES:
        raise ValueError(f"STG of {N} nodes has 2^{N} states; limit is {MAX_STG_NODES}")
    bits = _state_bits(N)
    p = prob_true_all(net, bits)
    up = (p > 0.0) & (bits == 0)
    down = (p < 1.0) & (bits == 1)
    return bits, p, up | down


def _label(bits_row) -> str:
    return str(np.asarray(bits_row, dtype=np.int64))


def compute_attractors(net: TruthTableNetwork) -> List[Set[Tuple[int, ...]]]:
    import networkx as nx

    bits, p, move = async_stg_edges(net)
    N = net.n_nodes
    labels = [_label(b) for b in bits]
    G = nx.DiGraph()
    flip = 1 << (N - 1 - np.arange(N))
    for s in range(bits.shape[0]):
        G.add_node(labels[s])
        cols = np.nonzero(move[s])[0]
        G.add_weighted_edges_from((labels[s], labels[s ^ int(flip[i])], float(p[s, i])) for i in cols)
    comps = list(nx.algorithms.components.attracting_components(G))
    return [set(tuple(int(x) for x in st.lstrip("[").rstrip("]").split()) for st in c) for c in comps]
