"""Network descriptors: the tables the HIP kernels stage in LDS.

Two dynamics families exist in the reference and both are represented here in
an integer-only form so that the device never touches floating point:

* :class:`PredictorNetwork` -- the Bittner engine (``gym_PBN/envs/bittner/base.py``).
  Each node owns a COD-weighted list of 3-input linear-threshold predictors
  (``Node.add_predictors`` ``base.py:30-45``). An async update draws
  ``r = random() * CODsum`` and takes the first predictor with
  ``cumCOD > r`` (``Node.Predstep`` ``base.py:93-97``), then evaluates
  ``Y = 0 if [x_in0, x_in1, x_in2, x_self] . A < 0 else 1`` (``base.py:100-118``).

  Exported per predictor: three input node indices, a 16-entry truth table
  evaluated with the reference's own ``np.matmul`` on the same array shapes, and
  an exact 53-bit threshold ``T_j`` such that, for ``random() == k53 * 2**-53``,
  ``cumCOD_j > random()*CODsum  <=>  k53 < T_j``. Predictor selection is then
  ``j = min(#{j : k53 >= T_j}, n_pred - 1)`` -- the ``min`` reproduces Python's
  ``for ... break`` falling through to the last predictor.

* :class:`TruthTableNetwork` -- the ``PBN``/``Node`` engine
  (``gym_PBN/envs/common/pbn.py:88-92``, ``common/node.py:31-38``). Each node has
  an input mask and a probability truth table indexed in C order by the masked
  inputs (lowest node index = most significant bit, ``node.py:32``). The draw
  ``u = numpy.random.uniform(0, 1) == k53 * 2**-53`` and ``u < p`` becomes
  ``k53 < ceil(p * 2**53)``, exact because scaling by 2**53 is exact.
"""

from __future__ import annotations

import math
from dataclasses import dataclass, field
from pathlib import Path
from typing import Sequence

import numpy as np

KIND_PREDICTOR_MIX = 1
KIND_PROB_TABLE = 2

TWO53 = 1 << 53
_INV53 = 1.0 / 9007199254740992.0  # exactly 2**-53, as CPython's random() uses
MAX_PRED_INPUTS = 3  # inputs per predictor (the self bit is the 4th pattern bit)

DATA_DIR = Path(__file__).resolve().parent / "data"


def n_words(n_nodes: int) -> int:
    return (int(n_nodes) + 63) // 64


def selection_threshold(cum: float, codsum: float) -> int:
    """Smallest k in [0, 2**53] with ``(k * 2**-53) * codsum >= cum`` (fp64).

    Mirrors ``r = random.random() * self.CODsum`` / ``if COD > r: break``
    (``base.py:94-97``): predictor j is skipped exactly when ``r >= cum_j``.
    ``fl(k * 2**-53 * c)`` is monotone in k, so the skipped set is a suffix
    ``[T_j, 2**53)`` and a binary search over k finds ``T_j``.
    """
    lo, hi = 0, TWO53  # invariant: answer in [lo, hi]; hi == 2**53 means "never skipped"
    while lo < hi:
        mid = (lo + hi) // 2
        if (float(mid) * _INV53) * codsum >= cum:
            hi = mid
        else:
            lo = mid + 1
    return lo


def probability_threshold(p: float) -> int:
    """``k53 < ceil(p * 2**53)``  <=>  ``k53 * 2**-53 < p`` (``node.py:37-38``)."""
    p = float(p)
    if not (p > 0.0):  # also catches NaN: u < NaN is False
        return 0
    t = math.ceil(p * float(TWO53))
    return min(t, (1 << 64) - 1)


def _predictor_truth_table(A: np.ndarray, n_inputs: int) -> int:
    """16-entry table over pattern ``x0<<3 | x1<<2 | x2<<1 | x_self``.

    Evaluated exactly like ``Node.Predstep`` (``base.py:100-118``): an fp64
    ``np.ones((len(IDs)+1, 1))`` column filled with the 0/1 inputs, then
    ``np.matmul(X.T, A)`` and ``Y = 0 if Ypred < 0. else 1``. Pattern bits for
    input slots the predictor does not have are ignored (table duplicated).
    """
    tt = 0
    for p in range(16):
        bits = [(p >> 3) & 1, (p >> 2) & 1, (p >> 1) & 1]
        xs = p & 1
        X = np.ones((n_inputs + 1, 1))
        for j in range(n_inputs):
            X[j] = bits[j]
        X[n_inputs] = xs
        Ypred = np.matmul(X.T, A)
        Y = 0 if Ypred < 0.0 else 1
        tt |= Y << p
    return tt


@dataclass
class PredictorNetwork:
    """Bittner predictor-mix network (``base.Graph`` of ``base.Node``)."""

    node_ids: np.ndarray  # int64 [N]
    pred_offsets: np.ndarray  # int32 [N+1]
    pred_inputs: np.ndarray  # int32 [P, 3] node indices (unused slots = self)
    pred_n_inputs: np.ndarray  # int32 [P]
    pred_tt: np.ndarray  # uint16 [P]
    pred_thr: np.ndarray  # uint64 [P]
    pred_cod: np.ndarray  # float64 [P] individual COD
    pred_cumcod: np.ndarray  # float64 [P]
    pred_A: np.ndarray  # float64 [P, 4]
    node_codsum: np.ndarray  # float64 [N]
    name: str = "bittner"
    kind: int = field(default=KIND_PREDICTOR_MIX, init=False)
    first_node: int = field(default=0, init=False)  # base.py:308 randint(0, N-1)

    @property
    def n_nodes(self) -> int:
        return int(self.node_ids.shape[0])

    @property
    def n_preds(self) -> int:
        return int(self.pred_tt.shape[0])

    @property
    def n_words(self) -> int:
        return n_words(self.n_nodes)

    @classmethod
    def from_predictor_sets(cls, predictor_sets: Sequence, node_ids: Sequence[int], name: str = "bittner"):
        """Build from the reference's predictor-set structure.

        ``predictor_sets[i]`` is the ``(3, n_pred)`` object array
        ``[COD; A; inputIDs]`` of node i (``predictor_sets.py:45,80-102``),
        ``node_ids[i]`` the gene ID of node i (``bittner/utils.py:81-88``).
        ``None`` CODs are skipped as in ``Node.add_predictors`` (``base.py:32-35``).
        """
        node_ids = [int(x) for x in node_ids]
        if len(node_ids) != len(predictor_sets):
            raise ValueError("node_ids and predictor_sets differ in length")
        index_of = {nid: i for i, nid in enumerate(node_ids)}
        if len(index_of) != len(node_ids):
            raise ValueError("duplicate node IDs")
        offs = [0]
        inputs, n_in, tts, thrs, cods, cums, As, codsums = [], [], [], [], [], [], [], []
        for i, ps in enumerate(predictor_sets):
            ps = np.asarray(ps, dtype=object)
            codsum = 0
            node_preds = []
            prev = None
            for COD, A, inputIDs in ps.T:  # same iteration as base.py:32
                if COD is None:
                    continue
                codsum += COD
                cum = COD if prev is None else prev + COD  # base.py:37-42
                prev = cum
                node_preds.append((COD, cum, np.asarray(A, dtype=np.float64), list(inputIDs)))
            if not node_preds:
                raise ValueError(f"node {i} has no predictors (Predstep would fail)")
            for COD, cum, A, ids in node_preds:
                k = len(ids)
                if not (1 <= k <= MAX_PRED_INPUTS):
                    raise ValueError(f"predictor with {k} inputs; 1..{MAX_PRED_INPUTS} supported")
                if A.shape != (k + 1, 1):
                    A = A.reshape(k + 1, 1)
                idx = []
                for gid in ids:
                    if int(gid) not in index_of:
                        raise ValueError(f"predictor input ID {gid} is not a node of the network")
                    idx.append(index_of[int(gid)])
                idx += [i] * (MAX_PRED_INPUTS - k)
                inputs.append(idx)
                n_in.append(k)
                tts.append(_predictor_truth_table(A, k))
                thrs.append(selection_threshold(float(cum), float(codsum)))
                cods.append(float(COD))
                cums.append(float(cum))
                a4 = np.zeros(4)
                a4[: k + 1] = A[:, 0]
                As.append(a4)
            codsums.append(float(codsum))
            offs.append(offs[-1] + len(node_preds))
        return cls(
            node_ids=np.asarray(node_ids, dtype=np.int64),
            pred_offsets=np.asarray(offs, dtype=np.int32),
            pred_inputs=np.asarray(inputs, dtype=np.int32).reshape(-1, MAX_PRED_INPUTS),
            pred_n_inputs=np.asarray(n_in, dtype=np.int32),
            pred_tt=np.asarray(tts, dtype=np.uint16),
            pred_thr=np.asarray(thrs, dtype=np.uint64),
            pred_cod=np.asarray(cods, dtype=np.float64),
            pred_cumcod=np.asarray(cums, dtype=np.float64),
            pred_A=np.asarray(As, dtype=np.float64).reshape(-1, 4),
            node_codsum=np.asarray(codsums, dtype=np.float64),
            name=name,
        )

    def save(self, path) -> None:
        np.savez_compressed(
            path, kind=np.int32(self.kind), name=np.array(self.name), node_ids=self.node_ids,
            pred_offsets=self.pred_offsets, pred_inputs=self.pred_inputs, pred_n_inputs=self.pred_n_inputs,
            pred_tt=self.pred_tt, pred_thr=self.pred_thr, pred_cod=self.pred_cod,
            pred_cumcod=self.pred_cumcod, pred_A=self.pred_A, node_codsum=self.node_codsum,
        )

    def validate(self) -> None:
        N, P = self.n_nodes, self.n_preds
        o = self.pred_offsets
        if o.shape != (N + 1,) or o[0] != 0 or o[-1] != P or np.any(np.diff(o) < 1):
            raise ValueError("bad pred_offsets")
        if self.pred_inputs.shape != (P, MAX_PRED_INPUTS):
            raise ValueError("bad pred_inputs shape")
        if P and (self.pred_inputs.min() < 0 or self.pred_inputs.max() >= N):
            raise ValueError("predictor input index out of range")
        for i in range(N):
            t = self.pred_thr[o[i]:o[i + 1]]
            if np.any(np.diff(t.astype(np.float64)) < 0):
                raise ValueError("thresholds must be non-decreasing within a node")

    def update_probability(self, state_bits: np.ndarray, node: int) -> float:
        """P(node -> 1 | state) = sum of selection masses of predictors voting 1.

        Used by the statistical tests of the Philox mode.
        """
        o0, o1 = int(self.pred_offsets[node]), int(self.pred_offsets[node + 1])
        prev = 0
        mass1 = 0
        for j in range(o0, o1):
            t = min(int(self.pred_thr[j]), TWO53) if j < o1 - 1 else TWO53
            w = t - prev
            prev = max(prev, t)
            x = [int(state_bits[self.pred_inputs[j, s]]) for s in range(3)]
            p = (x[0] << 3) | (x[1] << 2) | (x[2] << 1) | int(state_bits[node])
            if (int(self.pred_tt[j]) >> p) & 1:
                mass1 += max(w, 0)
        return mass1 / TWO53


@dataclass
class TruthTableNetwork:
    """Probability-truth-table network (``common/pbn.py`` ``PBN``)."""

    node_k: np.ndarray  # int32 [N]
    input_offsets: np.ndarray  # int32 [N+1]
    inputs: np.ndarray  # int32 [sum k] ascending node indices per node
    thr_offsets: np.ndarray  # int64 [N+1]
    thr: np.ndarray  # uint64 [sum 2**k]
    probs: np.ndarray  # float64 [sum 2**k]
    name: str = "pbn"
    kind: int = field(default=KIND_PROB_TABLE, init=False)
    first_node: int = field(default=1, init=False)  # pbn.py:131 randint(1, N-1)

    @property
    def n_nodes(self) -> int:
        return int(self.node_k.shape[0])

    @property
    def n_words(self) -> int:
        return n_words(self.n_nodes)

    @classmethod
    def from_pbn_data(cls, pbn_data: Sequence, name: str = "pbn"):
        """``PBN_DATA = [(input_mask, truth_table, name, is_control), ...]`` (``types.py:10``)."""
        N = len(pbn_data)
        ks, ioffs, ins, toffs, thr, probs = [], [0], [], [0], [], []
        for i, nd in enumerate(pbn_data):
            mask = np.asarray(nd[0], dtype=bool)
            if mask.shape != (N,):
                raise ValueError(f"node {i}: input mask must have length N={N}")
            tt = np.asarray(nd[1], dtype=np.float64)
            k = int(mask.sum())
            if tt.shape != (2,) * k:
                raise ValueError(f"node {i}: truth table shape {tt.shape} != {(2,) * k}")
            ks.append(k)
            ins.extend(np.nonzero(mask)[0].tolist())
            ioffs.append(ioffs[-1] + k)
            flat = tt.reshape(-1)  # C order == function.item(tuple(bits))
            probs.extend(flat.tolist())
            thr.extend(probability_threshold(p) for p in flat.tolist())
            toffs.append(toffs[-1] + flat.size)
        return cls(
            node_k=np.asarray(ks, dtype=np.int32),
            input_offsets=np.asarray(ioffs, dtype=np.int32),
            inputs=np.asarray(ins, dtype=np.int32),
            thr_offsets=np.asarray(toffs, dtype=np.int64),
            thr=np.asarray(thr, dtype=np.uint64),
            probs=np.asarray(probs, dtype=np.float64),
            name=name,
        )

    @classmethod
    def from_logic_funcs(cls, nodes: Sequence[str], node_functions: Sequence, name: str = "pbn"):
        """``PBN(logic_func_data=(nodes, node_functions))`` (``common/pbn.py:47-51``, ``converters.py:9-40``)."""
        from .io.logic import logic_funcs_to_pbn_data

        return cls.from_pbn_data(logic_funcs_to_pbn_data(nodes, node_functions), name=name)

    def save(self, path) -> None:
        np.savez_compressed(
            path, kind=np.int32(self.kind), name=np.array(self.name), node_k=self.node_k,
            input_offsets=self.input_offsets, inputs=self.inputs, thr_offsets=self.thr_offsets,
            thr=self.thr, probs=self.probs,
        )

    def validate(self) -> None:
        N = self.n_nodes
        if N < 2:
            raise ValueError("a PBN needs at least 2 nodes (node 0 is never updated)")
        if np.any(self.node_k < 0) or np.any(self.node_k > 16):
            raise ValueError("inputs per node must be in [0, 16]")
        if self.inputs.size and (self.inputs.min() < 0 or self.inputs.max() >= N):
            raise ValueError("input index out of range")
        exp = np.concatenate([[0], np.cumsum(1 << self.node_k.astype(np.int64))])
        if not np.array_equal(exp, self.thr_offsets):
            raise ValueError("thr_offsets inconsistent with node_k")


def load_network(path_or_name):
    """Load a descriptor ``.npz`` (path, or a bundled name such as ``"bittner199"``)."""
    p = Path(path_or_name)
    if not p.suffix:
        p = DATA_DIR / f"{path_or_name}.npz"
    with np.load(p, allow_pickle=False) as z:
        kind = int(z["kind"])
        name = str(z["name"])
        if kind == KIND_PREDICTOR_MIX:
            net = PredictorNetwork(
                node_ids=z["node_ids"], pred_offsets=z["pred_offsets"], pred_inputs=z["pred_inputs"],
                pred_n_inputs=z["pred_n_inputs"], pred_tt=z["pred_tt"], pred_thr=z["pred_thr"],
                pred_cod=z["pred_cod"], pred_cumcod=z["pred_cumcod"], pred_A=z["pred_A"],
                node_codsum=z["node_codsum"], name=name,
            )
        elif kind == KIND_PROB_TABLE:
            net = TruthTableNetwork(
                node_k=z["node_k"], input_offsets=z["input_offsets"], inputs=z["inputs"],
                thr_offsets=z["thr_offsets"], thr=z["thr"], probs=z["probs"], name=name,
            )
        else:
            raise ValueError(f"unknown network kind {kind}")
    net.validate()
    return net


def synthetic_truth_table_pbn(n_nodes: int = 200, k: int = 4, seed: int = 0):
    """random k-input masks, probabilities U[0,1) from default_rng(seed).

    Returns ``PBN_DATA`` (list of (input_mask, truth_table, name, is_control)).
    """
    rng = np.random.default_rng(seed)
    data = []
    for i in range(n_nodes):
        others = np.array([j for j in range(n_nodes) if j != i])
        inp = np.sort(rng.choice(others, size=k, replace=False))
        mask = np.zeros(n_nodes, dtype=bool)
        mask[inp] = True
        tt = rng.random((2,) * k)
        data.append((mask, tt, f"G{i}", False))
    return data


def synthetic_predictor_sets(n_nodes: int, max_preds: int = 5, seed: int = 0, ragged: bool = True):
    """Random predictor sets in the reference's pickle structure (``predictor_sets.py:45,80-102``).

    Node i gets 1..max_preds predictors (``ragged``) or exactly max_preds, each with 3
    distinct other nodes as inputs, a positive COD and a random 4x1 coefficient vector.
    Returns ``(predictor_sets, node_ids)`` for :meth:`PredictorNetwork.from_predictor_sets`.
    """
    rng = np.random.default_rng(seed)
    node_ids = np.arange(1000, 1000 + n_nodes)
    sets = []
    for i in range(n_nodes):
        k = int(rng.integers(1, max_preds + 1)) if ragged else max_preds
        ps = np.empty((3, k), dtype=object)
        others = np.array([j for j in range(n_nodes) if j != i])
        for q in range(k):
            ps[0, q] = float(rng.uniform(0.05, 1.0))
            ps[1, q] = rng.normal(size=(4, 1))
            ps[2, q] = [int(node_ids[j]) for j in rng.choice(others, size=3, replace=False)]
        sets.append(ps)
    return sets, node_ids
