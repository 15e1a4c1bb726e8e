"""Descriptor construction (host logic, CPU only): thresholds, truth tables, safe decoding."""

import math
import pickle
import random

import numpy as np
import pytest

from gym_pbn_amd.io.safe_pickle import UnsafePickleError, decode_pickle_bytes
from gym_pbn_amd.network import (
    TWO53,
    PredictorNetwork,
    TruthTableNetwork,
    load_network,
    probability_threshold,
    selection_threshold,
    synthetic_truth_table_pbn,
)


def _reference_pick(k53, cums, codsum):
    """base.py:94-97 verbatim: r = random()*CODsum; first COD > r, else the last."""
    r = (k53 * (1.0 / 9007199254740992.0)) * codsum
    j = 0
    for j, c in enumerate(cums):
        if c > r:
            break
    return j


def _threshold_pick(k53, thr):
    return min(sum(1 for t in thr if k53 >= t), len(thr) - 1)


@pytest.mark.parametrize("name", ["bittner28", "bittner199", "bittner70", "bittner100", "bittner149"])
def test_selection_thresholds_exact_at_boundaries(name):
    net = load_network(name)
    rng = random.Random(5)
    for i in range(net.n_nodes):
        o0, o1 = net.pred_offsets[i], net.pred_offsets[i + 1]
        cums, thr = net.pred_cumcod[o0:o1], [int(t) for t in net.pred_thr[o0:o1]]
        codsum = net.node_codsum[i]
        probes = [0, TWO53 - 1] + [rng.randrange(TWO53) for _ in range(20)]
        for t in thr:
            probes += [max(t - 2, 0), max(t - 1, 0), min(t, TWO53 - 1), min(t + 1, TWO53 - 1)]
        for k in probes:
            assert _reference_pick(k, cums, codsum) == _threshold_pick(k, thr), (name, i, k)


def test_selection_threshold_definition():
    c = 0.8666666639999999 * 3
    for cum in (0.1, 0.8666666639999999, 1.7333333279999998, c):
        t = selection_threshold(cum, c)
        assert (t * 2.0**-53) * c >= cum or t == TWO53
        assert t == 0 or ((t - 1) * 2.0**-53) * c < cum


def test_probability_threshold():
    for p in (0.0, 1e-300, 0.25, 0.5, 0.9999999999999999, 1.0, 1.0000000000000002):
        t = probability_threshold(p)
        for k in (0, 1, TWO53 // 2, TWO53 - 1, max(t - 1, 0), min(t, TWO53 - 1)):
            assert (k * 2.0**-53 < p) == (k < t)
    assert probability_threshold(float("nan")) == 0
    assert probability_threshold(-0.5) == 0


def test_truth_tables_match_predstep_expression():
    net = load_network("bittner199")
    for j in range(0, net.n_preds, 37):
        A = net.pred_A[j][:, None]
        for p in range(16):
            X = np.ones((4, 1))
            X[0], X[1], X[2], X[3] = (p >> 3) & 1, (p >> 2) & 1, (p >> 1) & 1, p & 1
            y = 0 if np.matmul(X.T, A) < 0.0 else 1
            assert ((int(net.pred_tt[j]) >> p) & 1) == y


def test_bundled_networks():
    shapes = {"bittner28": (28, 420), "bittner70": (70, 349), "bittner100": (100, 499), "bittner149": (149, 744),
              "bittner199": (199, 994)}
    for name, (n, p) in shapes.items():
        net = load_network(name)
        assert (net.n_nodes, net.n_preds) == (n, p)
        # no node predicts from itself (predictor_sets.py:47 drops the gene)
        for i in range(n):
            ins = net.pred_inputs[net.pred_offsets[i]:net.pred_offsets[i + 1]]
            k = net.pred_n_inputs[net.pred_offsets[i]:net.pred_offsets[i + 1]]
            assert all(i not in row[:kk] for row, kk in zip(ins, k))
    tt = load_network("tt200")
    assert tt.n_nodes == 200 and tt.thr.shape == (200 * 16,)


def test_from_predictor_sets_skips_none_and_builds_cumcod():
    A = np.array([[1.0], [-1.0], [0.5], [-0.25]])
    ps = np.empty((3, 3), dtype=object)
    ps[:, 0] = (0.5, A, np.array([11, 12, 13]))
    ps[:, 1] = (0.25, -A, np.array([12, 13, 11]))
    ps[:, 2] = (None, None, None)
    nets = [ps.copy() for _ in range(4)]
    ids = [10, 11, 12, 13]
    for i in range(4):
        nets[i][:, 0] = (0.5, A, np.array([x for x in ids if x != ids[i]]))
        nets[i][:, 1] = (0.25, -A, np.array([x for x in ids if x != ids[i]][::-1]))
    net = PredictorNetwork.from_predictor_sets(nets, ids)
    assert net.n_preds == 8
    assert np.allclose(net.pred_cumcod[:2], [0.5, 0.75]) and net.node_codsum[0] == 0.75
    net.validate()


def test_truth_table_network_c_order():
    data = synthetic_truth_table_pbn(6, 3, 2)
    net = TruthTableNetwork.from_pbn_data(data)
    for i, (mask, tt, _, _) in enumerate(data):
        ins = np.nonzero(mask)[0]
        assert list(net.inputs[net.input_offsets[i]:net.input_offsets[i + 1]]) == list(ins)
        for bits in np.ndindex(*tt.shape):
            flat = int("".join(map(str, bits)), 2)  # first masked node is the MSB (node.py:32)
            p = tt.item(bits)
            assert net.probs[net.thr_offsets[i] + flat] == p
            assert int(net.thr[net.thr_offsets[i] + flat]) == math.ceil(p * 2**53)


def test_safe_pickle_decodes_data_and_refuses_code():
    arr = np.empty((3, 2), dtype=object)
    arr[:, 0] = (0.5, np.arange(4.0).reshape(4, 1), np.array([1, 2, 3]))
    arr[:, 1] = (None, None, None)
    data = pickle.dumps([arr, {"k": (1, 2.5, "s", b"b", True)}], protocol=4)
    out = decode_pickle_bytes(data)
    assert out[1] == {"k": (1, 2.5, "s", b"b", True)}
    assert out[0].shape == (3, 2) and out[0][0, 0] == 0.5
    assert np.array_equal(out[0][1, 0], np.arange(4.0).reshape(4, 1))

    class Evil:
        def __reduce__(self):
            return (print, ("pwned",))

    with pytest.raises(UnsafePickleError):
        decode_pickle_bytes(pickle.dumps(Evil()))
    with pytest.raises(UnsafePickleError):
        decode_pickle_bytes(pickle.dumps(np.random.default_rng(0)))


def test_cabean_parse_kat():
    """parse_attractors(sample_cabean_out) (get_attractors_from_cabean.py:57-81)."""
    import json

    from conftest import GOLDEN
    from gym_pbn_amd.io.cabean import parse_attractors

    kat = json.loads((GOLDEN / "cabean_parse_kat.json").read_text())
    got = parse_attractors(kat["input"])
    assert {str(k): [list(t) for t in v] for k, v in got.items()} == kat["expected"]
