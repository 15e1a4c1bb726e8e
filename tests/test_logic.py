"""Logic-function import path (utils/logic/eval.py, utils/converters.py:9-40) vs reference KATs."""

import json
from itertools import product

import numpy as np
import pytest

from conftest import GOLDEN

KAT = json.loads((GOLDEN / "logic_kat.json").read_text())


@pytest.mark.parametrize("rec", KAT["expressions"], ids=lambda r: r["expr"])
def test_expression_evaluator_matches_reference(rec):
    from gym_pbn_amd.io.logic import LogicExpressionEvaluator

    e = rec["expr"]
    if "error" in rec and "symbols" not in rec:
        with pytest.raises(Exception):
            LogicExpressionEvaluator.get_symbols(e)
        return
    syms = LogicExpressionEvaluator.get_symbols(e)
    assert syms == rec["symbols"]
    order = sorted(set(syms))
    if "error" in rec:
        with pytest.raises(Exception):
            LogicExpressionEvaluator(dict(zip(order, [0] * len(order)))).evaluate(e)
        return
    got = [int(LogicExpressionEvaluator(dict(zip(order, bits))).evaluate(e))
           for bits in product([0, 1], repeat=len(order))]
    assert got == rec["values"]


@pytest.mark.parametrize("i", range(len(KAT["networks"])))
def test_logic_funcs_to_pbn_data_matches_reference(i):
    from gym_pbn_amd.io.logic import logic_funcs_to_pbn_data

    rec = KAT["networks"][i]
    funcs = [[tuple(f) for f in fs] for fs in rec["functions"]]
    if "error" in rec:
        with pytest.raises(Exception):
            logic_funcs_to_pbn_data(rec["nodes"], funcs)
        return
    data = logic_funcs_to_pbn_data(rec["nodes"], funcs)
    assert len(data) == len(rec["expected"])
    for d, exp in zip(data, rec["expected"]):
        assert d[0].astype(int).tolist() == exp["mask"]
        assert np.asarray(d[1]).reshape(-1).tolist() == exp["table"]  # exact float sums
        assert d[2] == exp["name"] and bool(d[3]) == exp["control"]


def test_truth_table_network_from_logic_funcs():
    from gym_pbn_amd.network import TruthTableNetwork

    rec = KAT["networks"][0]
    net = TruthTableNetwork.from_logic_funcs(rec["nodes"], [[tuple(f) for f in fs] for fs in rec["functions"]])
    net.validate()
    assert net.n_nodes == 5 and net.node_k.tolist() == [0, 2, 4, 3, 2]
