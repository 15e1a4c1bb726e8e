"""Export the reference's shipped networks into the build's descriptor format.

Runs ONLY in the build container (it reads ``/root/reference``). Outputs go to
``gym-pbn-stac_amd/gym_pbn_amd/data/*.npz`` and are committed; the GPU box never
reads the reference.

Node order (which gene ID is node i) is what ``spawn()`` produced when each
pickle was generated (``gym_PBN/envs/bittner/utils.py:54-91``):

* ``predictor_sets_28_15_median.pkl``: the 28 IDs of ``tests/test_bittner.py:83``
  in that order (``total_genes == len(include_ids)``, so no pad and no sort).
* ``predictor_sets_{70,100,150,200}_*``: ``pad_ids(7 target IDs, N, weight_ids)``
  (``utils.py:42-51``) in pad order -- the pickles predate the ``sorted()`` at
  ``utils.py:68`` (sorted order gives 8-13 self-reference violations, pad order 0).
  ``weight_ids`` come from the xls via ``oracle/tools/xls_ids.py``; the reader is
  pinned by ``tests/test_bittner.py:18`` (276 IDs) and ``:27`` (first 70 padded).
  The 150/200 pickles have N-1 nodes: ``drop_duplicates`` (``utils.py:72``)
  removed one ID. It is 295483: the only candidate that (a) no predictor
  references, (b) leaves zero self-references, and (c) shares its name
  ('ESTs') with another included gene, which ``drop_duplicates`` requires.

Safety: pickles are decoded with ``gym_pbn_amd.io.safe_pickle`` (no code runs).
"""

from __future__ import annotations

import json
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(REPO / "gym-pbn-stac_amd"))
sys.path.insert(0, str(Path(__file__).resolve().parent))

import numpy as np  # noqa: E402

import xls_ids  # noqa: E402
from gym_pbn_amd.io.safe_pickle import load_pickle_safely  # noqa: E402
from gym_pbn_amd.network import (  # noqa: E402
    DATA_DIR,
    PredictorNetwork,
    TruthTableNetwork,
    synthetic_truth_table_pbn,
)

REF = Path("/root/reference")
BITTNER_DATA = REF / "gym_PBN" / "envs" / "bittner" / "data"

TARGET_IDS = [234237, 324901, 759948, 25485, 266361, 108208, 130057]  # pbn_target_multi.py:326,354
IDS_28 = [234237, 324901, 759948, 25485, 324700, 43129, 266361, 108208, 40764, 130057, 39781, 49665, 39159,
          23185, 417218, 31251, 343072, 142076, 128100, 376725, 112500, 241530, 44563, 36950, 812276, 51018,
          306013, 418105]  # tests/test_bittner.py:83 (also pbn_target_multi.py:551-553, unsorted)
DROPPED_ID = 295483


def pad_ids(current, pad_to, pool):
    """Restatement of ``bittner/utils.py:42-51``."""
    new = list(current)
    for _id in pool:
        if _id not in new:
            new.append(_id)
            if len(new) == pad_to:
                break
    return new


def inputs_of(ps):
    s = set()
    for x in ps[2]:
        if x is not None:
            s.update(int(v) for v in x)
    return s


def main():
    DATA_DIR.mkdir(parents=True, exist_ok=True)
    sheets = xls_ids.read_sheets(str(BITTNER_DATA / "genedata.xls"))
    wsheet = sheets["WEIGHTED GENE LIST"]
    hr, hc = xls_ids.find_header(wsheet, "Image Clone ID")
    weight_ids = [int(x) for x in xls_ids.column(wsheet, hc, hr + 1)]
    assert len(weight_ids) == 276, len(weight_ids)  # tests/test_bittner.py:18
    meta = {"weight_ids_count": len(weight_ids), "networks": {}}

    jobs = [
        ("bittner28", "predictor_sets_28_15_median.pkl", IDS_28),
        ("bittner70", "predictor_sets_70_5_kmeans.pkl", pad_ids(TARGET_IDS, 70, weight_ids)),
        ("bittner100", "predictor_sets_100_5_kmeans.pkl", pad_ids(TARGET_IDS, 100, weight_ids)),
        ("bittner149", "predictor_sets_150_5_kmeans.pkl",
         [x for x in pad_ids(TARGET_IDS, 150, weight_ids) if x != DROPPED_ID]),
        ("bittner199", "predictor_sets_200_5_kmeans.pkl",
         [x for x in pad_ids(TARGET_IDS, 200, weight_ids) if x != DROPPED_ID]),
    ]
    for name, fname, ids in jobs:
        ps = load_pickle_safely(BITTNER_DATA / fname)
        assert len(ps) == len(ids), (name, len(ps), len(ids))
        viol = sum(ids[i] in inputs_of(p) for i, p in enumerate(ps))
        assert viol == 0, (name, viol)
        net = PredictorNetwork.from_predictor_sets(ps, ids, name=name)
        net.validate()
        net.save(DATA_DIR / f"{name}.npz")
        meta["networks"][name] = {
            "source": f"gym_PBN/envs/bittner/data/{fname}", "n_nodes": net.n_nodes, "n_preds": net.n_preds,
            "preds_per_node": [int(x) for x in np.unique(np.diff(net.pred_offsets))],
        }
        print(name, net.n_nodes, net.n_preds)

    tt = TruthTableNetwork.from_pbn_data(synthetic_truth_table_pbn(200, 4, 0), name="tt200")
    tt.validate()
    tt.save(DATA_DIR / "tt200.npz")
    meta["networks"]["tt200"] = {"source": "synthetic_truth_table_pbn(200, 4, seed=0)", "n_nodes": 200}
    tt8 = TruthTableNetwork.from_pbn_data(synthetic_truth_table_pbn(8, 3, 1), name="tt8")
    tt8.save(DATA_DIR / "tt8.npz")
    meta["networks"]["tt8"] = {"source": "synthetic_truth_table_pbn(8, 3, seed=1)", "n_nodes": 8}
    (DATA_DIR / "networks.json").write_text(json.dumps(meta, indent=1) + "\n")


if __name__ == "__main__":
    main()
