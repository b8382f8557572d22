"""eval_pipnet metric loop (pipnet/test.py:12-200): the oracle's restatement reproduces the
reference's own info dict, recorded by tests/golden/gen_golden_eval.py from the unchanged
reference, from the per-batch pooled / logits / weights the reference saw."""
import json

import numpy as np
import pytest
import torch

from golden_util import eval_golden_names, load_golden
from oracle import ref_cpu

NAMES = eval_golden_names()


def eval_batches(rec, meta):
    """[(pooled, out, w, ys)] per batch, w = the weight the reference's scores used."""
    w = torch.from_numpy(rec["w_initial"])
    out = []
    for i in range(meta["batches"]):
        w = torch.clamp(w - 1e-3, min=0.0)                     # test.py:73, in place each batch
        ws = torch.from_numpy(rec["count_class_weights"]) if "count_class_weights" in rec else w
        out.append((torch.from_numpy(rec[f"b{i}_pooled"]), torch.from_numpy(rec[f"b{i}_out"]), ws,
                    torch.from_numpy(rec[f"b{i}_ys"])))
    return out


@pytest.mark.parametrize("name", NAMES)
def test_oracle_eval_loop_matches_reference(name):
    meta, rec = load_golden(name)
    k = rec["cm"].shape[0]
    got = ref_cpu.eval_loop(eval_batches(rec, meta), k, meta["multiplier"])
    assert np.array_equal(got["confusion_matrix"], rec["cm"])
    assert got["abstained"] == meta["abstained"]
    for key, v in meta["info"].items():
        if key in got:
            assert got[key] == v, (key, got[key], v)      # exact: same float ops, same order


def test_eval_inventory():
    assert {"eval_pipnet_mid_addon", "eval_pipnet_c2", "eval_count_onehot"} <= set(NAMES)
