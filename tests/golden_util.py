"""Helpers to load the golden fixtures recorded from the reference (tests/golden/gen_golden.py)."""
from __future__ import annotations

import argparse
import json
import os

import numpy as np
import torch

from count_pipnet_amd.synthetic import synth_exponential, synth_images, synth_tensor

GOLDEN_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def golden_names():
    """Forward golden cases (eval_* fixtures belong to the eval_pipnet metric loop, input_*
    to the input transform, tests/test_input_oracle.py, train_* to the training iterations,
    tests/test_train_oracle.py, count_ste_bwd to the STE backward, tests/test_count_ste.py)."""
    return sorted(f[:-4] for f in os.listdir(GOLDEN_DIR)
                  if f.endswith(".npz") and not f.startswith(("eval_", "input_", "train_", "count_ste_")))


def eval_golden_names():
    return sorted(f[:-4] for f in os.listdir(GOLDEN_DIR) if f.startswith("eval_") and f.endswith(".npz"))


def load_golden(name: str):
    z = np.load(os.path.join(GOLDEN_DIR, name + ".npz"), allow_pickle=False)
    rec = {k: z[k] for k in z.files}
    meta = json.loads(str(rec.pop("meta")))
    return meta, rec


def golden_args(meta) -> argparse.Namespace:
    case = meta["case"]
    a = dict(disable_pretrained=True, positive_grad_strategy=None, backward_clamp_strategy="Gated")
    a.update({k: v for k, v in case.items() if k not in ("model", "num_classes", "batch", "size", "seed")})
    return argparse.Namespace(**a)


def golden_state_dict(meta):
    return {k: synth_tensor(k, tuple(s), meta["case"]["seed"], meta["profile"]) for k, s in meta["keys"]}


def golden_inputs(meta):
    c = meta["case"]
    xs = synth_images(c["batch"], c["size"], seed=c["seed"])
    assert abs(float(xs.double().sum()) - meta["input_sum"]) < 1e-6 * max(1.0, meta["input_abs"]), \
        "synthetic input generator drifted from the recorded fixture"
    return xs


def golden_noise(meta, shape):
    return synth_exponential(tuple(shape), meta["noise_seed"])


def proto_shape(meta, rec):
    c = meta["case"]
    p = rec["inf_pooled"].shape[1]
    if "inf_proto" in rec:
        return tuple(rec["inf_proto"].shape)
    hw = rec["inf_proto_pixmax"].shape[1:]
    return (c["batch"], p) + tuple(hw)


def eval_loader_batches(size: int, num_classes: int, nb: int, bs: int, label_seed: int):
    """The in-memory loader of the eval_* fixtures (tests/golden/gen_golden_eval.py):
    nb batches of (synthetic images, seeded labels)."""
    g = torch.Generator().manual_seed(label_seed)
    out = []
    for i in range(nb):
        xs = synth_images(bs, size, seed=label_seed * 100 + i)
        ys = torch.randint(0, num_classes, (bs,), generator=g)
        out.append((xs, ys))
    return out


def train_loader_batches(size: int, num_classes: int, nb: int, bs: int, seed: int):
    """The in-memory loader of the train_* fixtures (tests/golden/gen_golden_train.py):
    nb batches of (view-1 images, view-2 images, seeded labels)."""
    g = torch.Generator().manual_seed(seed)
    out = []
    for i in range(nb):
        xs1 = synth_images(bs, size, seed=seed * 100 + 2 * i)
        xs2 = synth_images(bs, size, seed=seed * 100 + 2 * i + 1)
        ys = torch.randint(0, num_classes, (bs,), generator=g)
        out.append((xs1, xs2, ys))
    return out


def train_golden_names():
    return sorted(f[:-4] for f in os.listdir(GOLDEN_DIR) if f.startswith("train_") and f.endswith(".npz"))


def load_train_golden(name: str):
    """(train meta, arrays, forward-case meta) of a train_* fixture."""
    meta, rec = load_golden(name)
    fwd_meta, _ = load_golden(meta["forward_case"])
    return meta, rec, fwd_meta


def train_step_lrs(meta):
    """Learning rate each iteration's optimizer step used: the initial lr, then the value
    the scheduler set after the previous iteration (train.py:120-122)."""
    return [meta["lr"]] + meta["info"]["lrs_class"][:-1]
