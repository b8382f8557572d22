"""Golden fixtures for the CountPIPNet count backward ("STE backward for
counts"), recorded by running the REFERENCE's own autograd Functions (unchanged) on CPU:

* ``ModifiedSTEFunction`` (pipnet/count_pipnet_utils.py:188-321) -- the one-hot encoder's
  backward, for every ``positive_grad_strategy`` (None, 'none', 'current_grad',
  'max_grad') x ``respect_active_grad`` -- on seeded counts and encoding gradients.  Cases:
  a mixed batch (zero counts, all-positive rows, ties), a batch with no all-positive row
  (the 'max_grad' batch-global branch falls back to the directional rule), and one whose
  gradients are sparse (rows of exact zeros, as a sparse classifier produces);
* ``ClampSTE`` (:58-84) "Gated" / "Identity" after ``STE_Round`` (:41-55), and the
  non-STE ``torch.clamp`` path of CountPIPNet.forward (count_pipnet.py:90-97).

Usage:  python tests/golden/gen_golden_ste.py   (writes tests/golden/count_ste_bwd.npz)
"""
from __future__ import annotations

import json
import os
import sys

sys.dont_write_bytecode = True            # /root/reference is read-only
HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference"

import numpy as np  # noqa: E402
import torch  # noqa: E402

STRATEGIES = [None, "none", "current_grad", "max_grad"]
MAX_COUNT = 3


def inputs(kind: str, seed: int):
    g = torch.Generator().manual_seed(seed)
    b, p = 6, 40
    # clamped counts (the encoder's input): 0..3 with soft offsets, some exact .5 (half-even)
    x = torch.randint(0, MAX_COUNT + 1, (b, p), generator=g).float()
    x = (x + (torch.rand(b, p, generator=g) - 0.5) * 0.9).clamp(0, MAX_COUNT)
    x[0, :4] = torch.tensor([0.5, 1.5, 2.5, 0.0])
    gr = torch.randn(b, p, MAX_COUNT, generator=g)
    if kind == "mixed":
        gr[1] = gr[1].abs() + 0.01                          # all-positive rows
        gr[2, :, 1] = gr[2, :, 0]                           # ties (first index wins)
    elif kind == "no_allpos":
        gr[:, :, 0] = -gr[:, :, 0].abs() - 0.01             # every row has a negative entry
    elif kind == "sparse":
        keep = torch.rand(b, p, 1, generator=g) < 0.5
        gr = gr * keep                                      # exact-zero rows
    return x, gr


def main():
    sys.path.insert(0, REF)
    from pipnet.count_pipnet_utils import ClampSTE, ModifiedSTEFunction, STE_Round
    rec, meta = {}, {"max_count": MAX_COUNT, "strategies": [str(s) for s in STRATEGIES], "cases": []}
    for ci, kind in enumerate(("mixed", "no_allpos", "sparse")):
        x, gr = inputs(kind, 40 + ci)
        rec[f"{kind}_x"] = x.numpy()
        rec[f"{kind}_g"] = gr.numpy()
        for si, strat in enumerate(STRATEGIES):
            for ra in (False, True):
                xi = x.clone().requires_grad_(True)
                enc = ModifiedSTEFunction.apply(xi, MAX_COUNT, ra, strat)
                rec[f"{kind}_enc"] = enc.detach().numpy()
                enc.backward(gr)
                rec[f"{kind}_dx_s{si}_ra{int(ra)}"] = xi.grad.numpy()
        meta["cases"].append(kind)
    # ClampSTE after STE_Round, and plain clamp (no STE)
    g = torch.Generator().manual_seed(77)
    counts = torch.rand(8, 32, generator=g) * 5 - 0.8           # raw soft counts, some < 0 and > max
    counts[0, :3] = torch.tensor([3.4, 3.5, 3.6])
    dcl = torch.randn(8, 32, generator=g)
    rec["clamp_counts"], rec["clamp_dclamped"] = counts.numpy(), dcl.numpy()
    for name, ident in (("gated", False), ("identity", True)):
        c = counts.clone().requires_grad_(True)
        ClampSTE.apply(STE_Round.apply(c), 0, MAX_COUNT, ident).backward(dcl)
        rec[f"clamp_dcounts_ste_{name}"] = c.grad.numpy()
    c = counts.clone().requires_grad_(True)
    torch.clamp(c, 0, MAX_COUNT).backward(dcl)
    rec["clamp_dcounts_plain"] = c.grad.numpy()
    meta["torch"] = torch.__version__
    rec["meta"] = np.array(json.dumps(meta))
    path = os.path.join(HERE, "count_ste_bwd.npz")
    np.savez_compressed(path, **rec)
    print(f"wrote {path}")


if __name__ == "__main__":
    main()
