"""Golden fixtures for the eval_pipnet metric loop, recorded by running
the REFERENCE's own ``pipnet/test.py:eval_pipnet`` (unchanged) on CPU.

For each case the reference model of a forward golden case (gen_golden.CASES, same
synthetic weights) is wrapped in ``nn.DataParallel`` (CPU: it calls the module directly)
and evaluated over a small in-memory loader of synthetic images with seeded labels.
The classifier is made sparse (3 of 4 weights zeroed, seeded) as in a trained PIP-Net, and
every other label is set to the class the model predicts (a pre-pass), so accuracy and the
confusion matrix are non-trivial.
Recorded per batch: the exact ``pooled`` / ``out`` the reference produced (captured with
a forward hook) and the labels; the classification weight batch i saw is the (i+1)-fold
in-place sparsify ``clamp(W - 1e-3, 0)`` of ``w_initial`` (pipnet/test.py:71-73; checked
here while recording); recorded at the end: every entry of the returned ``info`` dict
plus the printed "abstained" count and sparsity ratio.

Usage:  python tests/golden/gen_golden_eval.py
"""
from __future__ import annotations

import contextlib
import io
import json
import os
import re
import sys

sys.dont_write_bytecode = True            # /root/reference is read-only
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.nn as nn  # noqa: E402

import gen_golden as G  # noqa: E402

sys.path.insert(0, os.path.dirname(HERE))
from golden_util import eval_loader_batches  # noqa: E402

# name -> (forward golden case, batches, batch size, label seed)
EVAL_CASES = {
    "eval_pipnet_mid_addon": ("pipnet_mid_addon", 3, 6, 101),
    "eval_pipnet_c2": ("c2_pipnet_convnext26", 2, 3, 102),
    "eval_count_onehot": ("count_onehot", 3, 5, 103),
}


def run(name):
    fwd_case, nb, bs, label_seed = EVAL_CASES[name]
    net, case = G.build_reference(fwd_case)
    sys.path.insert(0, G.REF)
    from pipnet.test import eval_pipnet
    batches = eval_loader_batches(case["size"], case["num_classes"], nb, bs, label_seed)
    with torch.no_grad():    # a sparse classifier, as a trained PIP-Net has (keep 1 weight in 4)
        keep = torch.rand(net._classification.weight.shape, generator=torch.Generator().manual_seed(label_seed)) < 0.25
        net._classification.weight.mul_(keep)
    # every other label = the class the model will predict, so accuracy / confusion are non-trivial
    with torch.no_grad(), G.injected_exponential(seed=2000 + case["seed"]):
        w0 = net._classification.weight.detach().clone()
        for xs, ys in batches:
            net._classification.weight.copy_(torch.clamp(net._classification.weight - 1e-3, min=0.0))
            ys[::2] = net(xs, inference=True)[2].argmax(1)[::2]
        net._classification.weight.copy_(w0)
    dp = nn.DataParallel(net)
    rec = {"w_initial": net._classification.weight.detach().clone().numpy()}
    if hasattr(net, "_max_count"):   # eval_pipnet takes these once, before its loop (test.py:53-58)
        ptc = torch.stack([net.get_prototype_importance_per_class(i) for i in range(net._num_prototypes)], 0)
        rec["count_class_weights"] = ptc.detach().t().contiguous().numpy()   # [K, P]
    seen = []

    def hook(mod, inp, outp):
        seen.append((outp[1].detach().clone(), outp[2].detach().clone(),
                     mod._classification.weight.detach().clone()))

    h = net.register_forward_hook(hook)
    buf = io.StringIO()
    with G.injected_exponential(seed=2000 + case["seed"]), contextlib.redirect_stdout(buf), \
            contextlib.redirect_stderr(io.StringIO()):
        info = eval_pipnet(dp, batches, 0, torch.device("cpu"))
    h.remove()
    text = buf.getvalue()
    abst = int(re.search(r"abstained from a decision for (\d+) images", text).group(1))
    spars = float(re.search(r"sparsity ratio:\s+([0-9.eE+-]+)", text).group(1))
    for i, ((xs, ys), (pooled, out, w)) in enumerate(zip(batches, seen)):
        rec[f"b{i}_ys"] = ys.numpy()
        rec[f"b{i}_pooled"] = pooled.numpy()
        rec[f"b{i}_out"] = out.numpy()
        w_chk = torch.from_numpy(rec["w_initial"])
        for _ in range(i + 1):
            w_chk = torch.clamp(w_chk - 1e-3, min=0.0)
        assert torch.equal(w_chk, w), "per-batch weight is not the iterated sparsify of w_initial"
    rec["cm"] = info["confusion_matrix"]
    scal = {k: float(v) for k, v in info.items() if k != "confusion_matrix"}
    meta = dict(name=name, forward_case=fwd_case, batches=nb, batch_size=bs, label_seed=label_seed,
                info=scal, abstained=abst, sparsity_ratio=spars, noise_seed=2000 + case["seed"],
                multiplier=float(net._classification.normalization_multiplier.item()))
    rec["meta"] = np.array(json.dumps(meta))
    return rec


def main():
    torch.set_num_threads(os.cpu_count() or 8)
    for name in EVAL_CASES:
        rec = run(name)
        path = os.path.join(HERE, f"{name}.npz")
        np.savez_compressed(path, **rec)
        print(f"wrote {path} ({os.path.getsize(path) / 1e3:.1f} kB)", json.loads(str(rec["meta"]))["info"],
              flush=True)


if __name__ == "__main__":
    main()
