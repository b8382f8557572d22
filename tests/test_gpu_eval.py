"""eval_pipnet on the GPU (count_pipnet_amd.evaluate) against the reference's recorded run.

* metric kernel (pipnet_eval_batch_f32) fed the reference's own per-batch pooled / logits /
  weights: confusion matrix, abstain count, argmax and every accumulated mean EXACT
  (integer counts, fp32 means, fp64 running sums -- the reference's float semantics);
  confidence scores within 1e-6;
* end to end: count_pipnet_amd.evaluate.eval_pipnet on the HIP model with the same weights,
  labels and images: the returned info dict equals the reference's (exact where the
  forward's 1e-3-parity outputs decide no threshold, else within one prototype per image);
* the in-place sparsify kernel == torch.clamp(w - 1e-3, 0).
"""
import contextlib
import io

import numpy as np
import pytest
import torch

from count_pipnet_amd import kernels as K
from golden_util import eval_golden_names, load_golden
from oracle import ref_cpu
from test_eval_golden import eval_batches

pytestmark = pytest.mark.gpu
NAMES = eval_golden_names()


@pytest.mark.parametrize("name", NAMES)
def test_eval_batch_kernel_matches_reference(gpu, name):
    meta, rec = load_golden(name)
    k = rec["cm"].shape[0]
    cm = torch.zeros((k, k), dtype=torch.int64, device=gpu)
    acc = torch.zeros(5, dtype=torch.float64, device=gpu)
    abst = torch.zeros(1, dtype=torch.int64, device=gpu)
    mult = torch.tensor([meta["multiplier"]], device=gpu)
    for pooled, out, w, ys in eval_batches(rec, meta):
        ys_pred, conf = K.eval_batch(pooled.to(gpu), out.to(gpu), w.contiguous().to(gpu), ys.to(gpu), mult, 1e-3,
                                     cm, acc, abst)
        r = ref_cpu.eval_batch_metrics(pooled, out, w, ys, meta["multiplier"])
        assert torch.equal(ys_pred.cpu().long(), r["ys_pred"])
        assert torch.allclose(conf.cpu(), r["conf"], rtol=1e-6, atol=1e-7)
    nb = meta["batches"]
    a = acc.cpu().tolist()
    info = meta["info"]
    assert np.array_equal(cm.cpu().numpy(), rec["cm"])
    assert int(abst.item()) == meta["abstained"]
    assert a[0] / nb == info["local_size_for_true_class"]
    assert a[1] / nb == info["local_size_for_all_classes"]
    assert a[2] / nb == info["prototypes_per_class"]
    assert a[3] / nb == info["almost_nonzeros"]
    assert a[4] / nb == info["top1_accuracy"]


def test_sparsify_kernel(gpu):
    g = torch.Generator().manual_seed(5)
    w = torch.randn(200, 768, generator=g) * 1e-2
    wd = w.to(gpu)
    K.weight_sparsify_(wd, 1e-3)
    assert torch.equal(wd.cpu(), torch.clamp(w - 1e-3, min=0.0))


@pytest.mark.parametrize("name", ["eval_pipnet_mid_addon", "eval_pipnet_c2"])
def test_eval_pipnet_end_to_end(gpu, name):
    from count_pipnet_amd.dist import ShardedInference
    from count_pipnet_amd.evaluate import eval_pipnet
    from golden_util import eval_loader_batches
    from model_util import build_model
    meta, rec = load_golden(name)
    fmeta, _ = load_golden(meta["forward_case"])
    net = build_model(fmeta)
    with torch.no_grad():
        net._classification.weight.copy_(torch.from_numpy(rec["w_initial"]))
    case = fmeta["case"]
    batches = eval_loader_batches(case["size"], case["num_classes"], meta["batches"], meta["batch_size"],
                                  meta["label_seed"])
    for i, (_, ys) in enumerate(batches):
        ys.copy_(torch.from_numpy(rec[f"b{i}_ys"]))
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf), contextlib.redirect_stderr(io.StringIO()):
        info = eval_pipnet(ShardedInference(net.to(gpu)), batches, 0, gpu)
    assert f"abstained from a decision for {meta['abstained']} images" in buf.getvalue()
    ref = meta["info"]
    assert np.array_equal(info["confusion_matrix"], rec["cm"])
    assert info["test_accuracy"] == ref["test_accuracy"] and info["top1_accuracy"] == ref["top1_accuracy"]
    assert info["num non-zero prototypes"] == ref["num non-zero prototypes"]
    for key in ("local_size_for_true_class", "local_size_for_all_classes", "prototypes_per_class", "almost_nonzeros"):
        assert abs(info[key] - ref[key]) <= 1.0, (key, info[key], ref[key])
    assert torch.equal(net._classification.weight.detach().cpu(),
                       torch.from_numpy(eval_batches(rec, meta)[-1][2].numpy()))
