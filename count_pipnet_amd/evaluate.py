"""Evaluation loop -- drop-in for ``pipnet/test.py`` (``eval_pipnet``,
``evaluate_model_lightweight``, ``acc_from_cm``, ``compute_local_explanation_sizes``).

The reference's ``eval_pipnet`` (test.py:12-200) is the immediate caller of the hot path
(SURVEY.md 8f rank 1).  Per batch it sparsifies the classifier in place, runs
``net(xs, inference=True)``, materialises ``scores = pooled * W`` as a [K, B, P] tensor and
reduces it on the host side of ~B+5 synchronisations (``.item()`` per metric, a Python
loop over GPU scalars for the confusion matrix).  Here every batch stays on the device:
``pipnet_weight_sparsify_f32`` + the HIP forward + ``pipnet_eval_batch_f32`` (argmax,
confidence, abstain, top-1, confusion matrix, explanation sizes; fp64 running sums), and
the host reads the accumulators once after the loop.  The returned ``info`` dict, the
prints and the two-class report are the reference's.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn.functional as F

from . import kernels as K

THRESHOLD = 1e-3          # test.py:73 (sparsify), :104 (local sizes), :108, :121


def _module(net):
    return net.module if hasattr(net, "module") else net


def _bump_version(t: torch.Tensor) -> None:
    """The in-place HIP write bypasses autograd's version counter; bump it so that any
    version-stamped cache of this parameter sees the change."""
    inc = getattr(torch.autograd.graph, "increment_version", None)
    if inc is not None:
        inc(t)


@torch.no_grad()
def eval_pipnet(net, test_loader, epoch, device, log=None, progress_prefix: str = "Eval Epoch",
                enforce_weight_sparsity: bool = True, args=None) -> dict:
    """pipnet/test.py:12-200 with the per-batch metrics on the GPU (same ``info`` dict)."""
    from tqdm import tqdm
    net = net.to(device)
    net.eval()
    mod = _module(net)
    is_count_pipnet = hasattr(mod, "_max_count")
    nc = mod._num_classes
    dev = torch.device(device)
    cm = torch.zeros((nc, nc), dtype=torch.int64, device=dev)
    acc = torch.zeros(5, dtype=torch.float64, device=dev)
    abstained = torch.zeros(1, dtype=torch.int64, device=dev)

    if is_count_pipnet:          # test.py:50-62: taken once, before the loop
        ptc = torch.stack([mod.get_prototype_importance_per_class(i) for i in range(mod._num_prototypes)], dim=0)
        assert ptc.shape[0] == mod._num_prototypes and ptc.shape[1] == nc
        classification_weights = ptc.t().contiguous().float()      # [K, P]
    else:
        classification_weights = mod._classification.weight

    preds, scores, trues = [], [], []
    n_batches = 0
    test_iter = tqdm(enumerate(test_loader), total=len(test_loader), desc=progress_prefix + " %s" % epoch,
                     mininterval=5., ncols=0)
    for _, (xs, ys) in test_iter:
        xs, ys = xs.to(device, non_blocking=True), ys.to(device, non_blocking=True)
        if enforce_weight_sparsity:
            w = mod._classification.weight
            K.weight_sparsify_(w.detach(), THRESHOLD)
            _bump_version(w)
        _, pooled, out = net(xs, inference=True)
        w_scores = classification_weights if is_count_pipnet else mod._classification.weight
        ys_pred, score = K.eval_batch(pooled.contiguous(), out.contiguous(), w_scores.detach().contiguous(),
                                      ys.long().contiguous(), mod._classification.normalization_multiplier.detach(),
                                      THRESHOLD, cm, acc, abstained)
        preds.append(ys_pred)
        scores.append(score)
        trues.append(ys)
        n_batches += 1

    # the only host synchronisation of the loop
    nb = max(len(test_loader), 1)
    acc_h = acc.cpu().tolist()
    cm_h = cm.cpu().numpy().astype(int)
    y_preds = torch.cat(scores).cpu().tolist() if scores else []
    y_trues = torch.cat(trues).cpu().tolist() if trues else []
    y_preds_classes = torch.cat(preds).cpu().tolist() if preds else []
    print("PIP-Net abstained from a decision for", int(abstained.item()), "images", flush=True)
    info = dict()
    info["num non-zero prototypes"] = torch.gt(classification_weights, THRESHOLD).any(dim=0).sum().item()
    w = mod._classification.weight
    print("sparsity ratio: ", (torch.numel(w) - torch.count_nonzero(F.relu(w - THRESHOLD)).item()) / torch.numel(w),
          flush=True)
    info["confusion_matrix"] = cm_h
    info["test_accuracy"] = acc_from_cm(cm_h)
    info["top1_accuracy"] = acc_h[4] / nb
    info["local_size_for_true_class"] = acc_h[0] / nb
    info["local_size_for_all_classes"] = acc_h[1] / nb
    info["prototypes_per_class"] = acc_h[2] / nb
    info["almost_nonzeros"] = acc_h[3] / nb

    if nc == 2:                  # test.py:162-188
        from sklearn.metrics import balanced_accuracy_score, roc_auc_score
        tp, fn, fp, tn = cm_h[0][0], cm_h[0][1], cm_h[1][0], cm_h[1][1]
        print("TP: ", tp, "FN: ", fn, "FP:", fp, "TN:", tn, flush=True)
        sensitivity = tp / (tp + fn)
        specificity = tn / (tn + fp)
        print("\n Epoch", epoch, flush=True)
        print("Confusion matrix: ", cm_h, flush=True)
        try:
            for classname, classidx in test_loader.dataset.class_to_idx.items():
                if classidx == 0:
                    print("Accuracy positive class (", classname, classidx, ") (TPR, Sensitivity):", tp / (tp + fn))
                elif classidx == 1:
                    print("Accuracy negative class (", classname, classidx, ") (TNR, Specificity):", tn / (tn + fp))
        except (ValueError, AttributeError):
            pass
        print("Balanced accuracy: ", balanced_accuracy_score(y_trues, y_preds_classes), flush=True)
        print("Sensitivity: ", sensitivity, "Specificity: ", specificity, flush=True)
        try:
            print("AUC macro: ", roc_auc_score(y_trues, y_preds, average="macro"), flush=True)
            print("AUC weighted: ", roc_auc_score(y_trues, y_preds, average="weighted"), flush=True)
        except ValueError:
            pass
    return info


@torch.no_grad()
def evaluate_model_lightweight(net, loader, device):
    """pipnet/test.py:202-259: accuracy + confusion matrix, accumulated on the device."""
    from tqdm import tqdm
    net.eval()
    nc = _module(net)._num_classes
    cm = torch.zeros((nc, nc), dtype=torch.int64, device=torch.device(device))
    for inputs, targets in tqdm(loader, desc="Evaluating"):
        inputs, targets = inputs.to(device), targets.to(device)
        _, _, outputs = net(inputs, inference=True)
        _, predicted = outputs.max(1)
        cm.index_put_((targets.long(), predicted), torch.ones_like(predicted), accumulate=True)
    cm_h = cm.cpu().numpy()
    total = int(cm_h.sum())
    accuracy = float(np.trace(cm_h)) / total if total else 0.0
    labels_present = np.flatnonzero(cm_h.sum(0) + cm_h.sum(1))    # sklearn's confusion_matrix label set
    results = {"accuracy": accuracy, "confusion_matrix": cm_h[np.ix_(labels_present, labels_present)],
               "num_classes": nc}
    print(f"Evaluation completed. Accuracy: {accuracy:.4f}")
    return results


def acc_from_cm(cm: np.ndarray) -> float:
    """pipnet/test.py:261-276."""
    assert len(cm.shape) == 2 and cm.shape[0] == cm.shape[1]
    total = np.sum(cm)
    return 1 if total == 0 else np.trace(cm) / total


def compute_local_explanation_sizes(scores: torch.Tensor, ys_pred: torch.Tensor, threshold: float = 1e-3):
    """pipnet/test.py:278-319 (torch ops, any device): (any-class sizes, predicted-class sizes)."""
    relevant = torch.abs(scores) > threshold                         # [K, B, P]
    any_class_sizes = relevant.any(dim=0).sum(dim=1)
    local = relevant.sum(dim=2).float()                              # [K, B]
    pred_class_sizes = local.gather(0, ys_pred.view(1, -1)).view(-1)
    return any_class_sizes.float(), pred_class_sizes.float()
