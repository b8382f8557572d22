"""ORACLE -- CPU restatement of one PIP-Net training iteration after the forward
(pipnet/train.py:75-140 with calculate_loss :154-250 and align_loss :259-265), finetune
phase: loss values, the gradient of the loss w.r.t. the classifier, torch.optim.AdamW
(util/args.py:327-328) and the post-step clamps (train.py:134-140).

TEST INFRASTRUCTURE ONLY.  Only ``tests/`` (and ``bench.py``'s ``cpu_baseline`` leg) may
import this module, as the checker -- never as the product path (the product is
``count_pipnet_amd/csrc/train_ops.hip``).

The reference computes the gradient with autograd; here every derivative is written out
(softmax-minus-one-hot, log1p and pow backward, relu threshold backward), so this is an
independent statement of the same math.  Pinned against fixtures recorded by running the
reference's own ``train_pipnet`` (``tests/golden/gen_golden_train.py``).
"""
from __future__ import annotations

from typing import Dict, Optional, Tuple

import torch

Tensor = torch.Tensor

FINETUNE_WEIGHTS = (5.0, 2.0, 2.0)         # align, tanh, class (train.py:56-61)


def align_loss(pf1: Tensor, pf2: Tensor, eps: float = 1e-12) -> Tensor:
    """train.py:259-265 on [n, P] rows: -log(<a_n, b_n> + eps).mean()."""
    return -torch.log((pf1 * pf2).sum(dim=1) + eps).mean()


def proto_pixels(proto: Tensor) -> Tensor:
    """[B,P,h,w] -> [B*h*w, P] (train.py:160-161: flatten(2).permute(0,2,1).flatten(0,1))."""
    return proto.flatten(start_dim=2).permute(0, 2, 1).flatten(end_dim=1)


def loss_terms(proto: Tensor, pooled: Tensor, out: Tensor, ys1: Tensor, mult: float, enforce: bool = True,
               tanh_coeff: float = 1.0, is_count: bool = False, eps_tanh: float = 1e-8) -> Dict[str, Tensor]:
    """calculate_loss's three raw terms + accuracy (train.py:154-246)."""
    n = pooled.shape[0]
    pf1, pf2 = proto[: n // 2], proto[n // 2:]
    e1, e2 = proto_pixels(pf1), proto_pixels(pf2)
    a = (align_loss(e1, e2) + align_loss(e2, e1)) / 2.0
    p1, p2 = pooled[: n // 2], pooled[n // 2:]
    if is_count:
        p1, p2 = tanh_coeff * p1, tanh_coeff * p2
    t = -(torch.log(torch.tanh(p1.sum(dim=0)) + eps_tanh).mean()
          + torch.log(torch.tanh(p2.sum(dim=0)) + eps_tanh).mean()) / 2.0
    x = torch.log1p(out ** mult) if enforce else out
    ys = torch.cat([ys1, ys1])
    lsm = x - torch.logsumexp(x, dim=1, keepdim=True)
    cls = -lsm[torch.arange(n), ys].mean()
    correct = (out.argmax(dim=1) == ys).sum()
    return dict(align=a, tanh=t, cls=cls, correct=correct)


def d_out(out: Tensor, ys1: Tensor, mult: float, enforce: bool, w_class: float) -> Tensor:
    """d(w_class * NLL(log_softmax(log1p(out^m)), ys)) / d out, written out:
    (softmax - onehot) / N, then log1p backward 1/(1+out^m), then pow backward m out^(m-1)."""
    n = out.shape[0]
    ys = torch.cat([ys1, ys1])
    x = torch.log1p(out ** mult) if enforce else out
    g = torch.softmax(x, dim=1)
    g[torch.arange(n), ys] -= 1.0
    g = g * (w_class / n)
    if enforce:
        g = g / (1.0 + out ** mult)
        g = g * (mult * out ** (mult - 1.0)) if mult != 0.0 else torch.zeros_like(g)
    return g


def nonneg_linear_grads(g: Tensor, x: Tensor, w: Tensor) -> Tuple[Tensor, Tensor]:
    """pipnet.py:70-71 backward: dW = (W > 0) * g^T x, db = g.sum(0)."""
    dw = (g.t() @ x) * (w > 0).to(g.dtype)
    return dw, g.sum(dim=0)


def adamw(p: Tensor, g: Tensor, m: Tensor, v: Tensor, step: int, lr: float, betas=(0.9, 0.999),
          eps: float = 1e-8, wd: float = 0.0) -> Tuple[Tensor, Tensor, Tensor]:
    """torch.optim.AdamW (amsgrad off), returns new (p, m, v)."""
    b1, b2 = betas
    p = p * (1.0 - lr * wd)
    m = m + (1.0 - b1) * (g - m)
    v = v * b2 + (1.0 - b2) * g * g
    bc1 = 1.0 - b1 ** step
    bc2 = 1.0 - b2 ** step
    p = p - (lr / bc1) * (m / (v.sqrt() / bc2 ** 0.5 + eps))
    return p, m, v


def finetune_update(pooled: Tensor, out: Tensor, ys1: Tensor, w: Tensor, b: Optional[Tensor], mult: float,
                    state: Dict[str, Tensor], step: int, lr_w: float, lr_b: float, wd_w: float,
                    enforce: bool = True, w_class: float = FINETUNE_WEIGHTS[2]) -> Dict[str, Tensor]:
    """One finetune-phase classifier update (train.py:100-140 with finetune=True): gradient
    of w_class * class loss w.r.t. W (and b), AdamW, then W = max(W - 1e-3, 0),
    b = max(b, 0), multiplier = max(m, 1) (enforce_weight_sparsity)."""
    g = d_out(out, ys1, mult, enforce, w_class)
    dw, db = nonneg_linear_grads(g, pooled, w)
    nw, mw, vw = adamw(w, dw, state["w_m"], state["w_v"], step, lr_w, wd=wd_w)
    res = dict(dw=dw, db=db, w_m=mw, w_v=vw)
    if enforce:
        nw = torch.clamp(nw - 1e-3, min=0.0)
    res["w"] = nw
    if b is not None:
        nb, mb, vb = adamw(b, db, state["b_m"], state["b_v"], step, lr_b, wd=0.0)
        res.update(b=torch.clamp(nb, min=0.0) if enforce else nb, b_m=mb, b_v=vb)
    res["mult"] = max(mult, 1.0) if enforce else mult
    return res


# ---- CountPIPNet count backward (pretrain / joint phases) ---------------------------------
def onehot_ste_backward(x, g, strategy=None, respect_active=False):
    """ModifiedSTEFunction.backward (count_pipnet_utils.py:226-321) restated row by row in
    numpy: x [B,P] encoder input (clamped counts), g [B,P,M] encoding gradient -> dx [B,P].
    The reference's effective behaviour: `counts_grad[zero_mask][neg] = ...` (:317-319) and
    `final_grad_nz[std][dec] = ...` (:279-280) assign into temporaries, so zero-count rows
    and, in a 'max_grad' batch holding an all-positive row, the other rows get 0."""
    import numpy as np
    x = np.asarray(x, dtype=np.float32)
    g = np.asarray(g, dtype=np.float32).reshape(x.shape + (-1,))
    m = g.shape[-1]
    r = np.round(x)                                          # torch.round: half to even
    nz = ~(r < 0.1)
    mn, mi, mx = g.min(axis=-1), g.argmin(axis=-1), g.max(axis=-1)   # argmin: first index
    cur = np.clip(r.astype(np.int64) - 1, 0, m - 1)
    gcur = np.take_along_axis(g, cur[..., None], axis=-1)[..., 0]
    allpos = mn > 0
    dx = np.zeros_like(x)
    if strategy == "max_grad" and (allpos & nz).any():
        dx = np.where(allpos, mx, 0.0).astype(np.float32)
    else:
        mag = np.abs(mn)
        if strategy == "current_grad":
            mag = np.where(allpos, gcur, mag)
        dx = np.where(mi < cur, mag, np.where(mi > cur, -mag, 0.0)).astype(np.float32)
    if respect_active:
        dx = np.where(gcur < 0, 0.0, dx).astype(np.float32)
    return np.where(nz, dx, 0.0).astype(np.float32)


def count_clamp_backward(counts, d_clamped, max_count, use_ste, gated):
    """d raw counts through STE_Round (identity, count_pipnet_utils.py:52-55) + ClampSTE
    (:67-84, gate on its input rint(counts)), or torch.clamp on the raw counts without STE
    (count_pipnet.py:94-96: the train-mode forward does not round)."""
    import numpy as np
    c = np.asarray(counts, dtype=np.float32)
    xin = np.round(c) if use_ste else c
    keep = (xin >= 0) & (xin <= max_count) if gated else np.ones_like(c, dtype=bool)
    return np.where(keep, np.asarray(d_clamped, dtype=np.float32), 0.0).astype(np.float32)
