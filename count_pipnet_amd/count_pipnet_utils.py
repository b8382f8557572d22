"""Count-head building blocks -- drop-in for ``pipnet/count_pipnet_utils.py``.

Forward semantics are the reference's (cited per class).  The HIP inference path of
``CountPIPNet`` recognises these modules and runs their forwards as kernels; the torch
implementations here serve training (autograd, custom STE backwards) and the explicit
``torch_backend()`` mode.
"""
from __future__ import annotations

from typing import Optional, Tuple

import torch
import torch.nn as nn
import torch.nn.functional as F


class GumbelSoftmax(nn.Module):
    """count_pipnet_utils.py:7-38: soft Gumbel-softmax in training, hard (straight-through
    one-hot) in eval; fresh Exp(1) noise on every call.

    ``exp_noise`` (not part of the reference) lets a caller inject the Exp(1) draw
    (shape of the logits, NCHW) so two implementations can be compared on identical
    noise; ``None`` (default) draws fresh noise like the reference."""

    def __init__(self, dim: int = 1, tau: float = 1.0):
        super().__init__()
        self.dim = dim
        self.tau = tau
        self.exp_noise: Optional[torch.Tensor] = None

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if self.exp_noise is None:
            return F.gumbel_softmax(x, tau=self.tau, hard=not self.training, dim=self.dim)
        gumbels = (x - self.exp_noise.to(x.device, x.dtype).log()) / self.tau
        y_soft = gumbels.softmax(self.dim)
        if self.training:
            return y_soft
        index = y_soft.max(self.dim, keepdim=True)[1]
        y_hard = torch.zeros_like(x).scatter_(self.dim, index, 1.0)
        return y_hard - y_soft.detach() + y_soft


class STE_Round(torch.autograd.Function):
    """count_pipnet_utils.py:41-55: round (half to even) forward, identity backward."""

    @staticmethod
    def forward(ctx, x):
        return x.round()

    @staticmethod
    def backward(ctx, grad_output):
        return grad_output


class ClampSTE(torch.autograd.Function):
    """count_pipnet_utils.py:58-84: clamp forward; backward identity or gated to the range."""

    @staticmethod
    def forward(ctx, input, min_val, max_val, is_backward_identity: bool):
        ctx.save_for_backward(input)
        ctx.min_val, ctx.max_val, ctx.is_backward_identity = min_val, max_val, is_backward_identity
        return input.clamp(min_val, max_val)

    @staticmethod
    def backward(ctx, grad_output):
        (input,) = ctx.saved_tensors
        if not ctx.is_backward_identity:
            grad_output = grad_output * ((input >= ctx.min_val) & (input <= ctx.max_val)).float()
        return grad_output, None, None, None


def create_modified_encoding(x: torch.Tensor, max_count: int) -> torch.Tensor:
    """count_pipnet_utils.py:141-185: c > 0.1 -> one-hot at clamp(int(c) - 1, 0, C - 1),
    otherwise all zeros.  Returns [B, P, max_count]."""
    b, p = x.shape
    enc = torch.zeros(b, p, max_count, device=x.device)
    present = (x > 0.1).to(enc.dtype)
    slot = torch.clamp(x.long() - 1, 0, max_count - 1)
    return enc.scatter_(2, slot.unsqueeze(2), present.unsqueeze(2))


class ModifiedSTEFunction(torch.autograd.Function):
    """count_pipnet_utils.py:188-321: encode rounded counts; backward follows the bin with the
    most negative gradient.  The backward reproduces the reference's *effective* behaviour:
    its chained boolean-mask assignments (``a[m1][m2] = v``) write into temporaries, so
    zero-count entries and the non-all-positive rows of the 'max_grad' strategy receive 0."""

    @staticmethod
    def forward(ctx, counts, max_count, respect_active_grad, positive_grad_strategy=None):
        rounded = counts.round()
        ctx.save_for_backward(counts, rounded)
        ctx.max_count, ctx.respect_active_grad, ctx.strategy = max_count, respect_active_grad, positive_grad_strategy
        return create_modified_encoding(rounded, max_count)

    @staticmethod
    def backward(ctx, grad_output):
        counts, rounded = ctx.saved_tensors
        b, p = counts.shape
        if tuple(grad_output.shape) != (b, p, ctx.max_count):
            raise ValueError(f"Unexpected grad_output shape {tuple(grad_output.shape)}")
        grad = torch.zeros_like(counts)
        cur = torch.clamp(rounded.long() - 1, 0, ctx.max_count - 1)
        nz = ~(rounded < 0.1)
        if bool(nz.any()):
            g = grad_output[nz]                                   # [n, C]
            cur_nz = cur[nz]
            min_val, min_idx = torch.min(g, dim=1)
            all_pos = min_val > 0
            final = torch.zeros_like(min_val)
            if ctx.strategy == "max_grad" and bool(all_pos.any()):
                final = torch.where(all_pos, g.max(dim=1).values, final)
            else:
                mag = min_val.abs()
                if ctx.strategy == "current_grad" and bool(all_pos.any()):
                    mag = torch.where(all_pos, g.gather(1, cur_nz.unsqueeze(1)).squeeze(1), mag)
                final = torch.where(min_idx < cur_nz, mag, final)
                final = torch.where(min_idx > cur_nz, -mag, final)
            if ctx.respect_active_grad:
                final = torch.where(g.gather(1, cur_nz.unsqueeze(1)).squeeze(1) < 0, torch.zeros_like(final), final)
            grad[nz] = final
        return grad, None, None, None


class OneHotEncoder(nn.Module):
    """count_pipnet_utils.py:86-139 -> [B, P * num_bins] (p-major)."""

    def __init__(self, num_bins: int = 4, use_ste: bool = False, respect_active_grad: bool = False,
                 num_prototypes: int = None, device: Optional[torch.device] = None,
                 positive_grad_strategy: Optional[str] = None):
        super().__init__()
        self.num_bins = num_bins
        self.num_prototypes = num_prototypes
        self.device = device
        self.use_ste = use_ste
        self.respect_active_grad = respect_active_grad
        self.positive_grad_strategy = positive_grad_strategy

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if self.use_ste:
            enc = ModifiedSTEFunction.apply(x, self.num_bins, self.respect_active_grad, self.positive_grad_strategy)
        else:
            enc = create_modified_encoding(x, self.num_bins)
        return enc.view(enc.size(0), -1)

    def prototype_to_classifier_input_weights(self, prototype_idx):
        v = torch.zeros(self.num_prototypes * self.num_bins, device=self.device)
        v[prototype_idx * self.num_bins:(prototype_idx + 1) * self.num_bins] = 1.0
        return v


class BilinearIntermediate(nn.Module):
    """count_pipnet_utils.py:323-385: e = embed(x) (W_e[p*C + c, p] = c + 1), out = W(e) * V(e)."""

    def __init__(self, num_prototypes, max_count, expanded_dim=None, custom_init=False):
        super().__init__()
        self.num_prototypes = num_prototypes
        self.max_count = max_count
        self.expanded_dim = num_prototypes * max_count if expanded_dim is None else expanded_dim
        self.embed = nn.Linear(num_prototypes, self.expanded_dim, bias=False)
        self.W = nn.Linear(self.expanded_dim, self.expanded_dim, bias=False)
        self.V = nn.Linear(self.expanded_dim, self.expanded_dim, bias=False)
        with torch.no_grad():
            self.embed.weight.zero_()
            p = torch.arange(num_prototypes).repeat_interleave(max_count)
            c = torch.arange(max_count).repeat(num_prototypes)
            rows = p * max_count + c
            keep = rows < self.expanded_dim
            self.embed.weight[rows[keep], p[keep]] = (c[keep] + 1).to(self.embed.weight.dtype)
            if custom_init:
                nn.init.normal_(self.W.weight, mean=0.0, std=0.1)
                nn.init.normal_(self.V.weight, mean=0.0, std=0.1)
                self.W.weight.diagonal().add_(0.1)
                self.V.weight.diagonal().add_(0.1)

    def forward(self, x):
        e = self.embed(x)
        return self.W(e) * self.V(e)


class LinearFull(nn.Module):
    """count_pipnet_utils.py:387-444: dense Linear(P, P*C) with the structured init
    (c + 1 on the own prototype, 0.1 (c + 1) / P elsewhere), built vectorised."""

    def __init__(self, num_prototypes, max_count, expanded_dim=None):
        super().__init__()
        self.num_prototypes = num_prototypes
        self.max_count = max_count
        self.expanded_dim = num_prototypes * max_count if expanded_dim is None else expanded_dim
        self.linear = nn.Linear(num_prototypes, self.expanded_dim, bias=False)
        with torch.no_grad():
            w = self.linear.weight
            w.zero_()
            n = min(num_prototypes * max_count, self.expanded_dim)
            rows = torch.arange(n)
            p, c = rows // max_count, rows % max_count
            w[:n] = (0.1 * (c + 1).to(w.dtype) / num_prototypes).unsqueeze(1).expand(n, num_prototypes)
            w[rows, p] = (c + 1).to(w.dtype)

    def forward(self, x):
        return self.linear(x)

    def prototype_to_classifier_input_weights(self, prototype_idx):
        return self.linear.weight[:, prototype_idx]


class IdentityIntermediate(nn.Module):
    """count_pipnet_utils.py:446-469."""

    def __init__(self, num_prototypes, device):
        super().__init__()
        self.identity = nn.Identity()
        self.num_prototypes = num_prototypes
        self.device = device

    def forward(self, x):
        return self.identity(x)

    def prototype_to_classifier_input_weights(self, prototype_idx):
        return torch.eye(self.num_prototypes, device=self.device)[prototype_idx]


class LinearIntermediate(nn.Module):
    """count_pipnet_utils.py:471-539: per-prototype Linear(1, C), weight[i] = (i + 1) / max_count."""

    def __init__(self, num_prototypes, max_count, expansion_factor=None):
        super().__init__()
        self.num_prototypes = num_prototypes
        self.max_count = max_count
        self.expansion_factor = max_count if expansion_factor is None else expansion_factor
        self.linear = nn.Linear(1, self.expansion_factor, bias=False)
        with torch.no_grad():
            self.linear.weight.copy_((torch.arange(self.expansion_factor, dtype=torch.float32) + 1).unsqueeze(1)
                                     / self.max_count)

    def forward(self, x):
        b = x.shape[0]
        return self.linear(x.reshape(b * self.num_prototypes, 1)).view(b, self.num_prototypes * self.expansion_factor)

    def prototype_to_classifier_input_weights(self, prototype_idx):
        v = torch.zeros(self.num_prototypes * self.expansion_factor, device=self.linear.weight.device,
                        dtype=self.linear.weight.dtype)
        s = prototype_idx * self.expansion_factor
        v[s:s + self.expansion_factor] = self.linear.weight[:, 0]
        return v


__all__ = ["GumbelSoftmax", "STE_Round", "ClampSTE", "OneHotEncoder", "create_modified_encoding",
           "ModifiedSTEFunction", "BilinearIntermediate", "LinearFull", "IdentityIntermediate",
           "LinearIntermediate", "Tuple"]
