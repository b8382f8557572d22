"""Finetune-phase training iteration: the CPU oracle (oracle/train_ref.py) against the
reference's own train_pipnet run (tests/golden/train_*.npz, gen_golden_train.py), and the
host logic of count_pipnet_amd.train (no GPU).

* loss terms: align / tanh / class / accuracy of every recorded iteration from the
  recorded forward outputs (align only where the proto map is recorded);
* the classifier update chain: starting from the synthetic initial weights, the oracle's
  explicit-derivative gradient + AdamW + clamps reproduces every later iteration's weights,
  the final weights / bias / multiplier and the AdamW moments;
* stochastic-depth run splitting and mask generation; train_pipnet's phase guard.
"""
import numpy as np
import pytest
import torch

from count_pipnet_amd import train as T
from count_pipnet_amd.convnext_features import convnext_tiny_26_features, stochastic_depth_row_scales
from golden_util import load_train_golden, train_golden_names, train_step_lrs
from model_util import build_model
from oracle import train_ref

NAMES = train_golden_names()
FINETUNE = [n for n in NAMES if n.startswith("train_finetune_")]


def _loss_weights(meta):
    """(align, tanh, class) weights of train.py:51-61 for the fixture's phase (epoch 1)."""
    return {"pretrain": (0.5, 5.0, 0.0), "joint": (5.0, 2.0, 2.0), "finetune": (0.0, 0.0, 2.0),
            "count_finetune": (0.0, 0.0, 2.0), "count_pretrain": (0.5, 5.0, 0.0),
            "count_joint": (5.0, 2.0, 2.0), "full": (5.0, 2.0, 2.0), "count_full": (5.0, 2.0, 2.0)}[meta["phase"]]


def _t(a):
    return torch.from_numpy(np.ascontiguousarray(a))


@pytest.mark.parametrize("name", NAMES)
def test_oracle_loss_terms_match_reference(name):
    meta, rec, _ = load_train_golden(name)
    for i, comp in enumerate(meta["components"]):
        pooled, out, ys = _t(rec[f"s{i}_pooled"]), _t(rec[f"s{i}_out"]), _t(rec[f"s{i}_ys"])
        mult = float(rec[f"s{i}_mult"][0])
        proto = _t(rec[f"s{i}_proto"]) if f"s{i}_proto" in rec else torch.zeros(pooled.shape + (1, 1)) + 0.5
        got = train_ref.loss_terms(proto, pooled, out, ys, mult)
        assert float(got["tanh"]) == pytest.approx(comp["tanh"], rel=1e-5, abs=1e-6)
        if not meta["phase"].endswith("pretrain"):
            assert float(got["cls"]) == pytest.approx(comp["class"], rel=1e-5, abs=1e-6)
            assert float(got["correct"]) / (2 * len(ys)) == comp["acc"]
        wa, wt, wc = _loss_weights(meta)
        assert comp["loss"] == pytest.approx(wa * comp["align"] + wt * comp["tanh"] + wc * comp["class"], rel=1e-5)
        if f"s{i}_proto" in rec:
            assert float(got["align"]) == pytest.approx(comp["align"], rel=1e-5, abs=1e-6)


def _initial_classifier(name):
    meta, rec, fwd_meta = load_train_golden(name)
    net = build_model(fwd_meta)
    cls = net._classification
    w = cls.weight.detach().clone()
    b = None if cls.bias is None else cls.bias.detach().clone()
    return meta, rec, w, b, float(cls.normalization_multiplier.detach()[0])


@pytest.mark.parametrize("name", FINETUNE)
def test_oracle_update_chain_matches_reference(name):
    meta, rec, w, b, mult = _initial_classifier(name)
    if "s0_w" in rec:
        assert torch.equal(w, _t(rec["s0_w"]))       # synthetic weights == what the reference saw
    state = dict(w_m=torch.zeros_like(w), w_v=torch.zeros_like(w))
    if b is not None:
        state.update(b_m=torch.zeros_like(b), b_v=torch.zeros_like(b))
    lrs = train_step_lrs(meta)
    for i in range(meta["iterations"]):
        r = train_ref.finetune_update(_t(rec[f"s{i}_pooled"]), _t(rec[f"s{i}_out"]), _t(rec[f"s{i}_ys"]), w, b, mult,
                                      state, i + 1, lrs[i], lrs[i], meta["weight_decay"])
        w, b, mult = r["w"], r.get("b"), r["mult"]
        state = {k: r[k] for k in ("w_m", "w_v", "b_m", "b_v") if k in r}
        if f"s{i + 1}_w" in rec:
            torch.testing.assert_close(w, _t(rec[f"s{i + 1}_w"]), rtol=1e-5, atol=1e-6)
    if "final_w" in rec:
        torch.testing.assert_close(w, _t(rec["final_w"]), rtol=1e-5, atol=1e-6)
        torch.testing.assert_close(state["w_m"], _t(rec["final_w_exp_avg"]), rtol=1e-5, atol=1e-9)
        torch.testing.assert_close(state["w_v"], _t(rec["final_w_exp_avg_sq"]), rtol=1e-5, atol=1e-12)
    else:
        torch.testing.assert_close(w[:8], _t(rec["final_w_rows8"]), rtol=1e-5, atol=1e-6)
        np.testing.assert_allclose(w.double().sum(1).numpy(), rec["final_w_rowsum"], rtol=1e-5, atol=1e-4)
        torch.testing.assert_close(state["w_m"][:8], _t(rec["final_w_exp_avg_rows8"]), rtol=1e-5, atol=1e-9)
        torch.testing.assert_close(state["w_v"][:8], _t(rec["final_w_exp_avg_sq_rows8"]), rtol=1e-5, atol=1e-12)
    if b is not None:
        torch.testing.assert_close(b, _t(rec["final_b"]), rtol=1e-5, atol=1e-6)
        torch.testing.assert_close(state["b_m"], _t(rec["final_b_exp_avg"]), rtol=1e-5, atol=1e-9)
    assert mult == pytest.approx(float(rec["final_mult"][0]))


def test_oracle_adamw_matches_torch():
    g = torch.Generator().manual_seed(0)
    p0 = torch.randn(64, 33, generator=g)
    p = p0.clone().requires_grad_(True)
    opt = torch.optim.AdamW([p], lr=0.05, weight_decay=0.01, foreach=False)
    q, m, v = p0.clone(), torch.zeros_like(p0), torch.zeros_like(p0)
    for step in range(1, 4):
        grad = torch.randn(64, 33, generator=g)
        p.grad = grad.clone()
        opt.step()
        q, m, v = train_ref.adamw(q, grad, m, v, step, 0.05, wd=0.01)
        torch.testing.assert_close(q, p.detach(), rtol=1e-6, atol=1e-7)


def test_stochastic_depth_row_scales():
    feats = convnext_tiny_26_features().features
    masks = T.stochastic_depth_masks(feats, 8, torch.Generator().manual_seed(2))
    scales = stochastic_depth_row_scales(feats, masks, 8, "cpu")
    assert sorted(scales) == sorted(masks)
    for bid, sc in scales.items():
        keep = 1.0 - 0.1 * bid / 17
        want = masks[bid].to(torch.float32).div_(keep)      # StochasticDepth: noise.div_(keep)
        assert torch.equal(sc, want)


def test_stochastic_depth_masks_follow_module_probabilities():
    feats = convnext_tiny_26_features().features
    masks = T.stochastic_depth_masks(feats, 4096, torch.Generator().manual_seed(1))
    assert sorted(masks) == list(range(1, 18))           # block 0 has p = 0 (no draw)
    for bid, m in masks.items():
        p = 0.1 * bid / 17
        assert m.dtype == torch.bool and m.shape == (4096,)
        assert abs(1.0 - m.float().mean().item() - p) < 0.02


def test_train_pipnet_guards_other_phases():
    from count_pipnet_amd.pipnet import get_pipnet
    import argparse
    import contextlib
    import io
    args = argparse.Namespace(net="convnext_tiny_26", disable_pretrained=True, num_features=0, bias=False,
                              use_mid_layers=True, num_stages=1)
    with contextlib.redirect_stdout(io.StringIO()):
        net, _ = get_pipnet(5, args)
    opt = torch.optim.AdamW(net._classification.parameters(), lr=0.05)
    with pytest.raises(NotImplementedError):
        T.train_pipnet(net, [], opt, opt, None, None, None, 1, 1, "cpu", pretrain=True)
    with pytest.raises(NotImplementedError):   # CPU parameters: not the HIP finetune path
        T.train_pipnet(net, [], opt, opt, None, None, None, 1, 1, "cpu", finetune=True)
