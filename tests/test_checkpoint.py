"""Reference-format checkpoints (util/checkpoint_manager.py:118-125: DataParallel-wrapped
``state_dict`` under 'model_state_dict' + optimizer state) load into this package's models
through count_pipnet_amd.checkpoint with the safe loader, strict=True."""
import os

import pytest
import torch
import torch.nn as nn

from count_pipnet_amd.checkpoint import adapt_keys, load_checkpoint
from golden_util import load_golden
from model_util import build_model


def _save_reference_style(tmp_path, name):
    meta, _ = load_golden(name)
    net = build_model(meta)
    dp = nn.DataParallel(net)
    opt = torch.optim.AdamW(dp.parameters(), lr=1e-3)
    path = os.path.join(tmp_path, "net_pretrained")
    torch.save({"model_state_dict": dp.state_dict(), "optimizer_net_state_dict": opt.state_dict()}, path)
    return meta, net, path


@pytest.mark.parametrize("name", ["pipnet_mid_addon", "c1_count_identity"])
def test_reference_checkpoint_loads_strict(tmp_path, name):
    meta, net, path = _save_reference_style(tmp_path, name)
    fresh = build_model(dict(meta, case=dict(meta["case"], seed=meta["case"]["seed"] + 1)))
    assert any(not torch.equal(a, b) for a, b in zip(fresh.state_dict().values(), net.state_dict().values()))
    load_checkpoint(fresh, path, device=None)
    for (k1, v1), (k2, v2) in zip(net.state_dict().items(), fresh.state_dict().items()):
        assert k1 == k2 and torch.equal(v1, v2)
    # the same file into a DataParallel-style wrapper (keys keep the module. prefix)
    wrapped = nn.DataParallel(build_model(meta))
    load_checkpoint(wrapped, path, device=None)
    assert all(k.startswith("module.") for k in wrapped.state_dict())


def test_adapt_keys_both_ways():
    m = nn.Sequential(nn.Linear(2, 2))
    sd = {"module." + k: v for k, v in m.state_dict().items()}
    assert set(adapt_keys(sd, m)) == set(m.state_dict())
    assert set(adapt_keys(m.state_dict(), nn.DataParallel(m))) == set(sd)


@pytest.mark.gpu
def test_checkpoint_roundtrip_on_gpu(gpu, tmp_path):
    from golden_util import golden_inputs
    meta, net, path = _save_reference_style(tmp_path, "pipnet_mid_addon")
    net = net.to(gpu).eval()
    fresh = load_checkpoint(build_model(meta), path, device=gpu, warmup_image_size=meta["case"]["size"])
    xs = golden_inputs(meta).to(gpu)
    with torch.no_grad():
        a, b = net(xs, inference=True), fresh(xs, inference=True)
    for t1, t2 in zip(a, b):
        assert torch.equal(t1, t2)
