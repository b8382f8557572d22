"""CountPIPNet count backward (ModifiedSTEFunction / ClampSTE / STE_Round) against the
fixture recorded from the reference's own autograd Functions (tests/golden/gen_golden_ste.py):
the numpy oracle (oracle/train_ref.py) and the product's torch-path Functions on CPU; the
HIP kernels (pipnet_onehot_ste_bwd_f32 / pipnet_count_ste_bwd_f32) on the GPU."""
from __future__ import annotations

import json
import os

import numpy as np
import pytest
import torch

from oracle import train_ref

HERE = os.path.dirname(os.path.abspath(__file__))
REC = np.load(os.path.join(HERE, "golden", "count_ste_bwd.npz"))
META = json.loads(str(REC["meta"]))
STRATS = [None if s == "None" else s for s in META["strategies"]]
CASES = [(kind, si, ra) for kind in META["cases"] for si in range(len(STRATS)) for ra in (0, 1)]


@pytest.mark.parametrize("kind,si,ra", CASES)
def test_oracle_onehot_ste_matches_reference(kind, si, ra):
    dx = train_ref.onehot_ste_backward(REC[f"{kind}_x"], REC[f"{kind}_g"], STRATS[si], bool(ra))
    np.testing.assert_array_equal(dx, REC[f"{kind}_dx_s{si}_ra{ra}"])


@pytest.mark.parametrize("kind,si,ra", CASES)
def test_module_onehot_ste_matches_reference(kind, si, ra):
    from count_pipnet_amd.count_pipnet_utils import ModifiedSTEFunction
    x = torch.from_numpy(REC[f"{kind}_x"]).clone().requires_grad_(True)
    enc = ModifiedSTEFunction.apply(x, META["max_count"], bool(ra), STRATS[si])
    np.testing.assert_array_equal(enc.detach().numpy(), REC[f"{kind}_enc"])
    enc.backward(torch.from_numpy(REC[f"{kind}_g"]))
    np.testing.assert_array_equal(x.grad.numpy(), REC[f"{kind}_dx_s{si}_ra{ra}"])


@pytest.mark.parametrize("name,use_ste,gated", [("ste_gated", True, True), ("ste_identity", True, False),
                                                ("plain", False, True)])
def test_oracle_clamp_backward_matches_reference(name, use_ste, gated):
    d = train_ref.count_clamp_backward(REC["clamp_counts"], REC["clamp_dclamped"], META["max_count"], use_ste, gated)
    np.testing.assert_array_equal(d, REC[f"clamp_dcounts_{name}"])


@pytest.mark.gpu
@pytest.mark.parametrize("kind,si,ra", CASES)
def test_hip_onehot_ste_matches_reference(gpu, kind, si, ra):
    from count_pipnet_amd import kernels as K
    x = torch.from_numpy(REC[f"{kind}_x"]).to(gpu)
    g = torch.from_numpy(REC[f"{kind}_g"]).to(gpu).reshape(x.shape[0], -1).contiguous()
    dx = K.onehot_ste_backward(x, g, STRATS[si], bool(ra)).cpu().numpy()
    np.testing.assert_array_equal(dx, REC[f"{kind}_dx_s{si}_ra{ra}"])


@pytest.mark.gpu
@pytest.mark.parametrize("name,use_ste,gated", [("ste_gated", True, True), ("ste_identity", True, False),
                                                ("plain", False, True)])
def test_hip_clamp_backward_matches_reference(gpu, name, use_ste, gated):
    from count_pipnet_amd import kernels as K
    c = torch.from_numpy(REC["clamp_counts"]).to(gpu)
    d = K.count_ste_backward(c, torch.from_numpy(REC["clamp_dclamped"]).to(gpu), META["max_count"], use_ste, gated)
    np.testing.assert_array_equal(d.cpu().numpy(), REC[f"clamp_dcounts_{name}"])
