"""The oracle (oracle/ref_cpu.py) reproduces the reference's own outputs, recorded by
tests/golden/gen_golden.py from the unchanged reference code, on every golden case."""
import numpy as np
import pytest
import torch

from golden_util import golden_args, golden_inputs, golden_names, golden_noise, golden_state_dict, load_golden, proto_shape
from oracle import ref_cpu

NAMES = golden_names()


def run_oracle(meta, rec, inference):
    args, sd, xs = golden_args(meta), golden_state_dict(meta), golden_inputs(meta)
    with torch.no_grad():
        if meta["case"]["model"] == "pipnet":
            return ref_cpu.pipnet_forward(xs, sd, args, inference=inference)
        noise = golden_noise(meta, proto_shape(meta, rec))
        return ref_cpu.count_pipnet_forward(xs, sd, args, inference=inference, exp_noise=noise)


@pytest.mark.parametrize("name", NAMES)
def test_oracle_matches_reference_golden(name):
    meta, rec = load_golden(name)
    if meta["case"]["net"] == "resnet50" or meta["case"]["size"] >= 224:
        torch.set_num_threads(8)
    for inference in (True, False):
        tag = "inf" if inference else "raw"
        proto, pooled, out = run_oracle(meta, rec, inference)
        np.testing.assert_allclose(pooled.numpy(), rec[tag + "_pooled"], rtol=1e-5, atol=1e-6)
        np.testing.assert_allclose(out.numpy(), rec[tag + "_out"], rtol=1e-5, atol=1e-5)
        np.testing.assert_allclose(proto.sum(dim=(2, 3)).numpy(), rec[tag + "_proto_sum"], rtol=1e-5, atol=1e-5)
        np.testing.assert_allclose(proto.amax(dim=(2, 3)).numpy(), rec[tag + "_proto_max"], rtol=1e-5, atol=1e-6)
        if tag + "_proto" in rec:
            np.testing.assert_allclose(proto.numpy(), rec[tag + "_proto"], rtol=1e-5, atol=1e-6)


def test_golden_inventory():
    """Every BASELINE config except the multi-GPU sharding of C4 has a golden case."""
    for required in ("c1_count_identity", "c2_pipnet_convnext26", "c3_pipnet_resnet50", "c5_count_bilinear_2048"):
        assert required in NAMES


def test_bf16_build_tolerance_vs_reference():
    """The bf16 ResNet build's arithmetic (oracle.ref_cpu.pipnet_forward_bf16: bf16 weights
    and activations, fp32 accumulation) stays within the bf16 tolerance used by the GPU
    tests of the reference's fp32 outputs on the C3 golden (pooled 5e-2 abs, logits 5e-2 of
    scale, decisive argmax equal).  Measured: pooled 0.028, logits 1.2 % of scale."""
    meta, rec = load_golden("c3_pipnet_resnet50")
    torch.set_num_threads(8)
    args, sd, xs = golden_args(meta), golden_state_dict(meta), golden_inputs(meta)
    with torch.no_grad():
        _, pooled, out = ref_cpu.pipnet_forward_bf16(xs, sd, args, inference=True)
    g_pooled, g_out = torch.from_numpy(rec["inf_pooled"]), torch.from_numpy(rec["inf_out"])
    near = (g_pooled - 0.1).abs() < 5e-2
    assert torch.all((pooled - g_pooled).abs()[~near] <= 5e-2)
    gs = g_out.abs().max().clamp(min=1.0)
    assert (out - g_out).abs().max() <= 5e-2 * gs
    assert torch.equal(out.argmax(1), g_out.argmax(1))
