"""HIP-graph replay of the inference forward (count_pipnet_amd.graph.GraphedForward) equals
the eager HIP forward bit for bit, follows in-place classifier updates, and draws fresh
Gumbel noise per replay."""
import pytest
import torch

from golden_util import golden_inputs, load_golden
from model_util import build_model

pytestmark = pytest.mark.gpu


def _net(name, gpu):
    meta, rec = load_golden(name)
    return build_model(meta).to(gpu), golden_inputs(meta).to(gpu), meta


@pytest.mark.parametrize("name", ["c2_pipnet_convnext26", "pipnet_mid_addon", "c3_pipnet_resnet50"])
def test_graph_replay_equals_eager(gpu, name):
    from count_pipnet_amd.graph import GraphedForward
    net, xs, _ = _net(name, gpu)
    with torch.no_grad():
        ref = [t.clone() for t in net(xs, inference=True)]
    g = GraphedForward(net)
    for _ in range(2):
        outs = g(xs)
        torch.cuda.synchronize()
        for a, b in zip(outs, ref):
            assert torch.equal(a, b)
    # in-place classifier update (eval_pipnet sparsification) is seen by the replay
    with torch.no_grad():
        net._classification.weight.mul_(0.5)
        ref2 = net(xs, inference=True)[2].clone()
    out2 = g(xs)[2]
    torch.cuda.synchronize()
    assert torch.equal(out2, ref2)


def test_graph_count_injected_noise_equals_eager(gpu):
    from count_pipnet_amd.graph import GraphedForward
    from count_pipnet_amd.synthetic import synth_exponential
    net, xs, meta = _net("c1_count_identity", gpu)
    b, p = xs.shape[0], net._num_prototypes
    act = list(net._add_on)[-1]
    act.exp_noise = synth_exponential((b, p, 8, 8), seed=5).to(gpu)
    with torch.no_grad():
        ref = [t.clone() for t in net(xs, inference=True)]
    outs = GraphedForward(net)(xs)
    torch.cuda.synchronize()
    for a, r in zip(outs, ref):
        assert torch.equal(a, r)


def test_graph_count_fresh_noise_per_replay(gpu):
    from count_pipnet_amd.graph import GraphedForward
    net, xs, meta = _net("c1_count_identity", gpu)
    list(net._add_on)[-1].exp_noise = None
    g = GraphedForward(net)
    p1 = g(xs)[0].clone()
    p2 = g(xs)[0].clone()
    torch.cuda.synchronize()
    assert not torch.equal(p1, p2)                       # new Philox key per replay
    for p in (p1, p2):                                   # still hard one-hot maps
        s = p.sum(dim=1)
        assert torch.allclose(s, torch.ones_like(s))
        assert torch.equal((p > 0).sum(dim=1), torch.ones_like(s, dtype=torch.int64))


def test_stream_split_bit_identical_and_graph(gpu):
    """Opt-in stream split: a batch >= 32 runs as concurrent sub-batches on 2 (3) streams,
    outputs bit-identical to the one-stream forward, also under HIP-graph capture."""
    from count_pipnet_amd.graph import GraphedForward
    from count_pipnet_amd.pipnet import set_stream_split, stream_split
    from count_pipnet_amd.synthetic import synth_images
    net, _, _ = _net("pipnet_mid_addon", gpu)
    xs = synth_images(40, 64, seed=9).to(gpu)
    assert stream_split(net, xs) == 1                    # off by default
    set_stream_split(net, 2)
    assert stream_split(net, xs) == 2
    with torch.no_grad():
        split = [t.clone() for t in net(xs, inference=True)]
        set_stream_split(net, 1)
        one = [t.clone() for t in net(xs, inference=True)]
        set_stream_split(net, 3)
        three = [t.clone() for t in net(xs, inference=True)]
    for a, b, c in zip(split, one, three):
        assert torch.equal(a, b) and torch.equal(c, b)
    set_stream_split(net, 2)
    outs = GraphedForward(net)(xs)
    torch.cuda.synchronize()
    for a, b in zip(outs, one):
        assert torch.equal(a, b)


@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
def test_stream_split_resnet_default(gpu, dtype):
    """ResNet backbones split batches >= 32 over 2 streams by default (C3: +12 % bf16);
    bit-identical to the one-stream forward in both HIP dtypes."""
    from count_pipnet_amd.pipnet import set_hip_dtype, set_stream_split, stream_split
    from count_pipnet_amd.synthetic import synth_images
    net, _, _ = _net("c3_pipnet_resnet50", gpu)
    set_hip_dtype(net, dtype)
    xs = synth_images(36, 64, seed=11).to(gpu)
    assert stream_split(net, xs) == 2
    assert stream_split(net, xs[:16]) == 1               # small batches stay on one stream
    with torch.no_grad():
        split = [t.clone() for t in net(xs, inference=True)]
        set_stream_split(net, 1)
        one = [t.clone() for t in net(xs, inference=True)]
    for a, b in zip(split, one):
        assert torch.equal(a, b)


def test_stream_split_convnext_default(gpu):
    """The full ConvNeXt PIP-Net (C2's model) splits batches >= 32 over 2 streams by default;
    bit-identical to the one-stream forward.  CountPIPNet / mid-layer models stay on one."""
    from count_pipnet_amd.pipnet import set_stream_split, stream_split
    from count_pipnet_amd.synthetic import synth_images
    net, _, _ = _net("c2_pipnet_convnext26", gpu)
    xs = synth_images(34, 64, seed=12).to(gpu)
    assert stream_split(net, xs) == 2 and stream_split(net, xs[:16]) == 1
    with torch.no_grad():
        split = [t.clone() for t in net(xs, inference=True)]
        set_stream_split(net, 1)
        one = [t.clone() for t in net(xs, inference=True)]
    for a, b in zip(split, one):
        assert torch.equal(a, b)
    cnet, _, _ = _net("c5_count_bilinear_2048", gpu)
    assert stream_split(cnet, synth_images(40, 32, seed=1)) == 1


@pytest.mark.parametrize("noise", ["injected", "philox"])
def test_count_stream_split_bit_identical(gpu, noise):
    """CountPIPNet split forward (backbone + Gumbel head per sub-batch stream, count layers on
    the whole batch) == the one-stream forward: injected noise sliced per sub-batch, Philox
    noise offset to the sub-batch's first image."""
    from count_pipnet_amd.pipnet import set_stream_split, stream_split
    from count_pipnet_amd.synthetic import synth_exponential, synth_images
    net, _, _ = _net("c1_count_identity", gpu)
    xs = synth_images(40, 64, seed=13).to(gpu)
    act = list(net._add_on)[-1]
    b, p = xs.shape[0], net._num_prototypes
    act.exp_noise = synth_exponential((b, p, 8, 8), seed=6).to(gpu) if noise == "injected" else None
    outs = {}
    with torch.no_grad():
        for n in (1, 2, 3):
            set_stream_split(net, n)
            assert stream_split(net, xs) == n
            torch.manual_seed(1234)                      # same Philox key for every variant
            outs[n] = [t.clone() for t in net(xs, inference=True)]
    for n in (2, 3):
        for a, r in zip(outs[n], outs[1]):
            assert torch.equal(a, r)
