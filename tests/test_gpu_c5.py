"""BASELINE C5 at its real per-GPU size: CountPIPNet bilinear.yaml, 64 images of 128x128 per
GPU (bs=256 over 4 GPUs), 2048 prototypes, 16x16 grid (/root/reference/pipnet/count_pipnet.py:70-110,
GumbelSoftmax count_pipnet_utils.py:23-38, BilinearIntermediate :323-385).

The golden covers bs=2; here the Gumbel / count head runs at its real grid (64 x 256 pixels x
2048 channels) with an injected Exp(1) draw, and these size-independent properties hold:

* one-hot rows: every pixel's proto column has exactly one nonzero, equal to 1 within 1 ulp
  (``y_hard - y_soft + y_soft``) and at the argmax of logits - log(E) (checked for four images
  against the oracle, whole maps);
* counts = histogram: inference counts = clamp(round(sum over pixels), 0, 3), raw counts =
  the pixel sums, and both equal the per-image histogram of the one-hot argmax positions;
* logits = NonNegLinear(BilinearIntermediate(counts)) with the module's own weights, in fp64
  on the host (the reference's arithmetic restated by the oracle), at 1e-3 of scale;
* batch invariance: images 5..7 run alone give bit-identical proto / counts / logits;
* four images end to end against the oracle with the same noise: the one-hot position of
  every pixel whose Gumbel top-2 gap is >= 1e-3, and for images without such a near-tie the
  counts exactly and the logits at 1e-3.
"""
import numpy as np
import pytest
import torch

from count_pipnet_amd.synthetic import synth_exponential, synth_images
from golden_util import golden_args, load_golden
from model_util import build_model
from oracle import ref_cpu

pytestmark = pytest.mark.gpu
TOL = 1e-3
B, SIZE, P, GRID = 64, 128, 2048, 16
NO = 4      # images checked against the oracle


@pytest.fixture(scope="module")
def c5(gpu):
    meta, _ = load_golden("c5_count_bilinear_2048")
    net = build_model(meta).to(gpu)
    xs = synth_images(B, SIZE, seed=55)
    noise = synth_exponential((B, P, GRID, GRID), seed=56)
    net._add_on[-1].exp_noise = noise.to(gpu)
    with torch.no_grad():
        proto, counts, out = net(xs.to(gpu), inference=True)
        _, raw, out_raw = net(xs.to(gpu), inference=False)
        net._add_on[-1].exp_noise = noise[5:8].to(gpu)
        proto3, counts3, out3 = net(xs[5:8].to(gpu), inference=True)
    torch.cuda.synchronize()
    return dict(meta=meta, net=net, xs=xs, noise=noise, proto=proto, counts=counts, out=out, raw=raw,
                out_raw=out_raw, proto3=proto3, counts3=counts3, out3=out3)


def test_c5_shapes_and_one_hot_rows(c5):
    proto = c5["proto"]
    assert proto.shape == (B, P, GRID, GRID) and c5["counts"].shape == (B, P) and c5["out"].shape == (B, 9)
    nnz = (proto != 0).sum(dim=1)
    assert torch.equal(nnz, torch.ones_like(nnz)), "every pixel holds exactly one nonzero"
    top = proto.amax(dim=1)
    assert (top - 1.0).abs().max().item() <= 2 ** -23


def test_c5_counts_are_histograms(c5):
    proto, counts, raw = c5["proto"], c5["counts"], c5["raw"]
    idx = proto.argmax(dim=1).flatten(1)                                       # [B, 256]
    hist = torch.zeros(B, P, device=proto.device).scatter_add_(1, idx, torch.ones_like(idx, dtype=torch.float32))
    assert torch.allclose(raw, hist, atol=256 * 2 ** -23)                     # raw counts = pixel sums
    assert torch.equal(counts, hist.round().clamp(0, 3))                       # STE_Round + ClampSTE
    assert torch.equal(counts, raw.round().clamp(0, 3))


def test_c5_logits_from_counts(c5):
    """out = relu(W_cls) . (W(e) * V(e)), e = embed(counts): the intermediate and classifier
    recomputed in fp64 from the HIP counts with the module's own parameters.  With use_ste the
    classifier always sees the clamped counts (count_pipnet.py:90-110); inference=False only
    changes which counts are returned."""
    net = c5["net"]
    sd = {k: v.detach().cpu().double() for k, v in net.state_dict().items()}
    for counts, out in ((c5["counts"], c5["out"]), (c5["raw"].round().clamp(0, 3), c5["out_raw"])):
        c = counts.cpu().double()
        e = c @ sd["_intermediate.embed.weight"].t()
        inter = (e @ sd["_intermediate.W.weight"].t()) * (e @ sd["_intermediate.V.weight"].t())
        ref = inter @ sd["_classification.weight"].clamp(min=0).t()
        if "_classification.bias" in sd:
            ref = ref + sd["_classification.bias"]
        scale = ref.abs().clamp(min=1.0)
        assert ((out.cpu().double() - ref).abs() / scale).max().item() <= TOL


def test_c5_batch_invariance(c5):
    assert torch.equal(c5["proto"][5:8], c5["proto3"])
    assert torch.equal(c5["counts"][5:8], c5["counts3"])
    assert torch.equal(c5["out"][5:8], c5["out3"])


def test_c5_images_vs_oracle(c5):
    net, meta = c5["net"], c5["meta"]
    sd = {k: v.detach().cpu() for k, v in net.state_dict().items()}
    with torch.no_grad():
        r_proto, r_counts, r_out = ref_cpu.count_pipnet_forward(c5["xs"][:NO], sd, golden_args(meta), inference=True,
                                                                 exp_noise=c5["noise"][:NO])
        # images with a Gumbel near-tie (top-2 gap < 1e-3 somewhere) may pick the other channel
        feats = torch.nn.functional.conv2d(ref_cpu.backbone(c5["xs"][:NO], sd, golden_args(meta)),
                                           sd["_add_on.0.weight"], sd["_add_on.0.bias"])
        top2 = (feats - c5["noise"][:NO].log()).topk(2, dim=1).values
        decisive = (top2[:, 0] - top2[:, 1]) >= TOL                           # [NO, 16, 16]
        ok = decisive.flatten(1).all(dim=1).numpy()
    proto, counts, out = c5["proto"][:NO].cpu(), c5["counts"][:NO].cpu(), c5["out"][:NO].cpu()
    # the one-hot position of every decisive pixel of every image
    assert torch.equal(proto.argmax(dim=1)[decisive], r_proto.argmax(dim=1)[decisive])
    assert ok.any(), "every oracle image holds a Gumbel near-tie; pick other seeds"
    for i in np.nonzero(ok)[0]:
        assert torch.equal(counts[i], r_counts[i])
        assert ((out[i] - r_out[i]).abs() / r_out[i].abs().clamp(min=1)).max().item() <= TOL


# ---- the bilinear fold: in-tree fp64 kernel and its cache -------------------------

def test_matmul_f64acc_matches_float64(gpu):
    """pipnet_matmul_f64acc_f32 (csrc/fold_f64.hip) = float64 matmul rounded to fp32, on ragged
    shapes (no multiple of the 128 x 128 x 16 tile, odd K, N % 4 != 0) and on the C5 fold's own shape."""
    from count_pipnet_amd import kernels as K
    g = torch.Generator().manual_seed(7)
    for m, n, k in [(1, 1, 1), (37, 70, 19), (130, 65, 257), (129, 131, 33), (256, 258, 18), (6144, 2048, 6144)]:
        a = torch.randn(m, k, generator=g)
        b = torch.randn(k, n, generator=g)
        ref = (a.double() @ b.double()).float()
        out = K.matmul_f64acc(a.to(gpu), b.to(gpu)).cpu()
        # one fp32 rounding of an fp64 sum: equal except at rounding midpoints (1 ulp)
        ulp = torch.finfo(torch.float32).eps * ref.abs().clamp_min(1e-30)
        assert ((out - ref).abs() <= ulp).all(), (m, n, k)
        assert (out == ref).float().mean() > 0.999, (m, n, k)


def test_matmul2_f64acc_pair_equals_singles(gpu):
    """The one-launch pair form (W E, V E sharing E) is bitwise the two single products, ragged
    and full-size, and leaves nothing outside its outputs."""
    from count_pipnet_amd import kernels as K
    g = torch.Generator().manual_seed(11)
    for m, n, k in [(37, 70, 19), (300, 260, 100), (6144, 2048, 6144)]:
        a0, a1 = torch.randn(m, k, generator=g).to(gpu), torch.randn(m, k, generator=g).to(gpu)
        b = torch.randn(k, n, generator=g).to(gpu)
        c0, c1 = K.matmul2_f64acc(a0, a1, b)
        assert torch.equal(c0, K.matmul_f64acc(a0, b)) and torch.equal(c1, K.matmul_f64acc(a1, b)), (m, n, k)


def test_linear_pair_mul_equals_two_gemms(gpu):
    """pipnet_linear_pair_mul_f32 (one split-K GEMM over the stacked [W E; V E] + a reduction
    taking the product) = the two-GEMM form (V E x) * (W E x) bitwise when both split K into the
    same slabs, and the fp64 product at 1e-5 relative, on the C5 shape, short M, ragged M and long M
    (no split)."""
    from count_pipnet_amd import _lib
    from count_pipnet_amd import kernels as K
    g = torch.Generator().manual_seed(13)
    for m, nh, k in [(64, 6144, 2048), (3, 6144, 2048), (37, 256, 512), (1000, 128, 256)]:
        x = torch.randint(0, 4, (m, k), generator=g).float()
        w = torch.randn(2 * nh, k, generator=g) / k ** 0.5
        out = K.linear_pair_mul(x.to(gpu), w.to(gpu)).cpu()
        wd, xd = w.double(), x.double()
        ref = (xd @ wd[nh:].t()) * (xd @ wd[:nh].t())
        scale = ref.abs().max().clamp(min=1.0)
        assert ((out.double() - ref).abs() / scale).max().item() <= 1e-5, (m, nh, k)
        if 1 < K.splitk_factor(m, 2 * nh, k) == K.splitk_factor(m, nh, k):
            we = K.linear(x.to(gpu), w[:nh].contiguous().to(gpu))
            two = K.linear(x.to(gpu), w[nh:].contiguous().to(gpu), epilogue=_lib.EPI_MUL, r=we).cpu()
            assert torch.equal(out, two), (m, nh, k)


def test_bilinear_fold_tracks_weight_updates(gpu):
    """The folded (W E, V E) weights follow every in-place update that bumps a parameter's
    version (optimizer-style ``copy_``/``add_``, ``load_state_dict``); a ``.data`` write is
    invisible to the stamp until ``invalidate_weight_caches`` (documented limitation)."""
    from count_pipnet_amd import invalidate_weight_caches
    from count_pipnet_amd.count_pipnet import intermediate_hip
    from count_pipnet_amd.count_pipnet_utils import BilinearIntermediate
    torch.manual_seed(0)
    layer = BilinearIntermediate(96, 3, custom_init=True).to(gpu).eval()
    x = torch.randint(0, 4, (16, 96), device=gpu).float()

    def check():
        with torch.no_grad():
            e = x.double() @ layer.embed.weight.double().t()
            ref = (e @ layer.W.weight.double().t()) * (e @ layer.V.weight.double().t())
            out = intermediate_hip(layer, x).double()
        scale = ref.abs().max().item()
        return (out - ref).abs().max().item() / scale

    with torch.no_grad():
        assert check() < 1e-5
        layer.W.weight.add_(0.05 * torch.randn_like(layer.W.weight))          # optimizer-style
        assert check() < 1e-5
        sd = {k: v + 0.05 * torch.randn_like(v) for k, v in layer.state_dict().items()}
        layer.load_state_dict(sd)                                             # checkpoint load
        assert check() < 1e-5
        layer.V.weight.copy_(layer.V.weight * 0.5 + 0.01)                     # in-place copy_
        assert check() < 1e-5
        layer.embed.weight.data.mul_(1.5)                                     # bypasses _version
        assert check() > 1e-3                                                 # stale, as documented
        assert invalidate_weight_caches(layer) >= 1
        assert check() < 1e-5


# ---- the hard head's own Philox draw -------------------------------------------------------------

def test_count_gumbel_philox_draws_are_finite(gpu):
    """The Philox head on C5's full grid (64 x 256 pixels x 2,048 channels = 33.5M draws): every
    one-hot value finite and within 1 ulp of 1.  Before round 5's clamp the hardware log2 returned
    0 for uniforms within a few ulp of 1, giving log E = -inf, z = +inf and a NaN one-hot value
    about twice per forward (csrc/philox.hpp log_exp1_from_bits_fast)."""
    from count_pipnet_amd import kernels as K
    g = torch.Generator().manual_seed(21)
    logits = torch.randn(64, 16, 16, 2048, generator=g).to(gpu)
    for seed in (987654321, 5, 2 ** 61 + 3):
        proto, hist = K.count_gumbel(logits, 1.0, None, seed)
        assert torch.isfinite(proto).all(), seed
        nz = proto != 0
        assert torch.equal(nz.sum(dim=-1), torch.ones_like(nz.sum(dim=-1)))
        assert (proto[nz] - 1.0).abs().max().item() <= 2 ** -23
        assert hist.sum().item() == 64 * 256
