"""Generate the golden fixtures under tests/golden/ by running the REFERENCE itself.

Runs only in the build container (``/root/reference`` does not exist on the GPU box; the
fixtures it writes travel instead).  It imports the reference's own, unchanged
``pipnet/pipnet.py``, ``pipnet/count_pipnet.py``, ``pipnet/count_pipnet_utils.py``,
``features/convnext_features.py`` and ``features/resnet_features.py``.  The only
third-party package the reference needs that this image lacks, torchvision, is
replaced by the test-only stand-in in ``tests/golden/tv_standin``.

Weights: every parameter/buffer is overwritten with ``count_pipnet_amd.synthetic``
values keyed by its state_dict name (seed + profile are stored in the fixture).
Inputs: ``synth_images``.  Gumbel noise: ``torch.Tensor.exponential_`` is patched to
emit ``synth_exponential`` samples, so the reference's ``F.gumbel_softmax`` consumes
a recorded Exp(1) draw.

Usage:  python tests/golden/gen_golden.py [--only NAME]
"""
from __future__ import annotations

import argparse
import contextlib
import json
import os
import sys

sys.dont_write_bytecode = True            # /root/reference is read-only
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"

import numpy as np  # noqa: E402
import torch  # noqa: E402

sys.path.insert(0, REPO)
from count_pipnet_amd.synthetic import fill_module_, synth_exponential, synth_images  # noqa: E402

# name -> (model kind, args, num_classes, batch, image size, weight seed, profile, layer_scale)
CASES = {
    # C1: CountPIPNet identity.yaml (configs/identity.yaml), shapes 64x64, bs=16
    "c1_count_identity": dict(model="count_pipnet", net="convnext_tiny_26", use_mid_layers=True,
                              num_stages=3, num_features=16, activation="gumbel_softmax",
                              intermediate_layer="identity", max_count=3, use_ste=True, bias=False,
                              num_classes=9, batch=16, size=64, seed=11),
    # count heads on the same small backbone: every intermediate layer + softmax activation
    "count_onehot": dict(model="count_pipnet", net="convnext_tiny_26", use_mid_layers=True,
                         num_stages=3, num_features=16, activation="gumbel_softmax",
                         intermediate_layer="onehot", max_count=3, use_ste=True, bias=False,
                         num_classes=9, batch=4, size=64, seed=12),
    "count_linear": dict(model="count_pipnet", net="convnext_tiny_26", use_mid_layers=True,
                         num_stages=3, num_features=16, activation="gumbel_softmax",
                         intermediate_layer="linear", max_count=3, use_ste=False, bias=True,
                         num_classes=9, batch=4, size=64, seed=13),
    "count_linear_full": dict(model="count_pipnet", net="convnext_tiny_26", use_mid_layers=True,
                              num_stages=3, num_features=16, activation="softmax",
                              intermediate_layer="linear_full", max_count=3, use_ste=True, bias=False,
                              num_classes=9, batch=4, size=64, seed=14),
    "count_bilinear_small": dict(model="count_pipnet", net="convnext_tiny_26", use_mid_layers=True,
                                 num_stages=3, num_features=16, activation="gumbel_softmax",
                                 intermediate_layer="bilinear", max_count=3, use_ste=True, bias=False,
                                 num_classes=9, batch=4, size=96, seed=15),
    # C5: CountPIPNet bilinear.yaml with a 2048-prototype head at 128x128
    "c5_count_bilinear_2048": dict(model="count_pipnet", net="convnext_tiny_26", use_mid_layers=True,
                                   num_stages=3, num_features=2048, activation="gumbel_softmax",
                                   intermediate_layer="bilinear", max_count=3, use_ste=True, bias=False,
                                   num_classes=9, batch=2, size=128, seed=16),
    # C2: PIP-Net ConvNeXt-tiny-26, CUB 224x224 (configs/used_arguments/CUB_arguments.txt)
    "c2_pipnet_convnext26": dict(model="pipnet", net="convnext_tiny_26", num_features=0, bias=False,
                                 num_classes=200, batch=2, size=224, seed=21),
    "pipnet_convnext26_bias": dict(model="pipnet", net="convnext_tiny_26", num_features=0, bias=True,
                                   num_classes=196, batch=1, size=224, seed=22),
    "pipnet_convnext13": dict(model="pipnet", net="convnext_tiny_13", num_features=0, bias=False,
                              num_classes=200, batch=1, size=224, seed=23),
    "pipnet_mid_addon": dict(model="pipnet", net="convnext_tiny_26", use_mid_layers=True, num_stages=3,
                             num_features=32, bias=True, num_classes=10, batch=4, size=64, seed=24),
    # C3: PIP-Net ResNet50, 224x224
    "c3_pipnet_resnet50": dict(model="pipnet", net="resnet50", num_features=0, bias=False,
                               num_classes=200, batch=2, size=224, seed=31),
    # ResNet-50 PIP-Net at 64x64 (8x8 feature map): the forward case of the ResNet training
    # fixtures (gen_golden_train.py)
    "pipnet_resnet50_small": dict(model="pipnet", net="resnet50", num_features=0, bias=False,
                                  num_classes=10, batch=2, size=64, seed=32),
}
PROFILE = "trained"


def _import_reference():
    sys.path.insert(0, os.path.join(HERE, "tv_standin"))
    sys.path.insert(1, REF)
    import pipnet.count_pipnet as cp  # noqa: F401
    import pipnet.pipnet as pp  # noqa: F401
    return pp, cp


def make_args(case: dict) -> argparse.Namespace:
    a = dict(disable_pretrained=True, positive_grad_strategy=None, backward_clamp_strategy="Gated")
    a.update({k: v for k, v in case.items() if k not in ("model", "num_classes", "batch", "size", "seed")})
    return argparse.Namespace(**a)


@contextlib.contextmanager
def injected_exponential(seed: int):
    """Make the reference's F.gumbel_softmax draw recorded Exp(1) noise."""
    orig = torch.Tensor.exponential_
    drawn = []

    def fake(self, lambd=1.0, *, generator=None):
        e = synth_exponential(tuple(self.shape), seed + len(drawn))
        drawn.append(e)
        with torch.no_grad():
            self.copy_(e)
        return self

    torch.Tensor.exponential_ = fake
    try:
        yield drawn
    finally:
        torch.Tensor.exponential_ = orig


def build_reference(name: str):
    pp, cp = _import_reference()
    case = CASES[name]
    args = make_args(case)
    with contextlib.redirect_stdout(open(os.devnull, "w")):
        if case["model"] == "pipnet":
            net, _ = pp.get_pipnet(case["num_classes"], args)
        else:
            net, _ = cp.get_count_network(case["num_classes"], args, max_count=case["max_count"],
                                          use_ste=case["use_ste"])
    fill_module_(net, case["seed"], PROFILE)
    net.eval()
    return net, case


def run_case(name: str) -> dict:
    net, case = build_reference(name)
    xs = synth_images(case["batch"], case["size"], seed=case["seed"])
    rec = {}
    with torch.no_grad():
        for inference in (True, False):
            with injected_exponential(seed=1000 + case["seed"]) as drawn:
                proto, pooled, out = net(xs, inference=inference)
            tag = "inf" if inference else "raw"
            rec[f"{tag}_pooled"] = pooled.numpy()
            rec[f"{tag}_out"] = out.numpy()
            rec[f"{tag}_proto_sum"] = proto.sum(dim=(2, 3)).numpy()
            rec[f"{tag}_proto_max"] = proto.amax(dim=(2, 3)).numpy()
            rec[f"{tag}_proto_pixmax"] = proto.amax(dim=1).numpy()
            if proto.numel() <= 1 << 16:
                rec[f"{tag}_proto"] = proto.numpy()
            else:   # a deterministic slice: first image, first 8 prototypes
                rec[f"{tag}_proto_slice"] = proto[0, :8].numpy()
            rec[f"{tag}_noise_draws"] = np.array(len(drawn))
    sd = net.state_dict()
    meta = dict(name=name, case=case, profile=PROFILE, noise_seed=1000 + case["seed"],
                keys=[[k, list(v.shape)] for k, v in sd.items()],
                input_sum=float(xs.double().sum()), input_abs=float(xs.double().abs().sum()),
                torch=torch.__version__)
    rec["meta"] = np.array(json.dumps(meta))
    return rec


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default=None)
    a = ap.parse_args()
    torch.set_num_threads(os.cpu_count() or 8)
    for name in CASES:
        if a.only and name != a.only:
            continue
        rec = run_case(name)
        path = os.path.join(HERE, f"{name}.npz")
        np.savez_compressed(path, **rec)
        print(f"wrote {path} ({os.path.getsize(path) / 1e3:.1f} kB)", flush=True)


if __name__ == "__main__":
    main()
