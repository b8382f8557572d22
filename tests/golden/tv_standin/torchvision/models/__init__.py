"""TEST-ONLY restatement of torchvision's ConvNeXt-tiny (module tree + eval math).

Semantics:
  features = [Conv2dNormActivation(3,96,k4,s4,bias, LayerNorm2d(eps 1e-6), act=None)]
             + for (96,192,3),(192,384,3),(384,768,9),(768,None,3):
                 Sequential(CNBlock x n) and, if out is not None,
                 Sequential(LayerNorm2d(cin), Conv2d(cin,cout,k2,s2))
  CNBlock.block = [dwconv7x7 p3 groups=d, Permute(0,2,3,1), LayerNorm(d,1e-6),
                   Linear(d,4d), GELU(erf), Linear(4d,d), Permute(0,3,1,2)]
  CNBlock.forward = layer_scale * block(x) (+ stochastic depth, identity in eval) + x
"""
import torch
import torch.nn as nn
import torch.nn.functional as F


class LayerNorm2d(nn.LayerNorm):
    def forward(self, x):
        x = x.permute(0, 2, 3, 1)
        x = F.layer_norm(x, self.normalized_shape, self.weight, self.bias, self.eps)
        return x.permute(0, 3, 1, 2)


class Permute(nn.Module):
    def __init__(self, dims):
        super().__init__()
        self.dims = list(dims)

    def forward(self, x):
        return torch.permute(x, self.dims)


class StochasticDepth(nn.Module):
    def __init__(self, p, mode):
        super().__init__()
        self.p, self.mode = p, mode

    def forward(self, x):
        if not self.training or self.p == 0.0:
            return x
        keep = 1.0 - self.p
        shape = [x.shape[0]] + [1] * (x.ndim - 1)
        noise = torch.empty(shape, dtype=x.dtype, device=x.device).bernoulli_(keep)
        return x * noise.div_(keep)


class CNBlock(nn.Module):
    def __init__(self, dim, layer_scale, sd_prob):
        super().__init__()
        self.block = nn.Sequential(
            nn.Conv2d(dim, dim, kernel_size=7, padding=3, groups=dim, bias=True),
            Permute([0, 2, 3, 1]),
            nn.LayerNorm(dim, eps=1e-6),
            nn.Linear(dim, 4 * dim, bias=True),
            nn.GELU(),
            nn.Linear(4 * dim, dim, bias=True),
            Permute([0, 3, 1, 2]),
        )
        self.layer_scale = nn.Parameter(torch.ones(dim, 1, 1) * layer_scale)
        self.stochastic_depth = StochasticDepth(sd_prob, "row")

    def forward(self, x):
        result = self.layer_scale * self.block(x)
        result = self.stochastic_depth(result)
        result += x
        return result


class Conv2dNormActivation(nn.Sequential):
    def __init__(self, cin, cout, kernel_size, stride, norm_layer):
        super().__init__(nn.Conv2d(cin, cout, kernel_size=kernel_size, stride=stride,
                                   padding=0, bias=True),
                         norm_layer(cout))


class ConvNeXt(nn.Module):
    def __init__(self, stochastic_depth_prob=0.1, layer_scale=1e-6):
        super().__init__()
        setting = [(96, 192, 3), (192, 384, 3), (384, 768, 9), (768, None, 3)]
        norm = lambda c: LayerNorm2d(c, eps=1e-6)  # noqa: E731
        layers = [Conv2dNormActivation(3, 96, 4, 4, norm)]
        total = sum(n for _, _, n in setting)
        stage_block_id = 0
        for cin, cout, n in setting:
            stage = []
            for _ in range(n):
                sd = stochastic_depth_prob * stage_block_id / (total - 1.0)
                stage.append(CNBlock(cin, layer_scale, sd))
                stage_block_id += 1
            layers.append(nn.Sequential(*stage))
            if cout is not None:
                layers.append(nn.Sequential(norm(cin), nn.Conv2d(cin, cout, kernel_size=2, stride=2)))
        self.features = nn.Sequential(*layers)
        self.avgpool = nn.AdaptiveAvgPool2d(1)
        self.classifier = nn.Sequential(norm(768), nn.Flatten(1), nn.Linear(768, 1000))
        for m in self.modules():
            if isinstance(m, (nn.Conv2d, nn.Linear)):
                nn.init.trunc_normal_(m.weight, std=0.02)
                if m.bias is not None:
                    nn.init.zeros_(m.bias)

    def forward(self, x):
        x = self.features(x)
        x = self.avgpool(x)
        return self.classifier(x)


class ConvNeXt_Tiny_Weights:
    DEFAULT = "IMAGENET1K_V1"


def convnext_tiny(weights=None, **kwargs):
    if weights is not None:
        raise RuntimeError("stand-in: pretrained weights are unavailable offline")
    return ConvNeXt(stochastic_depth_prob=0.1, **kwargs)
