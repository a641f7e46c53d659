"""Inception-v3 feature extractor for FID, implemented natively (no torchvision dependency).

The reference's default FID model is ``torchvision.models.inception_v3(weights="DEFAULT")``
with ``fc = Identity`` behind a bilinear resize to 299x299 (torcheval/metrics/image/fid.py:
28-50), and ``import torcheval.metrics`` fails outright when torchvision is missing.  This
module re-implements the same architecture (module names follow torchvision's layout, so a
converted torchvision state dict loads with ``load_state_dict``), runs channels-last /
bf16-autocast friendly on ROCm (convolutions go to MIOpen), and is imported lazily.

Pretrained ImageNet weights are NOT bundled (no network in this environment): the model is
randomly initialised unless ``weights_path`` points to a local ``.safetensors`` /
``.pt`` state dict.  FID values are only comparable to published numbers with those weights.
"""

import warnings
from typing import Optional

import torch
import torch.nn as nn
import torch.nn.functional as F

__all__ = ["Inception3", "FIDInceptionV3", "inception_v3"]


class BasicConv2d(nn.Module):
    def __init__(self, cin: int, cout: int, **kwargs) -> None:
        super().__init__()
        self.conv = nn.Conv2d(cin, cout, bias=False, **kwargs)
        self.bn = nn.BatchNorm2d(cout, eps=0.001)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return F.relu(self.bn(self.conv(x)), inplace=True)


class InceptionA(nn.Module):
    def __init__(self, cin: int, pool_features: int) -> None:
        super().__init__()
        self.branch1x1 = BasicConv2d(cin, 64, kernel_size=1)
        self.branch5x5_1 = BasicConv2d(cin, 48, kernel_size=1)
        self.branch5x5_2 = BasicConv2d(48, 64, kernel_size=5, padding=2)
        self.branch3x3dbl_1 = BasicConv2d(cin, 64, kernel_size=1)
        self.branch3x3dbl_2 = BasicConv2d(64, 96, kernel_size=3, padding=1)
        self.branch3x3dbl_3 = BasicConv2d(96, 96, kernel_size=3, padding=1)
        self.branch_pool = BasicConv2d(cin, pool_features, kernel_size=1)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        b1 = self.branch1x1(x)
        b5 = self.branch5x5_2(self.branch5x5_1(x))
        b3 = self.branch3x3dbl_3(self.branch3x3dbl_2(self.branch3x3dbl_1(x)))
        bp = self.branch_pool(F.avg_pool2d(x, kernel_size=3, stride=1, padding=1))
        return torch.cat([b1, b5, b3, bp], 1)


class InceptionB(nn.Module):
    def __init__(self, cin: int) -> None:
        super().__init__()
        self.branch3x3 = BasicConv2d(cin, 384, kernel_size=3, stride=2)
        self.branch3x3dbl_1 = BasicConv2d(cin, 64, kernel_size=1)
        self.branch3x3dbl_2 = BasicConv2d(64, 96, kernel_size=3, padding=1)
        self.branch3x3dbl_3 = BasicConv2d(96, 96, kernel_size=3, stride=2)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        b3 = self.branch3x3(x)
        bd = self.branch3x3dbl_3(self.branch3x3dbl_2(self.branch3x3dbl_1(x)))
        bp = F.max_pool2d(x, kernel_size=3, stride=2)
        return torch.cat([b3, bd, bp], 1)


class InceptionC(nn.Module):
    def __init__(self, cin: int, channels_7x7: int) -> None:
        super().__init__()
        c7 = channels_7x7
        self.branch1x1 = BasicConv2d(cin, 192, kernel_size=1)
        self.branch7x7_1 = BasicConv2d(cin, c7, kernel_size=1)
        self.branch7x7_2 = BasicConv2d(c7, c7, kernel_size=(1, 7), padding=(0, 3))
        self.branch7x7_3 = BasicConv2d(c7, 192, kernel_size=(7, 1), padding=(3, 0))
        self.branch7x7dbl_1 = BasicConv2d(cin, c7, kernel_size=1)
        self.branch7x7dbl_2 = BasicConv2d(c7, c7, kernel_size=(7, 1), padding=(3, 0))
        self.branch7x7dbl_3 = BasicConv2d(c7, c7, kernel_size=(1, 7), padding=(0, 3))
        self.branch7x7dbl_4 = BasicConv2d(c7, c7, kernel_size=(7, 1), padding=(3, 0))
        self.branch7x7dbl_5 = BasicConv2d(c7, 192, kernel_size=(1, 7), padding=(0, 3))
        self.branch_pool = BasicConv2d(cin, 192, kernel_size=1)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        b1 = self.branch1x1(x)
        b7 = self.branch7x7_3(self.branch7x7_2(self.branch7x7_1(x)))
        bd = self.branch7x7dbl_1(x)
        for layer in (self.branch7x7dbl_2, self.branch7x7dbl_3, self.branch7x7dbl_4, self.branch7x7dbl_5):
            bd = layer(bd)
        bp = self.branch_pool(F.avg_pool2d(x, kernel_size=3, stride=1, padding=1))
        return torch.cat([b1, b7, bd, bp], 1)


class InceptionD(nn.Module):
    def __init__(self, cin: int) -> None:
        super().__init__()
        self.branch3x3_1 = BasicConv2d(cin, 192, kernel_size=1)
        self.branch3x3_2 = BasicConv2d(192, 320, kernel_size=3, stride=2)
        self.branch7x7x3_1 = BasicConv2d(cin, 192, kernel_size=1)
        self.branch7x7x3_2 = BasicConv2d(192, 192, kernel_size=(1, 7), padding=(0, 3))
        self.branch7x7x3_3 = BasicConv2d(192, 192, kernel_size=(7, 1), padding=(3, 0))
        self.branch7x7x3_4 = BasicConv2d(192, 192, kernel_size=3, stride=2)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        b3 = self.branch3x3_2(self.branch3x3_1(x))
        b7 = self.branch7x7x3_4(self.branch7x7x3_3(self.branch7x7x3_2(self.branch7x7x3_1(x))))
        bp = F.max_pool2d(x, kernel_size=3, stride=2)
        return torch.cat([b3, b7, bp], 1)


class InceptionE(nn.Module):
    def __init__(self, cin: int) -> None:
        super().__init__()
        self.branch1x1 = BasicConv2d(cin, 320, kernel_size=1)
        self.branch3x3_1 = BasicConv2d(cin, 384, kernel_size=1)
        self.branch3x3_2a = BasicConv2d(384, 384, kernel_size=(1, 3), padding=(0, 1))
        self.branch3x3_2b = BasicConv2d(384, 384, kernel_size=(3, 1), padding=(1, 0))
        self.branch3x3dbl_1 = BasicConv2d(cin, 448, kernel_size=1)
        self.branch3x3dbl_2 = BasicConv2d(448, 384, kernel_size=3, padding=1)
        self.branch3x3dbl_3a = BasicConv2d(384, 384, kernel_size=(1, 3), padding=(0, 1))
        self.branch3x3dbl_3b = BasicConv2d(384, 384, kernel_size=(3, 1), padding=(1, 0))
        self.branch_pool = BasicConv2d(cin, 192, kernel_size=1)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        b1 = self.branch1x1(x)
        b3 = self.branch3x3_1(x)
        b3 = torch.cat([self.branch3x3_2a(b3), self.branch3x3_2b(b3)], 1)
        bd = self.branch3x3dbl_2(self.branch3x3dbl_1(x))
        bd = torch.cat([self.branch3x3dbl_3a(bd), self.branch3x3dbl_3b(bd)], 1)
        bp = self.branch_pool(F.avg_pool2d(x, kernel_size=3, stride=1, padding=1))
        return torch.cat([b1, b3, bd, bp], 1)


class Inception3(nn.Module):
    """Inception-v3 trunk + 1000-way classifier (torchvision-compatible parameter names;
    the auxiliary classifier is omitted: it only runs in training mode)."""

    def __init__(self, num_classes: int = 1000, transform_input: bool = True, dropout: float = 0.5) -> None:
        super().__init__()
        self.transform_input = transform_input
        self.Conv2d_1a_3x3 = BasicConv2d(3, 32, kernel_size=3, stride=2)
        self.Conv2d_2a_3x3 = BasicConv2d(32, 32, kernel_size=3)
        self.Conv2d_2b_3x3 = BasicConv2d(32, 64, kernel_size=3, padding=1)
        self.maxpool1 = nn.MaxPool2d(kernel_size=3, stride=2)
        self.Conv2d_3b_1x1 = BasicConv2d(64, 80, kernel_size=1)
        self.Conv2d_4a_3x3 = BasicConv2d(80, 192, kernel_size=3)
        self.maxpool2 = nn.MaxPool2d(kernel_size=3, stride=2)
        self.Mixed_5b = InceptionA(192, pool_features=32)
        self.Mixed_5c = InceptionA(256, pool_features=64)
        self.Mixed_5d = InceptionA(288, pool_features=64)
        self.Mixed_6a = InceptionB(288)
        self.Mixed_6b = InceptionC(768, channels_7x7=128)
        self.Mixed_6c = InceptionC(768, channels_7x7=160)
        self.Mixed_6d = InceptionC(768, channels_7x7=160)
        self.Mixed_6e = InceptionC(768, channels_7x7=192)
        self.Mixed_7a = InceptionD(768)
        self.Mixed_7b = InceptionE(1280)
        self.Mixed_7c = InceptionE(2048)
        self.avgpool = nn.AdaptiveAvgPool2d((1, 1))
        self.dropout = nn.Dropout(p=dropout)
        self.fc: nn.Module = nn.Linear(2048, num_classes)
        for m in self.modules():
            if isinstance(m, (nn.Conv2d, nn.Linear)):
                nn.init.trunc_normal_(m.weight, mean=0.0, std=0.1, a=-2, b=2)
            elif isinstance(m, nn.BatchNorm2d):
                nn.init.constant_(m.weight, 1)
                nn.init.constant_(m.bias, 0)

    def _transform_input(self, x: torch.Tensor) -> torch.Tensor:
        if not self.transform_input:
            return x
        x0 = x[:, 0:1] * (0.229 / 0.5) + (0.485 - 0.5) / 0.5
        x1 = x[:, 1:2] * (0.224 / 0.5) + (0.456 - 0.5) / 0.5
        x2 = x[:, 2:3] * (0.225 / 0.5) + (0.406 - 0.5) / 0.5
        return torch.cat((x0, x1, x2), 1)

    def features(self, x: torch.Tensor) -> torch.Tensor:
        x = self._transform_input(x)
        for name in (
            "Conv2d_1a_3x3", "Conv2d_2a_3x3", "Conv2d_2b_3x3", "maxpool1", "Conv2d_3b_1x1",
            "Conv2d_4a_3x3", "maxpool2", "Mixed_5b", "Mixed_5c", "Mixed_5d", "Mixed_6a",
            "Mixed_6b", "Mixed_6c", "Mixed_6d", "Mixed_6e", "Mixed_7a", "Mixed_7b", "Mixed_7c",
        ):
            x = getattr(self, name)(x)
        return torch.flatten(self.avgpool(x), 1)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return self.fc(self.dropout(self.features(x)))


def inception_v3(weights_path: Optional[str] = None, **kwargs) -> Inception3:
    """Build Inception-v3; load a local state dict (safetensors or torch, weights only) if given."""
    model = Inception3(**kwargs)
    if weights_path is not None:
        if weights_path.endswith(".safetensors"):
            from safetensors.torch import load_file

            state = load_file(weights_path)
        else:
            state = torch.load(weights_path, map_location="cpu", weights_only=True)
        # the auxiliary classifier is not part of this feature model: drop it explicitly, then
        # load strictly - a renamed or partial checkpoint must not leave random weights behind
        state = {k: v for k, v in state.items() if not k.startswith("AuxLogits.")}
        missing, unexpected = _key_mismatch(model, state)
        if missing or unexpected:
            raise RuntimeError(
                f"Inception-v3 checkpoint {weights_path!r} does not match the model: "
                f"missing keys {missing[:8]}{' ...' if len(missing) > 8 else ''}, "
                f"unexpected keys {unexpected[:8]}{' ...' if len(unexpected) > 8 else ''}."
            )
        model.load_state_dict(state, strict=True)
    return model


def _key_mismatch(model: nn.Module, state: dict):
    want = set(model.state_dict().keys())
    have = set(state.keys())
    return sorted(want - have), sorted(have - want)


class FIDInceptionV3(nn.Module):
    """FID feature extractor: bilinear resize to 299x299 -> Inception-v3 pooled 2048-d features."""

    def __init__(self, weights: Optional[str] = "DEFAULT", weights_path: Optional[str] = None) -> None:
        super().__init__()
        self.model = inception_v3(weights_path=weights_path)
        self.model.fc = nn.Identity()
        if weights_path is None and weights is not None:
            warnings.warn(
                "Pretrained Inception-v3 weights are not available offline; FIDInceptionV3 is "
                "randomly initialised (pass weights_path=... to load a local checkpoint).",
                RuntimeWarning,
            )

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        x = F.interpolate(x, size=(299, 299), mode="bilinear", align_corners=False)
        return self.model(x)
