"""NCameraCNN restated — TEST INFRASTRUCTURE (oracle), never product code.

Follows ``argus/models.py:13-90`` line by line:
- ``NCameraCNNConfig`` (``models.py:13-23``): ``n_cams=2``, ``resnet_output_dim=1024``.
- ``__init__`` (``models.py:36-64``): ResNet-50 (with its original 2048->1000 ``fc`` constructed and
  initialised, consuming RNG, ``models.py:43``), ``avgpool`` replaced (``:55``), ``fc`` replaced by
  Linear(2048, 1024) (``:56``), ``output_mlp`` = Linear(2048,128), GELU, Linear(128,128), GELU,
  Linear(128,6) (``:58-64``).
- ``forward`` (``models.py:66-90``): assert 4-D (``:76``), reshape (B, 3n, H, W) -> (B n, 3, H, W)
  (``:81``), ResNet (``:84``), reshape (B, n*1024) (``:87``), exact-erf GELU (``:88``), MLP (``:90``).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Optional

import torch
import torch.nn as nn

from oracle.resnet import resnet50


@dataclass(frozen=True)
class NCameraCNNConfig:
    n_cams: int = 2
    resnet_output_dim: int = 1024


class NCameraCNN(nn.Module):
    def __init__(self, cfg: Optional[NCameraCNNConfig] = None) -> None:
        super().__init__()
        self.resnet = resnet50(weights="DEFAULT")
        if cfg is None:
            cfg = NCameraCNNConfig()
        self.num_channels = 3 * cfg.n_cams
        self.resnet_output_dim = cfg.resnet_output_dim
        self.n_cams = cfg.n_cams
        self.resnet.avgpool = nn.AdaptiveAvgPool2d((1, 1))
        self.resnet.fc = nn.Linear(self.resnet.fc.in_features, self.resnet_output_dim)
        self.output_mlp = nn.Sequential(
            nn.Linear(self.n_cams * self.resnet_output_dim, 128),
            nn.GELU(),
            nn.Linear(128, 128),
            nn.GELU(),
            nn.Linear(128, 6),
        )

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        assert len(x.shape) == 4, "The input images must be of shape (B, C, H, W)! If B=1, add a dummy dimension."
        B = x.shape[0]
        x = x.reshape(-1, 3, *(x.shape[-2:]))
        x = self.resnet(x)
        x = x.reshape(B, self.n_cams * self.resnet_output_dim)
        x = nn.GELU()(x)
        return self.output_mlp(x)


def build_reference_model(seed: int = 42, cfg: Optional[NCameraCNNConfig] = None) -> NCameraCNN:
    """Seeded construction in the reference's order (``argus/train.py:127-129,201``), on CPU."""
    torch.manual_seed(seed)
    return NCameraCNN(cfg)
