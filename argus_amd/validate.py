"""Per-example validation — the computational core of argus/validate.py:49-128 on the HIP path.

    python -m argus_amd.validate --model-path run.pth --dataset-config.dataset-path D [--use-train]

``ValConfig`` keeps the reference's fields (validate.py:49-83: ``model_path`` must end in ``.pth``
and exist, ``dataset_config``, ``model_config``, ``aug_config``, ``use_train``, ``device``).
``validate(cfg)`` loads the checkpoint (``module.`` / ``_orig_mod.`` prefixes stripped, so DDP and
torch.compile checkpoints of the reference load), runs the model in eval mode over the chosen split
one example at a time (validate.py:100-103,112-128: batch size 1, center crop, eval-mode BN) and
returns the per-example ``mean(geometric_loss_fn(pred, target))`` list the reference accumulates.

Not reproduced: the matplotlib pose plots and image dumps of validate.py:130-190 (visualisation,
out of scope) and the kornia photometric augmentations (the reference applies them only when
``use_train``; argus_amd.data warns about them). Batching (``batch_size`` > 1) gives the same
per-example losses, since eval-mode BN is per-sample.
"""
from __future__ import annotations

import os
from dataclasses import dataclass, field

import torch
from torch.utils.data import DataLoader

from argus_amd.data import AugmentationConfig, CameraCubePoseDataset, CameraCubePoseDatasetConfig
from argus_amd.losses import geometric_loss_fn
from argus_amd.models import NCameraCNN, NCameraCNNConfig


def _default_device() -> str:
    return "cuda"


@dataclass(frozen=True)
class ValConfig:
    """argus/validate.py:49-83."""

    model_path: str
    dataset_config: CameraCubePoseDatasetConfig
    model_config: NCameraCNNConfig = NCameraCNNConfig()
    aug_config: AugmentationConfig = AugmentationConfig()
    use_train: bool = False
    device: str = field(default_factory=_default_device)
    batch_size: int = 1  # extension: the reference validates one example at a time

    def __post_init__(self) -> None:
        assert self.dataset_config is not None, "The dataset config must be provided with a valid dataset path!"
        assert isinstance(self.model_path, str), "The model path must be a str!"
        assert self.model_path.endswith(".pth"), "The model path must end with '.pth'!"
        if not os.path.exists(self.model_path):
            raise FileNotFoundError(f"The specified path does not exist: {self.model_path}")


def load_model(model_path: str, model_config: NCameraCNNConfig | None = None, device="cuda",
               compute_dtype: str = "fp32") -> NCameraCNN:
    """NCameraCNN with the weights of a reference-format ``.pth`` (plain, DDP or compiled keys)."""
    model = NCameraCNN(model_config, compute_dtype=compute_dtype)
    sd = torch.load(model_path, map_location="cpu", weights_only=True)
    model.load_state_dict(sd)
    return model.to(device).eval()


def validate(cfg: ValConfig) -> list[float]:
    """Per-example validation losses of the checkpoint on the chosen split (validate.py:100-128)."""
    model = load_model(cfg.model_path, cfg.model_config, cfg.device)
    dataset = CameraCubePoseDataset(cfg.dataset_config, cfg_aug=cfg.aug_config, train=cfg.use_train, uint8=True)
    loader = DataLoader(dataset, batch_size=cfg.batch_size, shuffle=False)
    losses: list[float] = []
    with torch.no_grad():
        for example in loader:
            images = example["images"].to(cfg.device)
            target = example["cube_pose"].to(cfg.device).to(torch.float32)
            per = geometric_loss_fn(model(images), target)
            losses.extend(per.reshape(-1).cpu().tolist())
    return losses


def main(argv=None) -> list[float]:
    import argparse

    ap = argparse.ArgumentParser(description="argus_amd per-example validation (argus/validate.py)")
    ap.add_argument("--model-path", required=True)
    ap.add_argument("--dataset-config.dataset-path", dest="dataset_path", required=True)
    ap.add_argument("--dataset-config.center-crop", dest="center_crop", type=int, nargs=2, default=(256, 256))
    ap.add_argument("--use-train", action=argparse.BooleanOptionalAction, default=False)
    ap.add_argument("--device", default="cuda")
    ap.add_argument("--batch-size", type=int, default=1)
    a = ap.parse_args(argv)
    cfg = ValConfig(model_path=a.model_path,
                    dataset_config=CameraCubePoseDatasetConfig(a.dataset_path, center_crop=tuple(a.center_crop)),
                    use_train=a.use_train, device=a.device, batch_size=a.batch_size)
    losses = validate(cfg)
    print(f"{len(losses)} examples, mean loss {sum(losses) / max(1, len(losses)):.6f}")
    return losses


if __name__ == "__main__":
    main()
