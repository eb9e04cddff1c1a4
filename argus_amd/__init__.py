"""argus_amd — MI355X-native (gfx950) implementation of the argus training hot path.

Drop-in surface (mirrors the reference package ``argus``):
  argus_amd.models   NCameraCNN, NCameraCNNConfig            (argus/models.py)
  argus_amd.losses   geometric_loss_fn                        (argus/train.py:105-119)
  argus_amd.train    TrainConfig, train, CLI                  (argus/train.py)
  argus_amd.data     CameraCubePoseDataset(+Config), AugmentationConfig (argus/data.py)
  argus_amd.utils    pose-order conversions, get_pose, time_torch_fn   (argus/utils.py)
Compute: libargus_hip.so (include/argus_hip.h), hand-written HIP kernels for CDNA4.
"""
from pathlib import Path

ROOT = str(Path(__file__).resolve().parent.parent)
