"""Training entry point — drop-in for argus/train.py (TrainConfig, geometric_loss_fn, train, CLI).

    python -m argus_amd.train --dataset-config.dataset-path D [--batch-size 32] [--amp] [--multigpu] ...
    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 -m argus_amd.train ...

Same flag names as the reference's tyro CLI (train.py:58-88; tyro is not installed, a small
dataclass->argparse layer reproduces them), same loop semantics (train.py:264-361): per epoch
train over the loader, print the mean train loss, validate (eval mode, running BN stats), step
ReduceLROnPlateau(patience 5, factor 0.5) on the validation loss, save ``{run_id}.pth`` =
``model.state_dict()`` (reference keys / OIHW shapes) on rank 0 every ``save_epochs``.

The step itself is ``argus_amd.step.FusedTrainer`` (HIP kernels end to end, flat-buffer RCCL
all-reduce + clip + Adam) instead of autograd + DDP. ``--amp`` selects the bf16 kernels (the
reference's fp16 autocast; no GradScaler is needed in bf16). ``--multigpu``: one process per GPU —
either launched by torch.distributed.run (env RANK/WORLD_SIZE) or spawned here like the reference's
mp.spawn (train.py:376). Rendezvous on 127.0.0.1.

Multi-GPU buffers: before every validation pass the BN running statistics (and counters) of rank 0
are broadcast to every rank (``sync_bn_buffers``) — what DDP's ``broadcast_buffers=True`` makes the
reference's ranks validate with (train.py:199; its first no-grad forward after training syncs
buffers from rank 0). Rank 0's own buffers, the checkpointed ones, are never changed by it.

Documented deviations: validation loss is averaged over ALL ranks (the reference's is rank-local,
train.py:342-348, so its per-rank LR schedules can diverge); DDP checkpoints' ``module.`` key prefix
is not produced (the keys are the plain model keys; ``NCameraCNN.load_state_dict`` accepts
``module.`` / ``_orig_mod.`` prefixed checkpoints); ``TrainConfig`` does not require a GPU at
construction time (the reference asserts >= 1 GPU, train.py:99-102).
"""
from __future__ import annotations

import argparse
import typing
import dataclasses
import os
import random
import string
from dataclasses import dataclass, field
from pathlib import Path
from typing import Optional, get_type_hints

import numpy as np
import torch
import torch.distributed as dist
from torch.utils.data import DataLoader
from torch.utils.data.distributed import DistributedSampler

from argus_amd import ROOT
from argus_amd.data import AugmentationConfig, CameraCubePoseDataset, CameraCubePoseDatasetConfig
from argus_amd.losses import geometric_loss_fn
from argus_amd.models import NCameraCNN, NCameraCNNConfig

__all__ = ["TrainConfig", "geometric_loss_fn", "initialize_training", "train", "PlateauScheduler", "main",
           "sync_bn_buffers"]


def _gpu_count() -> int:
    return torch.cuda.device_count()


@dataclass(frozen=True)
class TrainConfig:
    """argus/train.py:29-102 (same fields and defaults)."""

    dataset_config: CameraCubePoseDatasetConfig
    model_config: NCameraCNNConfig = NCameraCNNConfig()
    compile_model: bool = False  # accepted; the HIP engine is not traced (no torch.compile)
    batch_size: int = 32
    learning_rate: float = 1e-4
    n_epochs: int = 100
    device: str = "cuda"
    max_grad_norm: float = 1.0
    num_gpus: int = field(default_factory=_gpu_count)
    random_seed: int = 42
    multigpu: bool = False
    amp: bool = False
    val_epochs: int = 1
    print_epochs: int = 1
    save_epochs: int = 5
    save_dir: str = ROOT + "/outputs/models"
    augmentation_config: AugmentationConfig = AugmentationConfig()
    use_augmentation: bool = True
    wandb_project: str = "argus-estimator"
    wandb_log: bool = True
    num_workers: int = -1  # extension: DataLoader workers (-1: the reference's 16 / 8 per rank, capped)

    def __post_init__(self) -> None:
        assert isinstance(self.save_dir, str)
        if not os.path.exists(self.save_dir):
            if os.path.exists(ROOT + "/" + self.save_dir):
                object.__setattr__(self, "save_dir", ROOT + "/" + self.save_dir)
            else:
                os.makedirs(self.save_dir, exist_ok=True)
        if self.multigpu:
            assert self.num_gpus > 0, "The number of GPUs must be greater than 0!"


class PlateauScheduler:
    """torch.optim.lr_scheduler.ReduceLROnPlateau('min', patience, factor) on the fused trainer's lr
    (defaults threshold 1e-4 rel, cooldown 0, min_lr 0, eps 1e-8)."""

    def __init__(self, trainer, patience: int = 5, factor: float = 0.5, threshold: float = 1e-4, eps: float = 1e-8):
        self.trainer, self.patience, self.factor, self.threshold, self.eps = trainer, patience, factor, threshold, eps
        self.best = float("inf")
        self.num_bad_epochs = 0

    def step(self, metric: float) -> None:
        if metric < self.best * (1.0 - self.threshold):
            self.best = metric
            self.num_bad_epochs = 0
        else:
            self.num_bad_epochs += 1
        if self.num_bad_epochs > self.patience:
            old = self.trainer.lr
            new = old * self.factor
            if old - new > self.eps:
                self.trainer.lr = new
            self.num_bad_epochs = 0


def _run_id() -> str:
    return "".join(random.SystemRandom().choice(string.ascii_lowercase + string.digits) for _ in range(8))


def rank_print(msg: str, rank: int = 0) -> None:
    if rank == 0:
        print(msg, flush=True)


def sync_bn_buffers(model: torch.nn.Module, src: int = 0, group=None) -> None:
    """Broadcast every buffer (BN running_mean / running_var / num_batches_tracked) from rank ``src``
    to all ranks (DDP broadcast_buffers semantics, argus/train.py:199). No-op when not distributed."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size(group) == 1:
        return
    for b in model.buffers():
        dist.broadcast(b.data, src=src, group=group)
    invalidate = getattr(model, "invalidate_bn_counters", None)
    if invalidate is not None:  # .data writes do not bump the counters' version: re-read them
        invalidate()


def _device_for(cfg: TrainConfig, rank: int) -> torch.device:
    """cuda:LOCAL_RANK under torch.distributed.run (multi-node safe), else the reference's
    cuda:rank for mp.spawn (train.py:131); ``cfg.device`` single-process."""
    if not cfg.multigpu:
        return torch.device(cfg.device)
    n = max(1, torch.cuda.device_count())
    local = int(os.environ.get("LOCAL_RANK", rank % n))
    return torch.device("cuda", local)


def make_loaders(cfg: TrainConfig, train_ds, val_ds, rank: int = 0, world: int = 1):
    """DataLoaders and DistributedSamplers of argus/train.py:150-191 (per-rank batch, shuffled
    DistributedSampler for training, ordered for validation). Workers are spawned, never forked: the
    caller has initialised the GPU by then, and a fork()ed child shares the HSA runtime's host-resident
    signal / queue pages copy-on-write, so the parent can miss GPU completions written to a page the
    fork split off (observed: a hang in the first copy of a later validation pass). Persistent workers
    pay the spawn once per loader. Returns (train_loader, val_loader, train_sampler, val_sampler)."""
    distributed = world > 1
    train_sampler = DistributedSampler(train_ds, num_replicas=world, rank=rank, shuffle=True) if distributed else None
    val_sampler = DistributedSampler(val_ds, num_replicas=world, rank=rank, shuffle=False) if distributed else None
    nw = cfg.num_workers
    if nw < 0:
        nw = (8 if distributed else 16) * (2 if cfg.amp else 1)
        nw = min(nw, max(1, (os.cpu_count() or 2) // max(1, world) - 1))
    kw = dict(batch_size=cfg.batch_size, num_workers=nw, pin_memory=True)
    if nw > 0:  # spawn, never fork (docstring)
        kw["multiprocessing_context"] = "spawn"
        kw["persistent_workers"] = True
    train_loader = DataLoader(train_ds, shuffle=train_sampler is None, sampler=train_sampler, **kw)
    val_loader = DataLoader(val_ds, shuffle=False, sampler=val_sampler, **kw)
    return train_loader, val_loader, train_sampler, val_sampler


def initialize_training(cfg: TrainConfig, rank: int = 0, world: int = 1):
    """Seeds, device, datasets/loaders, model, fused trainer, LR schedule (train.py:122-255)."""
    from argus_amd.augment import DeviceAugmentation
    from argus_amd.step import FusedTrainer

    torch.manual_seed(cfg.random_seed)
    np.random.seed(cfg.random_seed)
    if torch.cuda.is_available():
        torch.cuda.manual_seed_all(cfg.random_seed)
    device = _device_for(cfg, rank)
    if device.type != "cuda":
        raise RuntimeError("argus_amd trains on the MI355X HIP path only (device must be cuda)")
    if device.index is None:
        device = torch.device("cuda", torch.cuda.current_device())
    torch.cuda.set_device(device)

    # uint8 batches: 4x less host->device traffic; the /255 of argus/data.py:214-215 runs on the device
    train_ds = CameraCubePoseDataset(cfg.dataset_config, cfg_aug=cfg.augmentation_config, train=True, uint8=True,
                                     device_augmentation=True)
    val_ds = CameraCubePoseDataset(cfg.dataset_config, cfg_aug=cfg.augmentation_config, train=False, uint8=True)
    train_loader, val_loader, train_sampler, val_sampler = make_loaders(cfg, train_ds, val_ds, rank, world)
    distributed = world > 1

    model = NCameraCNN(cfg.model_config, compute_dtype="bf16" if cfg.amp else "fp32").to(device)
    if distributed:  # DDP's constructor broadcast (train.py:199): every rank starts from rank 0's weights
        for t in list(model.parameters()) + list(model.buffers()):
            dist.broadcast(t.data, src=0)
        model.invalidate_bn_counters()
    trainer = FusedTrainer(model, lr=cfg.learning_rate, max_grad_norm=cfg.max_grad_norm)
    scheduler = PlateauScheduler(trainer, patience=5, factor=0.5)
    # the reference's kornia augmentations of each training sample (data.py:222-224), on the device
    trainer.augment = DeviceAugmentation(cfg.augmentation_config, train=True, seed=cfg.random_seed + 1000 * rank)
    return train_loader, val_loader, model, trainer, scheduler, _run_id(), train_sampler, val_sampler, device


def train(cfg: TrainConfig, rank: int = 0) -> str:
    """Main training loop (train.py:264-361). Returns the checkpoint path (rank 0)."""
    world = 1
    if cfg.multigpu:
        if not dist.is_initialized():
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", "12355")
            dist.init_process_group("nccl", rank=rank, world_size=cfg.num_gpus)
        world = dist.get_world_size()
        rank = dist.get_rank()
    (train_loader, val_loader, model, trainer, scheduler, run_id, train_sampler, _vs,
     device) = initialize_training(cfg, rank, world)
    wandb = None
    if cfg.wandb_log and rank == 0:
        try:
            import wandb  # noqa: F811

            wandb.init(project=cfg.wandb_project, config=dataclasses.asdict(cfg), id=run_id, resume="allow")
        except Exception as e:  # not installed / offline
            rank_print(f"wandb logging disabled ({type(e).__name__}: {e})")
            wandb = None
    save_path = ""
    for epoch in range(cfg.n_epochs):
        if world > 1:
            dist.barrier()
            train_sampler.set_epoch(epoch)
        model.train()
        epoch_losses = []
        for example in train_loader:
            images = trainer.augment(example["images"].to(device, non_blocking=True))
            target = example["cube_pose"].to(device, non_blocking=True)
            losses = trainer.step(images, target)
            epoch_losses.append(losses.clone())
            if wandb is not None:
                wandb.log({"loss": losses.mean().item()})
        if epoch % cfg.print_epochs == 0 and epoch_losses:
            rank_print(f"    Avg. Loss in Epoch: {torch.mean(torch.cat(epoch_losses)).item()}", rank)
        if epoch % cfg.val_epochs == 0:
            sync_bn_buffers(model)  # every rank validates with rank 0's running statistics
            model.eval()
            tot = torch.zeros(2, dtype=torch.float64, device=device)
            with torch.no_grad():
                for example in val_loader:
                    pred = model(example["images"].to(device, non_blocking=True))
                    vl = geometric_loss_fn(pred, example["cube_pose"].to(device, non_blocking=True))
                    tot += torch.stack([vl.double().sum(), torch.tensor(float(vl.numel()), device=device,
                                                                         dtype=torch.float64)])
            if world > 1:
                dist.all_reduce(tot)
            val_loss = (tot[0] / tot[1].clamp_min(1)).item()
            if wandb is not None:
                wandb.log({"val_loss": val_loss})
            rank_print(f"    Validation loss: {val_loss}", rank)
            scheduler.step(val_loss)
        if epoch % cfg.save_epochs == 0:
            save_dir = Path(cfg.save_dir) if cfg.save_dir is not None else Path(ROOT + "/outputs/models")
            os.makedirs(save_dir, exist_ok=True)
            if rank == 0:
                save_path = str(save_dir / f"{run_id}.pth")
                torch.save({k: v.detach().cpu().contiguous().clone() for k, v in model.state_dict().items()},
                           save_path)
    if cfg.multigpu and dist.is_initialized():
        dist.destroy_process_group()
    return save_path


# ------------------------------------------------------------------------------ CLI (tyro-compatible)
def _flag(name: str) -> str:
    return "--" + name.replace("_", "-")


def _add_dataclass_args(ap: argparse.ArgumentParser, cls, prefix: str = "") -> None:
    hints = get_type_hints(cls)
    for f in dataclasses.fields(cls):
        name = prefix + f.name
        tp = hints[f.name]
        if dataclasses.is_dataclass(tp):
            _add_dataclass_args(ap, tp, name + ".")
            continue
        flag = "--" + ".".join(p.replace("_", "-") for p in name.split("."))
        if tp is bool:
            ap.add_argument(flag, dest=name, action=argparse.BooleanOptionalAction, default=None)
        elif tp in (int, float, str):
            ap.add_argument(flag, dest=name, type=tp, default=None)
        elif set(typing.get_args(tp)) == {str, type(None)}:  # Optional[str]: one string, kept verbatim
            ap.add_argument(flag, dest=name, type=str, default=None)
        else:  # Optional[str], tuples, unions: parse str / lists
            ap.add_argument(flag, dest=name, nargs="+", default=None)


def _build(cls, ns: dict, prefix: str = ""):
    hints = get_type_hints(cls)
    kw = {}
    for f in dataclasses.fields(cls):
        name = prefix + f.name
        tp = hints[f.name]
        if dataclasses.is_dataclass(tp):
            sub = _build(tp, ns, name + ".")
            if sub is not None:
                kw[f.name] = sub
            continue
        v = ns.get(name)
        if v is None:
            continue
        if isinstance(v, list):
            if len(v) == 1:
                v = v[0]
                try:
                    v = float(v) if "." in v else int(v)
                except ValueError:
                    pass
            else:
                v = tuple(float(x) if "." in x else int(x) for x in v)
        kw[f.name] = v
    if not kw and cls is not TrainConfig:
        return None
    return cls(**kw)


def parse_args(argv=None) -> TrainConfig:
    ap = argparse.ArgumentParser(description="argus_amd training (argus/train.py CLI)")
    _add_dataclass_args(ap, TrainConfig)
    ns = vars(ap.parse_args(argv))
    if ns.get("dataset_config.dataset_path") is None:
        ap.error("--dataset-config.dataset-path is required")
    return _build(TrainConfig, ns)


def _train_multigpu(rank: int, cfg: TrainConfig) -> None:
    train(cfg, rank=rank)


def main(argv=None) -> None:
    cfg = parse_args(argv)
    if cfg.multigpu and "WORLD_SIZE" not in os.environ:
        import torch.multiprocessing as mp

        mp.spawn(_train_multigpu, args=(cfg,), nprocs=cfg.num_gpus, join=True)
    else:
        rank = int(os.environ.get("RANK", "0"))
        if "LOCAL_RANK" in os.environ:
            torch.cuda.set_device(int(os.environ["LOCAL_RANK"]))
        train(cfg, rank=rank)


if __name__ == "__main__":
    main()
