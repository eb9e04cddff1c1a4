"""CPU: host-side logic — product model init/state_dict vs the golden schema, the train CLI, the
LR plateau scheduler, the flat parameter layout."""
import torch

from argus_amd.models import NCameraCNN, NCameraCNNConfig


def test_model_state_dict_and_seeded_init_match_reference(golden):
    from oracle.ncamera import build_reference_model

    torch.manual_seed(42)
    m = NCameraCNN()
    sd = m.state_dict()
    assert [[k, list(v.shape), str(v.dtype).replace("torch.", "")] for k, v in sd.items()] == golden["state_dict"]
    ref = build_reference_model(42).state_dict()
    assert all(torch.equal(sd[k], ref[k]) for k in sd)
    assert NCameraCNN(NCameraCNNConfig(n_cams=3)).output_mlp[0].in_features == 3 * 1024


def test_flat_params_keep_reference_views():
    from argus_amd.step import FlatParams

    torch.manual_seed(0)
    m = NCameraCNN()
    before = {k: v.clone() for k, v in m.state_dict().items()}
    fp = FlatParams(m)
    after = m.state_dict()
    assert all(torch.equal(before[k], after[k]) for k in before)
    w = m.resnet.layer1[0].conv2.weight
    assert w.shape == (64, 64, 3, 3) and w.data_ptr() >= fp.param.data_ptr()
    assert fp.G["resnet.layer1.0.conv2.weight"].shape == (64, 3, 3, 64)  # OHWI gradient slot
    assert all(o % FlatParams.ALIGN == 0 for o in fp.offset.values())
    m.load_state_dict(before)  # loading into the channels-last views works
    assert torch.equal(m.resnet.layer1[0].conv2.weight, before["resnet.layer1.0.conv2.weight"])


def test_plateau_scheduler_matches_torch():
    from argus_amd.train import PlateauScheduler

    class T:
        lr = 1e-4

    t = T()
    ours = PlateauScheduler(t, patience=5, factor=0.5)
    p = torch.nn.Parameter(torch.zeros(1))
    opt = torch.optim.SGD([p], lr=1e-4)
    ref = torch.optim.lr_scheduler.ReduceLROnPlateau(opt, "min", patience=5, factor=0.5)
    vals = [1.0, 0.9, 0.95, 0.95, 0.95, 0.95, 0.95, 0.95, 0.95, 0.8, 0.8] + [0.8] * 14
    for v in vals:
        ours.step(v)
        ref.step(v)
        assert abs(t.lr - opt.param_groups[0]["lr"]) < 1e-15


def test_cli_flag_names(tmp_path):
    from argus_amd.train import parse_args

    d = tmp_path / "ds"
    (d / "img").mkdir(parents=True)
    (d / "ds.hdf5").write_bytes(b"")
    cfg = parse_args(["--dataset-config.dataset-path", str(d), "--batch-size", "10", "--learning-rate", "1e-3",
                      "--n-epochs", "1", "--amp", "--no-wandb-log", "--model-config.n-cams", "2",
                      "--dataset-config.center-crop", "128", "128", "--save-dir", str(tmp_path / "out")])
    assert cfg.batch_size == 10 and cfg.learning_rate == 1e-3 and cfg.amp and not cfg.wandb_log
    assert cfg.dataset_config.center_crop == (128, 128) and cfg.model_config.n_cams == 2
    assert cfg.max_grad_norm == 1.0 and cfg.random_seed == 42 and not cfg.multigpu


def test_load_state_dict_strips_ddp_and_compile_prefixes(tmp_path):
    """Reference checkpoints saved from a DDP model (``module.``, argus/train.py:199,358) or a compiled
    one (``_orig_mod.``, train.py:61) load into NCameraCNN, also through a .pth file."""
    from argus_amd.models import strip_checkpoint_prefixes

    torch.manual_seed(1)
    src = NCameraCNN()
    sd = src.state_dict()
    for prefix in ("module.", "_orig_mod.", "module._orig_mod.", "_orig_mod.module."):
        path = tmp_path / "ckpt.pth"
        torch.save({prefix + k: v for k, v in sd.items()}, path)
        dst = NCameraCNN()
        res = dst.load_state_dict(torch.load(path, weights_only=True))
        assert not res.missing_keys and not res.unexpected_keys
        assert all(torch.equal(dst.state_dict()[k], sd[k]) for k in sd), prefix
    assert list(strip_checkpoint_prefixes({"module.resnet.fc.bias": 1})) == ["resnet.fc.bias"]


def test_bn_momentum_none_is_cumulative_average():
    """momentum=None -> torch's cumulative moving average factor 1/num_batches_tracked (after the
    increment), handed to the kernels per layer."""
    m = NCameraCNN()
    m.resnet.bn1.momentum = None
    m.resnet.bn1.num_batches_tracked.fill_(3)
    m.train()
    _, Bf = m._maps()
    assert Bf["resnet.bn1.momentum"] == 0.25
    assert Bf["resnet.layer1.0.bn1.momentum"] == 0.1
    # later train-mode forwards use the host shadow count (the finalize kernels increment the device
    # counter; nothing reads it back), a maps call for a backward does not advance it, and a write by
    # torch (load_state_dict, fill_) is picked up through the tensor's version counter
    assert m._maps(forward=False)[1]["resnet.bn1.momentum"] == 0.2
    assert m._maps()[1]["resnet.bn1.momentum"] == 0.2
    assert m._maps()[1]["resnet.bn1.momentum"] == 1 / 6
    m.resnet.bn1.num_batches_tracked.fill_(10)
    assert m._maps()[1]["resnet.bn1.momentum"] == 1 / 11
    # a .data write (dist.broadcast(b.data) in sync_bn_buffers) does not bump the version: the writer
    # invalidates the shadow, and the next forward re-reads the counter
    m.resnet.bn1.num_batches_tracked.data.fill_(20)
    m.invalidate_bn_counters()
    assert m._maps()[1]["resnet.bn1.momentum"] == 1 / 21


def test_spaghetti_draws_reference_arcs():
    """draw_spaghetti (argus/utils.py:252-275): black arcs only, deterministic under the np seed, and
    it consumes exactly six draws per arc (so a seeded worker stays in step with the reference)."""
    import numpy as np
    from PIL import Image

    from argus_amd.utils import draw_spaghetti

    base = Image.new("RGB", (64, 48), (200, 150, 100))
    np.random.seed(5)
    a = np.asarray(draw_spaghetti(base.copy(), 10))
    after_a = np.random.rand()
    np.random.seed(5)
    b = np.asarray(draw_spaghetti(base.copy(), 10))
    assert np.array_equal(a, b)
    changed = (a != np.asarray(base)).any(-1)
    assert changed.any() and (a[changed] == 0).all()
    np.random.seed(5)
    for _ in range(10):
        x0, y0 = np.random.randint(0, 64), np.random.randint(0, 48)
        np.random.randint(x0, 64), np.random.randint(y0, 48), np.random.randint(0, 360), np.random.randint(0, 360)
        np.random.uniform(1.0, 5.0)
    assert np.random.rand() == after_a
    assert np.array_equal(np.asarray(draw_spaghetti(base.copy(), 0)), np.asarray(base))


def test_validate_config_checks(tmp_path):
    import pytest

    from argus_amd.data import CameraCubePoseDatasetConfig
    from argus_amd.validate import ValConfig
    from tests.conftest import make_dummy_dataset

    d = make_dummy_dataset(tmp_path)
    with pytest.raises(AssertionError):
        ValConfig(model_path=str(tmp_path / "x.pt"), dataset_config=CameraCubePoseDatasetConfig(d))
    with pytest.raises(FileNotFoundError):
        ValConfig(model_path=str(tmp_path / "missing.pth"), dataset_config=CameraCubePoseDatasetConfig(d))


def test_train_loaders_never_fork(tmp_path):
    """argus_amd.train builds its DataLoaders spawned and persistent, never forked (the process has
    initialised the GPU by then: a fork()ed loader hung the GPU suite twice in round 2),
    for the default worker count, an explicit one and the distributed samplers; initialize_training
    builds its loaders only through make_loaders."""
    import inspect

    from argus_amd import train as T
    from argus_amd.data import CameraCubePoseDataset, CameraCubePoseDatasetConfig
    from tests.conftest import make_dummy_dataset

    path = make_dummy_dataset(tmp_path, hw=(32, 32))
    dcfg = CameraCubePoseDatasetConfig(dataset_path=path, center_crop=(32, 32))
    tr = CameraCubePoseDataset(dcfg, train=True, uint8=True)
    va = CameraCubePoseDataset(dcfg, train=False, uint8=True)
    for workers, world in ((-1, 1), (3, 1), (2, 2)):
        cfg = T.TrainConfig(dataset_config=dcfg, batch_size=4, num_workers=workers, wandb_log=False,
                            save_dir=str(tmp_path / "out"))
        loaders = T.make_loaders(cfg, tr, va, rank=world - 1, world=world)[:2]
        for ld in loaders:
            assert ld.num_workers > 0 and ld.persistent_workers
            ctx = ld.multiprocessing_context
            assert ctx is not None and ctx.get_start_method() == "spawn", (workers, world, ctx)
    src = inspect.getsource(T)
    assert '"fork"' not in src and "'fork'" not in src  # no fork start method named anywhere
    assert inspect.getsource(T.initialize_training).count("DataLoader(") == 0
