"""Data-parallel parity of FusedTrainer with two ranks on the GPU box.

Reference semantics (argus/train.py:137-168, 298-321 under DDP): every rank draws its own shard of
the global batch, BatchNorm statistics stay per rank (no SyncBN), the per-rank mean-loss gradients
are averaged, and every rank applies the same clip + Adam step.

The box has one GPU and RCCL refuses two ranks on one device. Both ranks therefore share cuda:0,
and the flat-gradient buckets go over gloo (CUDA tensors, staged through the host). FusedTrainer
issues the same bucketed all-reduce calls it issues over RCCL; only the transport differs.

Checks, fp32 parity path, global batch of 4 samples split 2 + 2:
- each rank's all-reduced flat gradient equals g(shard 0) + g(shard 1), both computed locally
  without the collective. The SUM of two addends is order-free, so this holds bit for bit;
- after the step the parameters are bitwise identical on both ranks;
- the per-rank BN running statistics are those of the rank's own shard (no SyncBN).
"""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _local_grads(x, T, dev):
    """g(shard) for each shard, with no collective: the engine schedule FusedTrainer.step runs."""
    import ctypes as C

    from argus_amd._lib import lib, ptr, stream
    from argus_amd.models import NCameraCNN
    from argus_amd.step import FlatParams

    torch.manual_seed(42)
    model = NCameraCNN().to(dev).train()
    flat = FlatParams(model)
    eng = model._engine(dev)
    P, Bf = model._maps()
    out = []
    for r in range(2):
        xs, ts = x[2 * r:2 * r + 2].to(dev), T[2 * r:2 * r + 2].to(dev).contiguous()
        pred = eng.forward(xs, P, Bf, True)
        loss = torch.empty(2, device=dev)
        dpred = torch.empty(2, 6, device=dev)
        lib().se3_loss(2, ptr(pred), ptr(ts), ptr(loss), ptr(dpred), C.c_float(0.5), stream())
        flat.grad.zero_()
        eng.backward(dpred, P, flat.G)
        torch.cuda.synchronize()
        out.append(flat.grad.clone())
    return out


def _worker(rank, port, x, T, outdir, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), HSA_ENABLE_IPC_MODE_LEGACY="0")
        import torch.distributed as dist

        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        dist.init_process_group("gloo", rank=rank, world_size=2)
        from argus_amd.models import NCameraCNN
        from argus_amd.step import FusedTrainer

        g0, g1 = _local_grads(x, T, dev)
        torch.manual_seed(42)
        model = NCameraCNN().to(dev).train()
        tr = FusedTrainer(model, lr=1e-3, max_grad_norm=1.0, bucket_mb=8.0)
        assert tr.distributed and tr.world == 2
        tr.step(x[2 * rank:2 * rank + 2].to(dev), T[2 * rank:2 * rank + 2].to(dev))
        torch.cuda.synchronize()
        grad_ok = bool(torch.equal(tr.flat.grad, g0 + g1))
        gmax = (tr.flat.grad - (g0 + g1)).abs().max().item()
        torch.save({"param": tr.flat.param.cpu(), "rm": model.resnet.bn1.running_mean.cpu()},
                   os.path.join(outdir, f"rank{rank}.pt"))
        dist.destroy_process_group()
        q.put((rank, grad_ok, gmax, None))
    except Exception as e:  # report, don't hang the parent
        q.put((rank, False, float("nan"), repr(e)))


def test_two_rank_step_matches_shard_gradient_sum(cuda, tmp_path):
    from oracle import se3

    g = torch.Generator().manual_seed(77)
    x = torch.randint(0, 256, (4, 6, 64, 64), generator=g, dtype=torch.uint8).float() / 255.0
    T = se3.random_targets(4, generator=g).float()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, port, x, T, str(tmp_path), q)) for r in range(2)]
    for p in procs:
        p.start()
    try:
        res = sorted(q.get(timeout=240) for _ in procs)
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    for rank, ok, gmax, err in res:
        assert err is None, f"rank {rank}: {err}"
        assert ok, f"rank {rank}: all-reduced gradient != g0 + g1 (max |diff| {gmax:.3e})"
    s0 = torch.load(tmp_path / "rank0.pt", weights_only=True)
    s1 = torch.load(tmp_path / "rank1.pt", weights_only=True)
    assert torch.equal(s0["param"], s1["param"]), "ranks diverged after the step"
    # per-rank BN (no SyncBN): the stem's running mean differs between the two shards
    assert not torch.equal(s0["rm"], s1["rm"])
