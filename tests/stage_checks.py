"""Shared GPU-test helper (not a test module): fp64 re-derivation of every backward stage of every
Bottleneck from the engine's own saved tensors (engine.debug captures)."""
import torch


def rel_max(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-30)).item()


def stage_checks(eng, P, debug, tol_max):
    """``tol_max``: one max-relative bar, or a dict stage -> bar. Each stage's kernel output vs fp64 torch on that stage's kernel inputs:
    dy3 / dy2 / dy1  BN backward (finalize + apply) from the masked dm;
    dz2 / dz1        dgrad + the fused BN-backward epilogue's ReLU mask (stored dm);
    dout             the previous block's dm3 = relu'(out) * (conv1 dgrad [+ downsample dgrad | skip]),
                     produced by this block's last dgrad with the fused epilogue;
    dW3 / dW2 / dW1  weight gradients (+ dWd of the downsample conv); a1 / a2 the materialised
                     relu(bn(y)) (bf16 schedule)."""
    nchw = lambda t: t.detach().double().cpu().permute(0, 3, 1, 2)  # noqa: E731
    col = lambda v: v[None, :, None, None]  # noqa: E731

    def bn_bwd(dm, y, mean, invstd, gamma):
        xh = (y - col(mean)) * col(invstd)
        n = dm.shape[0] * dm.shape[2] * dm.shape[3]
        S, Tt = dm.sum((0, 2, 3)), (dm * xh).sum((0, 2, 3))
        return col(gamma * invstd) * (dm - col(S) / n - xh * col(Tt) / n)

    worst = {}
    for idx, (b, a) in enumerate(zip(eng.blocks, eng.act)):
        pf = b.prefix
        st = {k: eng.bn_state[pf + k].double().cpu() for k in (".bn1", ".bn2", ".bn3")}
        gm = {k: P[pf + k + ".weight"].double().cpu() for k in (".bn1", ".bn2", ".bn3")}
        D = {k: nchw(debug[k + "." + pf]) for k in ("b_dout", "b_dy3", "b_dz2", "b_dy2", "b_dz1", "b_dy1")}
        out, y3, y2, y1 = nchw(a["out"]), nchw(a["y3"]), nchw(a["y2"]), nchw(a["y1"])
        z1 = torch.relu(y1 * col(st[".bn1"][2]) + col(st[".bn1"][3]))
        z2 = torch.relu(y2 * col(st[".bn2"][2]) + col(st[".bn2"][3]))
        checks = {}
        if eng.materialize:  # the materialised relu(bn(y)) the conv2/conv3 kernels consumed
            if a["a1"] is not None:
                checks["a1"] = (nchw(a["a1"]), z1)
                z1 = nchw(a["a1"])
            else:  # conv2 on the halo kernel: bn1 + ReLU applied in LDS, rounded to the compute dtype
                z1 = z1.to(a["y1"].dtype).double()
            checks["a2"] = (nchw(a["a2"]), z2)
            z2 = nchw(a["a2"])
        dm3 = D["b_dout"] * (out > 0)
        checks["dy3"] = (D["b_dy3"], bn_bwd(dm3, y3, st[".bn3"][0], st[".bn3"][1], gm[".bn3"]))
        w3 = P[pf + ".conv3.weight"].double().cpu()
        mask2 = (y2 * col(st[".bn2"][2]) + col(st[".bn2"][3])) > 0
        checks["dz2"] = (D["b_dz2"], torch.nn.grad.conv2d_input(y2.shape, w3, D["b_dy3"]) * mask2)
        checks["dy2"] = (D["b_dy2"], bn_bwd(D["b_dz2"] * mask2, y2, st[".bn2"][0], st[".bn2"][1], gm[".bn2"]))
        w2 = P[pf + ".conv2.weight"].double().cpu()
        mask1 = (y1 * col(st[".bn1"][2]) + col(st[".bn1"][3])) > 0
        checks["dz1"] = (D["b_dz1"], torch.nn.grad.conv2d_input(y1.shape, w2, D["b_dy2"], stride=b.stride, padding=1)
                         * mask1)
        checks["dy1"] = (D["b_dy1"], bn_bwd(D["b_dz1"] * mask1, y1, st[".bn1"][0], st[".bn1"][1], gm[".bn1"]))
        checks["dW3"] = (P[pf + ".conv3.weight"].grad, torch.nn.grad.conv2d_weight(z2, w3.shape, D["b_dy3"]))
        checks["dW2"] = (P[pf + ".conv2.weight"].grad,
                         torch.nn.grad.conv2d_weight(z1, w2.shape, D["b_dy2"], stride=b.stride, padding=1))
        # dW1 / the downsample dW: the block input h (the previous block's out, or the stem's max-pool
        # output) against dy1 / dyd. On the benched schedule the conv1 weight gradient stages dy1 =
        # ca*dm1 + cb*y1 + cc itself from dm1 (argus_conv_wgrad_apply); the captured dy1 is the same
        # formula stored by the dgrad's apply prologue, rounded alike.
        h_in = nchw(eng.act[idx - 1]["out"] if idx > 0 else eng.p0)
        w1 = P[pf + ".conv1.weight"]
        checks["dW1"] = (w1.grad, torch.nn.grad.conv2d_weight(h_in, w1.shape, D["b_dy1"]))
        if b.has_ds:
            wdp = P[pf + ".downsample.0.weight"]
            checks["dWd"] = (wdp.grad, torch.nn.grad.conv2d_weight(h_in, wdp.shape, nchw(debug["b_dyd." + pf]),
                                                                   stride=b.stride))
        if idx > 0:  # the previous block's dm3, from this block's conv1 (+ downsample) dgrad epilogue
            pb, pa = eng.blocks[idx - 1], eng.act[idx - 1]
            h = nchw(pa["out"])
            w1 = P[pf + ".conv1.weight"].double().cpu()
            v = torch.nn.grad.conv2d_input(h.shape, w1, D["b_dy1"])
            if b.has_ds:
                wd = P[pf + ".downsample.0.weight"].double().cpu()
                v = v + torch.nn.grad.conv2d_input(h.shape, wd, nchw(debug["b_dyd." + pf]), stride=b.stride)
            else:
                v = v + dm3
            checks["dout"] = (nchw(debug["b_dout." + pb.prefix]), v * (h > 0))
        for k, (got, want) in checks.items():
            r = rel_max(got, want)
            worst[k] = max(worst.get(k, 0.0), r)
            bar = tol_max[k] if isinstance(tol_max, dict) else tol_max
            assert r < bar, (pf, k, r)
    return worst
