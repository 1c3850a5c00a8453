"""The training step's device convolutions (csrc/gz_sgd.hip via gzero.sgd.train_forward:
conv0, the residual tower and the heads' 1x1 convs)
against torch autograd of the same PolicyValueNet in float64 on the CPU (the
reference's training.py:277-311 step: forward in train mode, CE + MSE loss,
backward), on identical weights and boards.

The float64 reference takes its ReLU masks from the device forward (the saved
activations, gz_sgd_saved): a pre-activation within ~1e-7 of zero can fall on
either side in any fp32 computation, and one such element moves a BatchNorm-bias
gradient, a sum with heavy cancellation, by up to ~1e-3 (measured: one flip in
3.7 M elements at |z| = 3e-7 carried all of a 1e-3 error; torch's own fp32 path
flips too).  With the masks matched the comparison sees the arithmetic only.

Tolerances, stated here: logits / value within 2e-5 (absolute, |logits| ~ 1),
the loss within 1e-6 relative, every parameter gradient within 1e-4 of the
float64 gradient's norm (relative Frobenius error; measured 1e-6 on the tower's
parameters, 6e-5 on the value head's one-element bias, a sum over the batch with
cancellation), every BatchNorm running
statistic within 1e-5, and at each of the five ReLUs at most 1e-5 of the
activations on the other side of zero than float64's own pre-activation (with the
device's masks upstream), each such element within 1e-5 of zero.  The biases of the convs that feed a BatchNorm have a zero
gradient (the batch mean cancels them); theirs must stay below 1e-6 of the
largest gradient norm.  The training-loop tests (test_gpu_train.py) run the same
kernels through DeviceTrainer against the reference's recorded losses (3e-3).
"""
import ctypes
import copy

import numpy as np
import pytest
import torch
import torch.nn as nn

from conftest import SEED

pytestmark = pytest.mark.gpu


def _net(seed=3, scale=1.0):
    from gzero import weights
    net = weights.PolicyValueNet()
    sd = weights.init_state_dict(seed)
    if scale != 1.0:
        for k in sd:
            if "conv" in k and k.endswith("weight"):
                sd[k] = sd[k] * scale
    net.load_state_dict(sd)
    return net


def _batch(B, seed):
    rng = np.random.default_rng(seed)
    cells = rng.choice(np.array([0, 0, 0, 1, 2], np.int8), size=(B, 225))
    x = np.stack([cells == 1, cells == 2, cells == 0], 1).reshape(B, 3, 15, 15).astype(np.float32)
    y = rng.integers(0, 225, B)
    v = rng.uniform(-1, 1, (B, 1)).astype(np.float32)
    return torch.from_numpy(x), torch.from_numpy(y), torch.from_numpy(v)


def _saved_masks(store):
    """Wrap the device Function's forward: after it runs, copy its saved activations
    (a0, h1, a1, h2) and its output a2 as float64 NCHW masks (> 0) into store."""
    from gzero import _lib, sgd
    orig = sgd._Tower.forward

    def fwd(ctx, x, net, *params):
        out = orig(ctx, x, net, *params)
        L = _lib.load()
        acts = []
        for i in (0, 1, 2, 3, 8):  # a0, h1, a1, h2 and the tower output a2
            t = torch.empty((ctx.B, 15, 15, 128), dtype=torch.float32, device="cuda")
            _lib.check(L.gz_sgd_saved(ctypes.c_void_p(ctx.ws.data_ptr()), ctx.B, i, ctypes.c_void_p(t.data_ptr()),
                                      ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)), "gz_sgd_saved")
            acts.append(t)
        store["masks"] = [(a > 0).permute(0, 3, 1, 2).double().cpu() for a in acts]
        return out
    return orig, fwd


def _masked_forward(net, x, m, pre=None):
    """PolicyValueNet.forward in float64 with relu(z) = z * m (the device's masks);
    pre: a list that receives the five pre-activations z (each computed with the
    device's masks upstream)."""
    def relu(z, k):
        if pre is not None:
            pre.append(z.detach())
        return z * m[k]
    a = relu(net.bn(net.conv(x)), 0)
    b0, b1 = net.residual_tower
    h = relu(b0.bn1(b0.conv1(a)), 1)
    a = relu(b0.bn2(b0.conv2(h)) + a, 2)
    h = relu(b1.bn1(b1.conv1(a)), 3)
    a = relu(b1.bn2(b1.conv2(h)) + a, 4)
    logits = net.policy_fc(torch.flatten(net.policy_conv(a), 1))
    v = torch.relu(net.value_fc1(torch.flatten(net.value_conv(a), 1)))
    return logits, torch.tanh(net.value_fc2(v))


def _step(net, fwd, x, y, v, loss_scale=1.0):
    net.train()
    net.zero_grad(set_to_none=True)
    lg, val = fwd(x)
    loss = nn.CrossEntropyLoss()(lg, y) + nn.MSELoss()(val, v.to(val.dtype))
    (loss * loss_scale).backward()
    grads = {k: p.grad.detach().double().cpu() for k, p in net.named_parameters()}
    bufs = {k: b.detach().double().cpu() for k, b in net.named_buffers()}
    return lg.detach().double().cpu(), val.detach().double().cpu(), float(loss), grads, bufs


def _compare(B, seed, scale=1.0, loss_scale=1.0, gtol=1e-4):
    from gzero import sgd
    net = _net(seed, scale)
    x, y, v = _batch(B, seed + 100)
    store = {}
    orig, spy = _saved_masks(store)
    sgd._Tower.forward = staticmethod(spy)
    try:
        dev_net = copy.deepcopy(net).cuda()
        got = _step(dev_net, lambda t: sgd.train_forward(dev_net, t), x.cuda(), y.cuda(), v.cuda(), loss_scale)
    finally:
        sgd._Tower.forward = staticmethod(orig)
    ref_net = copy.deepcopy(net).double()
    ref = _step(ref_net, lambda t: _masked_forward(ref_net, t, store["masks"]), x.double(), y, v.double(),
                loss_scale)
    # at each of the five ReLUs, the activations the device put on the other side of
    # zero than float64's own pre-activation (computed with the device's masks
    # upstream, so a flip is counted at the layer where it happens): at most 1e-5 of
    # the elements per layer, and only near-zero ones (|z| <= 1e-5)
    pre = []
    free = copy.deepcopy(net).double().train()
    with torch.no_grad():
        _masked_forward(free, x.double(), store["masks"], pre)
    flips, zmax = [], 0.0
    for z, m in zip(pre, store["masks"]):
        bad = (z > 0).double() != m
        flips.append(int(bad.sum()))
        if flips[-1]:
            zmax = max(zmax, float(z[bad].abs().max()))
        assert flips[-1] <= 1e-5 * z.numel(), (len(flips) - 1, flips[-1], z.numel())
    assert zmax <= 1e-5, zmax
    assert (got[0] - ref[0]).abs().max() < 2e-5 * max(1.0, float(ref[0].abs().max()))
    assert (got[1] - ref[1]).abs().max() < 2e-5
    assert abs(got[2] - ref[2]) <= 1e-6 * abs(ref[2])
    worst = {}
    top = max(float(g.norm()) for g in ref[3].values())
    for k, g in ref[3].items():
        if float(g.norm()) < 1e-9 * top:  # a bias in front of a BatchNorm
            assert float(got[3][k].norm()) < 1e-6 * top, k
            continue
        worst[k] = float((got[3][k] - g).norm()) / float(g.norm())
    for k, b in ref[4].items():
        assert torch.allclose(got[4][k], b, rtol=1e-5, atol=1e-6), k
    bad = {k: e for k, e in worst.items() if e > gtol}
    print("max rel grad error %.2e (%s), ReLU mask flips vs float64 per layer: %s, max |z| flipped %.2e" %
          (max(worst.values()), max(worst, key=worst.get), flips, zmax))
    assert not bad, bad


@pytest.mark.parametrize("B", [128, 7, 1])
def test_sgd_tower_vs_float64(B):
    """Batch 128 (a training step), a 7-board remainder batch and a single board."""
    _compare(B, SEED + B)


def test_sgd_tower_loss_scaled():
    """Gradients 1e-6 and 1e4 times larger: the input-gradient GEMM's power-of-two
    operand scaling keeps the same relative accuracy."""
    _compare(32, SEED + 5, loss_scale=1e-6)
    _compare(32, SEED + 6, loss_scale=1e4)


@pytest.mark.parametrize("scale", [0.1, 3.0])
def test_sgd_tower_scaled_weights(scale):
    """Conv weights x0.1 / x3 (BatchNorm renormalises; gradients through it grow / shrink)."""
    _compare(24, SEED + 9, scale=scale)


def test_sgd_tower_two_steps_match_torch_trainer():
    """Three Adam steps of DeviceTrainer (native tower) vs the same trainer on torch's
    GPU convolutions (native=False): the losses (each after the previous steps'
    updates, so ReLU-boundary flips of either path feed in) within 1e-3 and the
    BatchNorm running statistics within 1e-2 (Adam's first steps move weights whose
    gradient is rounding noise by +-lr either way; the statistics follow).
    (Parameters are not compared element-wise: Adam's first steps move weights whose
    gradient is rounding noise by +-lr either way.)"""
    from gzero.train import DeviceTrainer
    nets = [_net(SEED), _net(SEED)]
    x, y, v = _batch(128, SEED + 1)
    losses = []
    for native, net in zip((True, False), nets):
        tr = DeviceTrainer(net, native=native)
        ls = []
        for _ in range(3):
            if native:  # gzero.sgd.NetStep: tower, FC heads + loss and their backward on the device
                loss = tr.step_fn.step(x.cuda(), y.cuda(), v.cuda())
            else:
                tr.net.train()
                tr.optimizer.zero_grad()
                lg, val = tr._forward(x.cuda())
                loss = nn.CrossEntropyLoss()(lg, y.cuda()) + nn.MSELoss()(val, v.cuda())
                loss.backward()
            tr.clip_and_step()  # (grad_clip 0.8: DeviceAdam on the native trainer, torch's on the other)
            ls.append(float(loss))
        losses.append(ls)
    np.testing.assert_allclose(losses[0], losses[1], rtol=1e-3)
    for (k, a), (_, b) in zip(nets[0].named_buffers(), nets[1].named_buffers()):
        assert torch.allclose(a.float(), b.float(), rtol=1e-2, atol=1e-2), k



@pytest.mark.parametrize("B,scale", [(128, 1.0), (7, 0.25), (1, 1.0)])
def test_sgd_fc_loss_vs_float64(B, scale):
    """gz_sgd_fc_loss (the FC heads, CrossEntropy + MSE and their backward) against
    torch autograd in float64 on the same pin / vin: the loss within 1e-6 relative,
    dL/dpin, dL/dvin and the six FC gradients within 1e-5 of the float64 gradient's
    norm (relative Frobenius error), all scaled by `scale` except the loss."""
    import ctypes
    from gzero import _lib
    L = _lib.load()
    torch.manual_seed(SEED + B)
    net = _net(SEED + 3).cuda()
    pin = torch.randn(B, 450, device="cuda") * 0.5
    vin = torch.randn(B, 225, device="cuda") * 0.5
    y = torch.randint(0, 225, (B,), device="cuda")
    v = torch.rand(B, device="cuda") * 2 - 1
    fcs = [net.policy_fc.weight, net.policy_fc.bias, net.value_fc1.weight, net.value_fc1.bias,
           net.value_fc2.weight, net.value_fc2.bias]
    grads = [torch.full_like(t, float("nan")) for t in fcs]
    dpin, dvin = torch.empty_like(pin), torch.empty_like(vin)
    loss = torch.empty(3, device="cuda")
    ws = torch.empty(int(L.gz_sgd_fc_workspace_bytes(B)), dtype=torch.uint8, device="cuda")
    ptr = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    fc, fcg = _lib.SgdFc(*[t.data_ptr() for t in fcs]), _lib.SgdFc(*[t.data_ptr() for t in grads])
    _lib.check(L.gz_sgd_fc_loss(ctypes.byref(fc), B, ptr(pin), ptr(vin), ptr(y), ptr(v), scale, ptr(dpin),
                                ptr(dvin), ctypes.byref(fcg), ptr(loss), ptr(ws),
                                ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)), "gz_sgd_fc_loss")
    torch.cuda.synchronize()
    ref = [t.detach().double().cpu().requires_grad_() for t in fcs]
    p64 = pin.double().cpu().requires_grad_()
    v64 = vin.double().cpu().requires_grad_()
    lg = p64 @ ref[0].T + ref[1]
    val = torch.tanh(torch.relu(v64 @ ref[2].T + ref[3]) @ ref[4].T + ref[5])
    ce = nn.CrossEntropyLoss()(lg, y.cpu())
    mse = nn.MSELoss()(val, v.double().cpu().view(B, 1))
    ((ce + mse) * scale).backward()
    got = loss.double().cpu()
    for a, b in ((got[0], ce + mse), (got[1], ce), (got[2], mse)):
        assert abs(float(a) - float(b)) <= 1e-6 * max(1.0, abs(float(b))), (float(a), float(b))
    pairs = [(dpin, p64.grad), (dvin, v64.grad)] + list(zip(grads, [r.grad for r in ref]))
    for k, (a, b) in enumerate(pairs):
        err = float((a.double().cpu() - b).norm()) / max(float(b.norm()), 1e-30)
        assert err < 1e-5, (k, err)


def test_netstep_matches_the_autograd_path():
    """gzero.sgd.NetStep (no autograd: tower, FC heads + loss, backward on the device)
    against sgd.train_forward + torch's FC heads and loss under autograd, same weights
    and batch: the same tower kernels, so every gradient within 1e-5 (relative
    Frobenius) and the loss within 1e-6 relative; the BatchNorm running statistics
    and num_batches_tracked identical."""
    from gzero import sgd
    x, y, v = _batch(128, SEED + 21)
    nets = [_net(SEED + 4).cuda(), _net(SEED + 4).cuda()]
    step = sgd.NetStep(nets[0])
    nets[0].train()
    l0 = float(step.step(x.cuda(), y.cuda(), v.cuda()))
    nets[1].train()
    lg, val = sgd.train_forward(nets[1], x.cuda())
    loss = nn.CrossEntropyLoss()(lg, y.cuda()) + nn.MSELoss()(val, v.cuda())
    loss.backward()
    assert abs(l0 - float(loss)) <= 1e-6 * abs(float(loss))
    for (k, a), (_, b) in zip(nets[0].named_parameters(), nets[1].named_parameters()):
        err = float((a.grad - b.grad).norm()) / max(float(b.grad.norm()), 1e-30)
        top = max(float(p.grad.norm()) for p in nets[1].parameters())
        assert err < 1e-5 or float((a.grad - b.grad).norm()) < 1e-6 * top, (k, err)
    for (k, a), (_, b) in zip(nets[0].named_buffers(), nets[1].named_buffers()):
        assert torch.equal(a, b), k


def test_device_adam_matches_torch_adam_with_clipping():
    """gzero.optim.DeviceAdam.step(max_norm) against clip_grad_norm_ + torch.optim.Adam
    (the reference's training.py:303-304 pair) on the policy-value net's parameter
    shapes: 6 steps with fresh random gradients (one step unclipped: norm below
    max_norm), a learning-rate change half way (StepLR's), weight decay 1e-5.  The
    parameters within 1e-6 (relative, max-norm), the pre-clip norm within 1e-6."""
    from gzero.optim import DeviceAdam
    net = _net(SEED).cuda()
    ref = [p.detach().clone() for p in net.parameters()]
    mine = [p.detach().clone() for p in net.parameters()]
    opt_ref = torch.optim.Adam(ref, lr=8e-4, weight_decay=1e-5)
    opt = DeviceAdam(mine, lr=8e-4, weight_decay=1e-5)
    gen = torch.Generator(device="cuda").manual_seed(7)
    for k in range(6):
        scale = 1e-4 if k == 2 else 1.0  # step 2: total norm < max_norm, no clipping
        for a, b in zip(ref, mine):
            g = torch.randn(a.shape, generator=gen, device="cuda") * scale
            a.grad, b.grad = g.clone(), g.clone()
        if k == 3:
            for o in (opt_ref, opt):
                o.param_groups[0]["lr"] = 8e-4 * 0.85
        n_ref = float(nn.utils.clip_grad_norm_(ref, 0.8))
        opt_ref.step()
        v0 = [p._version for p in mine]
        opt.step(max_norm=0.8)
        # an update through raw pointers still bumps the version counters (the model's
        # packed-weight cache keys on them)
        assert all(p._version > v for p, v in zip(mine, v0))
        assert abs(float(opt.last_norm) - n_ref) <= 1e-6 * n_ref
        for a, b in zip(ref, mine):
            assert torch.allclose(a.grad, b.grad, rtol=1e-6, atol=0), k  # clipped in place
            err = float((a - b).abs().max()) / max(float(a.abs().max()), 1e-12)
            assert err < 1e-6, (k, err)
