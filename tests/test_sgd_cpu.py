"""Host side of the device training step (gzero/sgd.py, include/gzero.h gz_sgd_*),
without a GPU: the parameter order handed to gz_sgd_net, argument errors and the
workspace size (no compute call is made here)."""
import ctypes

import pytest
import torch

from gzero import _lib


def test_tower_params_follow_gz_sgd_net_order():
    """(gamma, beta) of bn, tower.0.bn1, tower.0.bn2, tower.1.bn1, tower.1.bn2, then
    (weight, bias) of tower.0.conv1, tower.0.conv2, tower.1.conv1, tower.1.conv2, conv0,
    policy_conv and value_conv."""
    from gzero import sgd, weights
    net = weights.PolicyValueNet()
    names = {id(p): k for k, p in net.named_parameters()}
    got = [names[id(p)] for p in sgd.tower_params(net)]
    bns = ["bn", "residual_tower.0.bn1", "residual_tower.0.bn2", "residual_tower.1.bn1", "residual_tower.1.bn2"]
    convs = ["residual_tower.0.conv1", "residual_tower.0.conv2", "residual_tower.1.conv1", "residual_tower.1.conv2"]
    want = [f"{m}.{p}" for m in bns + convs + ["conv", "policy_conv", "value_conv"] for p in ("weight", "bias")]
    assert got == want


def test_tower_rejects_other_architectures():
    from gzero import sgd, weights
    net = weights.PolicyValueNet(num_residual=3)
    with pytest.raises(ValueError, match="two residual blocks"):
        sgd.tower(net, torch.zeros(1, 3, 15, 15))
    net = weights.PolicyValueNet()
    net.bn.momentum = None
    with pytest.raises(ValueError, match="momentum"):
        sgd.tower(net, torch.zeros(1, 3, 15, 15))
    net = weights.PolicyValueNet()
    with pytest.raises(ValueError, match="CUDA"):  # CPU parameters: no silent fallback
        sgd.tower(net, torch.zeros(1, 3, 15, 15))


def test_gz_sgd_argument_errors_and_workspace():
    L = _lib.load()
    assert ctypes.sizeof(_lib.SgdNet) == 4 * 5 * 8 + 2 * 4 * 8 + 8 + 6 * 8
    assert ctypes.sizeof(_lib.SgdGrads) == 2 * 5 * 8 + 2 * 4 * 8 + 6 * 8
    assert L.gz_sgd_workspace_bytes(0) == 0
    w1, w128 = L.gz_sgd_workspace_bytes(1), L.gz_sgd_workspace_bytes(128)
    R = 128 * 225 * 128 * 4
    assert w128 > 16 * R and w1 < w128  # 16 activation-sized buffers at 128 boards
    net = _lib.SgdNet()
    rc = L.gz_sgd_forward(ctypes.byref(net), 4, None, None, None, None, None)
    assert rc == -1 and b"gz_sgd" in L.gz_last_error()
    assert L.gz_sgd_forward(None, 4, None, None, None, None, None) == -1
    ws = ctypes.c_void_p(1)  # never dereferenced: the parameters are checked first
    assert L.gz_sgd_forward(ctypes.byref(net), 0, None, None, None, ws, None) == -1
    assert L.gz_sgd_backward(ctypes.byref(net), 70000, None, None, None, None, ws, None) == -1
    assert L.gz_sgd_saved(ws, 4, 10, None, None) == -1


def test_gz_adam_argument_errors():
    L = _lib.load()
    assert L.gz_adam_workspace_bytes() >= 8
    t = (_lib.AdamTensor * 1)()
    ws = ctypes.c_void_p(1)  # never dereferenced: the arguments are checked first
    args = (ctypes.c_float(1e-3), ctypes.c_float(0.9), ctypes.c_float(0.999), ctypes.c_float(1e-8),
            ctypes.c_float(0.0))
    assert L.gz_adam_step(t, 0, *args, 1, ctypes.c_float(0.0), None, ws, None) == -1
    assert L.gz_adam_step(t, _lib.GZ_ADAM_MAX_TENSORS + 1, *args, 1, ctypes.c_float(0.0), None, ws, None) == -1
    assert L.gz_adam_step(t, 1, *args, 0, ctypes.c_float(0.0), None, ws, None) == -1  # step counts from 1
    t[0].numel = 5  # null tensor pointers
    assert L.gz_adam_step(t, 1, *args, 1, ctypes.c_float(0.0), None, ws, None) == -1
    assert b"gz_adam_step" in L.gz_last_error()
