"""Training-mode forward/backward of the policy-value net's residual tower on the
device (csrc/gz_sgd.hip, include/gzero.h gz_sgd_*), as a torch autograd Function.

``train_forward(net, x)`` is ``PolicyValueNet.forward`` (neural_network.py:132-159)
in training mode with the tower -- BN0 + ReLU and the two residual blocks
(neural_network.py:74-91), BatchNorm on batch statistics -- replaced by the HIP
kernels: f16x3 MFMA implicit-GEMM convolutions (forward and input gradient), fp32
MFMA weight gradients, BatchNorm statistics and backward in the conv epilogues.
conv0 (3 -> 128 channels) and the policy / value heads stay torch ops; the loss,
``clip_grad_norm_`` and Adam of ``training.train_epoch`` (training.py:277-311) are
unchanged.  The BatchNorm running statistics and ``num_batches_tracked`` are
updated as ``nn.BatchNorm2d.train()`` does.  There is no fallback: without the
library this raises ``GzeroUnavailable``.
"""
import ctypes

import torch
import torch.nn.functional as F

from . import _lib


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else ctypes.c_void_p(None)


def _stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def _bns(net):
    return [net.bn] + [m for blk in net.residual_tower for m in (blk.bn1, blk.bn2)]


def _convs(net):
    return [m for blk in net.residual_tower for m in (blk.conv1, blk.conv2)]


def tower_params(net):
    """The tower's parameters in the Function's order: (gamma, beta) of BN 0..4, then
    (weight, bias) of conv 1..4 (gz_sgd_net's order)."""
    out = []
    for bn in _bns(net):
        out += [bn.weight, bn.bias]
    for cv in _convs(net):
        out += [cv.weight, cv.bias]
    return out


def _check_net(net):
    if len(net.residual_tower) != 2:
        raise ValueError("gz_sgd: the device tower has two residual blocks (neural_network.py:98)")
    for bn in _bns(net):
        if bn.momentum is None or not bn.affine:
            raise ValueError("gz_sgd: BatchNorm needs affine parameters and an exponential momentum")
    for cv in _convs(net):
        if tuple(cv.weight.shape) != (128, 128, 3, 3) or cv.bias is None:
            raise ValueError("gz_sgd: residual convs must be 128 -> 128, 3x3, with bias")


class _Tower(torch.autograd.Function):
    @staticmethod
    def forward(ctx, y0, net, *params):
        lib = _lib.load()
        B = y0.shape[0]
        if not 1 <= B <= _lib.GZ_SGD_MAX_BOARDS:
            raise ValueError(f"gz_sgd: batch of {B} boards")
        y0n = y0.detach().permute(0, 2, 3, 1).contiguous()
        out = torch.empty_like(y0n)
        ws = torch.empty(int(lib.gz_sgd_workspace_bytes(B)), dtype=torch.uint8, device=y0.device)
        st = _lib.SgdNet()
        bns = _bns(net)
        for i, bn in enumerate(bns):
            st.bn_weight[i] = params[2 * i].data_ptr()
            st.bn_bias[i] = params[2 * i + 1].data_ptr()
            st.bn_running_mean[i] = bn.running_mean.data_ptr() if bn.track_running_stats else None
            st.bn_running_var[i] = bn.running_var.data_ptr() if bn.track_running_stats else None
        for i in range(4):
            st.conv_weight[i] = params[10 + 2 * i].data_ptr()
            st.conv_bias[i] = params[11 + 2 * i].data_ptr()
        st.momentum = float(bns[0].momentum)
        st.eps = float(bns[0].eps)
        _lib.check(lib.gz_sgd_forward(ctypes.byref(st), B, _ptr(y0n), _ptr(out), _ptr(ws), _stream()),
                   "gz_sgd_forward")
        for bn in bns:
            if bn.track_running_stats:
                bn.num_batches_tracked.add_(1)
        ctx.st, ctx.B, ctx.ws = st, B, ws
        ctx.keep = (y0n, out, params)  # the forward's pointers stay valid for the backward
        return out.permute(0, 3, 1, 2)

    @staticmethod
    def backward(ctx, gout):
        lib = _lib.load()
        y0n, out, params = ctx.keep
        dout = gout.permute(0, 2, 3, 1).contiguous()
        dy0 = torch.empty_like(y0n)
        grads = [torch.empty_like(p) for p in params]
        gr = _lib.SgdGrads()
        for i in range(5):
            gr.bn_weight[i] = grads[2 * i].data_ptr()
            gr.bn_bias[i] = grads[2 * i + 1].data_ptr()
        for i in range(4):
            gr.conv_weight[i] = grads[10 + 2 * i].data_ptr()
            gr.conv_bias[i] = grads[11 + 2 * i].data_ptr()
        _lib.check(lib.gz_sgd_backward(ctypes.byref(ctx.st), ctx.B, _ptr(y0n), _ptr(out), _ptr(dout), _ptr(dy0),
                                       ctypes.byref(gr), _ptr(ctx.ws), _stream()), "gz_sgd_backward")
        ctx.keep = ctx.ws = None
        return (dy0.permute(0, 3, 1, 2), None, *grads)


def tower(net, y0):
    """relu(BN0(y0)) through both residual blocks, training mode, on the device."""
    _check_net(net)
    params = tower_params(net)
    for p in params:
        if not (p.is_cuda and p.dtype == torch.float32 and p.is_contiguous()):
            raise ValueError("gz_sgd: tower parameters must be contiguous float32 CUDA tensors")
    return _Tower.apply(y0.float(), net, *params)


def train_forward(net, x):
    """(logits, value) of PolicyValueNet in training mode with the device tower."""
    h = tower(net, net.conv(x))
    logits = net.policy_fc(torch.flatten(net.policy_conv(h), 1))
    v = F.relu(net.value_fc1(torch.flatten(net.value_conv(h), 1)))
    return logits, torch.tanh(net.value_fc2(v))
