"""Training-mode forward/backward of the policy-value net's convolutional part on
the device (csrc/gz_sgd.hip, include/gzero.h gz_sgd_*), as a torch autograd Function.

``train_forward(net, x)`` is ``PolicyValueNet.forward`` (neural_network.py:132-159)
in training mode with everything up to the heads' flattened conv outputs -- conv0,
BN0 + ReLU, the two residual blocks (neural_network.py:74-91), BatchNorm on batch
statistics, and the 1x1 policy / value convs -- on the HIP kernels: f16x3 MFMA
implicit-GEMM convolutions (forward, input and weight gradients), BatchNorm
statistics and backward in the conv epilogues, conv0 and the 1x1 convs in fp32.
In ``train_forward`` the FC heads (policy_fc, value_fc1/2) stay torch ops under
autograd; ``NetStep`` runs the whole step without autograd: the tower forward, the
FC heads + loss and their backward (gz_sgd_fc_loss) and the tower backward, the
gradients written into every parameter's ``.grad`` (views of one flat buffer, which
is also the data-parallel all-reduce bucket).  ``clip_grad_norm_`` and Adam of
``training.train_epoch`` (training.py:277-311) follow (gzero.optim.DeviceAdam).  The
BatchNorm running statistics and ``num_batches_tracked`` are updated as
``nn.BatchNorm2d.train()`` does.  There is no fallback: without the
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
    """The parameters in the Function's order: (gamma, beta) of BN 0..4, (weight, bias)
    of conv 1..4 (gz_sgd_net's arrays), then conv0, policy_conv, value_conv."""
    out = []
    for bn in _bns(net):
        out += [bn.weight, bn.bias]
    for cv in _convs(net):
        out += [cv.weight, cv.bias]
    for cv in (net.conv, net.policy_conv, net.value_conv):
        out += [cv.weight, cv.bias]
    return out


_HEADS = ("conv0", "policy", "value")


def _check_net(net):
    if len(net.residual_tower) != 2:
        raise ValueError("gz_sgd: the device tower has two residual blocks (neural_network.py:98)")
    bns = _bns(net)
    for bn in bns:
        if bn.momentum is None or not bn.affine:
            raise ValueError("gz_sgd: BatchNorm needs affine parameters and an exponential momentum")
        # gz_sgd_net carries one momentum and one eps (taken from the first BatchNorm)
        if bn.momentum != bns[0].momentum or bn.eps != bns[0].eps:
            raise ValueError("gz_sgd: every BatchNorm must have the same momentum and eps")
    for cv in _convs(net):
        if tuple(cv.weight.shape) != (128, 128, 3, 3) or cv.bias is None:
            raise ValueError("gz_sgd: residual convs must be 128 -> 128, 3x3, with bias")
    if (tuple(net.conv.weight.shape) != (128, 3, 3, 3) or tuple(net.policy_conv.weight.shape) != (2, 128, 1, 1)
            or tuple(net.value_conv.weight.shape) != (1, 128, 1, 1)):
        raise ValueError("gz_sgd: conv0 must be 3 -> 128 (3x3), policy_conv 128 -> 2 and value_conv 128 -> 1 (1x1)")


class _Tower(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, net, *params):
        lib = _lib.load()
        B = x.shape[0]
        if not 1 <= B <= _lib.GZ_SGD_MAX_BOARDS or tuple(x.shape[1:]) != (3, 15, 15):
            raise ValueError(f"gz_sgd: input of shape {tuple(x.shape)}")
        xc = x.detach().contiguous()
        pin = torch.empty((B, 450), dtype=torch.float32, device=x.device)
        vin = torch.empty((B, 225), dtype=torch.float32, device=x.device)
        ws = torch.empty(int(lib.gz_sgd_workspace_bytes(B)), dtype=torch.uint8, device=x.device)
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
        for i, name in enumerate(_HEADS):
            setattr(st, f"{name}_weight", params[18 + 2 * i].data_ptr())
            setattr(st, f"{name}_bias", params[19 + 2 * i].data_ptr())
        st.momentum = float(bns[0].momentum)
        st.eps = float(bns[0].eps)
        _lib.check(lib.gz_sgd_forward(ctypes.byref(st), B, _ptr(xc), _ptr(pin), _ptr(vin), _ptr(ws), _stream()),
                   "gz_sgd_forward")
        counts = [bn.num_batches_tracked for bn in bns if bn.track_running_stats]
        if counts:
            torch._foreach_add_(counts, 1)  # one launch for the five counters
        ctx.st, ctx.B, ctx.ws = st, B, ws
        ctx.keep = (xc, params)  # the forward's pointers stay valid for the backward
        return pin, vin

    @staticmethod
    def backward(ctx, dpin, dvin):
        lib = _lib.load()
        if ctx.keep is None:
            raise RuntimeError("gz_sgd: the device tower's saved state is released by its first backward; a second "
                               "backward through the same graph (retain_graph=True) is not supported")
        xc, params = ctx.keep
        dpin = dpin.contiguous() if dpin is not None else torch.zeros((ctx.B, 450), device=xc.device)
        dvin = dvin.contiguous() if dvin is not None else torch.zeros((ctx.B, 225), device=xc.device)
        grads = [torch.empty_like(p) for p in params]
        gr = _lib.SgdGrads()
        for i in range(5):
            gr.bn_weight[i] = grads[2 * i].data_ptr()
            gr.bn_bias[i] = grads[2 * i + 1].data_ptr()
        for i in range(4):
            gr.conv_weight[i] = grads[10 + 2 * i].data_ptr()
            gr.conv_bias[i] = grads[11 + 2 * i].data_ptr()
        for i, name in enumerate(_HEADS):
            setattr(gr, f"{name}_weight", grads[18 + 2 * i].data_ptr())
            setattr(gr, f"{name}_bias", grads[19 + 2 * i].data_ptr())
        _lib.check(lib.gz_sgd_backward(ctypes.byref(ctx.st), ctx.B, _ptr(xc), _ptr(dpin), _ptr(dvin),
                                       ctypes.byref(gr), _ptr(ctx.ws), _stream()), "gz_sgd_backward")
        ctx.keep = ctx.ws = None
        return (None, None, *grads)


def tower(net, x):
    """(policy_conv output flattened [B, 450], value_conv output flattened [B, 225]) of
    the planes x [B, 3, 15, 15]: conv0, BN0, both residual blocks, training mode, on
    the device."""
    _check_net(net)
    params = tower_params(net)
    for p in params:
        if not (p.is_cuda and p.dtype == torch.float32 and p.is_contiguous()):
            raise ValueError("gz_sgd: tower parameters must be contiguous float32 CUDA tensors")
    return _Tower.apply(x.float(), net, *params)


def train_forward(net, x):
    """(logits, value) of PolicyValueNet in training mode with the device convolutions."""
    pin, vin = tower(net, x)
    logits = net.policy_fc(pin)
    v = F.relu(net.value_fc1(vin))
    return logits, torch.tanh(net.value_fc2(v))


class NetStep:
    """One training step of PolicyValueNet (training.py:292-297: forward in training
    mode, CrossEntropy + MSE, backward) on the device without autograd:
    gz_sgd_forward -> gz_sgd_fc_loss -> gz_sgd_backward.  ``grads`` is one flat
    buffer; every parameter's ``.grad`` is a view of it, overwritten by each step (no
    zero_grad needed; gradients are never accumulated).  ``step(x, y, v, scale)``
    returns the batch loss (a device scalar, unscaled); ``scale`` multiplies every
    gradient (a data-parallel rank's share of the global batch)."""

    def __init__(self, net):
        _check_net(net)
        self.net = net
        self.lib = _lib.load()
        self.params = list(net.parameters())
        for p in self.params:
            if not (p.is_cuda and p.dtype == torch.float32 and p.is_contiguous()):
                raise ValueError("gz_sgd: parameters must be contiguous float32 CUDA tensors")
        dev = self.params[0].device
        self.grads = torch.zeros(sum(p.numel() for p in self.params), dtype=torch.float32, device=dev)
        off = 0
        self._views = []
        for p in self.params:
            p.grad = self.grads[off:off + p.numel()].view_as(p)
            self._views.append((p, p.grad))
            off += p.numel()
        tp = tower_params(net)
        bns = _bns(net)
        st, gr = _lib.SgdNet(), _lib.SgdGrads()
        for i, bn in enumerate(bns):
            st.bn_weight[i], st.bn_bias[i] = tp[2 * i].data_ptr(), tp[2 * i + 1].data_ptr()
            st.bn_running_mean[i] = bn.running_mean.data_ptr() if bn.track_running_stats else None
            st.bn_running_var[i] = bn.running_var.data_ptr() if bn.track_running_stats else None
            gr.bn_weight[i], gr.bn_bias[i] = tp[2 * i].grad.data_ptr(), tp[2 * i + 1].grad.data_ptr()
        for i in range(4):
            st.conv_weight[i], st.conv_bias[i] = tp[10 + 2 * i].data_ptr(), tp[11 + 2 * i].data_ptr()
            gr.conv_weight[i], gr.conv_bias[i] = tp[10 + 2 * i].grad.data_ptr(), tp[11 + 2 * i].grad.data_ptr()
        for i, name in enumerate(_HEADS):
            setattr(st, f"{name}_weight", tp[18 + 2 * i].data_ptr())
            setattr(st, f"{name}_bias", tp[19 + 2 * i].data_ptr())
            setattr(gr, f"{name}_weight", tp[18 + 2 * i].grad.data_ptr())
            setattr(gr, f"{name}_bias", tp[19 + 2 * i].grad.data_ptr())
        st.momentum = float(bns[0].momentum)
        st.eps = float(bns[0].eps)
        fcs = (net.policy_fc.weight, net.policy_fc.bias, net.value_fc1.weight, net.value_fc1.bias,
               net.value_fc2.weight, net.value_fc2.bias)
        if (tuple(fcs[0].shape) != (225, 450) or tuple(fcs[2].shape) != (64, 225)
                or tuple(fcs[4].shape) != (1, 64)):
            raise ValueError("gz_sgd: FC heads must be policy_fc 450 -> 225, value_fc1 225 -> 64, value_fc2 64 -> 1")
        self.fc = _lib.SgdFc(*[t.data_ptr() for t in fcs])
        self.fcg = _lib.SgdFc(*[t.grad.data_ptr() for t in fcs])
        self.st, self.gr = st, gr
        self.counts = [bn.num_batches_tracked for bn in bns if bn.track_running_stats]
        self.loss = torch.zeros(3, dtype=torch.float32, device=dev)
        self._bufs = {}

    def _buffers(self, B, dev):
        b = self._bufs.get(B)
        if b is None:
            f32 = dict(dtype=torch.float32, device=dev)
            b = (torch.empty(int(self.lib.gz_sgd_workspace_bytes(B)), dtype=torch.uint8, device=dev),
                 torch.empty(int(self.lib.gz_sgd_fc_workspace_bytes(B)), dtype=torch.uint8, device=dev),
                 torch.empty((B, 450), **f32), torch.empty((B, 225), **f32),
                 torch.empty((B, 450), **f32), torch.empty((B, 225), **f32))
            self._bufs[B] = b
        return b

    def _bind(self):
        # the kernels write into the flat buffer: put the views back if something (a
        # zero_grad(set_to_none=True)) replaced a parameter's .grad
        for p, g in self._views:
            if p.grad is not g:
                p.grad = g

    def zero(self):
        self._bind()
        self.grads.zero_()

    def step(self, x, y, v, scale=1.0):
        B = int(x.shape[0])
        if not 1 <= B <= _lib.GZ_SGD_MAX_BOARDS or tuple(x.shape[1:]) != (3, 15, 15):
            raise ValueError(f"gz_sgd: input of shape {tuple(x.shape)}")
        xc = x.detach().float().contiguous()
        yc = y.detach().to(torch.int64).contiguous()
        vc = v.detach().float().reshape(B).contiguous()
        ws, fws, pin, vin, dpin, dvin = self._buffers(B, xc.device)
        self._bind()
        s = _stream()
        _lib.check(self.lib.gz_sgd_forward(ctypes.byref(self.st), B, _ptr(xc), _ptr(pin), _ptr(vin), _ptr(ws), s),
                   "gz_sgd_forward")
        if self.counts:
            torch._foreach_add_(self.counts, 1)
        _lib.check(self.lib.gz_sgd_fc_loss(ctypes.byref(self.fc), B, _ptr(pin), _ptr(vin), _ptr(yc), _ptr(vc),
                                           float(scale), _ptr(dpin), _ptr(dvin), ctypes.byref(self.fcg),
                                           _ptr(self.loss), _ptr(fws), s), "gz_sgd_fc_loss")
        _lib.check(self.lib.gz_sgd_backward(ctypes.byref(self.st), B, _ptr(xc), _ptr(dpin), _ptr(dvin),
                                            ctypes.byref(self.gr), _ptr(ws), s), "gz_sgd_backward")
        # a copy: the loss buffer is overwritten by the next step (a label outside
        # [0, 225) makes it NaN, and every gradient with it)
        return self.loss[0].clone()
