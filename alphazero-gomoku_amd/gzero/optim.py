"""The optimiser step of training.train_epoch (training.py:303-304) on the device:
``clip_grad_norm_`` followed by ``torch.optim.Adam`` in two HIP launches
(csrc/gz_train.hip, include/gzero.h gz_adam_step) instead of torch's multi-tensor
passes, whose 64-K-element chunks put a 0.75 M-parameter net on a dozen workgroups.

``DeviceAdam`` is a torch.optim.Optimizer (so StepLR and ``param_groups`` work as with
torch's Adam: L2 weight decay, bias-corrected moments); ``step(max_norm=c)`` clips the
gradients first, in place, by min(1, c / (||g||_2 + 1e-6)) over every parameter with a
gradient, as ``clip_grad_norm_(params, c)`` does.  There is no fallback: without the
library this raises ``GzeroUnavailable``.
"""
import ctypes

import torch
from torch.autograd.graph import increment_version

from . import _lib


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr())


class DeviceAdam(torch.optim.Optimizer):
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0):
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay))
        self._lib = _lib.load()
        for g in self.param_groups:
            for p in g["params"]:
                if not (p.is_cuda and p.dtype == torch.float32 and p.is_contiguous()):
                    raise ValueError("DeviceAdam: parameters must be contiguous float32 CUDA tensors")
        dev = self.param_groups[0]["params"][0].device
        self._ws = torch.empty(int(self._lib.gz_adam_workspace_bytes()), dtype=torch.uint8, device=dev)
        self.last_norm = torch.zeros(1, dtype=torch.float32, device=dev)
        self._tables = {}  # per group: (the tensors' data pointers, the ctypes table built from them)

    @torch.no_grad()
    def step(self, closure=None, max_norm=None):
        """One Adam step over every parameter with a gradient (after clipping them to
        max_norm when given).  Returns closure()'s loss, like torch's optimisers."""
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        live = [(g, p) for g in self.param_groups for p in g["params"] if p.grad is not None]
        if not live:
            return loss
        if max_norm is not None and len(self.param_groups) > 1:
            raise ValueError("DeviceAdam: clipping spans one parameter group")
        for group in self.param_groups:
            ps = [p for p in group["params"] if p.grad is not None]
            if not ps:
                continue
            if len(ps) > _lib.GZ_ADAM_MAX_TENSORS:
                raise ValueError(f"DeviceAdam: at most {_lib.GZ_ADAM_MAX_TENSORS} tensors per group")
            steps = set()
            for p in ps:
                st = self.state[p]
                if not st:
                    st["step"] = 0
                    st["exp_avg"] = torch.zeros_like(p)
                    st["exp_avg_sq"] = torch.zeros_like(p)
                steps.add(st["step"])
                if p.grad.dtype != torch.float32 or not p.grad.is_contiguous() or p.grad.is_sparse:
                    raise ValueError("DeviceAdam: gradients must be dense contiguous float32")
            if len(steps) != 1:
                raise ValueError("DeviceAdam: the parameters of a group must share their step count")
            step = steps.pop() + 1
            # the table is rebuilt only when a tensor moved (a trainer that keeps its
            # gradients in one buffer passes the same pointers every step)
            key = tuple((p.data_ptr(), p.grad.data_ptr(), self.state[p]["exp_avg"].data_ptr(),
                         self.state[p]["exp_avg_sq"].data_ptr(), p.numel()) for p in ps)
            cached = self._tables.get(id(group))
            if cached is not None and cached[0] == key:
                table = cached[1]
            else:
                table = (_lib.AdamTensor * len(ps))(*[_lib.AdamTensor(*k) for k in key])
                self._tables[id(group)] = (key, table)
            b1, b2 = group["betas"]
            _lib.check(self._lib.gz_adam_step(table, len(ps), float(group["lr"]), float(b1), float(b2),
                                              float(group["eps"]), float(group["weight_decay"]), step,
                                              float(max_norm) if max_norm is not None else 0.0,
                                              _ptr(self.last_norm), _ptr(self._ws),
                                              ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)),
                       "gz_adam_step")
            for p in ps:
                self.state[p]["step"] = step
            # the kernel wrote the parameters through raw pointers: bump their version
            # counters as an in-place torch op would, so that caches keyed on them (the
            # model's packed inference weights, neural_network.GomokuModel) see the update
            increment_version(ps)
        return loss
