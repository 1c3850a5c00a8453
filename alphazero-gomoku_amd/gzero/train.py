"""Device-resident training step: the replay stays on
the GPU as 80-byte records, batches are materialised by the gz_dataset_gather
kernel (augmentation included), and the policy-value SGD step runs data-parallel
with one RCCL all-reduce of the flat gradient per step.

Semantics follow the reference's training loop:

* ``DeviceDataset`` = ``GomokuSelfPlayDataset`` (training.py:104-134): every
  record, then the 8 symmetries of ``random.sample(range(n), max(1, int(n *
  augment_ratio)))`` drawn from the same ``random`` module, sample order
  identical (originals, then 8 per chosen record in (k_rot, flip) order).
* ``loader_order`` = the index order of ``DataLoader(ds, batch_size,
  shuffle)`` (training.py:453-454), produced by torch's own sampler over an index
  set so the torch RNG is consumed exactly as the reference's loader does.
* ``DeviceTrainer.train_epoch`` / ``validate_epoch`` = training.py:277-337:
  CrossEntropy(logits, move) + MSE(value, z), ``clip_grad_norm_`` at
  ``grad_clip``, Adam(lr 8e-4, wd 1e-5) and StepLR(2, 0.85) as in main()
  (training.py:387-388,379-381); the loss is the mean of per-batch float
  losses (accumulated on the device in float64, one host sync per epoch).

Data parallel (world size N): every rank holds the same dataset (records are
all-gathered at episode end, gzero.dist) and the same permutation; global batch
k is ``batch_size * N`` consecutive permutation entries and rank r trains on
its ``batch_size`` slice.  Each rank's loss is weighted by its share of the
global batch and the gradients are SUM-all-reduced, so the update is the
global-batch mean (BatchNorm statistics stay per rank, as in DDP).  N = 1 is the
reference's loop exactly.
"""
import ctypes
import random as _random

import numpy as np
import torch
import torch.nn as nn
import torch.distributed as dist
from torch.utils.data import DataLoader, Dataset

from . import _lib
from .boards import RECORD_DTYPE

SAMPLE_SHAPE = (3, 15, 15)


def _dev_ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


def _stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def records_to_device(records):
    """numpy RECORD_DTYPE array -> device uint8 tensor (80 B per record)."""
    raw = np.ascontiguousarray(records).view(np.uint8).reshape(-1)
    return torch.from_numpy(raw.copy()).to("cuda")


class DeviceDataset(Dataset):
    """GomokuSelfPlayDataset over device records (training.py:104-134)."""

    def __init__(self, records, use_augmentation=True, augment_ratio=0.5, fix_labels=False, rng=None,
                 n_records=None):
        if isinstance(records, torch.Tensor):
            self.d_records = records
            n = int(n_records if n_records is not None else records.numel() // RECORD_DTYPE.itemsize)
        else:
            records = np.asarray(records, RECORD_DTYPE)
            n = len(records)
            self.d_records = records_to_device(records)
        rng = _random if rng is None else rng
        sel = rng.sample(range(n), k=max(1, int(n * augment_ratio))) if (use_augmentation and n > 0) else []
        self.n = n
        self.m = len(sel)
        self.flags = _lib.GZ_AUG_FIX_LABELS if fix_labels else 0
        self.d_sel = torch.tensor(sel if sel else [0], dtype=torch.int32, device="cuda")

    def __len__(self):
        return self.n + 8 * self.m

    def check_ids(self, d_ids):
        check_ids(self, d_ids)

    def gather(self, d_ids, out=None, check=True):
        """Samples d_ids (device int64) -> (x [B,3,15,15] f32, y [B] int64, v [B,1] f32) on the device.
        ``check`` validates the ids first (one host sync; the trainer checks a whole
        epoch's ids once and passes False)."""
        if check:
            self.check_ids(d_ids)
        b = int(d_ids.numel())
        if out is None:
            out = (torch.empty((b,) + SAMPLE_SHAPE, dtype=torch.float32, device="cuda"),
                   torch.empty(b, dtype=torch.int64, device="cuda"),
                   torch.empty((b, 1), dtype=torch.float32, device="cuda"))
        x, y, v = out
        L = _lib.load()
        _lib.check(L.gz_dataset_gather(_dev_ptr(self.d_records), self.n, _dev_ptr(self.d_sel), self.m,
                                       _dev_ptr(d_ids), b, self.flags, _dev_ptr(x), _dev_ptr(y), _dev_ptr(v),
                                       _stream()), "gz_dataset_gather")
        return x, y, v

    def materialize(self):
        """The whole dataset (gz_dataset_build)."""
        s = len(self)
        x = torch.empty((s,) + SAMPLE_SHAPE, dtype=torch.float32, device="cuda")
        y = torch.empty(s, dtype=torch.int64, device="cuda")
        v = torch.empty((s, 1), dtype=torch.float32, device="cuda")
        L = _lib.load()
        _lib.check(L.gz_dataset_build(_dev_ptr(self.d_records), self.n, _dev_ptr(self.d_sel), self.m, self.flags,
                                      _dev_ptr(x), _dev_ptr(y), _dev_ptr(v), _stream()), "gz_dataset_build")
        return x, y, v

    def __getitem__(self, i):
        x, y, v = self.gather(torch.tensor([int(i)], dtype=torch.int64, device="cuda"))
        return x[0], y[0], v[0]


def check_ids(ds, d_ids):
    """Raise (GzeroError) if any sample id is outside [0, len(ds)): gz_dataset_gather
    would write label -1 and zero planes, and CrossEntropyLoss would turn that label
    into a device-side assert.  One host sync."""
    if d_ids.numel():
        lo, hi = int(d_ids.min().item()), int(d_ids.max().item())
        if lo < 0 or hi >= len(ds):
            raise _lib.GzeroError(f"gz_dataset_gather: sample id out of range [{lo}, {hi}] for {len(ds)} samples")


def rows_from_planes(x):
    """[B, 3, 15, 15] network input planes (black, white, empty: boards.planes_from_cells)
    -> [B, 16] int32 board rows (black words, then white: bit r * 16 + c), the input of
    the inference kernel -- on the device, no host round trip."""
    b = int(x.shape[0])
    bits = (x[:, :2] > 0.5).to(torch.int64)                      # [B, 2, 15, 15]
    bits = nn.functional.pad(bits, (0, 1)).reshape(b, 2, 240)    # column 15 empty
    bits = nn.functional.pad(bits, (0, 16)).reshape(b, 2, 8, 32)
    w = (bits << torch.arange(32, device=x.device, dtype=torch.int64)).sum(-1)
    w = torch.where(w >= 2 ** 31, w - 2 ** 32, w)                  # the uint32 word's int32 bits
    return w.to(torch.int32).reshape(b, 16)


def _gather(ds, ids):
    """A batch of an epoch whose ids were checked once (check_ids)."""
    return ds.gather(ids, check=False) if isinstance(ds, DeviceDataset) else ds.gather(ids)


class _IndexSet(Dataset):
    def __init__(self, n):
        self.n = n

    def __len__(self):
        return self.n

    def __getitem__(self, i):
        return i


def loader_order(n, batch_size=128, shuffle=True):
    """Index batches of DataLoader(<n samples>, batch_size, shuffle) with the same torch-RNG
    use, without iterating a DataLoader (one __getitem__ and collate per sample: 0.18 s
    per 77 k-sample epoch): the iterator draws its base seed from the global generator,
    then RandomSampler one seed for the generator of its randperm
    (test_train_cpu.test_loader_order_matches_dataloader)."""
    torch.empty((), dtype=torch.int64).random_()  # the DataLoader iterator's base seed
    if shuffle:
        g = torch.Generator()
        g.manual_seed(int(torch.empty((), dtype=torch.int64).random_().item()))
        perm = torch.randperm(n, generator=g)
    else:
        perm = torch.arange(n)
    return list(perm.split(batch_size)) if n else []


def loader_order_reference(n, batch_size=128, shuffle=True):
    """The same batches by iterating DataLoader itself (the checker of loader_order)."""
    return [b for b in DataLoader(_IndexSet(n), batch_size=batch_size, shuffle=shuffle)]


def _world(group):
    if dist.is_available() and dist.is_initialized():
        return dist.get_world_size(group), dist.get_rank(group)
    return 1, 0


class DeviceTrainer:
    """Adam + StepLR policy-value SGD of training.main (training.py:379-388) on the device.

    On a GPU the whole training step runs on the HIP kernels of csrc/gz_sgd.hip without
    autograd (``gzero.sgd.NetStep``: tower forward, FC heads + loss and their backward,
    tower backward, gradients into one flat buffer that is also the data-parallel
    all-reduce bucket; ``native=False``: torch's own modules under autograd, kept for
    comparison); on the CPU (gloo rehearsals of the data-parallel loop) it is torch's.
    With the native kernels, clip_grad_norm_ + Adam are gzero.optim.DeviceAdam
    (csrc/gz_train.hip: two launches per step)."""

    def __init__(self, model, lr=8e-4, weight_decay=1e-5, grad_clip=0.8, step_size=2, gamma=0.85, group=None,
                 device="cuda", native=None):
        self.gm = model
        self.net = model.model if hasattr(model, "model") else model
        self.device = torch.device(device)
        self.net.to(self.device)
        if hasattr(model, "device"):
            model.device = self.device
        self.grad_clip = grad_clip
        self.native = (self.device.type == "cuda") if native is None else bool(native)
        self.step_fn = None
        if self.native:
            from . import sgd
            self.step_fn = sgd.NetStep(self.net)
        self._forward = self.net
        self.group = group
        self.world, self.rank = _world(group)
        self.params = [p for p in self.net.parameters()]
        if self.native:
            from .optim import DeviceAdam
            self.optimizer = DeviceAdam(self.params, lr=lr, weight_decay=weight_decay)
        else:
            self.optimizer = torch.optim.Adam(self.params, lr=lr, weight_decay=weight_decay,
                                              fused=True if self.device.type == "cuda" else None)
        self.scheduler = torch.optim.lr_scheduler.StepLR(self.optimizer, step_size=step_size, gamma=gamma)
        self.ce, self.mse = nn.CrossEntropyLoss(), nn.MSELoss()
        if self.world > 1:
            # identical replicas: rank 0's parameters and BatchNorm buffers everywhere
            for t in list(self.net.state_dict().values()):
                dist.broadcast(t, 0, group=group)
            n = sum(p.numel() for p in self.params)
            self.flat = self.step_fn.grads if self.step_fn is not None else \
                torch.zeros(n, dtype=torch.float32, device=self.device)

    def _allreduce_grads(self):
        """One bucket: the whole gradient (2.85 MB) in a single SUM all-reduce (native:
        the gradients already live in that bucket)."""
        if self.step_fn is not None:
            dist.all_reduce(self.flat, op=dist.ReduceOp.SUM, group=self.group)
            return
        off = 0
        views = []
        for p in self.params:
            k = p.numel()
            g = self.flat[off:off + k]
            if p.grad is None:
                g.zero_()
            else:
                g.copy_(p.grad.reshape(-1))
            views.append((p, g))
            off += k
        dist.all_reduce(self.flat, op=dist.ReduceOp.SUM, group=self.group)
        for p, g in views:
            if p.grad is None:
                p.grad = torch.empty_like(p)
            p.grad.copy_(g.view_as(p))

    def clip_and_step(self):
        """clip_grad_norm_(params, grad_clip) then the Adam step (training.py:303-304)."""
        clip = self.grad_clip is not None and self.grad_clip > 0
        if self.native:
            self.optimizer.step(max_norm=self.grad_clip if clip else None)
            return
        if clip:
            nn.utils.clip_grad_norm_(self.params, self.grad_clip)
        self.optimizer.step()

    def _slices(self, order, batch_size):
        """Per-step (this rank's ids, local count, global count) of a permutation."""
        B = batch_size * self.world
        for k in range(0, len(order), B):
            glob = order[k:k + B]
            gcount = len(glob)
            # remainder batches: split as evenly as possible, rank r keeps slice r
            per = -(-gcount // self.world) if gcount < B else batch_size
            mine = glob[self.rank * per:(self.rank + 1) * per]
            yield mine, len(mine), gcount

    def _ids(self, indices, order):
        return order if indices is None else indices[order]

    def train_epoch(self, ds, batch_size=128, indices=None, shuffle=True):
        """One epoch over ds (or the subset ``indices``, a device int64 tensor); returns the mean batch loss."""
        self.net.train()
        n = len(ds) if indices is None else int(indices.numel())
        order = torch.cat(loader_order(n, batch_size * self.world if self.world > 1 else batch_size, shuffle)) \
            if n else torch.zeros(0, dtype=torch.int64)
        order = order.to(self.device)
        ids_all = self._ids(indices, order)
        check_ids(ds, ids_all)
        total = torch.zeros((), dtype=torch.float64, device=self.device)
        batches = 0
        for mine, local, gcount in self._slices(ids_all, batch_size):
            if self.step_fn is not None:  # every gradient is overwritten by the step
                if local > 0:
                    x, y, v = _gather(ds, mine)
                    lval = self.step_fn.step(x, y, v, scale=local / gcount if self.world > 1 else 1.0)
                else:
                    self.step_fn.zero()
                    lval = torch.zeros((), device=self.device)
                if self.world > 1:
                    self._allreduce_grads()
                    lval = lval * (local / gcount)
                    dist.all_reduce(lval, group=self.group)
                self.clip_and_step()
                total += lval.double()
                batches += 1
                continue
            # (torch's default, as training.py:292: fresh gradients are assigned, not added
            # into zero-filled ones -- about 60 fewer kernels per step)
            self.optimizer.zero_grad(set_to_none=True)
            if local > 0:
                x, y, v = _gather(ds, mine)
                logits, val = self._forward(x)
                loss = self.ce(logits, y) + self.mse(val, v)
                (loss * (local / gcount) if self.world > 1 else loss).backward()
                lval = loss.detach()
            else:
                lval = torch.zeros((), device=self.device)
            if self.world > 1:
                # the global-batch loss (for reporting) rides along with the gradient
                self._allreduce_grads()
                lval = lval * (local / gcount)
                dist.all_reduce(lval, group=self.group)
            self.clip_and_step()
            total += lval.double()
            batches += 1
        if self.world > 1:
            for t in self.net.buffers():  # BatchNorm running stats: rank 0's, as DDP's broadcast_buffers
                dist.broadcast(t, 0, group=self.group)
        return float(total.item()) / max(1, batches)

    @torch.no_grad()
    def validate_epoch(self, ds, batch_size=128, indices=None, chunk=512, kernel=None):
        """Mean per-batch validation loss (training.py:313-337).  Data parallel:
        batch k is evaluated by rank k mod N and the per-batch losses are
        SUM-all-reduced, so every rank returns the same global value (and each
        batch is evaluated once, not N times).  The batches are evaluated ``chunk``
        boards per forward (eval mode has no batch statistics, so the per-sample
        outputs do not depend on the batching; the last forward is padded to the same
        shape, whose convolution algorithms MIOpen then finds once per process instead
        of once per remainder size) and the per-sample losses are averaged per batch of
        ``batch_size``, as the reference's loop over its DataLoader does.

        ``kernel`` (default: the native trainer): the eval-mode forward is the inference
        kernel (gz_pv_forward, f16x3; logits within 3e-7 of fp32) on the
        samples' board rows, with the weights packed on the device from the current
        parameters and running statistics -- not the training graph's torch convolutions.
        This is a deliberate numeric difference from the reference, whose validation loss
        (and so training.main's improvement / early-stop decision) comes from the fp32
        eval-mode torch forward: the two agree within 1e-5 (checked every epoch in
        tests/test_gpu_train.py); kernel=False evaluates with the torch forward."""
        self.net.eval()
        kernel = self.native if kernel is None else bool(kernel)
        pvw = None
        if kernel:
            from . import device as _device, weights as _weights
            pvw = _device.PVWeights(_weights.pack_pv_weights_torch(self.net.state_dict(), self.device))
        n = len(ds) if indices is None else int(indices.numel())
        # iterate an (unshuffled) DataLoader as the reference does: it draws one torch seed
        order = loader_order(n, batch_size, shuffle=False)
        order = (torch.cat(order) if order else torch.zeros(0, dtype=torch.int64)).to(self.device)
        ids_all = self._ids(indices, order)
        check_ids(ds, ids_all)
        nb = -(-n // batch_size)
        mine = [bi for bi in range(nb) if bi % self.world == self.rank]
        total = torch.zeros((), dtype=torch.float64, device=self.device)
        per = max(1, chunk // batch_size)
        for c in range(0, len(mine), per):
            bis = mine[c:c + per]
            ids = torch.cat([ids_all[bi * batch_size:(bi + 1) * batch_size] for bi in bis])
            real = int(ids.numel())
            if real < per * batch_size:
                ids = torch.cat([ids, ids[:1].expand(per * batch_size - real)])
            x, y, v = _gather(ds, ids)
            if pvw is not None:
                b = int(ids.numel())
                lg, vl, _ = _device.pv_forward_dev(pvw, rows_from_planes(x), b)
                logits, val = lg.view(b, -1), vl.view(b, 1)
            else:
                logits, val = self.net(x)
            logits, val, y, v = logits[:real], val[:real], y[:real], v[:real]
            ce = nn.functional.cross_entropy(logits, y, reduction="none")
            se = (val.reshape(-1) - v.reshape(-1).to(val.dtype)) ** 2
            ks = [min(batch_size, n - bi * batch_size) for bi in bis]
            seg = torch.repeat_interleave(torch.arange(len(bis), device=self.device),
                                          torch.tensor(ks, device=self.device))
            cnt = torch.tensor(ks, dtype=torch.float64, device=self.device)
            sums = torch.zeros(len(bis), dtype=torch.float64, device=self.device)
            sums.index_add_(0, seg, ce.double()).div_(cnt)
            sse = torch.zeros(len(bis), dtype=torch.float64, device=self.device)
            sse.index_add_(0, seg, se.double()).div_(cnt)
            total += (sums + sse).sum()
        if self.world > 1:
            dist.all_reduce(total, group=self.group)
        return float(total.item()) / max(1, nb)

    def step_scheduler(self):
        self.scheduler.step()
