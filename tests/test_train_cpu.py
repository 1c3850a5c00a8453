"""Training-set construction and the SGD loop, CPU side.

* the numpy restatement (oracle/train_oracle.py) against the reference's
  fixtures: augment_sample (G8) and GomokuSelfPlayDataset's samples (G9);
* the host training loop (training.train_epoch / validate_epoch over
  GomokuSelfPlayDataset) reproduces the reference's two epochs bit for bit on
  CPU torch (G9 was recorded with 1 thread);
* the data-parallel step of gzero.train.DeviceTrainer on world_size 2 (gloo):
  two ranks x batch 64 give the single-process batch-128 update.
"""
import base64
import os
import random
import socket
import zlib

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp
import torch.nn as nn

from conftest import golden
import train_oracle as TO


def _records(g):
    cells = np.array([[int(ch) for ch in r["cells"]] for r in g["records"]], np.int8)
    moves = np.array([r["move"] for r in g["records"]], np.int64)
    players = np.array([r["player"] for r in g["records"]], np.int64)
    z = np.array([r["z"] for r in g["records"]], np.int64)
    return cells, moves, players, z


def _sel(g, n):
    rnd = random.Random(g["sel_seed"])
    sel = rnd.sample(range(n), k=max(1, int(n * 0.35)))
    return rnd, sel


def test_oracle_augment_matches_reference():
    cases = golden("augment")["cases"]
    for idx in range(225):
        c = np.zeros(225, np.int8)
        c[idx] = 1
        p = TO.planes_of(c)
        got = [[TO.transform_index(idx, k, f), int(np.argmax(TO.transform_planes(p, k, f)[0]))]
               for k in range(4) for f in (False, True)]
        assert got == cases[idx]


def test_oracle_dataset_matches_reference():
    g = golden("sgd")
    cells, moves, _, z = _records(g)
    _, sel = _sel(g, len(moves))
    x, y, v = TO.dataset_samples(cells, moves, z, sel)
    assert len(y) == g["n_samples"]
    assert y.tolist() == g["labels"]
    assert v.tolist() == g["values"]
    assert zlib.crc32(np.ascontiguousarray(x, np.float32).tobytes()) == g["planes_crc32"]


def test_oracle_fixed_labels_follow_planes():
    for idx in (0, 7, 14, 112, 210, 224):
        c = np.zeros(225, np.int8)
        c[idx] = 1
        p = TO.planes_of(c)
        for k in range(4):
            for f in (False, True):
                assert TO.transform_index(idx, k, f, fix=True) == int(np.argmax(TO.transform_planes(p, k, f)[0]))


def test_host_training_loop_matches_reference():
    """training.GomokuSelfPlayDataset + train_epoch + validate_epoch (CPU torch)
    == the reference's two epochs of training.main's optimiser loop."""
    import training
    from neural_network import GomokuModel
    from gzero import weights
    from torch.utils.data import DataLoader, Subset
    g = golden("sgd")
    cells, moves, players, z = _records(g)
    replay = training.SimpleReplay()
    for i in range(len(moves)):
        replay.add(TO.planes_of(cells[i]), int(moves[i]), int(players[i]))
        replay.outcomes.append(int(z[i]))
    nthr = torch.get_num_threads()
    torch.set_num_threads(1)
    saved = training.random
    try:
        rnd = random.Random(g["sel_seed"])
        training.random = rnd
        ds = training.GomokuSelfPlayDataset(replay, use_augmentation=True, augment_ratio=0.35)
        assert [int(s[1]) for s in ds.samples] == g["labels"]
        idx = list(range(len(ds)))
        rnd.shuffle(idx)
        split = int(len(ds) * 0.9)
        assert idx[:split] == g["train_idx"] and idx[split:] == g["val_idx"]
        m = GomokuModel(device="cpu")
        m.model.load_state_dict(weights.init_state_dict(seed=7))
        torch.manual_seed(g["torch_seed"])
        tl_loader = DataLoader(Subset(ds, idx[:split]), batch_size=128, shuffle=True)
        vl_loader = DataLoader(Subset(ds, idx[split:]), batch_size=128, shuffle=False)
        opt = torch.optim.Adam(m.model.parameters(), lr=8e-4, weight_decay=1e-5)
        tl, vl = [], []
        for _ in range(2):
            tl.append(training.train_epoch(m, tl_loader, opt, torch.device("cpu"), grad_clip=0.8))
            vl.append(training.validate_epoch(m, vl_loader, torch.device("cpu")))
    finally:
        training.random = saved
        torch.set_num_threads(nthr)
    assert tl == g["train_loss"] and vl == g["val_loss"]
    for k, t in m.model.state_dict().items():
        a = t.detach().float().numpy().reshape(-1)
        ref = np.frombuffer(base64.b64decode(g["param_sample_f32_b64"][k]), np.float32)
        assert np.array_equal(a[::max(1, a.size // 64)][:64], ref), k


# ---------------------------------------------------------------- data parallel (gloo, world 2)


class _TinyNet(nn.Module):
    """BatchNorm-free stand-in with the policy-value signature (x -> logits, value)."""

    def __init__(self):
        super().__init__()
        self.p = nn.Linear(675, 225)
        self.v = nn.Linear(675, 1)

    def forward(self, x):
        f = x.reshape(x.shape[0], -1)
        return self.p(f), torch.tanh(self.v(f))


class _TensorSet:
    def __init__(self, x, y, v):
        self.x, self.y, self.v = x, y, v

    def __len__(self):
        return len(self.y)

    def gather(self, ids):
        return self.x[ids], self.y[ids], self.v[ids]


def _data(n=300):
    g = torch.Generator().manual_seed(3)
    x = (torch.rand((n, 3, 15, 15), generator=g) < 0.3).float()
    y = torch.randint(0, 225, (n,), generator=g)
    v = torch.randint(-1, 2, (n, 1), generator=g).float()
    return _TensorSet(x, y, v)


def _train(world_rank=None):
    from gzero.train import DeviceTrainer
    torch.manual_seed(0)
    net = _TinyNet()
    tr = DeviceTrainer(net, device="cpu")
    ds = _data()
    torch.manual_seed(11)
    losses = [tr.train_epoch(ds, batch_size=128 if world_rank is None else 64) for _ in range(2)]
    return losses, [p.detach().clone() for p in net.parameters()]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _dp_worker(rank, ws, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    torch.set_num_threads(1)
    losses, params = _train(world_rank=rank)
    q.put((rank, losses, [p.numpy().tobytes() for p in params]))
    dist.destroy_process_group()


def test_data_parallel_step_equals_global_batch():
    torch.set_num_threads(1)
    ref_losses, ref_params = _train()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_dp_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=180) for _ in procs])
    for p in procs:
        p.join(timeout=60)
    (_, l0, p0), (_, l1, p1) = res
    assert p0 == p1 and l0 == l1  # replicas stay identical
    np.testing.assert_allclose(l0, ref_losses, rtol=1e-5)
    for a, b in zip(p0, ref_params):
        np.testing.assert_allclose(np.frombuffer(a, np.float32), b.numpy().reshape(-1), atol=2e-6)


@pytest.mark.parametrize("n", [1, 7, 128, 129, 5000])
@pytest.mark.parametrize("shuffle", [True, False])
def test_loader_order_matches_dataloader(n, shuffle):
    """gzero.train.loader_order (no DataLoader iteration) yields DataLoader's batches and
    leaves torch's global generator where iterating the DataLoader leaves it."""
    import torch
    from gzero.train import loader_order, loader_order_reference
    torch.manual_seed(11)
    a, ra = loader_order(n, 128, shuffle), torch.rand(4)
    torch.manual_seed(11)
    b, rb = loader_order_reference(n, 128, shuffle), torch.rand(4)
    assert len(a) == len(b) and all(torch.equal(x, y) for x, y in zip(a, b))
    assert torch.equal(ra, rb)


def test_rows_from_planes_matches_leaf_words():
    """gzero.train.rows_from_planes (the kernel validation's input) = boards.leaf_words of
    the same cells, every bit -- incl. the empty board, a full one and the corners."""
    from gzero import boards
    from gzero.train import rows_from_planes
    rng = np.random.default_rng(3)
    cells = rng.choice(3, size=(64, 225), p=[0.4, 0.3, 0.3]).astype(np.int8)
    cells[0] = 0
    cells[1] = rng.choice([1, 2], size=225)
    cells[2] = 0
    cells[2][[0, 14, 210, 224]] = [1, 2, 2, 1]
    bl, wh = boards.cells_to_words(cells)
    want = boards.leaf_words(bl, wh).view(np.int32)
    got = rows_from_planes(torch.from_numpy(boards.planes_from_cells(cells))).numpy()
    assert np.array_equal(got, want)
