"""Device SGD vs the G9 fixture under different torch backend settings (numerics probe)."""
import os
import random
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "tests"), os.path.join(REPO, "alphazero-gomoku_amd"), os.path.join(REPO, "oracle")]
from conftest import golden  # noqa: E402
from test_gpu_train import _records  # noqa: E402
from gzero import weights  # noqa: E402
from gzero.train import DeviceDataset, DeviceTrainer  # noqa: E402
from neural_network import GomokuModel  # noqa: E402


def run(tag):
    g = golden("sgd")
    _, rec = _records(g)
    rnd = random.Random(g["sel_seed"])
    ds = DeviceDataset(rec, augment_ratio=0.35, rng=rnd)
    idx = list(range(len(ds)))
    rnd.shuffle(idx)
    split = int(len(ds) * 0.9)
    tr_idx = torch.tensor(idx[:split], dtype=torch.int64, device="cuda")
    va_idx = torch.tensor(idx[split:], dtype=torch.int64, device="cuda")
    m = GomokuModel(device="cpu")
    m.model.load_state_dict(weights.init_state_dict(seed=7))
    tr = DeviceTrainer(m)
    torch.manual_seed(g["torch_seed"])
    tl, vl = [], []
    for _ in range(2):
        tl.append(tr.train_epoch(ds, 128, indices=tr_idx))
        vl.append(tr.validate_epoch(ds, 128, indices=va_idx))
    rel = np.abs(np.array(tl + vl) / np.array(g["train_loss"] + g["val_loss"]) - 1)
    print(tag, "train", tl, "val", vl, "max rel", rel.max(), flush=True)


run("default")
torch.backends.cudnn.allow_tf32 = False
torch.backends.cuda.matmul.allow_tf32 = False
run("no-tf32")
torch.backends.cudnn.deterministic = True
torch.backends.cudnn.benchmark = False
run("no-tf32+deterministic")
torch.backends.cudnn.enabled = False
run("no-miopen")
