"""Policy-value SGD step rate (batch 128, Adam, clip 0.8) under MIOpen settings."""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "alphazero-gomoku_amd"), REPO]
import torch  # noqa: E402
import torch.nn as nn  # noqa: E402

from gzero import weights  # noqa: E402


def run(tag, steps=60, bs=128, channels_last=False, native=False):
    torch.manual_seed(0)
    net = weights.PolicyValueNet().cuda()
    if channels_last:
        net = net.to(memory_format=torch.channels_last)
    opt = torch.optim.Adam(net.parameters(), lr=8e-4, weight_decay=1e-5, fused=native)
    ce, mse = nn.CrossEntropyLoss(), nn.MSELoss()
    x = (torch.rand((bs, 3, 15, 15), device="cuda") < 0.3).float()
    if channels_last:
        x = x.contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 225, (bs,), device="cuda")
    v = torch.rand((bs, 1), device="cuda")
    net.train()

    from gzero import sgd
    fwd = (lambda t: sgd.train_forward(net, t)) if native else net

    def step():
        opt.zero_grad()
        lg, val = fwd(x)
        loss = ce(lg, y) + mse(val, v)
        loss.backward()
        nn.utils.clip_grad_norm_(net.parameters(), 0.8)
        opt.step()

    for _ in range(5):
        step()
    torch.cuda.synchronize()
    t = time.time()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    dt = (time.time() - t) / steps
    print(f"{tag}: {dt * 1e3:.2f} ms/step, {bs * 3 * 267.38e6 / dt / 1e12:.1f} TFLOP/s", flush=True)


ONLY = sys.argv[1] if len(sys.argv) > 1 else None  # "native": just the device-tower runs (profiling)
run("native", native=True)
if ONLY != "native":
    run("default")
    torch.backends.cudnn.benchmark = True
    run("benchmark")
    run("benchmark+channels_last", channels_last=True)


def trainer_run(tag, n_records=4000, **kw):
    import random
    import numpy as np
    from gzero import boards
    from gzero.train import DeviceDataset, DeviceTrainer
    from neural_network import GomokuModel
    rng = np.random.default_rng(1)
    cells = rng.choice(np.array([0, 0, 0, 1, 2], np.int8), size=(n_records, 225))
    rec = np.zeros(n_records, boards.RECORD_DTYPE)
    rec["black"], rec["white"] = boards.cells_to_words(cells)
    rec["move"] = rng.integers(0, 225, n_records)
    rec["z"] = rng.integers(-1, 2, n_records)
    ds = DeviceDataset(rec, augment_ratio=0.35, rng=random.Random(0))
    m = GomokuModel(device="cpu")
    tr = DeviceTrainer(m, **kw)
    tr.train_epoch(ds, 128)
    torch.cuda.synchronize()
    t = time.time()
    tr.train_epoch(ds, 128)
    torch.cuda.synchronize()
    dt = time.time() - t
    steps = -(-len(ds) // 128)
    print(f"trainer {tag}: {len(ds)} samples, {steps} steps, {dt / steps * 1e3:.2f} ms/step", flush=True)


torch.backends.cudnn.benchmark = False
trainer_run("native", native=True)
trainer_run("native-2nd", native=True)
if ONLY != "native":
    trainer_run("miopen", native=False)

