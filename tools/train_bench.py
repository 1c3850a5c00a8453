"""BASELINE config 5: training.main's iteration on the device -- self-play
(medium AIs, 200 sims, beta 0.2, planner_steps 5 = the reference's default
AI), the augmented dataset, 2 epochs of data-parallel SGD (batch 128 per rank,
Adam 8e-4, clip 0.8) -- reported as iterations/hour, with the split between
self-play and SGD and the SGD step rate.

  python tools/train_bench.py --games 256 --iterations 2
  python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 tools/train_bench.py ...

One JSON line from rank 0.  The arena games of training.main (6 x easy, 60 sims)
are timed separately (--eval-games) and not part of the iteration figure.
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "alphazero-gomoku_amd"), REPO]

import torch  # noqa: E402


def dataset_bench(n, reps=5):
    """gz_dataset_build over n records with every record augmented (9n samples):
    HBM-bound writes, 2,712 B out per sample (planes 2,700 + label 8 + value 4)."""
    import random
    import numpy as np
    from gzero import boards
    from gzero.train import DeviceDataset
    rng = np.random.default_rng(1)
    cells = rng.choice(np.array([0, 0, 0, 1, 2], np.int8), size=(n, 225))
    rec = np.zeros(n, boards.RECORD_DTYPE)
    rec["black"], rec["white"] = boards.cells_to_words(cells)
    rec["move"] = rng.integers(0, 225, n)
    ds = DeviceDataset(rec, augment_ratio=1.0, rng=random.Random(0))
    ds.materialize()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        out = ds.materialize()
        del out
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    s = len(ds)
    byts = s * (2700 + 8 + 4) + n * 80
    return {"records": n, "samples": s, "ms": ms, "GB_per_s": byts / ms / 1e6, "bytes": byts,
            "note": "materialize() allocates its outputs inside the timed loop (caching allocator, no sync)"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--games", type=int, default=256, help="self-play games per rank per iteration")
    ap.add_argument("--iterations", type=int, default=2)
    ap.add_argument("--sims", type=int, default=200)
    ap.add_argument("--planner-steps", type=int, default=5)
    ap.add_argument("--eval-games", type=int, default=0)
    ap.add_argument("--seed", type=int, default=1234)
    ap.add_argument("--dataset-records", type=int, default=0,
                    help="also time gz_dataset_build on this many random records (x4.5 samples at ratio 0.35*10)")
    a = ap.parse_args()
    import random
    from gzero import dist as gdist
    from gzero.train import DeviceTrainer
    from neural_network import GomokuModel
    import training
    rank, ws = gdist.init_from_env()
    random.seed(a.seed)
    torch.manual_seed(a.seed)
    model = GomokuModel(device="cuda")
    trainer = DeviceTrainer(model)
    its = []
    for it in range(1, a.iterations + 1):
        if ws > 1:
            torch.distributed.barrier()
        torch.cuda.synchronize()
        t0 = time.time()
        r = training.run_iteration(model, trainer, it, a.games, num_simulations=a.sims,
                                   planner_steps=a.planner_steps, seed=a.seed, verbose=False)
        torch.cuda.synchronize()
        if ws > 1:
            torch.distributed.barrier()
        r["iteration_s"] = time.time() - t0
        its.append(r)
        if rank == 0:
            print(json.dumps({"progress": it, **{k: v for k, v in r.items() if not isinstance(v, dict)}}),
                  file=sys.stderr, flush=True)
    dsb = dataset_bench(a.dataset_records) if a.dataset_records and rank == 0 else None
    ev = None
    if a.eval_games and rank == 0:
        t = time.time()
        res = training.evaluate_model(model, None, games=a.eval_games, seed=a.seed, alternate=False)
        ev = {"games": a.eval_games, "seconds": time.time() - t, "win_rate": res["win_rate"]}
    if rank == 0:
        it_s = sum(r["iteration_s"] for r in its) / len(its)
        sgd_steps = sum(2 * -(-int(0.9 * r.get("samples", 0)) // (128 * ws)) for r in its)
        sgd_s = sum(r.get("sgd_s", 0.0) for r in its)
        print(json.dumps({
            "metric": "training iterations/hour (BASELINE config 5: self-play + policy-value SGD)",
            "value": 3600.0 / it_s, "unit": "iterations/h", "n_gpus": ws, "higher_is_better": True,
            "iteration_s": it_s, "selfplay_s": sum(r["selfplay_s"] for r in its) / len(its),
            "sgd_s": sgd_s / len(its), "sgd_steps_per_s": sgd_steps / max(1e-9, sgd_s),
            "records_per_iteration": sum(r["records"] for r in its) / len(its),
            "samples_per_iteration": sum(r.get("samples", 0) for r in its) / len(its),
            "config": {"games_per_rank": a.games, "sims": a.sims, "planner_steps": a.planner_steps,
                       "batch_per_rank": 128, "epochs": 2, "augment_ratio": 0.35},
            "eval": ev, "dataset_kernel": dsb, "dtype": "fp32 SGD (MIOpen), f16x3 self-play forwards",
            "data": "synthetic: self-play from the empty board, random-init weights"}), flush=True)


if __name__ == "__main__":
    main()
