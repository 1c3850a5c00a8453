#!/usr/bin/env python3
"""Config 5 alone (bench.config5: 512 games, 2 iterations) for a rocprofv3 kernel trace:
python tools/c5_trace.py [games] [iterations].  With GZ_PHASES=<file> the host phases of
run_iteration (self-play, dataset, each epoch's training and validation) are written
there as CLOCK_MONOTONIC ns intervals, to place the trace's idle gaps."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "alphazero-gomoku_amd"))
import bench  # noqa: E402

phases = []
if os.environ.get("GZ_PHASES"):
    import training
    from gzero import train as T

    def wrap(obj, name, label):
        f = getattr(obj, name)

        def g(*a, **k):
            t0 = time.monotonic_ns()
            try:
                return f(*a, **k)
            finally:
                phases.append((label, t0, time.monotonic_ns()))
        setattr(obj, name, g)
    wrap(training, "selfplay_device", "selfplay")
    wrap(T.DeviceDataset, "__init__", "dataset")
    wrap(T.DeviceTrainer, "train_epoch", "train_epoch")
    wrap(T.DeviceTrainer, "validate_epoch", "validate")
    wrap(training, "run_iteration", "iteration")

g = int(sys.argv[1]) if len(sys.argv) > 1 else 512
its = int(sys.argv[2]) if len(sys.argv) > 2 else 2
r = bench.config5(g, 200, 1234, iterations=its)
print(json.dumps({k: r[k] for k in ("value", "iteration_s", "selfplay_s", "sgd_s", "first_iteration_s")}))
if phases:
    json.dump(phases, open(os.environ["GZ_PHASES"], "w"))
