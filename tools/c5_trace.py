#!/usr/bin/env python3
"""Config 5 alone (bench.config5: 512 games, 2 iterations) for a rocprofv3 kernel trace:
python tools/c5_trace.py [games] [iterations]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "alphazero-gomoku_amd"))
import bench  # noqa: E402

g = int(sys.argv[1]) if len(sys.argv) > 1 else 512
its = int(sys.argv[2]) if len(sys.argv) > 2 else 2
r = bench.config5(g, 200, 1234, iterations=its)
print(json.dumps({k: r[k] for k in ("value", "iteration_s", "selfplay_s", "sgd_s", "first_iteration_s")}))
