"""gz_dataset_build throughput (HBM-bound writes); prints one line."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "alphazero-gomoku_amd"), os.path.join(REPO, "tools"), REPO]
from train_bench import dataset_bench  # noqa: E402

r = dataset_bench(int(sys.argv[1]) if len(sys.argv) > 1 else 200000, reps=10)
print(f"gz_dataset_build {r['samples']} samples: {r['ms']:.3f} ms, {r['GB_per_s']:.0f} GB/s")
