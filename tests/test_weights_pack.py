"""The device-side weight packer (gzero/weights.py:pack_pv_weights_torch) against the
host one (pack_pv_weights): the same float32 blob bit for bit -- on torch's CPU here,
on the GPU under -m gpu (neural_network.GomokuModel.device_weights packs there)."""
import os
import sys
import time

import numpy as np
import pytest
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "alphazero-gomoku_amd"))
from gzero import weights  # noqa: E402


def _same(a, b):
    a = np.ascontiguousarray(a, np.float32).view(np.uint32)
    b = np.ascontiguousarray(b, np.float32).view(np.uint32)
    assert a.shape == b.shape == (weights.TOTAL,)
    bad = np.flatnonzero(a != b)
    assert bad.size == 0, f"{bad.size} words differ, first at {bad[:5]}"


@pytest.mark.parametrize("seed,noise", [(0, True), (5, False)])
def test_torch_pack_matches_numpy_pack_cpu(seed, noise):
    sd = weights.init_state_dict(seed, bn_noise=noise)
    _same(weights.pack_pv_weights_torch(sd, "cpu").numpy(), weights.pack_pv_weights(sd))


@pytest.mark.gpu
@pytest.mark.parametrize("seed,scale", [(1, 1.0), (2, 0.1), (3, 3.0)])
def test_device_pack_matches_numpy_pack(seed, scale):
    sd = {k: (v * scale if k.endswith("weight") and v.dim() > 1 else v)
          for k, v in weights.init_state_dict(seed, bn_noise=True).items()}
    want = weights.pack_pv_weights(sd)
    got = weights.pack_pv_weights_torch(sd, "cuda")
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(5):
        got = weights.pack_pv_weights_torch(sd, "cuda")
    torch.cuda.synchronize()
    print(f"device pack {(time.perf_counter() - t) / 5 * 1e3:.1f} ms")
    _same(got.cpu().numpy(), want)
