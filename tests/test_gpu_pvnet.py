"""K6 policy-value forward (fp32 MFMA) against the reference GomokuModel
(golden, deterministic weights) and against a torch fp32 CPU forward.
Tolerance: 1e-4 absolute on logits / value / softmax (north star)."""
import base64

import numpy as np
import pytest
import torch

from conftest import golden
from gzero import boards, device, weights

pytestmark = pytest.mark.gpu
TOL = 1e-4


def _dec(s, shape):
    return np.frombuffer(base64.b64decode(s), np.float32).reshape(shape)


PRECS = ["fp32", "f16x3"]


@pytest.mark.parametrize("prec", PRECS)
def test_pv_forward_matches_reference_golden(oracle, prec):
    g = golden("pvnet")
    sd = weights.init_state_dict(seed=g["weights_seed"])
    w = device.PVWeights(weights.pack_pv_weights(sd), precision=prec)
    rows = []
    for c in g["cases"]:
        b = oracle.new_board(c["moves"])
        bl, wh = boards.cells_to_words(b.cells()[None])
        rows.append(boards.leaf_words(bl, wh)[0])
    n = len(rows)
    lg, v, pr = device.pv_forward(w, np.stack(rows))
    ref_lg = _dec(g["logits_f32_b64"], (n, 225))
    ref_v = _dec(g["value_f32_b64"], (n,))
    ref_p = _dec(g["probs_f32_b64"], (n, 225))
    assert np.abs(lg - ref_lg).max() < TOL, np.abs(lg - ref_lg).max()
    assert np.abs(v - ref_v).max() < TOL
    assert np.abs(pr - ref_p).max() < TOL


@pytest.mark.parametrize("prec", PRECS)
def test_pv_forward_matches_torch_fp32_large_batch(prec):
    rng = np.random.default_rng(3)
    n = 1500
    cells = rng.choice(3, size=(n, 225), p=[0.6, 0.2, 0.2]).astype(np.int8)
    sd = weights.init_state_dict(seed=11)
    w = device.PVWeights(weights.pack_pv_weights(sd), precision=prec)
    bl, wh = boards.cells_to_words(cells)
    lg, v, pr = device.pv_forward(w, boards.leaf_words(bl, wh))
    ref_lg, ref_v = weights.reference_forward(sd, boards.planes_from_cells(cells))
    ref_p = torch.softmax(torch.from_numpy(ref_lg), dim=1).numpy()
    assert np.abs(lg - ref_lg).max() < TOL
    assert np.abs(v - ref_v).max() < TOL
    assert np.abs(pr - ref_p).max() < TOL


@pytest.mark.parametrize("prec", PRECS)
def test_pv_forward_device_count(prec):
    """The count-on-device form evaluates only the first *d_count boards."""
    sd = weights.init_state_dict(seed=2)
    w = device.PVWeights(weights.pack_pv_weights(sd), precision=prec)
    rows = np.zeros((64, 16), np.uint32)
    d_b = torch.from_numpy(rows.view(np.int32)).cuda()
    d_cnt = torch.tensor([10], dtype=torch.int32, device="cuda")
    d_lg = torch.full((64 * 225,), 7.0, device="cuda")
    d_v = torch.full((64,), 7.0, device="cuda")
    device.pv_forward_dev(w, d_b, 64, d_count=d_cnt, d_logits=d_lg, d_value=d_v)
    torch.cuda.synchronize()
    v = d_v.cpu().numpy()
    assert np.all(v[10:] == 7.0) and np.all(np.abs(v[:10]) <= 1.0)


def test_pv_trained_scale_weights():
    """f16x3 on weights 10x larger than the init (trained-network scale): still 1e-4."""
    rng = np.random.default_rng(4)
    cells = rng.choice(3, size=(256, 225), p=[0.5, 0.25, 0.25]).astype(np.int8)
    sd = weights.init_state_dict(seed=5)
    for k in sd:
        if k.endswith("weight") and "conv" in k and "bn" not in k:
            sd[k] = sd[k] * 3.0
    ref_lg, ref_v = weights.reference_forward(sd, boards.planes_from_cells(cells))
    bl, wh = boards.cells_to_words(cells)
    for prec in PRECS:
        w = device.PVWeights(weights.pack_pv_weights(sd), precision=prec)
        lg, v, _ = device.pv_forward(w, boards.leaf_words(bl, wh))
        scale = max(1.0, float(np.abs(ref_lg).max()))
        assert np.abs(lg - ref_lg).max() < TOL * scale, (prec, np.abs(lg - ref_lg).max(), scale)
        assert np.abs(v - ref_v).max() < TOL
