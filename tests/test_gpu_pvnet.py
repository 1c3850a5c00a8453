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


def _check_weights(sd, cells, what):
    ref_lg, ref_v = weights.reference_forward(sd, boards.planes_from_cells(cells))
    bl, wh = boards.cells_to_words(cells)
    for prec in PRECS:
        w = device.PVWeights(weights.pack_pv_weights(sd), precision=prec)
        lg, v, _ = device.pv_forward(w, boards.leaf_words(bl, wh))
        scale = max(1.0, float(np.abs(ref_lg).max()))
        assert np.abs(lg - ref_lg).max() < TOL * scale, (what, prec, np.abs(lg - ref_lg).max(), scale)
        assert np.abs(v - ref_v).max() < TOL, (what, prec, np.abs(v - ref_v).max())


@pytest.mark.parametrize("mult", [0.1, 0.3, 3.0])
def test_pv_scaled_conv_weights(mult):
    """f16x3 with every conv weight scaled by `mult`: x0.1 / x0.3 push the residual
    weights' lo halves (|w| ~ 3e-3) deeper into fp16's subnormal range (the
    precision risk of DESIGN 3.3); x3 is a trained-network magnitude.  Logits within
    1e-4 relative to max(1, max |logit|), value within 1e-4 absolute."""
    rng = np.random.default_rng(4)
    cells = rng.choice(3, size=(256, 225), p=[0.5, 0.25, 0.25]).astype(np.int8)
    sd = weights.init_state_dict(seed=5)
    for k in sd:
        if k.endswith("weight") and "conv" in k and "bn" not in k:
            sd[k] = sd[k] * mult
    _check_weights(sd, cells, f"conv x{mult}")


def test_pv_after_device_sgd():
    """f16x3 on the weights DeviceTrainer produces (two epochs of the reference's
    SGD recipe, training.py:277-311, on 2,000 synthetic records; BN statistics
    updated in train mode) -- what config 5 feeds back into self-play."""
    import random

    from gzero.train import DeviceDataset, DeviceTrainer
    from neural_network import GomokuModel
    rng = np.random.default_rng(12)
    n = 2000
    cells = rng.choice(np.array([0, 0, 0, 1, 2], np.int8), size=(n, 225))
    rec = np.zeros(n, boards.RECORD_DTYPE)
    rec["black"], rec["white"] = boards.cells_to_words(cells)
    rec["move"] = rng.integers(0, 225, n)
    rec["player"] = rng.integers(1, 3, n)
    rec["z"] = rng.integers(-1, 2, n)
    ds = DeviceDataset(rec, augment_ratio=0.35, rng=random.Random(3))
    m = GomokuModel(device="cpu")
    m.model.load_state_dict(weights.init_state_dict(seed=9))
    tr = DeviceTrainer(m)
    torch.manual_seed(0)
    for _ in range(2):
        tr.train_epoch(ds, 128)
    sd = {k: v.detach().cpu() for k, v in m.model.state_dict().items()}
    eval_cells = rng.choice(3, size=(512, 225), p=[0.55, 0.225, 0.225]).astype(np.int8)
    _check_weights(sd, eval_cells, "after DeviceTrainer")


def _fixture_rows(oracle, g):
    rows, cells = [], []
    for c in g["cases"]:
        b = oracle.new_board(c["moves"])
        bl, wh = boards.cells_to_words(b.cells()[None])
        rows.append(boards.leaf_words(bl, wh)[0])
        cells.append(b.cells())
    return np.stack(rows), cells


@pytest.mark.parametrize("prec", PRECS)
def test_prior_matches_reference_and_oracle(oracle, prec):
    """a20 MCTSNode._get_prior_probability (ai_agent.py:564-582) on the device:
    * within 1e-4 of the reference's prior vectors (fixture prior: same boards and
      weights as pvnet; the float32 softmax differs from numpy's by ~1e-8);
    * bit-exact against the oracle's restatement fed the device's own softmax (the
      float64 pairwise sum and division round exactly like numpy's);
    * 0 at stones; the empty cells in row-major order = the reference's compact vector."""
    g, gp = golden("pvnet"), golden("prior")
    sd = weights.init_state_dict(seed=g["weights_seed"])
    ref = np.frombuffer(base64.b64decode(gp["prior_f64_b64"]), np.float64)
    w = device.PVWeights(weights.pack_pv_weights(sd), precision=prec)
    rows, cells = _fixture_rows(oracle, g)
    _, _, pr, prior = device.pv_forward(w, rows, want_prior=True)
    off = 0
    for i, cl in enumerate(cells):
        k = gp["counts"][i]
        empty = cl == 0
        assert int(empty.sum()) == k
        assert np.all(prior[i][~empty] == 0.0)
        got = prior[i][empty]
        assert np.abs(got - ref[off:off + k]).max() < TOL, i
        assert got.tobytes() == oracle.prior(pr[i], cl).tobytes(), i
        off += k


def test_prior_random_boards_exact_vs_oracle(oracle):
    """Prior on 600 random boards (1..225 empty cells: both pairwise-sum regimes,
    <= 128 and > 128 terms, and a single empty cell): bit-exact vs the oracle fed
    the device softmax."""
    rng = np.random.default_rng(21)
    n = 600
    fill = rng.uniform(0.0, 0.99, n)
    cells = np.where(rng.random((n, 225)) < fill[:, None], rng.integers(1, 3, (n, 225)), 0).astype(np.int8)
    cells[0] = 1
    cells[0, 17] = 0
    sd = weights.init_state_dict(seed=3)
    w = device.PVWeights(weights.pack_pv_weights(sd))
    bl, wh = boards.cells_to_words(cells)
    _, _, pr, prior = device.pv_forward(w, boards.leaf_words(bl, wh), want_prior=True)
    for i in range(n):
        empty = cells[i] == 0
        assert prior[i][empty].tobytes() == oracle.prior(pr[i], cells[i]).tobytes(), i
        assert np.all(prior[i][~empty] == 0.0)


def test_pvnet2_second_seed_full_and_tree_forward_vs_reference(oracle):
    """G4c: weight seed 29 on 288 boards in 16 families (root, 12 children, 5
    grandchildren through the first child) against the reference's own logits,
    value, softmax and prior (tests/golden/make_golden.py part_pvnet2):
    * the full f16x3 forward within 1e-4 (softmax, prior within 1e-4 as well);
    * the incremental tree forward -- roots full, children through pv_dg_kernel (delta
      of the root's accumulators), grandchildren through pv_sib_kernel -- within the
      same 1e-4 of the REFERENCE (not only of the full forward), within 2e-5 of the
      full forward (test_gpu_pvinc.DELTA_TOL), roots bit-identical to it."""
    g = golden("pvnet2")
    sd = weights.init_state_dict(seed=g["weights_seed"])
    w = device.PVWeights(weights.pack_pv_weights(sd), precision="f16x3")
    rows, cells = _fixture_rows(oracle, g)
    n = len(cells)
    meta = np.array([c["parent"] for c in g["cases"]], np.int32)
    ref_lg = _dec(g["logits_f32_b64"], (n, 225))
    ref_v = _dec(g["value_f32_b64"], (n,))
    ref_p = _dec(g["probs_f32_b64"], (n, 225))
    ref_prior = np.frombuffer(base64.b64decode(g["prior_f64_b64"]), np.float64)
    full = device.pv_forward(w, rows, want_prior=True)
    tree = device.pv_forward_tree(w, rows, meta)
    roots = int((meta == -1).sum())
    assert tree[4][1] == roots and tree[4][2] == 12 * roots and tree[4][4] == 5 * roots and tree[4][3] == 0, tree[4]
    for lg, v, pr, prior in (full[:4], tree[:4]):
        assert np.abs(lg - ref_lg).max() < TOL, np.abs(lg - ref_lg).max()
        assert np.abs(v - ref_v).max() < TOL
        assert np.abs(pr - ref_p).max() < TOL
        off = 0
        for i, cl in enumerate(cells):
            k = g["prior_counts"][i]
            empty = cl == 0
            assert int(empty.sum()) == k
            assert np.abs(prior[i][empty] - ref_prior[off:off + k]).max() < TOL, i
            off += k
    from test_gpu_pvinc import _close
    _close(full, tree, n, np.flatnonzero(meta == -1))
