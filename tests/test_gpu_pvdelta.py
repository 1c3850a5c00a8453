"""Delta tree forward of the root children (gz_pv_forward_tree, csrc/gz_pvdg.hip
pv_dg_kernel): a root child's pre-BN accumulators are the root's plus the
convolution of its one-stone input differences.  The network and its f16x3
(fp32-equivalent) arithmetic are the same as the full forward's, the order of the
additions is not, so the outputs are compared within tolerance, stated here:

* against the full f16x3 forward of the same boards: logits and value within
  DELTA_TOL = 2e-5 (measured ~1e-6), softmax within 1e-6, the fp64 masked prior
  within 1e-6 -- and roots and untagged boards (the full kernel) bit for bit the
  same;
* against the REFERENCE (tests/golden pvnet2, weight seed 29): within the
  north star's 1e-4, as the full forward;
* at weights x3 (larger activations and differences) within 1e-4 of torch fp32.
"""
import base64

import numpy as np
import pytest

from conftest import SEED, golden
from gzero import boards, weights
from test_gpu_pvinc import _close, _concat, _grand_family, _root_family, _rows

pytestmark = pytest.mark.gpu

@pytest.fixture(scope="module")
def pvw():
    from gzero.device import PVWeights
    return PVWeights(weights.pack_pv_weights(weights.init_state_dict(0)), precision="f16x3")


def test_delta_children_on_every_cell(pvw):
    """3 roots (4, 40 and 150 stones) with a child on every empty cell (edges and
    corners clip the squares), plus untagged deeper nodes: delta == full forward
    within DELTA_TOL; roots and untagged boards bitwise."""
    from gzero import device
    rng = np.random.default_rng(SEED)
    cells, meta, exact = [], [], []
    for ns in (4, 40, 150):
        root, kids = _root_family(rng, ns)
        r = len(cells)
        exact.append(r)
        cells.append(root)
        meta.append(-1)
        cells += kids
        meta += [r] * len(kids)
        for k in kids[:5]:
            g = k.copy()
            g[np.flatnonzero(g == 0)[0]] = 3 - (1 if ns % 2 == 0 else 2)
            exact.append(len(cells))
            cells.append(g)
            meta.append(-2)
    rows = _rows(cells)
    full = device.pv_forward(pvw, rows, want_prior=True)
    tree = device.pv_forward_tree(pvw, rows, meta)
    assert tree[4] == [3, 3, len(cells) - 3 - 15, 15, 0, 0]
    err = _close(full, tree, len(cells), exact)
    print("delta vs full:", err)


@pytest.mark.parametrize("planner", [False, True])
def test_delta_forward_of_real_searches(pvw, planner):
    """The leaves of 200-simulation searches (fused search: 256 slots; planner
    pipeline, config 4's tags: 64 slots) after a burn-in: the engine's delta forward
    is within DELTA_TOL of the full forward of the same leaves on every leaf."""
    from gzero import device, planner_nets
    from gzero.selfplay import SelfPlayEngine
    kw = dict(n_slots=256, beta=0.0)
    if planner:
        gnw = planner_nets.pack_planner_weights(planner_nets.init_graphnet_state(0), planner_nets.init_dqn_state(1))
        kw = dict(n_slots=64, beta=0.2, planner_steps=2, gn_weights=gnw)
    eng = SelfPlayEngine(num_simulations=200, seed=SEED, pv_weights=pvw, plies_per_step=1, pv_mode="tree", **kw)
    eng.advance(60 if not planner else 40)
    for _ in range(2):
        eng.step()
        c = eng.counters()
        n = int(c["leaves"])
        assert c["leaves_dropped"] == 0 and 0 < n <= eng.leaf_cap
        st = eng.tree_stats()
        assert st[1] == st[0] > 0 and st[1] + st[2] + st[3] + st[4] == n and st[2] > 0.5 * n and st[4] > 0, st
        rows = eng.d_leaves[: n * 16].cpu().numpy().view(np.uint32).reshape(n, 16)
        full = device.pv_forward(pvw, rows, want_prior=True)
        got = (eng.d_logits[: n * 225].cpu().numpy(), eng.d_value[:n].cpu().numpy(),
               eng.d_probs[: n * 225].cpu().numpy(), eng.d_prior[: n * 225].cpu().numpy())
        _close(full, got, n)


def test_delta_pvnet2_vs_reference(oracle):
    """tests/golden pvnet2 (weight seed 29, 288 reference boards in root / 12
    children / 5 grandchildren families): the delta tree forward within 1e-4 of the
    reference's own logits, value, softmax and prior."""
    from gzero import device
    from test_gpu_pvnet import TOL, _dec, _fixture_rows
    g = golden("pvnet2")
    sd = weights.init_state_dict(seed=g["weights_seed"])
    w = device.PVWeights(weights.pack_pv_weights(sd), precision="f16x3")
    rows, cells = _fixture_rows(oracle, g)
    n = len(cells)
    meta = np.array([c["parent"] for c in g["cases"]], np.int32)
    tree = device.pv_forward_tree(w, rows, meta)
    roots = int((meta == -1).sum())
    assert tree[4][2] == 12 * roots and tree[4][4] == 5 * roots, tree[4]
    lg, v, pr, prior = tree[:4]
    assert np.abs(lg - _dec(g["logits_f32_b64"], (n, 225))).max() < TOL
    assert np.abs(v - _dec(g["value_f32_b64"], (n,))).max() < TOL
    assert np.abs(pr - _dec(g["probs_f32_b64"], (n, 225))).max() < TOL
    ref_prior = np.frombuffer(base64.b64decode(g["prior_f64_b64"]), np.float64)
    off = 0
    for i, cl in enumerate(cells):
        k = g["prior_counts"][i]
        empty = cl == 0
        assert np.abs(prior[i][empty] - ref_prior[off:off + k]).max() < TOL, i
        off += k


@pytest.mark.parametrize("scale", [0.1, 3.0])
def test_delta_scaled_weights_vs_torch(scale):
    """Conv weights x0.1 / x3 (small and large activations and differences): the
    delta forward of root children and grandchildren within 1e-4 of a torch fp32
    forward of the same boards."""
    from gzero import device
    sd = weights.init_state_dict(0)
    for k in sd:
        if k.endswith("weight") and "conv" in k and "bn" not in k:
            sd[k] = sd[k] * scale
    w = device.PVWeights(weights.pack_pv_weights(sd), precision="f16x3")
    rng = np.random.default_rng(SEED + 9)
    cells, meta = _concat([_grand_family(rng, 30, [0, 112, 200], every=3), _grand_family(rng, 90, [14, 60], every=4)])
    rows = _rows(cells)
    tree = device.pv_forward_tree(w, rows, meta)
    ref_lg, ref_v = weights.reference_forward(sd, boards.planes_from_cells(np.asarray(cells, np.int8)))
    lscale = max(1.0, float(np.abs(ref_lg).max()))  # as test_gpu_pvnet.test_pv_scaled_conv_weights
    assert np.abs(tree[0] - ref_lg).max() < 1e-4 * lscale, (np.abs(tree[0] - ref_lg).max(), lscale)
    assert np.abs(tree[1] - ref_v).max() < 1e-4
