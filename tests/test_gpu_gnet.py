"""BG planner nets on the GPU (gz_gn_forward) vs the fp32 torch reference and
the reference's own outputs (tests/golden/gnet.json.gz)."""
import base64

import numpy as np
import pytest

from conftest import golden
from gzero import boards, planner_nets

pytestmark = pytest.mark.gpu


def _dec(s, shape):
    return np.frombuffer(base64.b64decode(s), dtype=np.float32).reshape(shape)


@pytest.fixture(scope="module")
def nets():
    from gzero import device
    g = golden("gnet")
    gsd = planner_nets.init_graphnet_state(g["gn_seed"])
    dsd = planner_nets.init_dqn_state(g["dqn_seed"])
    w = device.GNWeights(planner_nets.pack_planner_weights(gsd, dsd))
    return g, gsd, dsd, w


def _cells(moves):
    c = np.zeros(225, np.int8)
    p = 1
    for m in moves:
        c[m] = p
        p = 3 - p
    return c


def test_gnet_vs_reference_fixture(nets):
    from gzero import device
    g, gsd, dsd, w = nets
    n = len(g["cases"])
    cells = np.stack([_cells(c["moves"]) for c in g["cases"]])
    bl, wh = boards.cells_to_words(cells)
    p, q, lg = device.gn_forward(w, boards.leaf_words(bl, wh))
    np.testing.assert_allclose(lg, _dec(g["logits_f32_b64"], (n, 225)), rtol=0, atol=1e-4)
    np.testing.assert_allclose(p, _dec(g["p_f32_b64"], (n, 225)), rtol=0, atol=1e-6)
    np.testing.assert_allclose(q, _dec(g["q_f32_b64"], (n, 225)), rtol=0, atol=1e-4)


def test_gnet_vs_torch_random(nets):
    from gzero import device
    _, gsd, dsd, w = nets
    rng = np.random.default_rng(5)
    n = 700
    cells = rng.choice(3, size=(n, 225), p=[0.5, 0.25, 0.25]).astype(np.int8)
    cells[0] = 0  # empty board
    cells[1] = 1  # full board
    bl, wh = boards.cells_to_words(cells)
    p, q, lg = device.gn_forward(w, boards.leaf_words(bl, wh))
    planes = boards.planes_from_cells(cells)
    lr, pr, qr = planner_nets.reference_forward(gsd, dsd, planes)
    np.testing.assert_allclose(lg, lr, rtol=0, atol=1e-4)
    np.testing.assert_allclose(p, pr, rtol=0, atol=1e-6)
    np.testing.assert_allclose(q, qr, rtol=0, atol=1e-4)
