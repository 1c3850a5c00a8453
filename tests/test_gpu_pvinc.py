"""Incremental policy-value forward (gz_pv_forward_tree, csrc/gz_pvinc.hip).

A root child recomputes only the windows around its new stone from the root's
stored maps; every recomputed position takes the full kernel's products in the
full kernel's order, so the outputs -- logits, value, softmax, masked prior --
must equal the full forward's (gz_pv_forward, f16x3) BIT FOR BIT, for children
on every cell (corners and edges clip the windows), several roots in one launch,
deeper nodes (full forward), roots beyond the map capacity (their children fall
back to the full forward), and the leaves of real 200-simulation searches.
"""
import numpy as np
import pytest
import torch

from conftest import SEED
from gzero import boards, weights

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def pvw():
    from gzero.device import PVWeights
    return PVWeights(weights.pack_pv_weights(weights.init_state_dict(0)), precision="f16x3")


def _rows(cells):
    bl, wh = boards.cells_to_words(np.asarray(cells, np.int8).reshape(-1, 225))
    return boards.leaf_words(bl, wh)


def _same(a, b):
    return all(np.array_equal(x, y) for x, y in zip(a, b))


def _root_family(rng, n_stones, mover=None):
    """A root position and its children: one stone of the side to move on every empty cell."""
    cells = np.zeros(225, np.int8)
    idx = rng.choice(225, size=n_stones, replace=False)
    cells[idx[0::2]] = 1
    cells[idx[1::2]] = 2
    mover = mover or (1 if n_stones % 2 == 0 else 2)
    kids = []
    for c in np.flatnonzero(cells == 0):
        k = cells.copy()
        k[c] = mover
        kids.append(k)
    return cells, kids


def test_tree_children_on_every_cell_bitwise(pvw):
    """3 roots (4, 40 and 150 stones) with a child on every empty cell, plus deeper
    nodes: tree forward == full forward, bitwise, on every output."""
    from gzero import device
    rng = np.random.default_rng(SEED)
    cells, meta = [], []
    for ns in (4, 40, 150):
        root, kids = _root_family(rng, ns)
        r = len(cells)
        cells.append(root)
        meta.append(-1)
        cells += kids
        meta += [r] * len(kids)
        for k in kids[:5]:  # grandchildren: two stones from the root -> full forward
            g = k.copy()
            g[np.flatnonzero(g == 0)[0]] = 3 - (1 if ns % 2 == 0 else 2)
            cells.append(g)
            meta.append(-2)
    rows = _rows(cells)
    full = device.pv_forward(pvw, rows, want_prior=True)
    tree = device.pv_forward_tree(pvw, rows, meta)
    assert tree[4] == [3, 3, len(cells) - 3 - 15, 15]
    for name, a, b in zip(("logits", "value", "probs", "prior"), full, tree[:4]):
        bad = np.flatnonzero(~np.all(np.asarray(a).reshape(len(cells), -1) == np.asarray(b).reshape(len(cells), -1),
                                     axis=1))
        assert len(bad) == 0, (name, bad[:10], np.abs(np.asarray(a) - np.asarray(b)).max())


def test_tree_root_capacity_fallback(pvw):
    """root_cap smaller than the number of roots: the roots without a map slot and
    their children take the full forward; results unchanged."""
    from gzero import device
    rng = np.random.default_rng(SEED + 1)
    cells, meta = [], []
    for ns in (10, 11, 60):
        root, kids = _root_family(rng, ns)
        r = len(cells)
        cells.append(root)
        meta.append(-1)
        cells += kids[::7]
        meta += [r] * len(kids[::7])
    rows = _rows(cells)
    full = device.pv_forward(pvw, rows, want_prior=True)
    tree = device.pv_forward_tree(pvw, rows, meta, root_cap=1)
    assert tree[4][0] == 3 and tree[4][1] == 1
    assert _same(full, tree[:4])


def test_tree_forward_of_real_searches_bitwise(pvw):
    """The leaves of 200-simulation searches of 256 self-play slots after a burn-in
    (root children in the parallel phase, deeper nodes in the sequential phase):
    the engine's tree forward equals the full forward of the same leaves, bitwise."""
    from gzero import device
    from gzero.selfplay import SelfPlayEngine
    eng = SelfPlayEngine(n_slots=256, num_simulations=200, beta=0.0, seed=SEED, pv_weights=pvw, plies_per_step=1,
                         pv_mode="tree")
    eng.advance(60)
    for _ in range(2):
        eng.step()
        c = eng.counters()
        n = int(c["leaves"])
        assert c["leaves_dropped"] == 0 and 0 < n <= eng.leaf_cap
        st = eng.tree_stats()
        assert st[1] == st[0] and st[1] + st[2] + st[3] == n and st[2] > 0.5 * n
        rows = eng.d_leaves[: n * 16].cpu().numpy().view(np.uint32).reshape(n, 16)
        full = device.pv_forward(pvw, rows, want_prior=True)
        got = (eng.d_logits[: n * 225].cpu().numpy().reshape(n, 225), eng.d_value[:n].cpu().numpy(),
               eng.d_probs[: n * 225].cpu().numpy().reshape(n, 225), eng.d_prior[: n * 225].cpu().numpy().reshape(n, 225))
        assert _same(full, got)
