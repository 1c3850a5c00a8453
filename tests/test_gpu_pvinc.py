"""Incremental policy-value forward (gz_pv_forward_tree, csrc/gz_pvinc.hip).

A root child recomputes only the windows around its new stone from the root's
stored maps; every recomputed position takes the full kernel's products in the
full kernel's order, so the outputs -- logits, value, softmax, masked prior --
must equal the full forward's (gz_pv_forward, f16x3) BIT FOR BIT, for children
on every cell (corners and edges clip the windows), several roots in one launch,
grandchildren (a child of a root child: its windows come from the root's maps
overlaid with the parent's recomputed squares) on every cell around parents at
corners, edges and the centre, deeper nodes (full forward), roots beyond the map
capacity and parents beyond the patch capacity (full forward), and the leaves of
real 200-simulation searches.
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
        for k in kids[:5]:  # untagged grandchildren (meta -2) -> full forward
            g = k.copy()
            g[np.flatnonzero(g == 0)[0]] = 3 - (1 if ns % 2 == 0 else 2)
            cells.append(g)
            meta.append(-2)
    rows = _rows(cells)
    full = device.pv_forward(pvw, rows, want_prior=True)
    tree = device.pv_forward_tree(pvw, rows, meta)
    assert tree[4] == [3, 3, len(cells) - 3 - 15, 15, 0, 0]
    for name, a, b in zip(("logits", "value", "probs", "prior"), full, tree[:4]):
        bad = np.flatnonzero(~np.all(np.asarray(a).reshape(len(cells), -1) == np.asarray(b).reshape(len(cells), -1),
                                     axis=1))
        assert len(bad) == 0, (name, bad[:10], np.abs(np.asarray(a) - np.asarray(b)).max())


def _grand_family(rng, n_stones, parent_cells, every=1):
    """A root, its children on every empty cell, and for the children whose stone is
    on `parent_cells` a grandchild (the other side's stone) on every `every`-th empty
    cell; meta tags as the search writes them."""
    root, kids = _root_family(rng, n_stones)
    mover = 1 if n_stones % 2 == 0 else 2
    empties = np.flatnonzero(root == 0)
    cells, meta = [root], [-1]
    cells += kids
    meta += [0] * len(kids)
    for pc in parent_cells:
        if root[pc] != 0:
            continue
        p = 1 + int(np.flatnonzero(empties == pc)[0])
        for c in np.flatnonzero(cells[p] == 0)[::every]:
            g = cells[p].copy()
            g[c] = 3 - mover
            cells.append(g)
            meta.append(p)
    return cells, meta


def _concat(fams):
    cells, meta = [], []
    for c, m in fams:
        base = len(cells)
        cells += c
        meta += [x + base if x >= 0 else x for x in m]
    return cells, meta


def test_tree_grandchildren_every_cell_bitwise(pvw):
    """Grandchildren on every empty cell around parents at the corners, edges, next
    to each other and in the centre (parent and grandchild windows overlap, clip,
    or are disjoint), under 3 roots: tree forward == full forward, bitwise."""
    from gzero import device
    rng = np.random.default_rng(SEED + 2)
    corners = [0, 14, 210, 224]
    fams = [_grand_family(rng, 6, corners + [112, 113, 97]),
            _grand_family(rng, 41, [7, 105, 119, 217, 16], every=2),
            _grand_family(rng, 120, list(range(0, 225, 11)), every=5)]
    cells, meta = _concat(fams)
    meta_a = np.asarray(meta)
    n_kids = sum(1 for i, m in enumerate(meta) if m >= 0 and meta[m] == -1)
    n_grand = sum(1 for i, m in enumerate(meta) if m >= 0 and meta[m] >= 0)
    n_par = len(np.unique(meta_a[[i for i, m in enumerate(meta) if m >= 0 and meta[m] >= 0]]))
    rows = _rows(cells)
    full = device.pv_forward(pvw, rows, want_prior=True)
    tree = device.pv_forward_tree(pvw, rows, meta)
    assert tree[4] == [3, 3, n_kids, 0, n_grand, n_par], (tree[4], n_kids, n_grand, n_par)
    for name, a, b in zip(("logits", "value", "probs", "prior"), full, tree[:4]):
        bad = np.flatnonzero(~np.all(np.asarray(a).reshape(len(cells), -1) == np.asarray(b).reshape(len(cells), -1),
                                     axis=1))
        assert len(bad) == 0, (name, bad[:10], np.abs(np.asarray(a) - np.asarray(b)).max())


def test_tree_patch_capacity_fallback(pvw):
    """More parents with grandchildren than patch slots (16 per map slot): the
    grandchildren of parents without a slot take the full forward; results unchanged."""
    from gzero import device
    rng = np.random.default_rng(SEED + 3)
    cells, meta = _concat([_grand_family(rng, 30, list(range(0, 225, 3)), every=60)])
    n_grand = sum(1 for m in meta if m >= 0 and meta[m] >= 0)
    n_par = len({m for m in meta if m >= 0 and meta[m] >= 0})
    assert n_par > 32
    rows = _rows(cells)
    full = device.pv_forward(pvw, rows, want_prior=True)
    tree = device.pv_forward_tree(pvw, rows, meta, root_cap=1)
    st = tree[4]
    assert st[5] == n_par and 0 < st[4] < n_grand and st[3] == n_grand - st[4], st
    assert _same(full, tree[:4])


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
        assert st[1] == st[0] and st[1] + st[2] + st[3] + st[4] == n and st[2] > 0.5 * n
        assert st[4] > 0  # grandchildren of parents with a patch slot
        rows = eng.d_leaves[: n * 16].cpu().numpy().view(np.uint32).reshape(n, 16)
        full = device.pv_forward(pvw, rows, want_prior=True)
        got = (eng.d_logits[: n * 225].cpu().numpy().reshape(n, 225), eng.d_value[:n].cpu().numpy(),
               eng.d_probs[: n * 225].cpu().numpy().reshape(n, 225), eng.d_prior[: n * 225].cpu().numpy().reshape(n, 225))
        assert _same(full, got)


def test_tree_forward_of_planner_searches_bitwise(pvw):
    """Config-4 searches (BG-planner rollout plies, beta 0.2): the planner pipeline
    tags its leaves like the fused search (root, root children, their children), and
    the engine's tree forward equals the full forward of the same leaves, bitwise."""
    from gzero import device, planner_nets
    from gzero.selfplay import SelfPlayEngine
    gnw = planner_nets.pack_planner_weights(planner_nets.init_graphnet_state(0), planner_nets.init_dqn_state(1))
    eng = SelfPlayEngine(n_slots=64, num_simulations=200, beta=0.2, seed=SEED, pv_weights=pvw, plies_per_step=1,
                         planner_steps=2, gn_weights=gnw, pv_mode="tree")
    eng.advance(40)
    for _ in range(2):
        eng.step()
        c = eng.counters()
        n = int(c["leaves"])
        assert c["leaves_dropped"] == 0 and 0 < n <= eng.leaf_cap
        st = eng.tree_stats()
        assert st[1] == st[0] > 0 and st[1] + st[2] + st[3] + st[4] == n and st[2] > 0.5 * n and st[4] > 0, st
        rows = eng.d_leaves[: n * 16].cpu().numpy().view(np.uint32).reshape(n, 16)
        full = device.pv_forward(pvw, rows, want_prior=True)
        got = (eng.d_logits[: n * 225].cpu().numpy().reshape(n, 225), eng.d_value[:n].cpu().numpy(),
               eng.d_probs[: n * 225].cpu().numpy().reshape(n, 225), eng.d_prior[: n * 225].cpu().numpy().reshape(n, 225))
        assert _same(full, got)


def test_tree_wrong_tags_take_the_full_forward(pvw):
    """The tags are the caller's claim: a 'child' two stones from its root, a
    'grandchild' of such a node, and a node tagged with a non-root, non-child
    parent take the full forward -- the outputs stay bitwise those of the full
    forward; only the valid children are incremental."""
    from gzero import device
    rng = np.random.default_rng(SEED + 4)
    root, kids = _root_family(rng, 20)
    mover = 1  # 20 stones: black to move
    cells, meta = [root], [-1]
    cells += kids[:40]
    meta += [0] * 40
    bad = []
    for k in kids[40:50]:  # two stones more than the root, tagged as its children
        g = k.copy()
        g[np.flatnonzero(g == 0)[0]] = 3 - mover
        bad.append(len(cells))
        cells.append(g)
        meta.append(0)
    for p in bad[:3]:  # children of the invalid nodes
        g = cells[p].copy()
        g[np.flatnonzero(g == 0)[-1]] = mover
        cells.append(g)
        meta.append(p)
    g = cells[1].copy()  # valid grandchild of a valid child ...
    g[np.flatnonzero(g == 0)[-1]] = 3 - mover
    cells.append(g)
    meta.append(1)
    g2 = g.copy()  # ... and a node tagged with that grandchild as its parent (depth 3)
    g2[np.flatnonzero(g2 == 0)[-1]] = mover
    cells.append(g2)
    meta.append(len(cells) - 2)
    rows = _rows(cells)
    full = device.pv_forward(pvw, rows, want_prior=True)
    tree = device.pv_forward_tree(pvw, rows, meta)
    st = tree[4]
    assert st[:5] == [1, 1, 40, 10 + 3 + 1, 1], st
    assert _same(full, tree[:4])
