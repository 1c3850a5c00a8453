"""Incremental policy-value forward (gz_pv_forward_tree: csrc/gz_pvdg.hip for the
root children, csrc/gz_pvinc.hip for the grandchildren and the classification).

Roots and every board the tree forward runs through the full kernel (untagged nodes,
roots beyond the map capacity and their children, children of parents beyond the
patch capacity, wrongly tagged nodes) must equal the full forward (gz_pv_forward,
f16x3) BIT FOR BIT.  Root children are the root's pre-BN accumulators plus the
convolution of their input differences and grandchildren are computed from their
parent's recomputed squares: the same network in the same f16x3 arithmetic, the
additions in another order, so they are compared within the tolerance stated here:
logits and value within DELTA_TOL = 2e-5 of the full forward (measured ~2e-7),
softmax and the fp64 masked prior within 1e-6.  Covered: grandchildren on every
cell around parents at corners, edges and the centre, both capacity fallbacks and
wrong tags; children on every cell, real searches and the reference fixtures are in
tests/test_gpu_pvdelta.py.
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


DELTA_TOL = 2e-5


def _close(full, got, n, exact_rows=(), tol=DELTA_TOL):
    """Every row within the tolerance; the rows in exact_rows bitwise."""
    lg, v, p, pr = (np.asarray(x).reshape(n, -1) for x in got[:4])
    flg, fv, fp, fpr = (np.asarray(x).reshape(n, -1) for x in full[:4])
    err = {"logits": np.abs(lg - flg).max(), "value": np.abs(v - fv).max(), "probs": np.abs(p - fp).max(),
           "prior": np.abs(pr - fpr).max()}
    assert err["logits"] < tol and err["value"] < tol, err
    assert err["probs"] < 1e-6 and err["prior"] < 1e-6, err
    for i in exact_rows:
        assert np.array_equal(lg[i], flg[i]) and np.array_equal(v[i], fv[i]) and np.array_equal(p[i], fp[i]) \
            and np.array_equal(pr[i], fpr[i]), i
    return err


def _bitwise_rows(full, got, n):
    """How many rows equal the full forward bit for bit on every output."""
    eq = np.ones(n, bool)
    for a, b in zip(full[:4], got[:4]):
        eq &= np.all(np.asarray(a).reshape(n, -1) == np.asarray(b).reshape(n, -1), axis=1)
    return int(eq.sum())


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


def test_tree_grandchildren_every_cell(pvw):
    """Grandchildren on every empty cell around parents at the corners, edges, next
    to each other and in the centre (parent and grandchild windows overlap, clip,
    or are disjoint), under 3 roots: within DELTA_TOL of the full forward, roots
    bitwise."""
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
    print("grandchildren vs full:", _close(full, tree, len(cells), np.flatnonzero(meta_a == -1)))


def test_tree_patch_capacity_fallback(pvw):
    """More parents with grandchildren than patch slots (16 per map slot): the
    grandchildren of parents without a slot take the full forward (bitwise), the
    rest within DELTA_TOL."""
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
    _close(full, tree, len(cells))
    assert _bitwise_rows(full, tree, len(cells)) >= st[1] + st[3]


def test_tree_root_capacity_fallback(pvw):
    """root_cap smaller than the number of roots: the roots without a map slot and
    their children take the full forward (bitwise), the rest within DELTA_TOL."""
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
    st = tree[4]
    assert st[0] == 3 and st[1] == 1 and st[2] > 0 and st[3] > 0, st
    _close(full, tree, len(cells))
    assert _bitwise_rows(full, tree, len(cells)) >= st[1] + st[3]


def test_tree_wrong_tags_take_the_full_forward(pvw):
    """The tags are the caller's claim: a 'child' two stones from its root, a
    'grandchild' of such a node, and a node tagged with a non-root, non-child
    parent take the full forward -- their outputs stay bitwise those of the full
    forward; only the valid children and grandchild are incremental (DELTA_TOL)."""
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
    _close(full, tree, len(cells), [0] + bad + list(range(len(cells) - 5, len(cells) - 2)) + [len(cells) - 1])
