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


def test_gnet_sparse_boards_vs_torch(nets):
    """The batched heads run DQN fc0 only over the one-hot k-blocks that hold a stone
    on one of a workgroup's 32 boards (GN_HSKIP): whole workgroups of empty boards (no
    block), single stones in the first / last cell, one colour only, and a workgroup
    mixing them, against the fp32 torch nets."""
    from gzero import device
    _, gsd, dsd, w = nets
    rng = np.random.default_rng(11)
    cells = np.zeros((160, 225), np.int8)  # boards 0-31: empty (a workgroup with no block)
    for i in range(32, 64):  # one stone each, black or white, first and last cells included
        cells[i, [0, 224, 112, (7 * i) % 225][i % 4]] = 1 + (i % 2)
    for i in range(64, 96):  # white only, a few stones
        cells[i, rng.choice(225, size=1 + i % 5, replace=False)] = 2
    cells[96:128] = 0  # half empty, half sparse black
    for i in range(112, 128):
        cells[i, rng.choice(225, size=i % 3 + 1, replace=False)] = 1
    cells[128:160] = rng.choice(3, size=(32, 225), p=[0.9, 0.05, 0.05])
    bl, wh = boards.cells_to_words(cells)
    p, q, lg = device.gn_forward(w, boards.leaf_words(bl, wh))
    lr, pr, qr = planner_nets.reference_forward(gsd, dsd, boards.planes_from_cells(cells))
    np.testing.assert_allclose(lg, lr, rtol=0, atol=1e-4)
    np.testing.assert_allclose(p, pr, rtol=0, atol=1e-6)
    np.testing.assert_allclose(q, qr, rtol=0, atol=1e-4)


GN_TAG = np.dtype([("mode", "<i4"), ("base", "<i4"), ("job", "<i4"), ("cell", "<i4"), ("nst", "<i4"),
                   ("st", "u1", (6,)), ("pad", "u1", (2,)), ("pad2", "<i4")])


def _chain_forward(w, cells, tags, d_slots):
    import torch
    from gzero import _lib, device
    lib = _lib.load()
    n = len(cells)
    bl, wh = boards.cells_to_words(np.asarray(cells, np.int8))
    rows = boards.leaf_words(bl, wh)
    d_b = torch.from_numpy(np.ascontiguousarray(rows, np.uint32).view(np.int32).copy()).cuda()
    d_t = torch.from_numpy(np.ascontiguousarray(tags).view(np.uint8).copy()).cuda()
    d_p = torch.empty(n * 225, dtype=torch.float32, device="cuda")
    d_q = torch.empty(n * 225, dtype=torch.float32, device="cuda")
    ws = torch.empty(lib.gz_gn_chain_workspace_bytes(n), dtype=torch.uint8, device="cuda")
    _lib.check(lib.gz_gn_forward_chain(device.ptr(w.tensor), device.ptr(d_b), n, device.ptr(d_t),
                                       device.ptr(d_slots), device.ptr(d_p), device.ptr(d_q), device.ptr(ws),
                                       device.stream()), "gz_gn_forward_chain")
    torch.cuda.synchronize()
    p, q, _ = device.gn_forward(w, rows)
    return d_p.cpu().numpy().reshape(n, 225), d_q.cpu().numpy().reshape(n, 225), p, q


def test_incremental_graphnet_chains_bitwise(nets):
    """gn_inc_kernel on explicit chains: bases (full forward, maps kept), then 6 plies
    adding one stone each -- centre, edges and corners, stones near each other and
    far apart, a full forward in the middle of some chains -- p and q bit-identical to
    gz_gn_forward of the same boards at every ply."""
    import torch
    from gzero import _lib
    _, _, _, w = nets
    lib = _lib.load()
    rng = np.random.default_rng(11)
    R = 40
    base = rng.choice(3, size=(R, 225), p=[0.7, 0.15, 0.15]).astype(np.int8)
    base[0] = 0  # the empty board
    d_slots = torch.empty(3 * R * lib.gz_gn_slot_bytes(), dtype=torch.uint8, device="cuda")
    tags = np.zeros(R, GN_TAG)
    tags["mode"], tags["job"] = 0, np.arange(R)
    p, q, pf, qf = _chain_forward(w, base, tags, d_slots)
    assert p.view(np.uint32).tolist() == pf.view(np.uint32).tolist() and (q.view(np.uint32) == qf.view(np.uint32)).all()
    cur = base.copy()
    stones = [[] for _ in range(R)]
    bj = np.zeros(R, bool)
    corners = [0, 14, 210, 224, 7, 105, 119, 217]
    for ply in range(6):
        tags = np.zeros(R, GN_TAG)
        for r in range(R):
            empty = np.flatnonzero(cur[r] == 0)
            pref = [c for c in corners if cur[r][c] == 0]
            c = int(pref[(r + ply) % len(pref)]) if (r % 3 == 0 and pref) else int(rng.choice(empty))
            cur[r][c] = 1 + (ply + r) % 2
            full = r % 5 == 4 and ply == 2  # a full forward inside the chain
            t = tags[r]
            t["job"] = R + r
            if full:
                t["mode"], t["base"] = 0, R + r
                bj[r], stones[r] = True, []
            else:
                t["mode"], t["cell"] = 1, c
                t["base"] = R + r if bj[r] else r
                t["nst"] = 0 if bj[r] else len(stones[r])
                for k, s in enumerate(stones[r]):
                    t["st"][k] = s
                if not bj[r]:
                    stones[r].append(c)
        p, q, pf, qf = _chain_forward(w, cur, tags, d_slots)
        bad = [r for r in range(R) if not ((p[r].view(np.uint32) == pf[r].view(np.uint32)).all()
                                           and (q[r].view(np.uint32) == qf[r].view(np.uint32)).all())]
        if bad:  # which stored map first differs from the full forward's (diagnostics)
            ft = np.zeros(R, GN_TAG)
            ft["mode"], ft["job"] = 0, 2 * R + np.arange(R)
            _chain_forward(w, cur, ft, d_slots)
            sb = lib.gz_gn_slot_bytes()
            raw = d_slots.cpu().numpy()
            r = bad[0]
            job = raw[(R + r) * sb:(R + r + 1) * sb]
            ref = raw[(2 * R + r) * sb:(2 * R + r + 1) * sb]
            c = int(tags[r]["cell"]) if tags[r]["mode"] == 1 else 0
            diag = []
            for m in range(4):
                mj = job[m * 57600:(m + 1) * 57600].view(np.float16).reshape(16, 225, 8)
                mr = ref[m * 57600:(m + 1) * 57600].view(np.float16).reshape(16, 225, 8)
                sq = [pp for pp in range(225) if abs(pp // 15 - c // 15) <= m + 1 and abs(pp % 15 - c % 15) <= m + 1]
                nb = sum(not np.array_equal(mj[:, pp].view(np.uint16), mr[:, pp].view(np.uint16)) for pp in sq)
                diag.append((m, nb, len(sq)))
            pj = job[230400:230400 + 1800].view(np.float32)
            pr_ = ref[230400:230400 + 1800].view(np.float32)
            diag.append(("pol", int((pj.view(np.uint32) != pr_.view(np.uint32)).sum()), float(np.abs(pj - pr_).max())))
            assert not bad, (ply, bad[:8], float(np.abs(p - pf).max()), float(np.abs(q - qf).max()), c, diag)


@pytest.mark.parametrize("n", [1, 17, 700, 5000])
def test_small_launch_heads_bitwise(nets, n):
    """The heads split over output tiles (gn_hn0/1/2_kernel: 16 boards x 4 tiles per
    workgroup, dense fc0 -- the planner's small sequential-round launches) against
    gn_heads_kernel (32 boards, 4 waves, fc0 over the stone-holding k-blocks) on the same
    records: p and q bit for bit.  A launch that asks for logits takes gn_heads_kernel;
    one that does not, below 2 x 32 boards per CU, the split.  Sparse and empty boards
    included."""
    import torch
    from gzero import device
    _, gsd, dsd, w = nets
    rng = np.random.default_rng(23)
    cells = rng.choice(3, size=(n, 225), p=[0.6, 0.2, 0.2]).astype(np.int8)
    cells[: min(n, 40) // 2] = 0
    for i in range(min(n, 40) // 2, min(n, 40)):
        cells[i] = 0
        cells[i, rng.choice(225, size=1 + i % 3, replace=False)] = 1 + i % 2
    bl, wh = boards.cells_to_words(cells)
    d_b = torch.from_numpy(boards.leaf_words(bl, wh).view(np.int32).copy()).cuda()
    d_lg = torch.empty(n * 225, dtype=torch.float32, device="cuda")
    p_big, q_big, _ = device.gn_forward_dev(w, d_b, n, d_logits=d_lg)
    p_big, q_big = p_big.clone(), q_big.clone()
    p_sm, q_sm, _ = device.gn_forward_dev(w, d_b, n)
    torch.cuda.synchronize()
    assert torch.equal(p_sm.view(torch.int32), p_big.view(torch.int32))
    assert torch.equal(q_sm.view(torch.int32), q_big.view(torch.int32))
    _, pr, qr = planner_nets.reference_forward(gsd, dsd, boards.planes_from_cells(cells))
    np.testing.assert_allclose(p_sm.cpu().numpy().reshape(n, 225), pr, rtol=0, atol=1e-6)
    np.testing.assert_allclose(q_sm.cpu().numpy().reshape(n, 225), qr, rtol=0, atol=1e-4)
