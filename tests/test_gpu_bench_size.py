"""The headline's timed path pinned at the size it is timed (bench.py config 2):
4096 self-play slots, 200 simulations, beta 0, the tree forward (pv_mode="tree",
f16x3) after the bench's 600-ply burn-in -- the engine bench.py builds, one step.

Every node the searches create (ai_agent.py:522-523, ~745 k leaves) is compared
with the full forward (gz_pv_forward, f16x3) of the same board:

* root children (pv_dg_kernel, csrc/gz_pvdg.hip) and grandchildren
  (pv_sib_kernel, csrc/gz_pvinc.hip): logits and value within DELTA_TOL = 2e-5,
  softmax and the fp64 masked prior (ai_agent.py:564-582) within 1e-6;
* roots and every node the full kernel ran (untagged nodes, capacity
  fallbacks): bit for bit;
* 1,024 sampled leaves against a torch fp32 forward of the reference network
  (neural_network.py:74-91,132-159): logits and value within the north star's
  1e-4.

The capacity-dependent paths are asserted too: every root gets a map slot
(root_cap maps), no tagged node falls back to the full kernel for want of a
patch slot (16 per map slot), and the list sizes add up to the leaf count.
"""
import numpy as np
import pytest
import torch

from conftest import SEED
from gzero import boards, weights

pytestmark = pytest.mark.gpu

DELTA_TOL = 2e-5  # as tests/test_gpu_pvinc.py


def test_bench_workload_every_leaf_vs_full_forward():
    from gzero import _lib
    from gzero.device import PVWeights, ptr, stream
    from gzero.selfplay import SelfPlayEngine
    sd = weights.init_state_dict(0)
    w = PVWeights(weights.pack_pv_weights(sd), precision="f16x3")
    eng = SelfPlayEngine(n_slots=4096, num_simulations=200, c_puct=1.6, exploration=0.05, beta=0.0, seed=SEED,
                         pv_weights=w, plies_per_step=1, pv_mode="tree")
    assert eng.tree
    eng.advance(600)
    eng.step()
    torch.cuda.synchronize()
    c = eng.counters()
    n = int(c["leaves"])
    assert c["leaves_dropped"] == 0 and c["moves"] == 4096 and 600_000 < n <= eng.leaf_cap, (n, c)
    st = eng.tree_stats()  # roots seen, roots with maps, children, full, grandchildren, patches
    meta = eng.d_meta[:n].clone()
    n_roots = int((meta == -1).sum())
    n_other = int((meta == -2).sum())
    fallbacks = st[3] - n_other
    print(f"leaves {n}: roots {st[1]}/{st[0]}, children {st[2]}, grandchildren {st[4]} ({st[5]} patch slots), "
          f"full {st[3]} (untagged {n_other}, capacity fallbacks {fallbacks})")
    assert st[0] == n_roots and st[1] == st[0], "every root has a map slot"
    assert st[1] + st[2] + st[3] + st[4] == n
    assert st[2] > 0.85 * n and st[4] > 0 and st[5] <= 16 * eng.root_cap
    assert fallbacks == 0, "no tagged node took the full kernel for want of a map / patch slot"

    tree = [t.clone() for t in (eng.d_logits[: n * 225], eng.d_value[:n], eng.d_probs[: n * 225],
                                eng.d_prior[: n * 225])]
    lib = eng.lib
    _lib.check(lib.gz_pv_forward(ptr(w.tensor), ptr(eng.d_leaves), eng.leaf_cap, ptr(eng.d_counters[4:8]),
                                 ptr(eng.d_logits), ptr(eng.d_value), ptr(eng.d_probs), ptr(eng.d_prior),
                                 ptr(w.workspace_for(eng.leaf_cap)), w.mode, stream()), "full")
    torch.cuda.synchronize()
    full = (eng.d_logits[: n * 225], eng.d_value[:n], eng.d_probs[: n * 225], eng.d_prior[: n * 225])
    exact = meta < 0  # roots (-1) and untagged (-2) nodes ran the full kernel
    err = {}
    for name, a, b, k in zip(("logits", "value", "probs", "prior"), tree, full, (225, 1, 225, 225)):
        a2, b2 = a.view(n, k), b.view(n, k)
        err[name] = float((a2.double() - b2.double()).abs().max())
        assert torch.equal(a2[exact], b2[exact]), f"{name}: roots / full-kernel nodes not bitwise"
    print("tree vs full forward, max |diff| over", n, "leaves:", err)
    assert err["logits"] < DELTA_TOL and err["value"] < DELTA_TOL, err
    assert err["probs"] < 1e-6 and err["prior"] < 1e-6, err

    # 1,024 sampled leaves (roots, children and grandchildren alike) vs torch fp32
    sel = np.sort(np.random.default_rng(SEED).choice(n, size=1024, replace=False))
    rows = eng.d_leaves[: n * 16].view(n, 16)[torch.from_numpy(sel).cuda()].cpu().numpy().view(np.uint32)
    cells = boards.words_to_cells(rows[:, :8], rows[:, 8:])
    ref_lg, ref_v = weights.reference_forward(sd, boards.planes_from_cells(cells))
    lg = tree[0].view(n, 225)[torch.from_numpy(sel).cuda()].cpu().numpy()
    v = tree[1][torch.from_numpy(sel).cuda()].cpu().numpy()
    e_ref = (float(np.abs(lg - ref_lg).max()), float(np.abs(v - ref_v).max()))
    print("tree vs torch fp32 (1,024 leaves): logits %.2e value %.2e" % e_ref)
    assert e_ref[0] < 1e-4 and e_ref[1] < 1e-4, e_ref
