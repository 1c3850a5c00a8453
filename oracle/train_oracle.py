"""TEST INFRASTRUCTURE ONLY -- numpy restatement of the reference's training-set
construction (the checker for gz_dataset_build / gz_dataset_gather).

Only tests/ may import this module; the product never does.  Pinned by the
golden fixtures augment.json.gz (G8: training.augment_sample) and sgd.json.gz
(G9: GomokuSelfPlayDataset sample order, labels, values, planes CRC).

* planes [black, white, empty] of a cell array (training.py:203-210 records
  get_board_tensor, gomoku_board.py:239-260);
* _transform_planes: k counter-clockwise np.rot90 on axes (1, 2), then
  np.flip(axis=2) (training.py:44-51);
* _transform_index: k times (r, c) -> (c, n-1-r), then c -> n-1-c
  (training.py:53-61) -- which does not match the planes for k = 1, 3; the
  corrected map (r, c) -> (n-1-c, r) is the ``fix`` variant;
* GomokuSelfPlayDataset: all records, then 8 samples per chosen record in
  (k_rot 0..3) x (flip False, True) order (training.py:104-124).
"""
import numpy as np

N = 15


def planes_of(cells):
    c = np.asarray(cells).reshape(N, N)
    return np.stack([(c == 1), (c == 2), (c == 0)]).astype(np.float32)


def transform_planes(planes, k, flip):
    x = planes
    for _ in range(k % 4):
        x = np.rot90(x, k=1, axes=(1, 2))
    if flip:
        x = np.flip(x, axis=2)
    return np.ascontiguousarray(x)


def transform_index(idx, k, flip, fix=False):
    r, c = divmod(int(idx), N)
    for _ in range(k % 4):
        r, c = (N - 1 - c, r) if fix else (c, N - 1 - r)
    if flip:
        c = N - 1 - c
    return r * N + c


def dataset_samples(cells, moves, z, sel, fix=False):
    """-> (planes float32 [S,3,15,15], labels int64 [S], values float32 [S])."""
    xs, ys, vs = [], [], []
    for i in range(len(moves)):
        xs.append(planes_of(cells[i]))
        ys.append(int(moves[i]))
        vs.append(float(z[i]))
    for i in sel:
        p = planes_of(cells[i])
        for k in range(4):
            for f in (False, True):
                xs.append(transform_planes(p, k, f))
                ys.append(transform_index(moves[i], k, f, fix))
                vs.append(float(z[i]))
    if not xs:
        return np.zeros((0, 3, N, N), np.float32), np.zeros(0, np.int64), np.zeros(0, np.float32)
    return np.stack(xs), np.asarray(ys, np.int64), np.asarray(vs, np.float32)
