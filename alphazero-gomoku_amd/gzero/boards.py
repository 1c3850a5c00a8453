"""Host-side conversions between the reference's board representation and the
device bit planes (layout: include/gzero.h; row r in word r>>1, bit
(r&1)*16 + c).

The reference stores a board as an int array with 0 empty / 1 black / 2 white
(gomoku_board.py:47) and feeds the network three float planes
[black, white, empty] (gomoku_board.py:239-260).
"""
import numpy as np

N = 15
CELLS = 225

STATE_DTYPE = np.dtype([("black", "<u4", (8,)), ("white", "<u4", (8,)), ("n_moves", "<i4"),
                        ("player", "<i4"), ("over", "<i4"), ("winner", "<i4")])
assert STATE_DTYPE.itemsize == 80

RECORD_DTYPE = np.dtype([("black", "<u4", (8,)), ("white", "<u4", (8,)), ("game_id", "<i8"),
                         ("ply", "<i2"), ("move", "<i2"), ("player", "i1"), ("z", "i1"), ("pad", "i1", (2,))])
assert RECORD_DTYPE.itemsize == 80

_idx = np.arange(CELLS)
_bit = (_idx // N) * 16 + (_idx % N)
_word = _bit >> 5
_shift = (_bit & 31).astype(np.uint64)


def cells_to_words(cells):
    """[..., 225] cells (0/1/2) -> (black, white) uint32 words [..., 8]."""
    cells = np.asarray(cells)
    lead = cells.shape[:-1]
    c = cells.reshape(-1, CELLS)
    out = []
    for colour in (1, 2):
        bits = (c == colour).astype(np.uint64) << _shift[None, :]
        w = np.zeros((c.shape[0], 8), np.uint64)
        for k in range(8):
            w[:, k] = bits[:, _word == k].sum(axis=1)
        out.append(w.astype(np.uint32).reshape(lead + (8,)))
    return out[0], out[1]


def words_to_cells(black, white):
    """(black, white) uint32 words [..., 8] -> cells int8 [..., 225]."""
    black = np.asarray(black, dtype=np.uint32)
    white = np.asarray(white, dtype=np.uint32)
    lead = black.shape[:-1]
    b = black.reshape(-1, 8).astype(np.uint64)
    w = white.reshape(-1, 8).astype(np.uint64)
    bb = (b[:, _word] >> _shift[None, :]) & 1
    ww = (w[:, _word] >> _shift[None, :]) & 1
    cells = (bb + 2 * ww).astype(np.int8)
    return cells.reshape(lead + (CELLS,))


def make_states(cells, n_moves=None, player=None, over=0, winner=0):
    """Structured gz_board_state array from cell arrays.  By default the move
    count is the stone count and the side to move follows from its parity."""
    cells = np.asarray(cells).reshape(-1, CELLS)
    st = np.zeros(cells.shape[0], STATE_DTYPE)
    st["black"], st["white"] = cells_to_words(cells)
    stones = (cells != 0).sum(axis=1)
    st["n_moves"] = stones if n_moves is None else n_moves
    st["player"] = np.where(stones % 2 == 0, 1, 2) if player is None else player
    st["over"] = over
    st["winner"] = winner
    return st


def leaf_words(black, white):
    """[n, 16] uint32 leaf rows (black words then white words) as the PV kernel reads them."""
    return np.concatenate([np.asarray(black, np.uint32), np.asarray(white, np.uint32)], axis=-1)


def planes_from_cells(cells):
    """Reference network input float32 [n, 3, 15, 15]: [black, white, empty]."""
    c = np.asarray(cells).reshape(-1, N, N)
    return np.stack([(c == 1), (c == 2), (c == 0)], axis=1).astype(np.float32)


def legal_int(mask4):
    """[4] uint64 row-major legal mask -> Python int (bit i = cell i)."""
    m = [int(x) for x in np.asarray(mask4, dtype=np.uint64)]
    return m[0] | (m[1] << 64) | (m[2] << 128) | (m[3] << 192)
