#!/usr/bin/env python3
"""Executed MFMA rows of pv_dg_kernel's tap-skipping gather for 16-row tiles
(v_mfma_f32_16x16x32_f16, shipped) and 32-row tiles (v_mfma_f32_32x32x16_f16, VERDICT r05
item 2b), simulated on the kernel's own row classification (csrc/gz_pvdg.hip dg_rows_all):
rows of a pass = the on-board positions of its nodes' output squares, counting-sorted by the
class (ty-set, tx-set) in the kernel's rank order, cut into tiles, each tile running the
union of its rows' taps.  Chunks: 6 children of a random root with stones on consecutive
empty cells in descending row-major order (the search expands the highest empty cell
first, ai_agent.py:224-249).  Prints executed tile-taps x rows per child."""
import numpy as np

BN = 15
RANK = {7: 0, 3: 1, 1: 2, 6: 3, 2: 4, 4: 5}  # tap sets {-1,0,1},{-1,0},{-1},{0,1},{0},{1}
GROUP = {0: 6, 1: 3, 2: 2, 3: 1}  # nodes per pass of layer L


def pass_rows(cells, L):
    RO, RIN = L + 2, L + 1
    rows = []
    for cell in cells:
        cr, cc = divmod(cell, BN)
        for dy in range(-RO, RO + 1):
            for dx in range(-RO, RO + 1):
                pr, pc = cr + dy, cc + dx
                if not (0 <= pr < BN and 0 <= pc < BN):
                    continue
                ty = tx = 0
                for d in (-1, 0, 1):
                    qy, qx = dy + d, dx + d
                    if -RIN <= qy <= RIN and 0 <= cr + qy < BN:
                        ty |= 1 << (d + 1)
                    if -RIN <= qx <= RIN and 0 <= cc + qx < BN:
                        tx |= 1 << (d + 1)
                if not ty or not tx:
                    continue
                taps = {(a, b) for a in range(3) if ty >> a & 1 for b in range(3) if tx >> b & 1}
                rows.append((RANK[ty] * 6 + RANK[tx], taps))
    rows.sort(key=lambda r: r[0])
    return rows


def tile_taps(rows, T):
    n = 0
    for i in range(0, len(rows), T):
        u = set()
        for _, t in rows[i:i + T]:
            u |= t
        n += len(u)
    return n


def main():
    rng = np.random.default_rng(1)
    tot = {16: 0, 32: 0}
    row_taps = 0
    kids = 0
    for _ in range(400):
        ns = int(rng.integers(4, 80))
        occ = set(rng.choice(225, size=ns, replace=False).tolist())
        empty = [c for c in range(224, -1, -1) if c not in occ]
        s = int(rng.integers(0, len(empty) - 6))
        chunk = empty[s:s + 6]
        for L in range(4):
            g = GROUP[L]
            for k in range(0, 6, g):
                rows = pass_rows(chunk[k:k + g], L)
                row_taps += sum(len(t) for _, t in rows)
                for T in (16, 32):
                    tot[T] += tile_taps(rows, T) * T
        kids += 6
    print(f"per child: ideal row-taps {row_taps / kids:.0f}; executed rows x taps: 16-row tiles "
          f"{tot[16] / kids:.0f} ({tot[16] / 16 / kids:.1f} tile-taps), 32-row tiles {tot[32] / kids:.0f} "
          f"(+{(tot[32] / tot[16] - 1) * 100:.1f} % MFMA work)")


if __name__ == "__main__":
    main()
