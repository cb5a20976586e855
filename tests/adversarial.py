"""Adversarial boards for the general kernels' capacity limits (test helper).

The reference accepts any board a caller writes into `env.board.board`
(board.py:65-74 promotes a 2-D array; the tests in tests/board/ hand-build
boards the same way), and a cascade on such a board can be far larger than on
a generated one.  These boards aim at the LDS lists of the general kernels
(tmg_board.hip ListStore): long special-activation chains (DFS depth), many
first-pass and perpendicular lines (line pool), and whole-board cookie
combinations.  Colour specials carry colours 1..k, cookies colour 0 / type -1.
"""
import numpy as np

MODES = ("laser_sea", "stripes", "cookie_field", "combo_grid")


def adversarial_boards(n, R, C, k, smask, seed, mode):
    rs = np.random.default_rng(seed)
    b = np.zeros((n, 2, R, C), np.int8)
    sp_types = [t for bit, t in ((2, 2), (4, 3), (8, 4)) if smask & bit]
    cookie = bool(smask & 1)
    rr, cc = np.meshgrid(np.arange(R), np.arange(C), indexing="ij")
    for i in range(n):
        col = rs.integers(1, k + 1, (R, C))
        typ = np.ones((R, C), np.int64)
        if mode == "laser_sea":
            # almost every cell a laser / bomb: one activation reaches the whole board depth-first
            if sp_types:
                typ = rs.choice(sp_types, (R, C))
                typ[rs.random((R, C)) < 0.05] = 1
        elif mode == "stripes":
            # two-wide vertical colour stripes with a shifted row: long vertical lines in
            # every column plus 3-long perpendicular runs from each of their cells
            col = 1 + ((cc // 2 + (rr == R - 1)) % k)
            col[rs.random((R, C)) < 0.03] = rs.integers(1, k + 1)
            if sp_types:
                m = rs.random((R, C)) < 0.3
                typ[m] = rs.choice(sp_types, int(m.sum()))
        elif mode == "cookie_field":
            # many cookies among lasers: cookie activations chain through every colour
            if sp_types:
                typ = rs.choice(sp_types, (R, C))
            if cookie:
                m = rs.random((R, C)) < 0.15
                typ[m] = -1
        elif mode == "combo_grid":
            # a single colour with specials everywhere: every swap is a combination
            col[:] = 1 + rs.integers(0, min(k, 2))
            if sp_types:
                typ = rs.choice(sp_types + ([-1] if cookie else []), (R, C))
        col = np.where(typ == -1, 0, col)
        b[i, 0], b[i, 1] = col, typ
    return b


def effective_actions(board):
    """Per board, one action the oracle finds effective (else 0)."""
    from oracle import oracle as orc
    out = np.zeros(board.shape[0], np.int32)
    rs = np.random.default_rng(board.shape[0])
    for i in range(board.shape[0]):
        m, _ = orc.effective_mask(board[i])
        nz = np.nonzero(m)[0]
        if nz.size:
            out[i] = nz[rs.integers(nz.size)]
    return out
