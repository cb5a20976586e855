"""What an incremental effective-action mask could skip.

After an effective move, an action's effectiveness can only change if its
window (tile_match_env.py:118-124 -> board.py:735-787: the two swapped cells
and the cells up to two away along both axes) touches a cell the move changed.
The device scan (scan_effective_clean) takes 64 vertical and 64 horizontal
actions per pass, so work is saved only when a whole pass has no such action.
This runs the oracle (random actions, num_moves = 30, autoreset) and reports,
over effective moves: the mean fraction of actions whose window touches a
changed cell, and the fraction of scan passes no changed cell reaches.

    python tools/incremental_mask_stats.py [R C k smask] [--envs 4096 --steps 60]
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tile-match-gym_amd"))
from oracle import oracle as orc                                     # noqa: E402
from tile_match_gym_amd.seeding import batch_rng_words               # noqa: E402


def windows(R, C):
    """[A, R*C] bool: cells of each action's window (the swapped pair +-2 along both axes)."""
    acts = []
    for i in range(C * (R - 1)):                      # vertical actions first (board.py:77-93)
        r, c = divmod(i, C)
        acts.append(((r, c), (r + 1, c)))
    for i in range(R * (C - 1)):
        r, c = divmod(i, C - 1)
        acts.append(((r, c), (r, c + 1)))
    win = np.zeros((len(acts), R * C), bool)
    for a, cells in enumerate(acts):
        for (r, c) in cells:
            for d in range(-2, 3):
                if 0 <= r + d < R:
                    win[a, (r + d) * C + c] = True
                if 0 <= c + d < C:
                    win[a, r * C + c + d] = True
    return win, C * (R - 1)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("shape", nargs="*", type=int, default=[10, 10, 4, 0])
    ap.add_argument("--envs", type=int, default=4096)
    ap.add_argument("--steps", type=int, default=60)
    a = ap.parse_args()
    R, C, k, sm = a.shape
    n = a.envs
    o = orc.OracleBatch(R, C, k, sm, 30, batch_rng_words(range(n)), threads=8)
    o.reset()
    win, nv = windows(R, C)
    A = win.shape[0]
    nh = A - nv
    passes = (max(nv, nh) + 63) // 64
    rs = np.random.default_rng(7)
    touched, skippable, moves = 0.0, np.zeros(passes), 0
    for t in range(a.steps):
        before = o.board.reshape(n, 2, R * C).copy()
        o.step(rs.integers(0, A, n, dtype=np.int32), autoreset=True)
        after = o.board.reshape(n, 2, R * C)
        eff = (o.reward > 0) & ((o.flags & 8) == 0)             # effective, not an episode end
        for e in np.nonzero(eff)[0]:
            ch = (before[e] != after[e]).any(axis=0)
            hit = (win & ch).any(axis=1)                          # [A]
            touched += hit.mean()
            for p in range(passes):
                lo, hi = 64 * p, 64 * (p + 1)
                if not hit[lo:min(hi, nv)].any() and not hit[nv + lo:nv + min(hi, nh)].any():
                    skippable[p] += 1
            moves += 1
    print(f"{R}x{C} k{k} smask {sm}: {moves} effective moves; actions whose window touches a changed cell: "
          f"{touched / moves:.1%}; scan passes with none (per pass of {passes}): "
          + ", ".join(f"{s / moves:.1%}" for s in skippable))


if __name__ == "__main__":
    main()
