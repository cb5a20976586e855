#!/usr/bin/env python3
"""Golden counts for utils.compute_num_states (src/tile_match_gym/utils/utils.py:6-26).

Runs ONLY in the build container (it reads /root/reference).  It imports the
reference with make_goldens.py's inert stand-ins and calls the reference's own
`is_valid_state` on every colouring (itertools.product order, as
compute_num_states does — single process instead of its multiprocessing pool),
recording (sum of has_poss_move and no matches, sum of no matches) per shape
into tests/golden/fn_count_states.npz (data only).

The hard-coded counts in the comment block of utils.py:33-46 do not match the
reference's current code for the playable column (e.g. (3, 3, 2) is listed
as (94, 102)); the fixture holds what the current code returns.

Usage:  python tests/golden/make_count_states.py
"""
from __future__ import annotations

import os
import sys
import time
from itertools import product

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from make_goldens import install_stubs  # noqa: E402

SHAPES = [(3, 2, 2), (3, 2, 3), (3, 3, 2), (4, 3, 2), (3, 3, 3), (2, 4, 3), (5, 2, 3), (3, 4, 2)]


def main():
    install_stubs()
    from tile_match_gym.board import Board
    from tile_match_gym.utils.utils import is_valid_state
    rows = []
    for (R, C, k) in SHAPES:
        t0 = time.time()
        board = Board(R, C, k, [], [], np.random.default_rng(0))     # as compute_num_states, utils.py:8-9
        board.board = np.ones((2, R, C), dtype=np.int32)
        playable = line_free = 0
        for b in product(range(1, k + 1), repeat=R * C):
            a, c = is_valid_state(R, C, board, b)
            playable += int(a)
            line_free += int(c)
        rows.append((R, C, k, playable, line_free))
        print(f"{(R, C, k)}: ({playable}, {line_free})  {time.time() - t0:.1f}s", flush=True)
    arr = np.array(rows, dtype=np.int64)
    np.savez(os.path.join(HERE, "fn_count_states.npz"), shapes=arr[:, :3], playable=arr[:, 3], line_free=arr[:, 4])


if __name__ == "__main__":
    main()
