"""How much work one generate_board is: remove_colour_lines redraws and colours drawn.

A plain numpy restatement of board.py:95-131 (generate_board / remove_colour_lines
with get_colour_lines' first line, :149-193) that counts, per board, the redraw
iterations and the colours drawn (the PCG64 words the stream must advance by).
Statistics only: the device path is checked against tmg_oracle.c, not this.

    python tools/gen_stats.py [--boards 200] [R C k ...]
"""
import argparse

import numpy as np


def first_line_row(b):
    """Row of the first coord of get_colour_lines()[0], or -1 (no line)."""
    R, C = b.shape
    for r in range(R - 1, -1, -1):                 # bottom-up, first row holding a line
        for c in range(C):                         # left to right, vertical first
            if r > 1 and b[r, c] == b[r - 1, c] == b[r - 2, c]:
                s = r - 2
                while s > 0 and b[s - 1, c] == b[r, c]:
                    s -= 1
                return s                           # a vertical line starts at its top
            if c < C - 2 and b[r, c] == b[r, c + 1] == b[r, c + 2]:
                return r
    return -1


def generate(R, C, k, rng):
    b = rng.integers(1, k + 1, (R, C))
    iters, colours = 0, R * C
    while (r := first_line_row(b)) >= 0:
        row = min(R - 1, r + 1)
        b[:row + 1] = rng.integers(1, k + 1, (row + 1, C))
        iters += 1
        colours += (row + 1) * C
    return iters, colours


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--boards", type=int, default=200)
    ap.add_argument("shape", nargs="*", type=int, default=[20, 20, 6, 10, 10, 4])
    a = ap.parse_args()
    rng = np.random.default_rng(1)
    for i in range(0, len(a.shape), 3):
        R, C, k = a.shape[i:i + 3]
        res = np.array([generate(R, C, k, rng) for _ in range(a.boards)])
        print(f"{R}x{C} k{k}: {res[:, 0].mean():.0f} redraws, {res[:, 1].mean():.0f} colours "
              f"({res[:, 1].mean() / 128:.0f} batches of 64 PCG64 outputs) per generate_board, {a.boards} boards")


if __name__ == "__main__":
    main()
