"""utils.compute_num_states of the reference (src/tile_match_gym/utils/utils.py:6-26),
enumerated on the GPU by libtmg.so's `tmg_count_states` kernel instead of a
multiprocessing pool over itertools.product."""
from __future__ import annotations

from . import _native


def compute_num_states(num_rows, num_cols, num_colours, num_processes=None, colour_specials=(),
                       colourless_specials=(), device: int = 0):
    """(number of line-free boards with a possible move, number of line-free
    boards) over all num_colours^(R*C) colourings of an all-normal board —
    the reference's return value (utils.py:22-24).  `num_processes` and the
    specials are accepted for signature compatibility and unused, as in the
    reference (it builds the Board with no specials, utils.py:8).
    Needs R*C <= 16."""
    return _native.count_states(device, num_rows, num_cols, num_colours)
