#!/usr/bin/env python3
"""Records the reference's OWN hand-built edge cases as fixtures.  Runs ONLY in
the build container (it reads /root/reference, which never travels to the GPU
box).

The reference's board tests (``/root/reference/tests/board/*.py``: test_move.py
:35-337, test_activation.py:9-434, test_combination_match.py:6-417,
test_match_detection.py:15-346, test_gravity, test_refill,
test_resolve_colour_match, test_generate_board, test_move_valid,
test_possible_move) build boards by hand and call Board methods on them.  This
script runs those test functions with the Board methods wrapped by recorders:
every OUTERMOST call (not the nested ones a method makes itself) is stored
with its inputs and the reference's outputs.  The fixtures are data only —
``tests/golden/ref_<kind>.npz`` in the ``fn_<kind>.npz`` record layout of
make_goldens.py, so the same loaders and checks apply:

* move      board, action, rng_in -> out, rng_out, res   (Board.move)
* activate  board, cell, combo -> out, n_act              (activate_special)
* combo     board, action -> out, n_act                   (combination_match)
* lines     board -> get_colour_lines + process_colour_lines
* gravity   board -> out
* effective board -> mask over every action, possible     (is_move_effective)
* generate  rng_in -> out, rng_out                        (generate_board)

A call whose coordinates are given in the reverse of the action table's order
(e.g. combination_match((1, 3), (1, 2))) is kept only when the reference gives
the same result for the table's order, so it can be replayed by action index.
Stand-ins for the absent numba / gymnasium / pygame come from make_goldens.py.

Usage:  python tests/golden/make_ref_cases.py
"""
from __future__ import annotations

import glob
import importlib.util
import os
import sys
import traceback

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import make_goldens as mg  # noqa: E402

REF_TESTS = "/root/reference/tests"

_depth = [0]
RECS = {k: [] for k in ("move", "activate", "combo", "lines", "gravity", "effective", "generate")}
SKIPPED = {"reversed_order_differs": 0, "not_adjacent": 0, "bad_type_arg": 0, "error": 0}


def smask_of(b):
    return sum(mg.SPECIAL_BITS[s] for s in b.specials)


def shape_of(b):
    return (b.num_rows, b.num_cols, b.num_colours, smask_of(b))


def action_of(b, c1, c2):
    """(action, reversed) for a pair of adjacent coords, or (None, None)."""
    c1, c2 = tuple(int(x) for x in c1), tuple(int(x) for x in c2)
    for a, (p, q) in enumerate(b.action_to_coords):
        if (p, q) == (c1, c2):
            return a, False
        if (p, q) == (c2, c1):
            return a, True
    return None, None


def outermost(fn):
    def wrap(*a, **k):
        top = _depth[0] == 0
        _depth[0] += 1
        try:
            return fn(top, *a, **k)
        finally:
            _depth[0] -= 1
    return wrap


def install_recorders():
    import tile_match_gym.board as B
    Board = B.Board
    orig = {n: getattr(Board, n) for n in ("move", "activate_special", "combination_match", "get_colour_lines",
                                            "gravity", "generate_board", "possible_move")}
    orig_eff = B.is_move_effective

    def clone(b):
        c = Board(b.num_rows, b.num_cols, b.num_colours, [s for s in b.specials if s == "cookie"],
                  [s for s in b.specials if s != "cookie"], mg.gen_from_words(mg.rng_state_words(b.np_random)),
                  board=b.board.copy())
        return c

    @outermost
    def move(top, self, c1, c2):
        if not top:
            return orig["move"](self, c1, c2)
        board0 = self.board.astype(np.int8).copy()
        rng0 = mg.rng_state_words(self.np_random)
        a, rev = action_of(self, c1, c2)
        alt = None
        if a is not None and rev:
            t = clone(self)
            p, q = self.action_to_coords[a]
            try:
                alt = (orig["move"](t, p, q), t.board.copy(), mg.rng_state_words(t.np_random))
            except Exception:
                alt = None
        res = orig["move"](self, c1, c2)
        if a is None:
            SKIPPED["not_adjacent"] += 1
            return res
        if rev and (alt is None or alt[0] != res or not np.array_equal(alt[1], self.board)
                    or not np.array_equal(alt[2], mg.rng_state_words(self.np_random))):
            SKIPPED["reversed_order_differs"] += 1
            return res
        RECS["move"].append(dict(shape=shape_of(self), board=board0, action=a, rng_in=rng0,
                                 out=self.board.astype(np.int8).copy(), rng_out=mg.rng_state_words(self.np_random),
                                 res=np.array([int(res[0]), int(res[1]), int(res[2]), int(res[3]), int(res[4])],
                                              np.int32), err=0))
        return res

    @outermost
    def activate_special(top, self, coord, tile_type, tile_colour, is_combination_match=False):
        if not top:
            return orig["activate_special"](self, coord, tile_type, tile_colour, is_combination_match)
        r, c = int(coord[0]), int(coord[1])
        board0 = self.board.astype(np.int8).copy()
        n0 = getattr(self, "num_specials_activated", 0)
        out = orig["activate_special"](self, coord, tile_type, tile_colour, is_combination_match)
        if int(board0[1, r, c]) != int(tile_type) or int(board0[0, r, c]) != int(tile_colour):
            SKIPPED["bad_type_arg"] += 1           # the oracle reads type / colour from the board
            return out
        RECS["activate"].append(dict(shape=shape_of(self), board=board0, cell=r * self.num_cols + c,
                                     combo=int(bool(is_combination_match)), out=self.board.astype(np.int8).copy(),
                                     n_act=int(self.num_specials_activated - n0)))
        return out

    @outermost
    def combination_match(top, self, c1, c2):
        if not top:
            return orig["combination_match"](self, c1, c2)
        board0 = self.board.astype(np.int8).copy()
        n0 = getattr(self, "num_specials_activated", 0)
        a, rev = action_of(self, c1, c2)
        alt = None
        if a is not None and rev:
            t = clone(self)
            t.num_specials_activated = 0
            p, q = self.action_to_coords[a]
            orig["combination_match"](t, p, q)
            alt = (t.board.copy(), t.num_specials_activated)
        out = orig["combination_match"](self, c1, c2)
        if a is None:
            SKIPPED["not_adjacent"] += 1
            return out
        n_act = int(self.num_specials_activated - n0)
        if rev and (not np.array_equal(alt[0], self.board) or alt[1] != n_act):
            SKIPPED["reversed_order_differs"] += 1
            return out
        RECS["combo"].append(dict(shape=shape_of(self), board=board0, action=a, out=self.board.astype(np.int8).copy(),
                                  n_act=n_act))
        return out

    @outermost
    def get_colour_lines(top, self):
        lines = orig["get_colour_lines"](self)
        if top:
            lens, cells = mg.encode_lines(lines, self.num_cols)
            try:
                pc, pn, pcol = self.process_colour_lines([list(l) for l in lines]) if lines else ([], [], [])
                perr = 0
            except Exception:
                pc, pn, pcol, perr = [], [], [], 1
            plens, pcells = mg.encode_lines(pc, self.num_cols)
            RECS["lines"].append(dict(shape=shape_of(self), board=self.board.astype(np.int8).copy(), lens=lens,
                                      cells=cells, plens=plens, pcells=pcells,
                                      pnames=np.array([mg.TYPE_CODE[n] for n in pn], np.int8),
                                      pcols=np.array([int(x) for x in pcol], np.int8), perr=perr))
        return lines

    @outermost
    def gravity(top, self):
        board0 = self.board.astype(np.int8).copy()
        out = orig["gravity"](self)
        if top:
            RECS["gravity"].append(dict(shape=shape_of(self), board=board0, out=self.board.astype(np.int8).copy()))
        return out

    @outermost
    def generate_board(top, self):
        rng0 = mg.rng_state_words(self.np_random)
        out = orig["generate_board"](self)
        if top:
            RECS["generate"].append(dict(shape=shape_of(self), rng_in=rng0, out=self.board.astype(np.int8).copy(),
                                         rng_out=mg.rng_state_words(self.np_random)))
        return out

    def record_effective(self_or_none, board):
        b = np.asarray(board)
        R, C = b.shape[1:]
        if self_or_none is not None:
            shape, coords = shape_of(self_or_none), self_or_none.action_to_coords
        else:
            t = Board(R, C, 4, [], [], np.random.default_rng(0), board=b.copy())
            shape, coords = (R, C, max(1, int(b[0].max())), 0), t.action_to_coords
        eff = np.array([bool(orig_eff(b.copy(), p, q)) for (p, q) in coords], bool)
        RECS["effective"].append(dict(shape=shape, board=b.astype(np.int8).copy(), eff=eff, possible=bool(eff.any())))

    @outermost
    def possible_move(top, self, grid=None):
        out = orig["possible_move"](self, grid)
        if top:
            record_effective(self, self.board if grid is None else grid)
        return out

    @outermost
    def is_move_effective(top, board, c1, c2):
        out = orig_eff(board, c1, c2)
        if top:
            record_effective(None, board)
        return out

    Board.move = move
    Board.activate_special = activate_special
    Board.combination_match = combination_match
    Board.get_colour_lines = get_colour_lines
    Board.gravity = gravity
    Board.generate_board = generate_board
    Board.possible_move = possible_move
    B.is_move_effective = is_move_effective


def run_reference_tests():
    sys.path.insert(0, os.path.dirname(REF_TESTS))
    ran, failed = 0, 0
    for path in sorted(glob.glob(os.path.join(REF_TESTS, "board", "test_*.py"))):
        name = "reftests_" + os.path.splitext(os.path.basename(path))[0]
        spec = importlib.util.spec_from_file_location(name, path)
        mod = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(mod)
        for fn in sorted(n for n in dir(mod) if n.startswith("test")):
            f = getattr(mod, fn)
            if not callable(f):
                continue
            try:
                f()
                ran += 1
            except Exception:
                failed += 1
                SKIPPED["error"] += 1
                print(f"  {os.path.basename(path)}::{fn} raised:", traceback.format_exc().splitlines()[-1])
    return ran, failed


def dedupe(recs):
    seen, out = set(), []
    for r in recs:
        key = tuple((k, np.asarray(v).tobytes()) for k, v in sorted(r.items()))
        if key not in seen:
            seen.add(key)
            out.append(r)
    return out


def main():
    mg.install_stubs()
    import tile_match_gym  # noqa: F401
    install_recorders()
    ran, failed = run_reference_tests()
    print(f"reference board tests: {ran} ran, {failed} raised; skipped records: {SKIPPED}")
    for kind, recs in RECS.items():
        recs = dedupe(recs)
        if recs:
            mg.pack_records(recs, os.path.join(HERE, f"ref_{kind}.npz"))
        print(f"ref_{kind}: {len(recs)} records")


if __name__ == "__main__":
    main()
