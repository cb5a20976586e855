#!/usr/bin/env python3
"""Golden-vector generator.  Runs ONLY in the build container (it reads
/root/reference, which never travels to the GPU box).

It imports the reference package ``tile_match_gym`` (akshilpatel/tile-match-gym
v1.0.6, ``/root/reference/src``) and records inputs + outputs of the reference
itself into small ``.npz`` fixtures under ``tests/golden/``.  The fixtures are
data only (boards, actions, RNG states, counters, masks); no reference source
is copied.

The reference depends on three packages that are absent in this image:

* ``numba`` (pinned 0.59.1, ``pyproject.toml:18``) — used only as ``@njit`` on
  two pure integer functions (``board.py:729,735``) and for an unused jitclass
  spec (``board.py:28-39``).  ``njit`` is replaced by the identity decorator,
  which is semantically exact for those functions.
* ``gymnasium`` (``pyproject.toml:17``) — ``TileMatchEnv`` subclasses
  ``gym.Env`` and builds ``spaces``.  A minimal inert stand-in supplies
  ``Env`` (with the lazily created ``np_random`` property) and the space
  constructors.  None of it is on the transition path.
* ``pygame`` — imported by ``renderer.py`` only; an empty module.

Usage:  python tests/golden/make_goldens.py  [--quick]
"""
from __future__ import annotations

import argparse
import os
import signal
import sys
import tempfile
import textwrap
import time

import numpy as np

REF_SRC = "/root/reference/src"
OUT_DIR = os.path.dirname(os.path.abspath(__file__))

TYPE_CODE = {"normal": 0, "vertical_laser": 1, "horizontal_laser": 2, "bomb": 3, "cookie": 4}
SPECIAL_BITS = {"cookie": 1, "vertical_laser": 2, "horizontal_laser": 4, "bomb": 8}


# --------------------------------------------------------------------------
# stub modules (written to a temp dir, prepended to sys.path)
# --------------------------------------------------------------------------
_STUB_NUMBA = '''
def njit(*args, **kwargs):
    if len(args) == 1 and callable(args[0]) and not kwargs:
        return args[0]
    def deco(f):
        return f
    return deco
class _Inert:
    def __getattr__(self, name):
        return _Inert()
    def __call__(self, *a, **k):
        return _Inert()
    def __getitem__(self, k):
        return _Inert()
types = _Inert()
def typeof(x):
    return _Inert()
'''

_STUB_GYM = '''
import numpy as np
from . import spaces
from .core import Env, ObservationWrapper, RewardWrapper
'''
_STUB_GYM_CORE = '''
import numpy as np
class Env:
    _np_random = None
    @property
    def np_random(self):
        if self._np_random is None:
            self._np_random = np.random.default_rng()
        return self._np_random
    @np_random.setter
    def np_random(self, value):
        self._np_random = value
    @property
    def unwrapped(self):
        return self
class Wrapper(Env):
    def __init__(self, env):
        self.env = env
    @property
    def unwrapped(self):
        return self.env.unwrapped
class ObservationWrapper(Wrapper):
    pass
class RewardWrapper(Wrapper):
    pass
'''
_STUB_GYM_SPACES = '''
class _Space:
    def __init__(self, *a, seed=None, **k):
        self.args = a
        self.kwargs = k
class Discrete(_Space):
    def __init__(self, n, seed=None, start=0):
        self.n = n
class Box(_Space):
    pass
class Dict(_Space):
    def __init__(self, d=None, seed=None, **k):
        self.spaces = d
'''
_STUB_GYM_REG = '''
def register(*a, **k):
    pass
'''


def install_stubs() -> str:
    d = tempfile.mkdtemp(prefix="tmg_stubs_")
    os.makedirs(os.path.join(d, "numba"))
    os.makedirs(os.path.join(d, "gymnasium", "envs"))
    os.makedirs(os.path.join(d, "pygame"))
    files = {
        "numba/__init__.py": _STUB_NUMBA,
        "gymnasium/__init__.py": _STUB_GYM,
        "gymnasium/core.py": _STUB_GYM_CORE,
        "gymnasium/spaces.py": _STUB_GYM_SPACES,
        "gymnasium/envs/__init__.py": "",
        "gymnasium/envs/registration.py": _STUB_GYM_REG,
        "pygame/__init__.py": "",
    }
    for rel, txt in files.items():
        with open(os.path.join(d, rel), "w") as f:
            f.write(textwrap.dedent(txt))
    sys.path.insert(0, REF_SRC)
    sys.path.insert(0, d)
    return d


# --------------------------------------------------------------------------
# helpers
# --------------------------------------------------------------------------
def rng_state_words(gen: np.random.Generator) -> np.ndarray:
    """numpy PCG64 state -> 5 uint64 words [state_lo, state_hi, inc_lo, inc_hi, has<<32|uinteger]."""
    st = gen.bit_generator.state
    s = st["state"]["state"]
    inc = st["state"]["inc"]
    m = (1 << 64) - 1
    return np.array([s & m, s >> 64, inc & m, inc >> 64,
                     (int(st["has_uint32"]) << 32) | int(st["uinteger"])], dtype=np.uint64)


def gen_from_words(w) -> np.random.Generator:
    w = [int(x) for x in w]
    bg = np.random.PCG64()
    bg.state = {"bit_generator": "PCG64",
                "state": {"state": w[0] | (w[1] << 64), "inc": w[2] | (w[3] << 64)},
                "has_uint32": w[4] >> 32, "uinteger": w[4] & 0xFFFFFFFF}
    return np.random.Generator(bg)


def specials_lists(mask: int):
    colourless = ["cookie"] if mask & 1 else []
    colour = []
    # order of the list does not matter to the reference (it builds a set, board.py:61)
    if mask & 8:
        colour.append("bomb")
    if mask & 2:
        colour.append("vertical_laser")
    if mask & 4:
        colour.append("horizontal_laser")
    return colourless, colour


class Timeout(Exception):
    pass


def _alarm(signum, frame):
    raise Timeout()


signal.signal(signal.SIGALRM, _alarm)


def encode_lines(lines, C):
    """list of lines (lists of (r,c)) -> (lengths int16[n], cells int16[sum])."""
    lens = np.array([len(l) for l in lines], dtype=np.int16)
    cells = np.array([r * C + c for l in lines for (r, c) in l], dtype=np.int16)
    return lens, cells


def random_board(rs: np.random.Generator, R, C, k, smask, p_special=0.12, p_cookie=0.04, p_ccookie=0.01, p_empty=0.0):
    col = rs.integers(1, k + 1, size=(R, C))
    typ = np.ones((R, C), dtype=np.int64)
    allowed = [t for t, b in ((2, 2), (3, 4), (4, 8)) if smask & b]
    u = rs.random((R, C))
    if allowed:
        sp = u < p_special
        typ[sp] = rs.choice(allowed, size=int(sp.sum()))
    if smask & 1:
        ck = (u >= p_special) & (u < p_special + p_cookie)
        typ[ck] = -1
        col[ck] = 0
        cc = (u >= p_special + p_cookie) & (u < p_special + p_cookie + p_ccookie)
        typ[cc] = -1  # coloured cookie: reachable via remove_colour_lines (board.py:128-129)
    if p_empty > 0:
        e = rs.random((R, C)) < p_empty
        col[e] = 0
        typ[e] = 0
    return np.array([col, typ], dtype=np.int32)


SHAPES = [
    # R, C, k, specials mask
    (3, 4, 3, 15), (4, 5, 4, 15), (5, 5, 3, 15), (6, 6, 4, 15), (8, 8, 3, 15),
    (10, 10, 4, 15), (10, 10, 4, 14), (10, 10, 4, 0), (7, 9, 5, 15), (9, 7, 3, 15),
    (6, 6, 4, 2), (6, 6, 4, 4), (6, 6, 4, 8), (6, 6, 4, 1), (6, 6, 4, 3), (6, 6, 4, 9),
    (5, 8, 2, 15), (12, 12, 6, 15), (20, 20, 6, 15), (3, 3, 3, 15), (4, 3, 5, 0),
]


# --------------------------------------------------------------------------
# function-level goldens
# --------------------------------------------------------------------------
def gen_function_goldens(n_per_shape: int, seed: int = 777):
    from tile_match_gym.board import Board, is_move_effective
    rs = np.random.default_rng(seed)

    recs = {k: [] for k in ("lines", "effective", "gravity", "activate", "combo", "resolve", "move", "generate")}

    for (R, C, k, smask) in SHAPES:
        cl, co = specials_lists(smask)
        for it in range(n_per_shape):
            # ---------------- get_colour_lines / process_colour_lines ----------
            dense = rs.random() < 0.5
            b0 = random_board(rs, R, C, k if not dense else max(2, k - 1), smask)
            b = Board(R, C, k, cl, co, np.random.default_rng(0), board=b0.copy())
            lines = b.get_colour_lines()
            lens, cells = encode_lines(lines, C)
            try:
                pcoords, pnames, pcols = b.process_colour_lines([list(l) for l in lines]) if lines else ([], [], [])
                perr = 0
            except Exception:
                pcoords, pnames, pcols, perr = [], [], [], 1
            plens, pcells = encode_lines(pcoords, C)
            recs["lines"].append(dict(shape=(R, C, k, smask), board=b0.astype(np.int8), lens=lens, cells=cells,
                                      plens=plens, pcells=pcells,
                                      pnames=np.array([TYPE_CODE[n] for n in pnames], np.int8),
                                      pcols=np.array([int(x) for x in pcols], np.int8), perr=perr))

            # ---------------- is_move_effective / possible_move --------------
            b0 = random_board(rs, R, C, k, smask, p_special=0.05, p_cookie=0.03, p_ccookie=0.02)
            b = Board(R, C, k, cl, co, np.random.default_rng(0), board=b0.copy())
            eff = np.array([bool(is_move_effective(b.board, c1, c2)) for (c1, c2) in b.action_to_coords], dtype=bool)
            assert np.array_equal(b.board, b0)
            recs["effective"].append(dict(shape=(R, C, k, smask), board=b0.astype(np.int8), eff=eff,
                                          possible=bool(b.possible_move())))

            # ---------------- gravity ----------------------------------------
            b0 = random_board(rs, R, C, k, smask, p_empty=0.3)
            b = Board(R, C, k, cl, co, np.random.default_rng(0), board=b0.copy())
            b.gravity()
            recs["gravity"].append(dict(shape=(R, C, k, smask), board=b0.astype(np.int8), out=b.board.astype(np.int8)))

            # ---------------- activate_special --------------------------------
            if smask & 14 or smask & 1:
                b0 = random_board(rs, R, C, k, smask, p_special=0.2, p_cookie=0.05, p_ccookie=0.02)
                spec = np.argwhere((b0[1] != 0) & (b0[1] != 1))
                if len(spec):
                    r, c = spec[rs.integers(len(spec))]
                    combo = bool(rs.random() < 0.2)
                    b = Board(R, C, k, cl, co, np.random.default_rng(0), board=b0.copy())
                    b.num_specials_activated = 0
                    b.activate_special((int(r), int(c)), int(b0[1, r, c]), int(b0[0, r, c]), combo)
                    recs["activate"].append(dict(shape=(R, C, k, smask), board=b0.astype(np.int8), cell=int(r * C + c),
                                                 combo=int(combo), out=b.board.astype(np.int8),
                                                 n_act=int(b.num_specials_activated)))

            # ---------------- combination_match ------------------------------
            if smask:
                b0 = random_board(rs, R, C, k, smask, p_special=0.25, p_cookie=0.08, p_ccookie=0.02)
                coords_tab = Board(R, C, k, cl, co, np.random.default_rng(0), board=b0.copy()).action_to_coords
                acts = [a for a, (c1, c2) in enumerate(coords_tab)
                        if (b0[1][c1] not in (0, 1) and b0[1][c2] not in (0, 1)) or b0[1][c1] < 0 or b0[1][c2] < 0]
                if acts:
                    a = acts[rs.integers(len(acts))]
                    c1, c2 = coords_tab[a]
                    b = Board(R, C, k, cl, co, np.random.default_rng(0), board=b0.copy())
                    b.num_specials_activated = 0
                    b.combination_match(c1, c2)
                    recs["combo"].append(dict(shape=(R, C, k, smask), board=b0.astype(np.int8), action=a,
                                              out=b.board.astype(np.int8), n_act=int(b.num_specials_activated)))

            # ---------------- detect + resolve (one cascade iteration) -------
            b0 = random_board(rs, R, C, max(2, k - 1), smask, p_special=0.1, p_cookie=0.03, p_ccookie=0.01)
            b = Board(R, C, k, cl, co, np.random.default_rng(0), board=b0.copy())
            b.num_specials_activated = 0
            b.num_new_specials = 0
            try:
                locs, names, cols = b.detect_colour_matches()
                if locs:
                    b.resolve_colour_matches(locs, names, cols)
                err = 0
            except Exception:
                err = 1
            recs["resolve"].append(dict(shape=(R, C, k, smask), board=b0.astype(np.int8), out=b.board.astype(np.int8),
                                        n_act=int(b.num_specials_activated), n_new=int(b.num_new_specials), err=err))

            # ---------------- full move() incl. refill RNG + ensure-playable --
            gseed = int(rs.integers(1 << 31))
            g = np.random.default_rng(gseed)
            b = Board(R, C, k, cl, co, g)
            try:
                signal.alarm(20)
                b.generate_board()
                signal.alarm(0)
            except Timeout:
                signal.alarm(0)
                continue
            gen_board = b.board.copy()
            # sprinkle specials onto the generated board to exercise every branch
            bb = random_board(rs, R, C, k, smask, p_special=0.15, p_cookie=0.05, p_ccookie=0.015)
            sp = (bb[1] != 1) & (rs.random((R, C)) < 0.7)
            start = gen_board.copy()
            start[:, sp] = bb[:, sp]
            # fill some cells with a second random colouring so that matches exist
            if rs.random() < 0.3:
                m = rs.random((R, C)) < 0.3
                start[0][m & (start[1] > 0)] = rs.integers(1, k + 1, size=int((m & (start[1] > 0)).sum()))
            b.board = start.copy()
            eff = [a for a, (c1, c2) in enumerate(b.action_to_coords) if is_move_effective(b.board, c1, c2)]
            A = len(b.action_to_coords)
            a = eff[rs.integers(len(eff))] if (eff and rs.random() < 0.85) else int(rs.integers(A))
            rng_in = rng_state_words(b.np_random)
            c1, c2 = b.action_to_coords[a]
            try:
                signal.alarm(20)
                out = b.move(c1, c2)
                signal.alarm(0)
                err = 0
            except Timeout:
                signal.alarm(0)
                continue
            except Exception:
                signal.alarm(0)
                out, err = (0, False, 0, 0, False), 1
            recs["move"].append(dict(shape=(R, C, k, smask), board=start.astype(np.int8), action=a, rng_in=rng_in,
                                     out=b.board.astype(np.int8), rng_out=rng_state_words(b.np_random),
                                     res=np.array([int(out[0]), int(out[1]), int(out[2]), int(out[3]), int(out[4])], np.int32),
                                     err=err))
            if it < max(2, n_per_shape // 4):
                recs["generate"].append(dict(shape=(R, C, k, smask), seed=gseed, out=gen_board.astype(np.int8)))
    return recs


def pack_records(recs, path):
    """Store a list of heterogeneous dict records as concatenated arrays + offsets."""
    out = {}
    if not recs:
        return
    keys = recs[0].keys()
    out["n"] = np.array(len(recs))
    for key in keys:
        vals = [r[key] for r in recs]
        if key == "shape":
            out["shape"] = np.array(vals, dtype=np.int32)
            continue
        arrs = [np.asarray(v) for v in vals]
        if all(a.ndim == 0 for a in arrs):
            out[key] = np.array([a.item() for a in arrs]) if arrs[0].dtype != np.uint64 else np.array([int(a) for a in arrs], np.uint64)
            continue
        flat = [a.reshape(-1) for a in arrs]
        out[key] = np.concatenate(flat) if flat else np.zeros(0)
        out[key + "_off"] = np.concatenate([[0], np.cumsum([f.size for f in flat])]).astype(np.int64)
    np.savez_compressed(path, **out)


# --------------------------------------------------------------------------
# env trajectories (TileMatchEnv.reset/step, tile_match_env.py:84-112)
# --------------------------------------------------------------------------
def gen_trajectory(name, R, C, k, num_moves, smask, seeds, n_steps, act_seed, p_eff=0.5, actions_fixed=None):
    from tile_match_gym.tile_match_env import TileMatchEnv
    cl, co = specials_lists(smask)
    A = 2 * R * C - R - C
    ev_env, ev_kind, ev_action, ev_reward, ev_flags, ev_nnew, ev_nact = [], [], [], [], [], [], []
    ev_board, ev_eff, ev_rng = [], [], []
    init_rng = []
    ars = np.random.default_rng(act_seed)
    for e, seed in enumerate(seeds):
        env = TileMatchEnv(R, C, k, num_moves, cl, co, seed=int(seed))
        init_rng.append(rng_state_words(env.board.np_random))
        obs, info = env.reset()

        def rec(kind, a, rew, flags, nn, na, eff_list):
            m = np.zeros(A, dtype=bool)
            m[list(eff_list)] = True
            ev_env.append(e); ev_kind.append(kind); ev_action.append(a); ev_reward.append(rew)
            ev_flags.append(flags); ev_nnew.append(nn); ev_nact.append(na)
            ev_board.append(env.board.board.astype(np.int8).copy()); ev_eff.append(m)
            ev_rng.append(rng_state_words(env.board.np_random))

        rec(0, -1, 0, 0, 0, 0, info["effective_actions"])
        eff = info["effective_actions"]
        for t in range(n_steps):
            if actions_fixed is not None:
                a = int(actions_fixed[t])
            elif eff and ars.random() < p_eff:
                a = int(eff[ars.integers(len(eff))])
            else:
                a = int(ars.integers(A))
            obs, rew, done, trunc, info = env.step(a)
            flags = int(done) | (int(info["is_combination_match"]) << 1) | (int(info["shuffled"]) << 2)
            rec(1, a, int(rew), flags, int(info["num_new_specials"]), int(info["num_specials_activated"]),
                info["effective_actions"])
            eff = info["effective_actions"]
            if done:
                if t == n_steps - 1:
                    break
                obs, info = env.reset()
                rec(0, -1, 0, 0, 0, 0, info["effective_actions"])
                eff = info["effective_actions"]
    np.savez_compressed(
        os.path.join(OUT_DIR, f"traj_{name}.npz"),
        shape=np.array([R, C, k, smask, num_moves], np.int32), seeds=np.array(seeds, np.int64),
        init_rng=np.array(init_rng, np.uint64),
        env=np.array(ev_env, np.int32), kind=np.array(ev_kind, np.int8), action=np.array(ev_action, np.int32),
        reward=np.array(ev_reward, np.int32), flags=np.array(ev_flags, np.int8),
        n_new=np.array(ev_nnew, np.int32), n_act=np.array(ev_nact, np.int32),
        board=np.array(ev_board, np.int8), eff=np.packbits(np.array(ev_eff, bool), axis=1),
        rng=np.array(ev_rng, np.uint64))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--quick", action="store_true")
    args = ap.parse_args()
    install_stubs()
    import tile_match_gym  # noqa: F401  (registers the gym id through the stub)

    t0 = time.time()
    npf = 6 if args.quick else 40
    recs = gen_function_goldens(npf)
    for key, rs in recs.items():
        pack_records(rs, os.path.join(OUT_DIR, f"fn_{key}.npz"))
        print(f"fn_{key}: {len(rs)} records")
    print(f"function goldens {time.time() - t0:.1f}s")

    q = args.quick
    # BASELINE.json configs[0]: 8x8, 3 colours, no specials, seed=0, 30 random steps (plumbing).
    A1 = 2 * 8 * 8 - 8 - 8
    gen_trajectory("c1_plumbing", 8, 8, 3, 30, 0, [0], 30, 0,
                   actions_fixed=np.random.default_rng(12345).integers(0, A1, 30))
    # reference test scenario tests/test_env.py:5-88 (inputs only; outputs recorded from the reference)
    gen_trajectory("env3x5", 3, 5, 3, 4, 15, [3], 4, 0, actions_fixed=[6, 16, 19, 19])
    cfgs = [
        # name, R, C, k, moves, smask, n_seeds, n_steps
        ("c2_10x10k4", 10, 10, 4, 30, 0, 12, 75),
        ("c3_10x10k4_vhb", 10, 10, 4, 30, 14, 12, 75),
        ("c5_20x20k6_all", 20, 20, 6, 30, 15, 4, 40),
        ("s5x5k3_all", 5, 5, 3, 30, 15, 24, 75),
        ("s6x6k4_cookie", 6, 6, 4, 20, 1, 12, 50),
        ("s6x7k3_v", 6, 7, 3, 20, 2, 12, 50),
        ("s7x6k3_h", 7, 6, 3, 20, 4, 12, 50),
        ("s6x6k3_bomb", 6, 6, 3, 20, 8, 12, 50),
        ("s8x8k3_all", 8, 8, 3, 30, 15, 12, 75),
        ("s4x4k3_all", 4, 4, 3, 10, 15, 24, 40),
    ]
    for (name, R, C, k, mv, sm, ns, st) in cfgs:
        t1 = time.time()
        if q:
            ns, st = max(2, ns // 4), max(10, st // 3)
        gen_trajectory(name, R, C, k, mv, sm, list(range(100, 100 + ns)), st, 4242 + R * 31 + C)
        print(f"traj_{name}: {time.time() - t1:.1f}s")
    print(f"total {time.time() - t0:.1f}s")


if __name__ == "__main__":
    main()
