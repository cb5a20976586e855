"""TileMatchEnv — drop-in for the reference's single Gymnasium env
(src/tile_match_gym/tile_match_env.py:14-150), backed by the HIP kernels.

Same constructor, attributes, spaces, reset/step signatures, return values,
info keys and exceptions as the reference.  The board transition runs on the
GPU through libtmg.so (one env = a batch of one); the host keeps a numpy
mirror of the board (`env.board.board`, int32 [2,R,C]) and of the RNG state,
uploaded before and downloaded after every call, so code that edits
`env.board.board` by hand (as tests/test_env.py:91-120 of the reference does)
behaves as with the reference.  Differences: `obs["board"]` is a copy rather
than an alias of the internal array (equality, not identity, is the
contract), and `np_random` returns a Generator snapshot of the device stream.
"""
from __future__ import annotations

from collections import OrderedDict
from typing import List, Optional

import numpy as np
import torch

from . import _native
from .seeding import generator_from_words, rng_words_from_generator, rng_words_from_seed
from .spaces import Box, Dict, Discrete

try:  # the reference subclasses gymnasium.Env (tile_match_env.py:14)
    import gymnasium as _gym
    _EnvBase = _gym.Env
except Exception:  # gymnasium absent in this image
    _EnvBase = object


def action_to_coords(num_rows: int, num_cols: int):
    """board.py:77-93."""
    out = []
    for i in range(2 * num_rows * num_cols - num_rows - num_cols):
        if i < num_cols * (num_rows - 1):
            out.append(((i // num_cols, i % num_cols), (i // num_cols + 1, i % num_cols)))
        else:
            j = i - num_cols * (num_rows - 1)
            out.append(((j // (num_cols - 1), j % (num_cols - 1)), (j // (num_cols - 1), j % (num_cols - 1) + 1)))
    return tuple(out)


class Board:
    """The reference's Board (board.py:41-93) as a host mirror of one device
    board: same constructor and public fields (`board` int32 [2,R,C],
    `np_random`, `specials`, `action_to_coords`, ...), and the transition
    entry points the reference's callers and tests use, run by the HIP kernels
    on a batch of one:

    * `generate_board()` (board.py:95-131) -> tmg_reset,
    * `move(coord1, coord2)` (board.py:330-395) -> tmg_step with an untrusted
      mask (the exact effectiveness test), returning the same 5-tuple,
    * `possible_move()` (board.py:558-569) / `is_move_effective(board, c1, c2)`
      (module level, board.py:735-787) -> tmg_effective.

    `board` and the RNG position are uploaded before and downloaded after
    every call, so hand edits of `board.board` behave as with the reference.
    The order of coord1 / coord2 does not change the reference's result
    (swap_coords and combination_match are symmetric in them), so a move is
    replayed as the action of the table (board.py:77-93) holding that pair."""

    def __init__(self, num_rows, num_cols, num_colours, colourless_specials=("cookie",),
                 colour_specials=("vertical_laser", "horizontal_laser", "bomb"), np_random=None, board=None,
                 device=None, _env=None):
        self.num_rows, self.num_cols, self.num_colours = num_rows, num_cols, num_colours
        self.colourless_specials = list(colourless_specials)
        self.colour_specials = list(colour_specials)
        self.specials = set(self.colourless_specials + self.colour_specials)
        self.rng_words = rng_words_from_generator(np_random if np_random is not None else np.random.default_rng(0))
        if board is not None:                                                # board.py:64-74
            board = np.array(board, dtype=np.int32) if isinstance(board, list) else board
            self.board = np.array([board, np.ones_like(board)]) if len(board.shape) < 3 else board
            self.num_rows, self.num_cols = self.board.shape[1], self.board.shape[2]
        else:
            self.board = np.ones((2, self.num_rows, self.num_cols), dtype=np.int32)
        self.flat_size = int(self.num_rows * self.num_cols)
        self.num_actions = int(2 * self.num_rows * self.num_cols - self.num_rows - self.num_cols)
        self.action_to_coords = action_to_coords(self.num_rows, self.num_cols)
        self._coord_to_action = {c: a for a, c in enumerate(self.action_to_coords)}
        self._env = _env
        self._device = device
        self._dev = None                       # lazily: context + device buffers of a batch of one
        self.num_specials_activated = 0
        self.num_new_specials = 0

    @property
    def np_random(self) -> np.random.Generator:
        return generator_from_words(self.rng_words)

    @np_random.setter
    def np_random(self, gen):
        self.rng_words = rng_words_from_generator(gen)

    # ----------------------------------------------------------- device side
    def _buffers(self):
        if self._dev is None:
            dev = self._device
            if dev is None:
                if not torch.cuda.is_available():
                    raise _native.TmgError("Board needs a HIP device (no CPU fallback)")
                dev = torch.device("cuda", torch.cuda.current_device())
            dev = torch.device(dev)
            R, C = self.num_rows, self.num_cols
            smask = _native.specials_mask(self.colourless_specials, self.colour_specials)
            ctx = _native.Context(dev.index if dev.index is not None else 0, R, C, self.num_colours, smask, 1 << 30)
            kw = dict(device=dev)
            self._dev = dict(dev=dev, ctx=ctx, board=torch.zeros((1, 2, R, C), dtype=torch.int8, **kw),
                             rng=torch.zeros((1, 5), dtype=torch.int64, **kw),
                             timer=torch.zeros(1, dtype=torch.int32, **kw),
                             eff=torch.zeros((1, ctx.mask_words), dtype=torch.int64, **kw),
                             out=torch.zeros((3, 1), dtype=torch.int32, **kw),
                             flags=torch.zeros(1, dtype=torch.uint8, **kw),
                             act=torch.zeros(1, dtype=torch.int32, **kw))
        return self._dev

    def _stream(self, d):
        return torch.cuda.current_stream(d["dev"]).cuda_stream

    def _upload(self, d):
        b = self.board
        if b.shape != (2, self.num_rows, self.num_cols):
            raise ValueError("board has the wrong shape")
        d["board"].copy_(torch.from_numpy(np.ascontiguousarray(b, dtype=np.int8)).unsqueeze(0))
        d["rng"].copy_(torch.from_numpy(self.rng_words.view(np.int64)).unsqueeze(0))

    def _download(self, d):
        self.board = d["board"][0].to(torch.int32).cpu().numpy()
        self.rng_words = d["rng"][0].cpu().numpy().view(np.uint64).copy()

    # -------------------------------------------------------------- methods
    def generate_board(self):                                                # board.py:95-109
        d = self._buffers()
        self._upload(d)
        d["ctx"].reset(1, d["board"].data_ptr(), d["rng"].data_ptr(), d["timer"].data_ptr(), d["eff"].data_ptr(),
                       None, self._stream(d))
        self._download(d)

    def is_move_legal(self, coord1, coord2) -> bool:                         # board.py:242-267
        (r1, c1), (r2, c2) = coord1, coord2
        if not (0 <= r1 < self.num_rows and 0 <= c1 < self.num_cols):
            return False
        if not (0 <= r2 < self.num_rows and 0 <= c2 < self.num_cols):
            return False
        if (r1, c1) == (r2, c2):
            return False
        return (r1 == r2 or c1 == c2) and abs(r1 - r2) <= 1 and abs(c1 - c2) <= 1

    def move(self, coord1, coord2):                                          # board.py:330-395
        self.num_specials_activated = 0
        self.num_new_specials = 0
        if not self.is_move_legal(coord1, coord2):
            raise ValueError(f"Invalid move: {coord1}, {coord2}")
        key = (tuple(int(x) for x in coord1), tuple(int(x) for x in coord2))
        a = self._coord_to_action.get(key)
        if a is None:
            a = self._coord_to_action[(key[1], key[0])]
        d = self._buffers()
        self._upload(d)
        d["timer"].zero_()
        d["act"].fill_(a)
        out = d["out"]
        d["ctx"].step(1, d["board"].data_ptr(), d["rng"].data_ptr(), d["timer"].data_ptr(), d["act"].data_ptr(),
                      out[0].data_ptr(), out[1].data_ptr(), out[2].data_ptr(), d["flags"].data_ptr(),
                      d["eff"].data_ptr(), 0, 0, self._stream(d))
        self._download(d)
        o = out[:, 0].cpu().numpy()
        flags = int(d["flags"][0].item())
        if flags & (_native.FLAG_ERROR | _native.FLAG_OVERFLOW):
            raise _native.TmgError("device reported an error for this move")
        self.num_new_specials, self.num_specials_activated = int(o[1]), int(o[2])
        return (int(o[0]), bool(flags & _native.FLAG_COMBO), self.num_new_specials, self.num_specials_activated,
                bool(flags & _native.FLAG_SHUFFLED))

    def effective_actions(self) -> List[int]:
        """Ascending actions a with is_move_effective(board, *action_to_coords[a])."""
        return _effective_actions(self.board, self._device)

    def possible_move(self, grid=None) -> bool:                              # board.py:558-569
        """Whether any of THIS board's actions (self.action_to_coords, in index
        order) is effective on `grid` (default: self.board), as the reference
        loops over its own action table whatever grid is passed: a grid of
        another shape is checked at those coordinates, and one that is too
        small for them raises IndexError where numpy would."""
        if grid is None:
            return bool(_effective_actions(self.board, self._device))
        g = np.asarray(grid)
        if g.ndim == 2:                                                      # board.py:64-74 promotion
            g = np.array([g, np.ones_like(g)])
        R, C = g.shape[1], g.shape[2]
        if (R, C) == (self.num_rows, self.num_cols):
            return bool(_effective_actions(g, self._device))
        eff = set(_effective_actions(g, self._device)) if R * C > 1 else set()
        for (r1, c1), (r2, c2) in self.action_to_coords:
            if max(r1, r2) >= R or max(c1, c2) >= C:
                raise IndexError(f"action {((r1, c1), (r2, c2))} is outside a {R}x{C} grid")
            a = r1 * C + c1 if c1 == c2 else C * (R - 1) + r1 * (C - 1) + c1      # the grid's own action index
            if a in eff:
                return True
        return False


def _effective_actions(board, device=None) -> List[int]:
    """is_move_effective (board.py:735-787) for every action of one board of
    any shape, on the device (effective_kernel) through a cached scan-only
    context (tmg_create_scan: no viability test, like the reference, which
    accepts any board here)."""
    b = np.asarray(board)
    if b.ndim == 2:                                                          # board.py:64-74 promotion
        b = np.array([b, np.ones_like(b)])
    if device is None:
        if not torch.cuda.is_available():
            raise _native.TmgError("is_move_effective needs a HIP device (no CPU fallback)")
        device = torch.device("cuda", torch.cuda.current_device())
    device = torch.device(device)
    idx = device.index if device.index is not None else 0
    R, C = b.shape[1], b.shape[2]
    ctx = _native.scan_context(idx, R, C)
    d_board = torch.from_numpy(np.ascontiguousarray(b, dtype=np.int8)).unsqueeze(0).to(device)
    d_eff = torch.zeros((1, ctx.mask_words), dtype=torch.int64, device=device)
    ctx.effective(1, d_board.data_ptr(), d_eff.data_ptr(), torch.cuda.current_stream(device).cuda_stream)
    w = d_eff[0].cpu().numpy().view(np.uint64)
    bits = np.unpackbits(w.view(np.uint8), bitorder="little")[:ctx.num_actions]
    return [int(a) for a in np.nonzero(bits)[0]]


def is_move_effective(board, coord1, coord2) -> bool:
    """board.py:735-787 on the device (effective_kernel) for one board and one
    pair of adjacent coords.  The board may hold any colours / types and have
    any shape; the answer does not depend on the colour count or the enabled
    specials."""
    b = np.asarray(board)
    R, C = b.shape[-2], b.shape[-1]
    table = {c: a for a, c in enumerate(action_to_coords(R, C))}
    key = (tuple(int(x) for x in coord1), tuple(int(x) for x in coord2))
    a = table.get(key)
    if a is None:
        a = table[(key[1], key[0])]
    return a in _effective_actions(b)


class TileMatchEnv(_EnvBase):
    metadata = {"render_modes": ["string", "human", "rgb_array"], "render_fps": 2}

    def __init__(self, num_rows: int, num_cols: int, num_colours: int, num_moves: int,
                 colourless_specials: List[str], colour_specials: List[str], seed: Optional[int] = 1,
                 render_mode: str = "string", device=None) -> None:
        self.num_rows, self.num_cols, self.num_colours = num_rows, num_cols, num_colours
        self.colourless_specials = colourless_specials
        self.colour_specials = colour_specials
        self.num_moves = num_moves
        self.renderer = None
        if render_mode == "string":   # gym.Env's lazily created unseeded generator (tile_match_env.py:37-38)
            self.colour_map = np.random.default_rng().choice(range(105, 230), size=self.num_colours + 1, replace=False)
        elif render_mode in ("human", "rgb_array"):
            raise NotImplementedError("pygame rendering is out of scope; use render_mode='string'")
        self.render_mode = render_mode
        self.num_colour_specials = len(self.colour_specials)
        self.num_colourless_specials = len(self.colourless_specials)
        self.seed = seed

        if device is None:
            if not torch.cuda.is_available():
                raise _native.TmgError("TileMatchEnv needs a HIP device (no CPU fallback)")
            device = torch.device("cuda", torch.cuda.current_device())
        self.device = torch.device(device)
        smask = _native.specials_mask(colourless_specials, colour_specials)
        self._ctx = _native.Context(self.device.index if self.device.index is not None else 0,
                                    num_rows, num_cols, num_colours, smask, num_moves)
        self.board = Board(num_rows, num_cols, num_colours, colourless_specials, colour_specials,
                           device=self.device, _env=self)
        self.board.rng_words = rng_words_from_seed(seed)                     # tile_match_env.py:49
        R, C = num_rows, num_cols
        obs_low = np.array([np.zeros((R, C), dtype=np.int32),
                            np.full((R, C), -self.num_colourless_specials, dtype=np.int32)])
        obs_high = np.array([np.full((R, C), self.num_colours, dtype=np.int32),
                             np.full((R, C), self.num_colour_specials + 2, dtype=np.int32)])
        self.num_actions = int((R * C * 2) - R - C)
        self._action_to_coords = self.board.action_to_coords
        self._board_observation_space = Box(low=obs_low, high=obs_high, shape=(2, R, C), dtype=np.int32, seed=self.seed)
        self._moves_left_observation_space = Discrete(self.num_moves + 1, seed=self.seed)
        self.observation_space = Dict({"board": self._board_observation_space,
                                       "num_moves_left": self._moves_left_observation_space})
        self.last_board = None
        self.timer = None
        self.action_space = Discrete(self.num_actions, seed=self.seed)
        self._coord_to_action = {c: a for a, c in enumerate(self._action_to_coords)}
        # device buffers for a batch of one
        kw = dict(device=self.device)
        self._d_board = torch.zeros((1, 2, R, C), dtype=torch.int8, **kw)
        self._d_rng = torch.zeros((1, 5), dtype=torch.int64, **kw)
        self._d_timer = torch.zeros(1, dtype=torch.int32, **kw)
        self._d_eff = torch.zeros((1, self._ctx.mask_words), dtype=torch.int64, **kw)
        self._d_out = torch.zeros((3, 1), dtype=torch.int32, **kw)
        self._d_flags = torch.zeros(1, dtype=torch.uint8, **kw)
        self._d_act = torch.zeros(1, dtype=torch.int32, **kw)

    # reference attribute: env.np_random is the board's generator (tile_match_env.py:51)
    @property
    def np_random(self):
        return self.board.np_random

    @np_random.setter
    def np_random(self, gen):
        self.board.np_random = gen

    def set_seed(self, seed: int) -> None:                                   # tile_match_env.py:79-82
        self.action_space.seed = seed
        self.observation_space.seed = seed
        self.board.np_random = np.random.default_rng(seed=seed)

    # ------------------------------------------------------------- device sync
    def _stream(self):
        return torch.cuda.current_stream(self.device).cuda_stream

    def _upload(self):
        b = self.board.board
        if b.shape != (2, self.num_rows, self.num_cols):
            raise ValueError("board has the wrong shape")
        self._d_board.copy_(torch.from_numpy(np.ascontiguousarray(b, dtype=np.int8)).unsqueeze(0))
        self._d_rng.copy_(torch.from_numpy(self.board.rng_words.view(np.int64)).unsqueeze(0))

    def _download(self):
        self.board.board = self._d_board[0].to(torch.int32).cpu().numpy()
        self.board.rng_words = self._d_rng[0].cpu().numpy().view(np.uint64).copy()

    def _eff_list(self) -> List[int]:
        w = self._d_eff[0].cpu().numpy().view(np.uint64)
        bits = np.unpackbits(w.view(np.uint8), bitorder="little")[:self.num_actions]
        return [int(a) for a in np.nonzero(bits)[0]]

    # ------------------------------------------------------------------- API
    def reset(self, seed: Optional[int] = None, options: Optional[dict] = None):   # tile_match_env.py:84-91
        if seed is not None:
            self.set_seed(seed)
        self._upload()
        self._ctx.reset(1, self._d_board.data_ptr(), self._d_rng.data_ptr(), self._d_timer.data_ptr(),
                        self._d_eff.data_ptr(), None, self._stream())
        self._download()
        self.timer = 0
        obs = self._get_obs()
        info = {"effective_actions": self._eff_list()}
        return obs, info

    def step(self, action: int):                                              # tile_match_env.py:93-112
        if self.timer is None or self.timer >= self.num_moves:
            raise Exception("You must call reset before calling step")
        coord1, coord2 = self._action_to_coords[action]
        a = self._coord_to_action[(coord1, coord2)]
        self._upload()
        self._d_timer.fill_(self.timer)
        self._d_act.fill_(a)
        out = self._d_out
        self._ctx.step(1, self._d_board.data_ptr(), self._d_rng.data_ptr(), self._d_timer.data_ptr(),
                       self._d_act.data_ptr(), out[0].data_ptr(), out[1].data_ptr(), out[2].data_ptr(),
                       self._d_flags.data_ptr(), self._d_eff.data_ptr(), 0, 0, self._stream())
        self._download()
        o = out[:, 0].cpu().numpy()
        flags = int(self._d_flags[0].item())
        if flags & (_native.FLAG_ERROR | _native.FLAG_OVERFLOW):
            raise _native.TmgError(f"device reported {'an error' if flags & _native.FLAG_ERROR else 'an overflow'} "
                                   "for this move")
        num_eliminations, num_new_specials, num_specials_activated = int(o[0]), int(o[1]), int(o[2])
        self.timer += 1
        done = self.timer == self.num_moves
        info = {
            "is_combination_match": bool(flags & _native.FLAG_COMBO),
            "num_new_specials": num_new_specials,
            "num_specials_activated": num_specials_activated,
            "shuffled": bool(flags & _native.FLAG_SHUFFLED),
            "effective_actions": [] if done else self._eff_list(),
        }
        next_obs = self._get_obs()
        return next_obs, num_eliminations, done, False, info

    def _get_obs(self):                                                       # tile_match_env.py:114-115
        return OrderedDict([("board", self.board.board.copy()), ("num_moves_left", self.num_moves - self.timer)])

    def _get_effective_actions(self) -> List[int]:                            # tile_match_env.py:118-124
        if self.timer == self.num_moves:
            return []
        self._upload()
        self._ctx.effective(1, self._d_board.data_ptr(), self._d_eff.data_ptr(), self._stream())
        return self._eff_list()

    def render(self):
        if self.render_mode == "string":                                      # tile_match_env.py:127-143
            color = lambda i, c: "\033[48;5;16m" + f"\033[38;5;{self.colour_map[i]}m{c}\033[0m"
            b = self.board.board
            print(" " + "-" * (b.shape[2] * 2 + 1))
            for r in range(b.shape[1]):
                print("| ", end="\033[48;5;16m")
                for c in range(b.shape[2]):
                    print(color(b[0, r, c], b[1, r, c]), end="\033[48;5;16m ")
                    print("\033[0m", end="")
                print("|", end="\n")
            print(" " + "-" * (b.shape[2] * 2 + 1))
        return None

    def close(self) -> None:
        self._ctx.close()
