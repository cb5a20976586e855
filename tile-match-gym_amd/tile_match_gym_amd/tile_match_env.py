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
    """Host view of the device board (mirror of board.py:41-93's public fields)."""

    def __init__(self, env: "TileMatchEnv", num_rows, num_cols, num_colours, colourless_specials, colour_specials):
        self._env = env
        self.num_rows, self.num_cols, self.num_colours = num_rows, num_cols, num_colours
        self.flat_size = num_rows * num_cols
        self.colourless_specials = colourless_specials
        self.colour_specials = colour_specials
        self.specials = set(list(colourless_specials) + list(colour_specials))
        self.num_actions = 2 * num_rows * num_cols - num_rows - num_cols
        self.action_to_coords = action_to_coords(num_rows, num_cols)
        self.board = np.ones((2, num_rows, num_cols), dtype=np.int32)
        self.rng_words = np.zeros(5, dtype=np.uint64)

    @property
    def np_random(self) -> np.random.Generator:
        return generator_from_words(self.rng_words)

    @np_random.setter
    def np_random(self, gen):
        self.rng_words = rng_words_from_generator(gen)


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
        self.board = Board(self, num_rows, num_cols, num_colours, colourless_specials, colour_specials)
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
