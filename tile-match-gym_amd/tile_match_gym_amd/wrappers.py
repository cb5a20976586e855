"""Observation / reward wrappers of the reference (src/tile_match_gym/wrappers.py),
with the one-hot encoding run by libtmg.so's `tmg_onehot` kernel.

* `OneHotWrapper(env)` — same constructor, attributes (`board_obs_space`,
  `observation_space`, `type_slices`, `num_type_slices`, ...) and observation
  layout as wrappers.py:17-69: channels = colours 1..k, then one channel per
  enabled special in the order cookie, v-laser, h-laser, bomb.  Like the
  reference it returns float64 arrays (wrappers.py:60 builds np.zeros).
* `ProportionRewardWrapper(env)` — reward / (R*C) (wrappers.py:71-77).
* `VecOneHot(vec_env, dtype=torch.float32)` — the batched form for
  `TileMatchVecEnv`: (N, channels, R, C) device tensors, no host round trip.

gymnasium is absent in this image; the wrappers keep gymnasium's
Wrapper surface (`env`, `unwrapped`, attribute pass-through, reset/step).
"""
from __future__ import annotations

from collections import OrderedDict

import numpy as np
import torch

from . import _native
from .spaces import Box, Dict

COLOURLESS_SPECIALS = {"cookie": -1}                                         # wrappers.py:9
COLOUR_SPECIALS = {"vertical_laser": 2, "horizontal_laser": 3, "bomb": 4}    # wrappers.py:10

_TORCH_DTYPES = {torch.float32: _native.DTYPE_F32, torch.uint8: _native.DTYPE_U8, torch.int32: _native.DTYPE_I32}


class _Wrapper:
    def __init__(self, env):
        self.env = env

    @property
    def unwrapped(self):
        e = self.env
        while isinstance(e, _Wrapper):
            e = e.env
        return e

    def __getattr__(self, name):
        if name.startswith("__"):
            raise AttributeError(name)
        return getattr(self.env, name)

    def close(self):
        return self.env.close()


def _type_slices(colourless_specials, colour_specials):
    """wrappers.py:37-46: the type-plane slices kept, as sorted(id + 1)."""
    glob = {**COLOURLESS_SPECIALS, **COLOUR_SPECIALS}
    ids = [idx for sp, idx in glob.items() if sp in colour_specials or sp in colourless_specials]
    return np.array(sorted(ids), dtype=np.int64) + len(COLOURLESS_SPECIALS)


class OneHotWrapper(_Wrapper):
    """wrappers.py:17-69 for the single env (TileMatchEnv)."""

    def __init__(self, env):
        super().__init__(env)
        u = self.unwrapped
        self.num_colours = u.num_colours
        self.num_colour_specials = u.num_colour_specials
        self.num_colourless_specials = u.num_colourless_specials
        self.num_rows = u.num_rows
        self.num_cols = u.num_cols
        self.board_obs_space = Box(low=0, high=1, dtype=np.int32,
                                   shape=(self.num_colours + self.num_colour_specials + self.num_colourless_specials,
                                          self.num_rows, self.num_cols))
        self.observation_space = Dict({"board": self.board_obs_space,
                                       "num_moves_left": u._moves_left_observation_space})
        self.colour_specials = u.colour_specials
        self.colourless_specials = u.colourless_specials
        self.global_num_colourless_specials = len(COLOURLESS_SPECIALS)
        self.global_num_colour_specials = len(COLOUR_SPECIALS)
        self._global_specials = {**COLOURLESS_SPECIALS, **COLOUR_SPECIALS}
        self.type_slices = _type_slices(self.colourless_specials, self.colour_specials)
        self.num_type_slices = len(self.type_slices)
        self._ctx = u._ctx
        ch = self._ctx.onehot_channels()
        self._d_out = torch.zeros((1, ch, self.num_rows, self.num_cols), dtype=torch.float32, device=u.device)

    def reset(self, seed=None, options=None):
        obs, info = self.env.reset(seed=seed, options=options)
        return self.observation(obs), info

    def step(self, action):
        obs, reward, done, truncated, info = self.env.step(action)
        return self.observation(obs), reward, done, truncated, info

    def observation(self, obs) -> dict:                                      # wrappers.py:50-53
        return OrderedDict([("board", self._one_hot_encode_board(obs["board"])),
                            ("num_moves_left", obs["num_moves_left"])])

    def _one_hot_encode_board(self, board: np.ndarray) -> np.ndarray:        # wrappers.py:56-69
        u = self.unwrapped
        d = torch.from_numpy(np.ascontiguousarray(board, dtype=np.int8)).to(u.device).reshape(1, 2, self.num_rows,
                                                                                               self.num_cols)
        self._ctx.onehot(1, d.data_ptr(), self._d_out.data_ptr(), _native.DTYPE_F32,
                         torch.cuda.current_stream(u.device).cuda_stream)
        return self._d_out[0].cpu().numpy().astype(np.float64)


class ProportionRewardWrapper(_Wrapper):
    """wrappers.py:71-77: reward as a fraction of the board size."""

    def __init__(self, env):
        super().__init__(env)
        self.flat_size = self.unwrapped.num_rows * self.unwrapped.num_cols

    def reset(self, seed=None, options=None):
        return self.env.reset(seed=seed, options=options)

    def step(self, action):
        obs, reward, done, truncated, info = self.env.step(action)
        return obs, self.reward(reward), done, truncated, info

    def reward(self, reward):
        return reward / self.flat_size


class VecOneHot:
    """One-hot boards of a TileMatchVecEnv: `encode()` -> (N, channels, R, C) on the env's device.

    fused=True: the planes are kept by the step / reset kernels themselves
    (TileMatchVecEnv.attach_onehot -> tmg_step_onehot), rewritten only for
    the boards a step changes; `encode()` then just returns them."""

    def __init__(self, vec_env, dtype=torch.float32, fused=False):
        if dtype not in _TORCH_DTYPES:
            raise ValueError(f"dtype must be one of {list(_TORCH_DTYPES)}")
        self.env = vec_env
        self.dtype = dtype
        self.fused = bool(fused)
        self.channels = vec_env.ctx.onehot_channels()
        self.type_slices = _type_slices(vec_env.colourless_specials, vec_env.colour_specials)
        if self.fused:
            self.out = vec_env.attach_onehot(dtype)
        else:
            self.out = torch.empty((vec_env.num_envs, self.channels, vec_env.num_rows, vec_env.num_cols),
                                   dtype=dtype, device=vec_env.device)

    def encode(self, board=None) -> torch.Tensor:
        if self.fused and board is None:
            self.env.join()
            return self.out
        b = self.env.board if board is None else board
        if b.dtype != torch.int8 or not b.is_contiguous() or b.shape != self.env.board.shape:
            raise ValueError("board must be a contiguous int8 (N, 2, R, C) tensor")
        self.env.ctx.onehot(self.env.num_envs, b.data_ptr(), self.out.data_ptr(), _TORCH_DTYPES[self.dtype],
                            torch.cuda.current_stream(self.env.device).cuda_stream)
        return self.out
